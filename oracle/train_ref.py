"""fp32 CPU restatement of one xattn train step (``src/train.py:200-228``).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Step = zero_grad -> FusionModel.forward (ResNet18 trunk in train-mode BN, frozen
WavLM under no_grad, xattn head) -> CrossEntropyLoss -> backward -> Adam
(``torch.optim.Adam(lr, weight_decay)``, L2-style decay added to the gradient,
``train.py:902``).  Only parameters that receive a gradient are updated (torch's
Adam skips ``grad is None``): the ResNet18 trunk and the used head parameters.
Dropout / drop-path are identity here (deterministic variant).
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch

from . import fusion_ref, resnet18_ref, wavlm_ref

Tensor = torch.Tensor


def model_forward(p: Dict[str, Tensor], video: Tensor, audio: Tensor, *, num_heads: int = 4,
                  xattn_head: str = "concat", use_prior: bool = False, bn_training: bool = True):
    """``FusionModel.forward`` xattn branch end to end (fusion.py:366-411)."""
    b, t, c, h, w = video.shape
    vf = resnet18_ref.resnet18_trunk(p, video.reshape(b * t, c, h, w), bn_training,
                                     prefix="video_model.backbone.").reshape(b, t, -1)
    with torch.no_grad():
        a_seq = wavlm_ref.wavlm_forward(p, audio, prefix="audio_model.wavlm.")
    logits, _ = fusion_ref.xattn_forward(p, vf, a_seq, num_heads=num_heads, xattn_head=xattn_head,
                                         use_prior=use_prior)
    return logits


class AdamRef:
    """Restatement of ``torch.optim.Adam`` (single-tensor path, amsgrad=False, maximize=False): per-parameter
    step counts (``state[p]['step']``), parameters whose ``.grad`` is None untouched."""

    def __init__(self, params: List[Tensor], lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        self.params = params
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, weight_decay
        self.steps = [0] * len(params)
        self.m = [torch.zeros_like(q) for q in params]
        self.v = [torch.zeros_like(q) for q in params]

    @torch.no_grad()
    def step(self) -> None:
        for i, (q, m, v) in enumerate(zip(self.params, self.m, self.v)):
            if q.grad is None:
                continue
            self.steps[i] += 1
            t = self.steps[i]
            bc1 = 1.0 - self.b1 ** t
            bc2 = 1.0 - self.b2 ** t
            g = q.grad + self.wd * q
            m.mul_(self.b1).add_(g, alpha=1.0 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1.0 - self.b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            q.addcdiv_(m, denom, value=-self.lr / bc1)


def train_step(p: Dict[str, Tensor], trainable: List[str], opt: AdamRef, video: Tensor, audio: Tensor,
               labels: Tensor, **kw) -> float:
    for n in trainable:
        p[n].grad = None
    logits = model_forward(p, video, audio, **kw)
    loss = fusion_ref.cross_entropy(logits, labels)
    loss.backward()
    opt.step()
    return float(loss.detach())
