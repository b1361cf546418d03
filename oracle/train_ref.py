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


def encoders_forward(p: Dict[str, Tensor], video: Tensor, audio: Tensor, bn_training: bool = True):
    """The two encoders' outputs: ResNet18 frame features ``[B, T, 512]`` (video.py:21-23 via ``backbone``) and the
    frozen WavLM hidden states ``[B, Ta, 768]`` (wavlm_audio.py:165-183, eval semantics, no grad)."""
    b, t, c, h, w = video.shape
    vf = resnet18_ref.resnet18_trunk(p, video.reshape(b * t, c, h, w), bn_training,
                                     prefix="video_model.backbone.").reshape(b, t, -1)
    with torch.no_grad():
        hidden = wavlm_ref.wavlm_forward(p, audio, prefix="audio_model.wavlm.")
    return vf, hidden


def audio_encode(p: Dict[str, Tensor], hidden: Tensor, embedding_dim: int = 768) -> Tensor:
    """``WavLMAudioEncoder.encode`` after ``encode_sequence`` (wavlm_audio.py:146-163): mean temporal pooling, then
    ``classifier[0]`` only when the pooled width differs from ``embedding_dim`` (not for WavLM-base: 768)."""
    a_emb = hidden.mean(dim=1)
    if a_emb.shape[-1] != embedding_dim:
        a_emb = fusion_ref.linear(a_emb, p, "audio_model.classifier.0")
    return a_emb


def video_encode(vf: Tensor) -> Tensor:
    """``VideoNet.encode`` after the backbone (video.py:34-40): mean temporal pooling of the frame features."""
    return vf.mean(dim=1)


def embedding_model_forward(p: Dict[str, Tensor], mode: str, video: Tensor, audio: Tensor,
                            bn_training: bool = True, return_embeddings: bool = False):
    """``FusionModel.forward`` for the non-xattn modes with the real encoders:

    * ``late`` (fusion.py:358-363): mean of the softmaxes of ``WavLMAudioEncoder.forward`` (wavlm_audio.py:121-144:
      pool, classifier Linear-ReLU-Dropout-Linear) and ``VideoNet.forward`` (video.py:42-44: encode, Linear) --
      probabilities;
    * ``concat`` / ``gated`` (fusion.py:413-435): ``encode`` of both encoders, then the projection + MLP / gate head
      (dropouts and ModalityDropout identity: the deterministic variant)."""
    vf, hidden = encoders_forward(p, video, audio, bn_training)
    a_emb, v_emb = audio_encode(p, hidden), video_encode(vf)
    if mode == "late":
        h = torch.relu(fusion_ref.linear(hidden.mean(dim=1), p, "audio_model.classifier.0"))
        a_logits = fusion_ref.linear(h, p, "audio_model.classifier.3")
        v_logits = fusion_ref.linear(v_emb, p, "video_model.classifier")
        out = fusion_ref.late_forward(a_logits, v_logits)
    else:
        out = fusion_ref.embedding_fusion_forward(p, mode, a_emb, v_emb)
    return (out, a_emb, v_emb) if return_embeddings else out


def train_step_mode(p: Dict[str, Tensor], trainable: List[str], opt: AdamRef, mode: str, video: Tensor,
                    audio: Tensor, labels: Tensor) -> float:
    """One train step (train.py:200-228) of a non-xattn model: CE, or late NLL(log(p + 1e-8))."""
    for n in trainable:
        p[n].grad = None
    out = embedding_model_forward(p, mode, video, audio)
    loss = fusion_ref.late_nll(out, labels) if mode == "late" else fusion_ref.cross_entropy(out, labels)
    loss.backward()
    opt.step()
    return float(loss.detach())
