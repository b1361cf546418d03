"""fp32 CPU restatement of the ResNet18 frame trunk used as ``VideoNet.backbone``.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

``src/models/video.py:21-23`` wraps torchvision's ``resnet18`` (0.25.0 per
``uv.lock``) as ``nn.Sequential(*children[:-1])``: indices 0 conv1, 1 bn1, 2 relu,
3 maxpool, 4..7 layer1..4, 8 avgpool -> ``[N,512,1,1]``.  torchvision is absent in
this image, so this restatement of its published topology (BasicBlock [2,2,2,2],
conv 7x7/2 + maxpool 3/2, 1x1/2 downsample + BN) is **parity unpinned**: it is
checked structurally (parameter count 11,176,512 and output shape) only.

BatchNorm is restated for both modes: train mode normalises with the batch
statistics and updates running stats in place (momentum 0.1, unbiased var).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

STAGES = ((64, 1), (128, 2), (256, 2), (512, 2))


def param_shapes(prefix: str = "backbone.") -> List[Tuple[str, Tuple[int, ...]]]:
    out = [(prefix + "0.weight", (64, 3, 7, 7))]
    out += _bn(prefix + "1.", 64)
    cin = 64
    for si, (c, stride) in enumerate(STAGES):
        for bi in range(2):
            n = f"{prefix}{4 + si}.{bi}."
            s = stride if bi == 0 else 1
            out.append((n + "conv1.weight", (c, cin, 3, 3)))
            out += _bn(n + "bn1.", c)
            out.append((n + "conv2.weight", (c, c, 3, 3)))
            out += _bn(n + "bn2.", c)
            if bi == 0 and (s != 1 or cin != c):
                out.append((n + "downsample.0.weight", (c, cin, 1, 1)))
                out += _bn(n + "downsample.1.", c)
            cin = c
    return out


def _bn(n: str, c: int):
    return [(n + "weight", (c,)), (n + "bias", (c,)), (n + "running_mean", (c,)),
            (n + "running_var", (c,)), (n + "num_batches_tracked", ())]


def batch_norm(x: Tensor, p: Dict[str, Tensor], n: str, training: bool) -> Tensor:
    """nn.BatchNorm2d (momentum 0.1): train mode normalises with batch stats, updates the running
    stats (unbiased var) and counts the batch in ``num_batches_tracked``; eval uses running stats."""
    if training and (n + "num_batches_tracked") in p:
        with torch.no_grad():
            p[n + "num_batches_tracked"].add_(1)
    return F.batch_norm(x, p[n + "running_mean"], p[n + "running_var"], p[n + "weight"], p[n + "bias"],
                        training=training, momentum=0.1, eps=1e-5)


def basic_block(x: Tensor, p: Dict[str, Tensor], n: str, stride: int, training: bool) -> Tensor:
    out = F.conv2d(x, p[n + "conv1.weight"], stride=stride, padding=1)
    out = F.relu(batch_norm(out, p, n + "bn1.", training))
    out = F.conv2d(out, p[n + "conv2.weight"], stride=1, padding=1)
    out = batch_norm(out, p, n + "bn2.", training)
    if (n + "downsample.0.weight") in p:
        idt = F.conv2d(x, p[n + "downsample.0.weight"], stride=stride)
        idt = batch_norm(idt, p, n + "downsample.1.", training)
    else:
        idt = x
    return F.relu(out + idt)


def resnet18_trunk(p: Dict[str, Tensor], x: Tensor, training: bool, prefix: str = "backbone.") -> Tensor:
    """``[N,3,H,W] -> [N,512,1,1]``; in train mode BN running stats in ``p`` are updated in place."""
    x = F.conv2d(x, p[prefix + "0.weight"], stride=2, padding=3)
    x = F.relu(batch_norm(x, p, prefix + "1.", training))
    x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
    for si, (_, stride) in enumerate(STAGES):
        for bi in range(2):
            x = basic_block(x, p, f"{prefix}{4 + si}.{bi}.", stride if bi == 0 else 1, training)
    return F.adaptive_avg_pool2d(x, (1, 1))
