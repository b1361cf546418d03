"""Loss modules of the train step (``src/train.py:1030-1033`` and ``212-225``) on the HIP kernels."""
from __future__ import annotations

import torch
from torch import nn

from . import kernels as K


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, label_smoothing, late):
        logits = logits.contiguous().float()
        loss = torch.empty((), device=logits.device, dtype=torch.float32)
        dlogits = torch.empty_like(logits)
        preds = torch.empty(logits.shape[0], device=logits.device, dtype=torch.int64)
        K.cross_entropy(logits, labels.contiguous(), loss, dlogits, label_smoothing, late, preds=preds)
        ctx.save_for_backward(dlogits)
        ctx.mark_non_differentiable(preds)
        return loss, preds

    @staticmethod
    def backward(ctx, gloss, gpreds=None):
        (dlogits,) = ctx.saved_tensors
        out = torch.empty_like(dlogits)
        K.scale_dev(dlogits, gloss.contiguous().float().reshape(1), out)
        return out, None, None, None


class CrossEntropyLoss(nn.Module):
    """``nn.CrossEntropyLoss(label_smoothing=...)`` with mean reduction (train.py:1033).  The same kernel writes
    the rows' top-1 indices (``outputs.argmax(dim=1)``, train.py:220) to ``last_preds``."""

    def __init__(self, label_smoothing: float = 0.0) -> None:
        super().__init__()
        self.label_smoothing = float(label_smoothing)
        self.last_preds = None

    def forward(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        loss, self.last_preds = _CEFn.apply(logits, labels, self.label_smoothing, False)
        return loss


class LateNLLLoss(nn.Module):
    """late-mode loss ``NLLLoss()(log(probs + 1e-8), labels)`` (train.py:1031, 212-214), given probabilities;
    ``last_preds`` = ``outputs.argmax(dim=1)`` (train.py:216)."""

    def __init__(self) -> None:
        super().__init__()
        self.last_preds = None

    def forward(self, probs: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        loss, self.last_preds = _CEFn.apply(probs, labels, 0.0, True)
        return loss


class _AddScaledFn(torch.autograd.Function):
    """out = x + w * y over 0-d device losses (train.py:225: cls_loss + fusion_align_weight * align_loss)."""

    @staticmethod
    def forward(ctx, x, y, w):
        out = torch.empty((), device=x.device, dtype=torch.float32)
        K.add_scaled_scalar(x.contiguous().float(), y.contiguous().float(), w, out)
        ctx.w = float(w)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().float().reshape(())
        gy = torch.empty((), device=g.device, dtype=torch.float32)
        zero = torch.zeros((), device=g.device, dtype=torch.float32)
        K.add_scaled_scalar(zero, g, ctx.w, gy)  # d/dy = w * g
        return g, gy, None


def add_scaled(x: torch.Tensor, y: torch.Tensor, w: float) -> torch.Tensor:
    return _AddScaledFn.apply(x, y, float(w))
