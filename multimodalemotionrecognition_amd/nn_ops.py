"""Autograd-aware building blocks (Linear / ReLU+Dropout) on the fp32 HIP kernels, for the small
classifier heads of ``VideoNet`` / ``WavLMAudioEncoder`` (video.py:30-44, wavlm_audio.py:49-56)."""
from __future__ import annotations

import torch

from . import kernels as K


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        out = torch.empty(x2.shape[0], w.shape[0], device=x.device, dtype=torch.float32)
        K.linear_fwd(x2, w, b, out, act=act)
        ctx.save_for_backward(x2, w, out)
        ctx.act, ctx.shape, ctx.bias = act, x.shape, b
        return out.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from .fusion import grad_buffer

        x2, w, out = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous().float()
        if ctx.act == "relu":
            dy2 = dy2.clone()
            K.relu_dropout_bwd_(dy2, out, 0.0, None)
        elif ctx.act != "none":
            raise NotImplementedError(ctx.act)
        dx = torch.empty(x2.shape, device=dy.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        dw = grad_buffer(w) if ctx.needs_input_grad[1] else None
        db = grad_buffer(ctx.bias) if ctx.needs_input_grad[2] else None
        K.linear_bwd(x2, w, dy2, dx=dx, dw=dw, db=db)
        return (dx.view(ctx.shape) if dx is not None else None), dw, db, None


def hip_linear(x: torch.Tensor, layer: torch.nn.Linear, act: str = "none") -> torch.Tensor:
    return _LinearFn.apply(x, layer.weight, layer.bias, act)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, rng):
        y = x.contiguous().clone()
        K.dropout_(y.view(-1, y.shape[-1]), p, rng)
        ctx.p, ctx.rng = p, rng
        return y

    @staticmethod
    def backward(ctx, dy):
        g = dy.contiguous().clone()
        K.dropout_(g.view(-1, g.shape[-1]), ctx.p, ctx.rng)  # same (base, index) -> same mask and scale
        return g, None, None


def draw_seed(p: float, training: bool):
    """The host seed ``hip_dropout(x, p, training)`` would draw (None when it draws nothing)."""
    if not training or p <= 0:
        return None
    return int(torch.randint(0, 2 ** 62, (1,)).item())  # host draw: torch.manual_seed reproduces it


def hip_dropout(x: torch.Tensor, p: float, training: bool, seed=None) -> torch.Tensor:
    """``seed``: drawn ahead by ``draw_seed`` (same draw, earlier), else drawn here."""
    if not training or p <= 0:
        return x
    seed = draw_seed(p, training) if seed is None else seed
    rng = torch.full((1,), seed, dtype=torch.int64, device=x.device)  # a fill kernel: no host buffer in flight
    return _DropoutFn.apply(x, p, rng)
