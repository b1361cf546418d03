"""``TemporalPooler`` mirror (``src/models/temporal.py``): same constructor, submodule names and
state-dict keys.  All three modes run on the HIP kernels: 'mean' (``mer_mean_pool_fwd``, the fusion
default), 'attn' and 'transformer' through the explicit schedules of ``temporal_hip.py`` (one autograd
node per pooler).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import kernels as K
from . import temporal_hip as TH


class TemporalAttentionPooling(nn.Module):
    def __init__(self, dim: int, dropout: float = 0.1) -> None:
        super().__init__()
        hidden_dim = max(1, dim // 2)
        self.score = nn.Sequential(nn.LayerNorm(dim), nn.Linear(dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                   nn.Linear(hidden_dim, 1))


class SinusoidalPositionalEncoding(nn.Module):
    def __init__(self, dim: int, max_len: int = 4096) -> None:
        super().__init__()
        position = torch.arange(max_len).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, dim, 2) * (-math.log(10000.0) / max(1, dim)))
        pe = torch.zeros(max_len, dim)
        pe[:, 0::2] = torch.sin(position * div_term)
        if dim > 1:
            pe[:, 1::2] = torch.cos(position * div_term[: pe[:, 1::2].shape[1]])
        self.register_buffer("pe", pe.unsqueeze(0), persistent=False)


class TemporalTransformerPooling(nn.Module):
    def __init__(self, dim: int, num_heads: int = 4, num_layers: int = 1, dropout: float = 0.1,
                 mlp_ratio: float = 4.0) -> None:
        super().__init__()
        ffn_dim = max(dim * 2, int(dim * mlp_ratio))
        layer = nn.TransformerEncoderLayer(d_model=dim, nhead=num_heads, dim_feedforward=ffn_dim, dropout=dropout,
                                           activation="gelu", batch_first=True, norm_first=True)
        self.pos_encoding = SinusoidalPositionalEncoding(dim)
        self.encoder = nn.TransformerEncoder(layer, num_layers=num_layers, enable_nested_tensor=False)
        self.pool = TemporalAttentionPooling(dim=dim, dropout=dropout)


class _MeanPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous().float()
        B, L, D = x.shape
        y = torch.empty(B, D, device=x.device, dtype=torch.float32)
        K.mean_pool_fwd(x, y)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty(ctx.shape, device=dy.device, dtype=torch.float32)
        K.mean_pool_bwd(dy.contiguous().float(), dx)
        return dx


class _PoolFn(torch.autograd.Function):
    """'attn' / 'transformer' pooling of x [B, L, D] on the HIP schedule (temporal_hip.py)."""

    @staticmethod
    def forward(ctx, x, pooler, training, rng, names, *params):
        from .fusion import grad_buffer  # noqa: F401  (imported for backward)

        x = x.contiguous().float()
        B, L, D = x.shape
        p = dict(zip(names, params))
        y = torch.empty(B, D, device=x.device, dtype=torch.float32)
        ctx.pctx = TH.pool_forward(p, "pool", pooler.mode, x, y, num_heads=pooler.num_heads,
                                   num_layers=pooler.num_layers, dropout=pooler.dropout if training else 0.0, rng=rng)
        ctx.names, ctx.params = names, params
        return y

    @staticmethod
    def backward(ctx, dy):
        from .fusion import grad_buffer

        p = dict(zip(ctx.names, ctx.params))
        grads = {n: grad_buffer(t) for n, t in p.items() if t.requires_grad}
        dx = TH.pool_backward(p, "pool", ctx.pctx, dy.contiguous().float(), grads)
        return (dx, None, None, None, None, *[grads.get(n) for n in ctx.names])


class TemporalPooler(nn.Module):
    """Configurable temporal aggregation: mean, attention, or transformer (temporal.py:78-110)."""

    def __init__(self, dim: int, mode: str = "mean", num_heads: int = 4, num_layers: int = 1,
                 dropout: float = 0.1) -> None:
        super().__init__()
        self.mode = mode
        self.num_heads, self.num_layers, self.dropout = num_heads, num_layers, float(dropout)
        if mode == "mean":
            self.pool = None
        elif mode == "attn":
            self.pool = TemporalAttentionPooling(dim=dim, dropout=dropout)
        elif mode == "transformer":
            self.pool = TemporalTransformerPooling(dim=dim, num_heads=num_heads, num_layers=num_layers, dropout=dropout)
        else:
            raise ValueError(f"Unsupported temporal pooling mode: {mode}")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.ndim != 3:
            raise ValueError(f"TemporalPooler expects [B, T, D], got shape={tuple(x.shape)}")
        if self.pool is None:
            if not x.is_cuda:
                raise RuntimeError("TemporalPooler runs on the MI355X kernels; move the input to the GPU")
            return _MeanPoolFn.apply(x)
        if not x.is_cuda:
            raise RuntimeError("TemporalPooler runs on the MI355X kernels; move the input to the GPU")
        names, params = zip(*self.named_parameters())
        rng = None
        if self.training and self.dropout > 0:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())  # host draw: torch.manual_seed reproduces it
            rng = torch.full((1,), seed, dtype=torch.int64, device=x.device)
        return _PoolFn.apply(x, self, self.training, rng, tuple(names), *params)
