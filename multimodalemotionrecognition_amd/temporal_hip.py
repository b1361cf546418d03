"""HIP schedule of ``TemporalPooler`` 'attn' and 'transformer' (src/models/temporal.py:9-110).

* attn (``TemporalAttentionPooling``, temporal.py:9-26): LayerNorm -> Linear(D, D/2) -> GELU -> Dropout
  -> Linear(D/2, 1) -> softmax over time -> weighted sum of the UN-normalised input.
* transformer (``TemporalTransformerPooling``, temporal.py:46-75): x + sinusoidal PE, then ``num_layers``
  pre-LN ``nn.TransformerEncoderLayer`` (norm_first=True, GELU, dim_feedforward=max(2D, 4D)):
  x = x + drop(SA(LN1(x)));  x = x + drop(FF(LN2(x))),  FF = Linear2(drop(gelu(Linear1(.)))),
  then the attention pooling above.

Explicit forward/backward schedules over the fp32 kernels (GEMM on f32 MFMA, LayerNorm, the MFMA MHA
core, GELU/dropout, residual add, attention-pool softmax); parameter gradients accumulate into
caller-provided buffers (``grads[name]``, e.g. FusedAdam's flat-buffer views).  Parameter names are the
reference's state-dict names under ``prefix`` (e.g. ``v_temporal_pool.pool``).
Dropout masks come from the step's device RNG base (``rng``) and constant sites ``site0 + k``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

from . import kernels as K


@dataclass
class PoolCtx:
    mode: str
    saved: Dict[str, object] = field(default_factory=dict)


def _e(shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


def param_names(prefix: str, mode: str, num_layers: int = 1):
    """State-dict names of a pooler's parameters (``prefix`` = '<TemporalPooler>.pool')."""
    def attn(pfx):
        return [f"{pfx}.score.0.weight", f"{pfx}.score.0.bias", f"{pfx}.score.1.weight", f"{pfx}.score.1.bias",
                f"{pfx}.score.4.weight", f"{pfx}.score.4.bias"]
    if mode == "attn":
        return attn(prefix)
    names = []
    for i in range(num_layers):
        ln = f"{prefix}.encoder.layers.{i}"
        names += [f"{ln}.self_attn.in_proj_weight", f"{ln}.self_attn.in_proj_bias", f"{ln}.self_attn.out_proj.weight",
                  f"{ln}.self_attn.out_proj.bias", f"{ln}.linear1.weight", f"{ln}.linear1.bias",
                  f"{ln}.linear2.weight", f"{ln}.linear2.bias", f"{ln}.norm1.weight", f"{ln}.norm1.bias",
                  f"{ln}.norm2.weight", f"{ln}.norm2.bias"]
    return names + attn(prefix + ".pool")


# ---------------------------------------------------------------------------------------------
# attention pooling
# ---------------------------------------------------------------------------------------------
def _attn_pool_fwd(p, pfx, x3, out, ldo, drop, rng, site):
    B, L, D = x3.shape
    rows = B * L
    x2 = x3.reshape(rows, D)
    h, mu, rs = _e((rows, D), x2), _e((rows,), x2), _e((rows,), x2)
    K.add_ln_fwd(x2, None, p[pfx + ".score.0.weight"], p[pfx + ".score.0.bias"], h, None, mu, rs, L)
    w1 = p[pfx + ".score.1.weight"]
    z = K.linear_fwd(h, w1, p[pfx + ".score.1.bias"], _e((rows, w1.shape[0]), x2))
    g = K.gelu_dropout_fwd(z, _e(z.shape, x2), drop, rng, site)
    sc = K.linear_fwd(g, p[pfx + ".score.4.weight"], p[pfx + ".score.4.bias"], _e((rows, 1), x2))
    attn = _e((B, L), x2)
    K.attn_pool_fwd(x3, sc, attn, out, ldo)
    return dict(x3=x3, h=h, mu=mu, rs=rs, z=z, g=g, attn=attn)


def _attn_pool_bwd(p, pfx, sv, dy, grads, drop, rng, site):
    x3 = sv["x3"]
    B, L, D = x3.shape
    rows = B * L
    dx = _e((B, L, D), x3)
    ds = _e((rows, 1), x3)
    K.attn_pool_bwd(x3, sv["attn"], dy, dx, ds)
    g, z, h = sv["g"], sv["z"], sv["h"]
    dg = _e(g.shape, x3)
    K.linear_bwd(g, p[pfx + ".score.4.weight"], ds, dx=dg, dw=grads.get(pfx + ".score.4.weight"),
                 db=grads.get(pfx + ".score.4.bias"))
    dz = K.gelu_dropout_bwd(dg, z, _e(z.shape, x3), drop, rng, site)
    dh = _e((rows, D), x3)
    K.linear_bwd(h, p[pfx + ".score.1.weight"], dz, dx=dh, dw=grads.get(pfx + ".score.1.weight"),
                 db=grads.get(pfx + ".score.1.bias"))
    dxl = _e((rows, D), x3)
    K.add_ln_bwd(dh, x3.reshape(rows, D), sv["mu"], sv["rs"], p[pfx + ".score.0.weight"], dxl, None,
                 grads.get(pfx + ".score.0.weight"), grads.get(pfx + ".score.0.bias"), L)
    dx2 = dx.view(rows, D)
    K.add_dropout(dx2, dxl, dx2)
    return dx


# ---------------------------------------------------------------------------------------------
# multi-head self-attention with a materialised-score backward for long sequences
# ---------------------------------------------------------------------------------------------
def _mha_bwd(q, k, v, P, do, dq, dk, dv, B, H, L, drop, rng, site):
    dh = do.shape[1] // H
    # the fused kernel's LDS image must fit in 160 KiB (mer.h mer_mha_bwd)
    if fused_mha_ok(L, dh) and K.mha_bwd_lds_bytes(L, L, dh) <= 160 * 1024:
        K.mha_bwd(q, k, v, P, do, dq, dk, dv, None, B, H, L, L, drop, rng, site)
        return
    scale = dh ** -0.5
    dpp, ds, pd = _e((B, L, L), q), _e((B, L, L), q), _e((B, L, L), q)
    sc = torch.full((1,), scale, device=q.device, dtype=torch.float32)
    for h in range(H):
        o = h * dh
        K.gemm_batched(do[:, o:], v[:, o:], dpp, M=L, N=L, K=dh, sam=do.stride(0), sak=1, bsa=L * do.stride(0),
                       sbk=1, sbn=v.stride(0), bsb=L * v.stride(0), ldc=L, bsc=L * L, batch=B)
        K.softmax_dropout_bwd(P, dpp, ds, pd, h, drop, rng, site)
        K.scale_dev(ds, sc, ds)
        K.gemm_batched(ds, k[:, o:], dq[:, o:], M=L, N=dh, K=L, sam=L, sak=1, bsa=L * L, sbk=k.stride(0), sbn=1,
                       bsb=L * k.stride(0), ldc=dq.stride(0), bsc=L * dq.stride(0), batch=B)
        K.gemm_batched(ds, q[:, o:], dk[:, o:], M=L, N=dh, K=L, sam=1, sak=L, bsa=L * L, sbk=q.stride(0), sbn=1,
                       bsb=L * q.stride(0), ldc=dk.stride(0), bsc=L * dk.stride(0), batch=B)
        K.gemm_batched(pd, do[:, o:], dv[:, o:], M=L, N=dh, K=L, sam=1, sak=L, bsa=L * L, sbk=do.stride(0), sbn=1,
                       bsb=L * do.stride(0), ldc=dv.stride(0), bsc=L * dv.stride(0), batch=B)


def fused_mha_ok(L: int, dh: int) -> bool:
    """Shapes the fused MFMA MHA kernels (attn.hip) take: head_dim % 4 == 0, <= 64, L <= 256."""
    return dh % 4 == 0 and dh <= 64 and L <= 256


def _mha_fwd(q, k, v, o, P, B, H, L, drop, rng, site):
    """Self-attention core; the materialised-score path (batched f32 MFMA GEMMs + a softmax/dropout pass per head)
    for head widths > 64 -- the encoders' transformer pooling (512 / 768 wide, 4 heads: head_dim 128 / 192)."""
    D = o.shape[1]
    dh = D // H
    if fused_mha_ok(L, dh):
        K.mha_fwd(q, k, v, None, o, P, B, H, L, L, drop, rng, site)
        return
    S, Pd = _e((B, L, L), q), _e((B, L, L), q)
    for h in range(H):
        c = h * dh
        K.gemm_batched(q[:, c:], k[:, c:], S, M=L, N=L, K=dh, sam=q.stride(0), sak=1, bsa=L * q.stride(0),
                       sbk=1, sbn=k.stride(0), bsb=L * k.stride(0), ldc=L, bsc=L * L, batch=B)
        K.softmax_dropout_fwd(S, dh ** -0.5, P, Pd, h, drop, rng, site)
        K.gemm_batched(Pd, v[:, c:], o[:, c:], M=L, N=dh, K=L, sam=L, sak=1, bsa=L * L, sbk=v.stride(0), sbn=1,
                       bsb=L * v.stride(0), ldc=o.stride(0), bsc=L * o.stride(0), batch=B)


# ---------------------------------------------------------------------------------------------
# transformer pooling
# ---------------------------------------------------------------------------------------------
def _layer_fwd(p, ln, x, B, L, H, drop, rng, site):
    rows, D = x.shape
    sv = {"x": x}
    h1, m1, r1 = _e((rows, D), x), _e((rows,), x), _e((rows,), x)
    K.add_ln_fwd(x, None, p[ln + ".norm1.weight"], p[ln + ".norm1.bias"], h1, None, m1, r1, L)
    qkv = K.linear_fwd(h1, p[ln + ".self_attn.in_proj_weight"], p[ln + ".self_attn.in_proj_bias"], _e((rows, 3 * D), x))
    o, P = _e((rows, D), x), _e((B, H, L, L), x)
    _mha_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, P, B, H, L, drop, rng, site)
    sa = K.linear_fwd(o, p[ln + ".self_attn.out_proj.weight"], p[ln + ".self_attn.out_proj.bias"], _e((rows, D), x))
    x1 = K.add_dropout(x, sa, _e((rows, D), x), None, drop, rng, site + 1)
    h2, m2, r2 = _e((rows, D), x), _e((rows,), x), _e((rows,), x)
    K.add_ln_fwd(x1, None, p[ln + ".norm2.weight"], p[ln + ".norm2.bias"], h2, None, m2, r2, L)
    w1 = p[ln + ".linear1.weight"]
    z = K.linear_fwd(h2, w1, p[ln + ".linear1.bias"], _e((rows, w1.shape[0]), x))
    g = K.gelu_dropout_fwd(z, _e(z.shape, x), drop, rng, site + 2)
    f = K.linear_fwd(g, p[ln + ".linear2.weight"], p[ln + ".linear2.bias"], _e((rows, D), x))
    x2 = K.add_dropout(x1, f, _e((rows, D), x), None, drop, rng, site + 3)
    sv.update(h1=h1, m1=m1, r1=r1, qkv=qkv, o=o, P=P, x1=x1, h2=h2, m2=m2, r2=r2, z=z, g=g)
    return x2, sv


def _layer_bwd(p, ln, sv, dx2, grads, B, L, H, drop, rng, site):
    rows, D = dx2.shape
    gr = grads.get
    df = dx2.clone()
    K.dropout_(df, drop, rng, site + 3)
    g, z = sv["g"], sv["z"]
    dg = _e(g.shape, dx2)
    K.linear_bwd(g, p[ln + ".linear2.weight"], df, dx=dg, dw=gr(ln + ".linear2.weight"), db=gr(ln + ".linear2.bias"))
    dz = K.gelu_dropout_bwd(dg, z, _e(z.shape, dx2), drop, rng, site + 2)
    dh2 = _e((rows, D), dx2)
    K.linear_bwd(sv["h2"], p[ln + ".linear1.weight"], dz, dx=dh2, dw=gr(ln + ".linear1.weight"),
                 db=gr(ln + ".linear1.bias"))
    t = _e((rows, D), dx2)
    K.add_ln_bwd(dh2, sv["x1"], sv["m2"], sv["r2"], p[ln + ".norm2.weight"], t, None, gr(ln + ".norm2.weight"),
                 gr(ln + ".norm2.bias"), L)
    dx1 = K.add_dropout(dx2, t, _e((rows, D), dx2))
    dsa = dx1.clone()
    K.dropout_(dsa, drop, rng, site + 1)
    do = _e((rows, D), dx2)
    K.linear_bwd(sv["o"], p[ln + ".self_attn.out_proj.weight"], dsa, dx=do, dw=gr(ln + ".self_attn.out_proj.weight"),
                 db=gr(ln + ".self_attn.out_proj.bias"))
    qkv = sv["qkv"]
    dqkv = _e((rows, 3 * D), dx2)
    _mha_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], sv["P"], do, dqkv[:, :D], dqkv[:, D:2 * D],
             dqkv[:, 2 * D:], B, H, L, drop, rng, site)
    dh1 = _e((rows, D), dx2)
    K.linear_bwd(sv["h1"], p[ln + ".self_attn.in_proj_weight"], dqkv, dx=dh1,
                 dw=gr(ln + ".self_attn.in_proj_weight"), db=gr(ln + ".self_attn.in_proj_bias"))
    K.add_ln_bwd(dh1, sv["x"], sv["m1"], sv["r1"], p[ln + ".norm1.weight"], t, None, gr(ln + ".norm1.weight"),
                 gr(ln + ".norm1.bias"), L)
    return K.add_dropout(dx1, t, _e((rows, D), dx2))


# ---------------------------------------------------------------------------------------------
def pool_forward(p: Dict[str, torch.Tensor], prefix: str, mode: str, x3: torch.Tensor, out: torch.Tensor,
                 ldo: Optional[int] = None, num_heads: int = 4, num_layers: int = 1, dropout: float = 0.0,
                 rng: Optional[torch.Tensor] = None, site0: int = 100, pe: Optional[torch.Tensor] = None) -> PoolCtx:
    """TemporalPooler.forward (temporal.py:105-110) for 'attn' / 'transformer' on x3 [B, L, D] (fp32,
    contiguous): writes the pooled [B, D] rows into ``out`` (row stride ``ldo``) and returns the context
    for ``pool_backward``.  ``dropout`` is the active drop probability (0 in eval mode)."""
    B, L, D = x3.shape
    ldo = out.stride(0) if ldo is None else ldo
    ctx = PoolCtx(mode)
    ctx.saved.update(dims=(B, L, D), heads=num_heads, layers=num_layers, drop=dropout, rng=rng, site0=site0)
    if mode == "attn":
        ctx.saved["pool"] = _attn_pool_fwd(p, prefix, x3, out, ldo, dropout, rng, site0)
        return ctx
    if mode != "transformer":
        raise ValueError(f"Unsupported temporal pooling mode: {mode}")
    if D % num_heads:
        raise ValueError(f"embed_dim {D} must be divisible by num_heads {num_heads}")
    if pe is None:
        pe = sinusoidal_pe(L, D, x3.device)
    rows = B * L
    x = K.add_dropout(x3.reshape(rows, D), pe[:L].contiguous(), _e((rows, D), x3), L)
    layers = []
    for i in range(num_layers):
        x, sv = _layer_fwd(p, f"{prefix}.encoder.layers.{i}", x, B, L, num_heads, dropout, rng, site0 + 8 * (i + 1))
        layers.append(sv)
    ctx.saved["layers"] = layers
    ctx.saved["pool"] = _attn_pool_fwd(p, prefix + ".pool", x.view(B, L, D), out, ldo, dropout, rng, site0)
    return ctx


def pool_backward(p: Dict[str, torch.Tensor], prefix: str, ctx: PoolCtx, dy: torch.Tensor,
                  grads: Dict[str, torch.Tensor]) -> torch.Tensor:
    """Reverse of ``pool_forward`` given dy [B, D] (row-strided): returns dx [B, L, D]; parameter
    gradients accumulate into ``grads`` (names missing from it are not computed)."""
    sv = ctx.saved
    B, L, D = sv["dims"]
    drop, rng, site0 = sv["drop"], sv["rng"], sv["site0"]
    if ctx.mode == "attn":
        return _attn_pool_bwd(p, prefix, sv["pool"], dy, grads, drop, rng, site0)
    dx = _attn_pool_bwd(p, prefix + ".pool", sv["pool"], dy, grads, drop, rng, site0).view(B * L, D)
    for i in reversed(range(sv["layers"].__len__())):
        dx = _layer_bwd(p, f"{prefix}.encoder.layers.{i}", sv["layers"][i], dx, grads, B, L, sv["heads"], drop, rng,
                        site0 + 8 * (i + 1))
    return dx.view(B, L, D)  # the positional encoding is a constant: its gradient is the identity


_PE_CACHE: Dict[tuple, torch.Tensor] = {}


def sinusoidal_pe(length: int, dim: int, device) -> torch.Tensor:
    """SinusoidalPositionalEncoding (temporal.py:29-43) rows [length, dim], fp32 on the device (cached)."""
    key = (length, dim, str(device))
    pe = _PE_CACHE.get(key)
    if pe is None:
        position = torch.arange(length).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, dim, 2) * (-math.log(10000.0) / max(1, dim)))
        pe = torch.zeros(length, dim)
        pe[:, 0::2] = torch.sin(position * div_term)
        if dim > 1:
            pe[:, 1::2] = torch.cos(position * div_term[: pe[:, 1::2].shape[1]])
        pe = _PE_CACHE[key] = pe.to(device)
    return pe
