"""Thin tensor-level wrappers over the C-ABI (``include/mer.h``).

PyTorch is plumbing here: it owns device memory (caching allocator) and the current
HIP stream; every byte of math runs in ``libmer_hip.so``.  Wrappers validate shapes
and dtypes on the host before launching (a mis-sized launch is a GPU fault, not an
exception), then pass raw pointers and the current stream.
"""
from __future__ import annotations

import os

import torch

from ._lib import LIB, MerKernelError

F32, BF16 = 0, 1
ACT = {"none": 0, "relu": 1, "gelu": 2}


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


class KernelProbe:
    """Brackets launches of ONE kernel (by name + shape key) with HIP events on the launching stream, so
    bench.py can report that kernel's average device time inside the timed region."""

    def __init__(self, name: str, key: tuple, units: float):
        self.name, self.key, self.units = name, tuple(key), units  # units = algorithmic FLOP or bytes / launch
        self.pairs = []
        self.active = False

    def matches(self, name, key):
        return self.active and name == self.name and tuple(key) == self.key

    def avg_ms(self):
        if not self.pairs:
            return None
        return sum(a.elapsed_time(b) for a, b in self.pairs) / len(self.pairs)

    def record(self, name, pair):
        self.pairs.append(pair)


class MultiProbe:
    """Brackets every launch of the named kernels (any shape) with HIP events: per-kernel average device time
    (bench.py's head-core roofline entry)."""

    def __init__(self, names):
        self.names = tuple(names)
        self.by_name = {n: [] for n in self.names}
        self.active = False

    def matches(self, name, key):
        return self.active and name in self.by_name

    def record(self, name, pair):
        self.by_name[name].append(pair)

    def avg_ms(self, name):
        p = self.by_name.get(name) or []
        return sum(a.elapsed_time(b) for a, b in p) / len(p) if p else None


PROBE = None


def _launch(name, key, fn, *args):
    if PROBE is not None and PROBE.matches(name, key) and not torch.cuda.is_current_stream_capturing():
        s = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        LIB(fn, *args)
        b.record(s)
        PROBE.record(name, (a, b))
    else:
        LIB(fn, *args)


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported dtype {t.dtype}")


def _ptr(t):
    return 0 if t is None else t.data_ptr()


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("MI355X kernels need device tensors (HIP); got a CPU tensor")


def gemm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, *, trans_a: bool = False, trans_b: bool = False,
         bias=None, beta: int = 0, act: str = "none", splitk: int = 1) -> torch.Tensor:
    """out[M,N] (+)= op(a) @ op(b) (+ bias) on the fp32 MFMA GEMM.

    ``a`` is [M,K] (or [K,M] with trans_a), ``b`` is [K,N] (or [N,K] with trans_b); both may be
    strided 2-D views with one unit stride.  ``out`` is fp32 [M,N] with unit column stride.
    """
    _check_dev(a, b, out, bias)
    if trans_a:
        K, M = a.shape
        sam, sak = a.stride(1), a.stride(0)
    else:
        M, K = a.shape
        sam, sak = a.stride(0), a.stride(1)
    if trans_b:
        N, K2 = b.shape
        sbk, sbn = b.stride(1), b.stride(0)
    else:
        K2, N = b.shape
        sbk, sbn = b.stride(0), b.stride(1)
    if K != K2 or tuple(out.shape) != (M, N) or out.stride(1) != 1 or out.dtype != torch.float32:
        raise ValueError(f"gemm shape mismatch: a{tuple(a.shape)} b{tuple(b.shape)} out{tuple(out.shape)}")
    if bias is not None and (bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("bias must be contiguous [N]")
    if splitk > 1:
        splitk = max(1, min(splitk, (K + 255) // 256))
    ws = _workspace(splitk * M * N, out.device) if splitk > 1 else None
    LIB("mer_gemm_f32", M, N, K, a.data_ptr(), _dt(a), sam, sak, 0, b.data_ptr(), _dt(b), sbk, sbn, 0,
        out.data_ptr(), out.stride(0), 0, _ptr(bias), int(beta), ACT[act], int(splitk), 1, _ptr(ws), stream_ptr())
    return out


def auto_splitk(M: int, N: int, K: int) -> int:
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    if tiles >= 128 or K < 1024:
        return 1
    return int(max(1, min(32, 256 // tiles, K // 512)))


def linear_fwd(x2d, w, b, out, act="none"):
    """nn.Linear: out = x W^T + b."""
    return gemm(x2d, w, out, trans_b=True, bias=b, act=act)


def linear_bwd(x2d, w, dy, dx=None, dw=None, db=None, dx_beta=0):
    """Given dy [M,N] for out = x W^T + b: dx (+)= dy W ; dw += dy^T x ; db += colsum(dy).

    dw / db must be initialised (they are accumulated; split-K slices and colsum partials are added in a
    fixed order, so the result is run-to-run reproducible).
    """
    M, N = dy.shape
    K = x2d.shape[1]
    if dx is not None:
        gemm(dy, w, dx, beta=dx_beta)
    if dw is not None:
        gemm(dy, x2d, dw, trans_a=True, beta=1, splitk=auto_splitk(N, K, M))
    if db is not None:
        colsum(dy, db)


def _workspace(floats, device):
    """fp32 scratch for the fixed-order reductions; freed back to torch's stream-ordered cache on return."""
    return torch.empty(max(1, int(floats)), device=device, dtype=torch.float32)


def colsum(x2d, out):
    _check_dev(x2d, out)
    M, N = x2d.shape
    ws = _workspace((M + 15) // 16 * N, out.device)  # MER_COLSUM_WS_FLOATS
    LIB("mer_colsum_f32", M, N, x2d.data_ptr(), x2d.stride(0), out.data_ptr(), ws.data_ptr(), stream_ptr())


def rng_ptr(rng):
    """Device address of a step's RNG base (int64 [1] tensor, see mer_site_seed) or 0 (no dropout)."""
    if rng is None:
        return 0
    if rng.dtype != torch.int64 or rng.numel() != 1 or not rng.is_cuda:
        raise ValueError("the RNG base must be a device int64 tensor of one element")
    return rng.data_ptr()


def rng_advance(rng):
    """rng = splitmix64(rng): the next step's RNG base, on the device (capturable in a hipGraph)."""
    LIB("mer_rng_advance", rng_ptr(rng), stream_ptr())


def mha_fwd(q, k, v, bias, out, P, B, H, Lq, Lk, drop_p=0.0, rng=None, site=0):
    d = out.shape[-1]
    dh = d // H
    LIB("mer_mha_fwd", B, H, Lq, Lk, dh, q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(),
        v.stride(0), _ptr(bias), out.data_ptr(), out.stride(0), P.data_ptr(), float(dh ** -0.5), float(drop_p),
        rng_ptr(rng), int(site), stream_ptr())


def mha_bwd(q, k, v, P, dout, dq, dk, dv, dbias, B, H, Lq, Lk, drop_p=0.0, rng=None, site=0):
    d = dout.shape[-1]
    dh = d // H
    LIB("mer_mha_bwd", B, H, Lq, Lk, dh, q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(),
        v.stride(0), P.data_ptr(), dout.data_ptr(), dout.stride(0), dq.data_ptr(), dq.stride(0), dk.data_ptr(),
        dk.stride(0), dv.data_ptr(), dv.stride(0), _ptr(dbias), float(dh ** -0.5), float(drop_p), rng_ptr(rng),
        int(site), stream_ptr())


def add_ln_fwd(x, r, gamma, beta, y, s_out, mean, rstd, rows_per_sample, dp_p=0.0, rng=None, site=0, eps=1e-5):
    rows, d = x.shape
    LIB("mer_add_ln_fwd", rows, d, rows_per_sample, x.data_ptr(), _ptr(r), float(dp_p), rng_ptr(rng), int(site),
        gamma.data_ptr(), beta.data_ptr(), float(eps), y.data_ptr(), _ptr(s_out), _ptr(mean), _ptr(rstd),
        stream_ptr())


def add_ln_bwd(dy, s, mean, rstd, gamma, dx, dr, dgamma, dbeta, rows_per_sample, dp_p=0.0, rng=None, site=0):
    rows, d = dy.shape
    LIB("mer_add_ln_bwd", rows, d, rows_per_sample, dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
        gamma.data_ptr(), float(dp_p), rng_ptr(rng), int(site), dx.data_ptr(), _ptr(dr), _ptr(dgamma), _ptr(dbeta),
        _workspace((rows + 15) // 16 * 2 * d, dy.device).data_ptr(), stream_ptr())  # MER_ADD_LN_WS_FLOATS


def mean_pool_fwd(x3d, y, ldy=None):
    B, L, D = x3d.shape
    LIB("mer_mean_pool_fwd", B, L, D, x3d.data_ptr(), y.data_ptr(), int(ldy if ldy is not None else y.stride(0)),
        stream_ptr())


def mean_pool_bwd(dy, dx3d, accumulate=False):
    B, L, D = dx3d.shape
    LIB("mer_mean_pool_bwd", B, L, D, dy.data_ptr(), dy.stride(0), dx3d.data_ptr(), int(accumulate), stream_ptr())


def gelu_dropout_fwd(z, y, p=0.0, rng=None, site=0):
    rows, cols = z.shape
    LIB("mer_gelu_dropout_fwd", rows, cols, z.data_ptr(), z.stride(0), y.data_ptr(), y.stride(0), float(p),
        rng_ptr(rng), int(site), stream_ptr())
    return y


def gelu_dropout_bwd(dy, z, dz, p=0.0, rng=None, site=0):
    rows, cols = z.shape
    LIB("mer_gelu_dropout_bwd", rows, cols, dy.data_ptr(), dy.stride(0), z.data_ptr(), z.stride(0), dz.data_ptr(),
        dz.stride(0), float(p), rng_ptr(rng), int(site), stream_ptr())
    return dz


def add_dropout(x, r, y, r_period=None, p=0.0, rng=None, site=0):
    """y = x + dropout(r[row % r_period]); all contiguous [rows, cols]."""
    rows, cols = x.shape
    _check_dev(x, r, y)
    if not (x.is_contiguous() and r.is_contiguous() and y.is_contiguous()):
        raise ValueError("add_dropout operands must be contiguous")
    LIB("mer_add_dropout", rows, cols, x.data_ptr(), r.data_ptr(), int(r_period or rows), float(p), rng_ptr(rng),
        int(site), y.data_ptr(), stream_ptr())
    return y


def attn_pool_fwd(x3d, scores, attn, y, ldy=None):
    B, L, D = x3d.shape
    LIB("mer_attn_pool_fwd", B, L, D, x3d.data_ptr(), scores.data_ptr(), attn.data_ptr(), y.data_ptr(),
        int(ldy if ldy is not None else y.stride(0)), stream_ptr())


def attn_pool_bwd(x3d, attn, dy, dx3d, dscores, accumulate=False):
    B, L, D = x3d.shape
    LIB("mer_attn_pool_bwd", B, L, D, x3d.data_ptr(), attn.data_ptr(), dy.data_ptr(), dy.stride(0), dx3d.data_ptr(),
        int(accumulate), dscores.data_ptr(), stream_ptr())


def softmax_dropout_bwd(P, dpp, ds, pd, h, p=0.0, rng=None, site=0):
    B, H, Lq, Lk = P.shape
    LIB("mer_softmax_dropout_bwd", B, H, int(h), Lq, Lk, P.data_ptr(), dpp.data_ptr(), ds.data_ptr(), pd.data_ptr(),
        float(p), rng_ptr(rng), int(site), stream_ptr())


def gemm_batched(a, b, out, *, M, N, K, sam, sak, bsa, sbk, sbn, bsb, ldc, bsc, batch, beta=0):
    """out_z[M,N] (+)= A_z B_z over a batch of strided fp32 matrices (views into larger buffers)."""
    _check_dev(a, b, out)
    LIB("mer_gemm_f32", M, N, K, a.data_ptr(), _dt(a), sam, sak, bsa, b.data_ptr(), _dt(b), sbk, sbn, bsb,
        out.data_ptr(), ldc, bsc, 0, int(beta), 0, 1, int(batch), 0, stream_ptr())
    return out


def cross_entropy(logits, labels, loss, dlogits, label_smoothing=0.0, late=False, preds=None):
    B, C = logits.shape
    if labels.dtype != torch.int64 or labels.numel() != B:
        raise ValueError("labels must be int64 [B]")
    if preds is not None and (preds.dtype != torch.int64 or preds.numel() != B):
        raise ValueError("preds must be int64 [B]")
    LIB("mer_cross_entropy", B, C, logits.data_ptr(), labels.data_ptr(), float(label_smoothing), int(late),
        loss.data_ptr(), _ptr(dlogits), _ptr(preds), stream_ptr())


def scale_dev(x, s, y):
    LIB("mer_scale_dev", x.numel(), x.data_ptr(), s.data_ptr(), y.data_ptr(), stream_ptr())


def dropout_(x2d, p, rng=None, site=0):
    if p > 0:
        LIB("mer_dropout_inplace", x2d.shape[0], x2d.shape[1], x2d.data_ptr(), x2d.stride(0), float(p), rng_ptr(rng),
            int(site), stream_ptr())


def relu_dropout_bwd_(dy, y, p, rng=None, site=0):
    LIB("mer_relu_dropout_bwd", dy.shape[0], dy.shape[1], dy.data_ptr(), dy.stride(0), y.data_ptr(), y.stride(0),
        float(p), rng_ptr(rng), int(site), stream_ptr())


def gate_mix_fwd(z, v, a, out, g):
    B, D = out.shape
    LIB("mer_gate_mix_fwd", B, D, z.data_ptr(), v.data_ptr(), v.stride(0), a.data_ptr(), a.stride(0),
        out.data_ptr(), g.data_ptr(), stream_ptr())


def gate_mix_bwd(g, v, a, dout, dz, dv, da):
    B, D = dout.shape
    LIB("mer_gate_mix_bwd", B, D, g.data_ptr(), v.data_ptr(), v.stride(0), a.data_ptr(), a.stride(0),
        dout.data_ptr(), dz.data_ptr(), dv.data_ptr(), dv.stride(0), da.data_ptr(), da.stride(0), stream_ptr())


def token_bias_fwd(qt, qp, kt, kp, scale, out):
    B, Lq, Lk = out.shape
    LIB("mer_token_bias_fwd", B, Lq, Lk, qt.data_ptr(), qp.data_ptr(), kt.data_ptr(), kp.data_ptr(),
        scale.data_ptr(), out.data_ptr(), stream_ptr())


def token_bias_bwd(qt, qp, kt, kp, scale, dbias, dqt, dkt, dqp, dkp, dscale_part):
    B, Lq, Lk = dbias.shape
    LIB("mer_token_bias_bwd", B, Lq, Lk, qt.data_ptr(), qp.data_ptr(), kt.data_ptr(), kp.data_ptr(),
        scale.data_ptr(), dbias.data_ptr(), dqt.data_ptr(), dkt.data_ptr(), dqp.data_ptr(), dkp.data_ptr(),
        dscale_part.data_ptr(), stream_ptr())


def vec_sum(x, out, accumulate=False):
    LIB("mer_vec_sum", x.numel(), x.data_ptr(), out.data_ptr(), int(accumulate), stream_ptr())


def adam_step(p, g, m, v, lr, b1, b2, eps, wd, step, grad_scale=1.0):
    LIB("mer_adam_step", p.numel(), p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), float(lr), float(b1),
        float(b2), float(eps), float(wd), int(step), float(grad_scale), stream_ptr())


def _aligned16(*ts):
    for t in ts:
        if t is not None and t.data_ptr() % 16:
            raise ValueError("bf16 GEMM operands must be 16-byte aligned")


def _train_args(drop_p, rng, site, skip, skip_bit):
    """(drop_p, seed ptr, site, skip-mask ptr, bit) of the *_tr entry points, validated."""
    if drop_p > 0 and rng is None:
        raise ValueError("dropout needs the step's device RNG base")
    if skip is not None and (skip.dtype != torch.int64 or skip.numel() != 1 or not skip.is_cuda):
        raise ValueError("the LayerDrop mask must be a device int64 tensor of one element")
    return float(drop_p), rng_ptr(rng) if drop_p > 0 else 0, int(site), _ptr(skip), int(skip_bit)


def gemm_bf16(a, w, out, *, M=None, K=None, rows=None, bias=None, residual=None, act="none", variant=-1,
              drop_p=0.0, rng=None, site=0, skip=None, skip_bit=0):
    """out[M,N] = act(A W^T + bias) (+ residual) on bf16 MFMA.

    ``a``: bf16 [M,K] (row stride a.stride(0)), or a raw bf16 buffer with ``rows=(rpg, rstride, gstride)``
    describing the channel-last Conv1d im2col rows.  ``w``: bf16 [N,K].  ``out``: bf16 or fp32 [M,N].
    Train mode: ``drop_p`` / ``rng`` / ``site`` dropout after the activation (before the residual);
    ``skip`` / ``skip_bit``: LayerDrop (the launch is a no-op when that bit of the device mask is set).
    """
    N = w.shape[0]
    if rows is None:
        M, K = a.shape
        rows = (M, a.stride(0), 0)
    if w.dtype != torch.bfloat16 or a.dtype != torch.bfloat16 or w.shape[1] != K or w.stride(1) != 1:
        raise ValueError("gemm_bf16 expects bf16 A and W[N,K]")
    if out.shape[-1] != N or out.numel() != M * N:
        raise ValueError(f"gemm_bf16 out shape {tuple(out.shape)} != ({M},{N})")
    _aligned16(a, w)
    ldc = N if out.dim() < 2 else out.stride(-2)
    ldr = 0 if residual is None else residual.stride(-2)
    if drop_p > 0 or skip is not None:
        _launch("gemm_bf16", (M, N, K), "mer_gemm_bf16_tr", M, N, K, a.data_ptr(), rows[2], rows[1], rows[0],
                w.data_ptr(), w.stride(0), out.data_ptr(), _dt(out), ldc, _ptr(bias), _ptr(residual), ldr, ACT[act],
                *_train_args(drop_p, rng, site, skip, skip_bit), int(variant), stream_ptr())
        return out
    _launch("gemm_bf16", (M, N, K), "mer_gemm_bf16_ex", M, N, K, a.data_ptr(), rows[2], rows[1], rows[0], w.data_ptr(),
            w.stride(0), out.data_ptr(), _dt(out), ldc, _ptr(bias), _ptr(residual), ldr, ACT[act], int(variant),
            stream_ptr())
    return out


def posconv_gemm_bf16(x, wp, out, B, L, C, groups, taps, pad, bias, residual, act="gelu", variant=-1):
    """``variant`` -1: the Toeplitz strip kernel where it applies; 0: the gather GEMM (its bit-exact reference)."""
    LIB("mer_posconv_gemm_bf16", B, L, C, groups, taps, pad, x.data_ptr(), x.stride(-2), wp.data_ptr(), out.data_ptr(),
        _dt(out), out.stride(-2), _ptr(bias), _ptr(residual), 0 if residual is None else residual.stride(-2),
        ACT[act], int(variant), stream_ptr())


def wavlm_conv0_gn_gelu(wav, w0, gamma, beta, out, eps=1e-5):
    """conv0 -> GroupNorm(512, 512) -> GELU of the WavLM feature extractor (deterministic two-pass)."""
    B, S = wav.shape
    Lout = out.shape[1]
    if tuple(out.shape) != (B, (S - 10) // 5 + 1, 512) or out.dtype != torch.bfloat16:
        raise ValueError(f"wavlm_conv0_gn_gelu out {tuple(out.shape)}")
    ws = torch.empty(B * ((Lout + 127) // 128 + 1) * 1024 + 16384, device=wav.device, dtype=torch.float32)
    LIB("mer_wavlm_conv0_gn_gelu", B, S, Lout, wav.data_ptr(), w0.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
        float(eps), ws.data_ptr(), out.data_ptr(), stream_ptr())


def layernorm(x2d, gamma, beta, y2d, eps=1e-5, drop_p=0.0, rng=None, site=0, skip=None, skip_bit=0):
    rows, d = x2d.shape
    if drop_p > 0 or skip is not None:
        LIB("mer_layernorm_tr", rows, d, x2d.data_ptr(), _dt(x2d), x2d.stride(0), gamma.data_ptr(), beta.data_ptr(),
            float(eps), y2d.data_ptr(), _dt(y2d), y2d.stride(0), *_train_args(drop_p, rng, site, skip, skip_bit),
            stream_ptr())
        return
    LIB("mer_layernorm", rows, d, x2d.data_ptr(), _dt(x2d), x2d.stride(0), gamma.data_ptr(), beta.data_ptr(),
        float(eps), y2d.data_ptr(), _dt(y2d), y2d.stride(0), stream_ptr())


def wavlm_attention(qkv, x, gate_w, gate_b, gate_const, rel_emb, bucket, out, B, L, H, scale, drop_p=0.0, rng=None,
                    site=0, skip=None, skip_bit=0):
    """``bucket`` None: ``rel_emb`` is the per-head bias table [H][2L-1] (``rel_emb[bucket].t()``)."""
    if drop_p > 0 or skip is not None:
        LIB("mer_wavlm_attention_tr", B, L, H, qkv.data_ptr(), qkv.stride(0), x.data_ptr(), x.stride(0),
            gate_w.data_ptr(), gate_b.data_ptr(), gate_const.data_ptr(), rel_emb.data_ptr(), _ptr(bucket),
            out.data_ptr(), out.stride(0), float(scale), *_train_args(drop_p, rng, site, skip, skip_bit), stream_ptr())
        return
    LIB("mer_wavlm_attention", B, L, H, qkv.data_ptr(), qkv.stride(0), x.data_ptr(), x.stride(0), gate_w.data_ptr(),
        gate_b.data_ptr(), gate_const.data_ptr(), rel_emb.data_ptr(), _ptr(bucket), out.data_ptr(),
        out.stride(0), float(scale), stream_ptr())


def wavlm_time_mask(h, B, L, embed, mask_prob, mask_len, min_masks, rng, site, mask_out=None):
    """SpecAugment time masking of the projected WavLM features h bf16 [B*L, D] in place."""
    D = h.shape[-1]
    if h.dtype != torch.bfloat16 or h.numel() != B * L * D or embed.numel() != D:
        raise ValueError("wavlm_time_mask shapes")
    if mask_len > L:
        raise ValueError(f"`mask_length` has to be smaller than `sequence_length`, but got `mask_length`: {mask_len} "
                         f"and `sequence_length`: {L}`")  # TF:863-867
    if mask_out is not None and (mask_out.dtype != torch.uint8 or mask_out.numel() != B * L):
        raise ValueError("mask_out must be uint8 [B, L]")
    LIB("mer_wavlm_time_mask", B, L, D, h.data_ptr(), h.stride(-2), embed.detach().contiguous().data_ptr(),
        float(mask_prob), int(mask_len), int(min_masks), rng_ptr(rng), int(site), _ptr(mask_out), stream_ptr())


def bf16_convert(x, y):
    if x.dtype != torch.bfloat16 or not x.is_contiguous() or not y.is_contiguous() or x.numel() != y.numel():
        raise ValueError("bf16_convert: contiguous bf16 source of the same size")
    LIB("mer_bf16_convert", x.numel(), x.data_ptr(), y.data_ptr(), _dt(y), stream_ptr())
    return y


def permute3_bf16(src, shape3, strides3, dst, scale=None):
    n0, n1, n2 = shape3
    LIB("mer_permute3_bf16", n0, n1, n2, src.data_ptr(), strides3[0], strides3[1], strides3[2], _ptr(scale),
        dst.data_ptr(), stream_ptr())


def weightnorm_scale(v, g, scale):
    n01 = v.shape[0] * v.shape[1]
    LIB("mer_weightnorm_scale", n01, v.shape[2], v.data_ptr(), g.data_ptr(), scale.data_ptr(), stream_ptr())


def cast_bf16(x, y):
    LIB("mer_cast_bf16", x.numel(), x.data_ptr(), y.data_ptr(), stream_ptr())


BN_STAT_PARTS = 64  # MER_BN_STAT_PARTS (include/mer.h)


def bn_stat_rows(M: int) -> int:
    """MER_BN_STAT_ROWS(M): rows of a conv forward's BatchNorm statistics buffer (one per <=64-row output tile,
    plus 64 finalize scratch rows)."""
    return (M + 63) // 64 + 64


def bn_red_rows(M: int) -> int:
    """MER_BN_RED_ROWS(M): rows of a fused BN-backward reduction buffer of a dgrad with M output pixels."""
    return (M + 63) // 64 + 4 + 64


BN_RED_WS_ROWS = 576  # MER_BN_RED_WS_ROWS: bn_bwd_reduce workspace rows


def bn_stats_buffer(C, device, M=None):
    """Zeroed BatchNorm partial-sum buffer: conv_fwd statistics float[bn_stat_rows(M)][C][2] when the output
    pixel count M is given, else the striped backward-reduction layout float[BN_STAT_PARTS][C][2]."""
    rows = BN_STAT_PARTS if M is None else bn_stat_rows(M)
    return torch.zeros(rows, C, 2, device=device, dtype=torch.float32)


def conv_fwd(x, wp, y, stats, R, S, stride, pad, variant=-1):
    N, H, W, C = x.shape
    Kc = y.shape[-1]
    Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    if tuple(y.shape) != (N, Ho, Wo, Kc) or tuple(wp.shape) != (Kc, R * S * C):
        raise ValueError(f"conv_fwd shapes x{tuple(x.shape)} w{tuple(wp.shape)} y{tuple(y.shape)}")
    if stats is not None and (stats.numel() != bn_stat_rows(N * Ho * Wo) * Kc * 2 or not stats.is_contiguous()):
        raise ValueError("conv_fwd stats must be a contiguous zeroed float[bn_stat_rows(M)][K][2] buffer")
    _launch("conv_fwd", (N, H, W, C, Kc, R, stride), "mer_conv_fwd_ex", N, H, W, C, Kc, R, S, stride, pad, x.data_ptr(),
            wp.data_ptr(), y.data_ptr(), _ptr(stats), int(variant), stream_ptr())
    if stats is not None:
        return _partial_rows("mer_conv_fwd_rows", N, H, W, C, Kc, R, S, stride, pad, x.data_ptr(), wp.data_ptr(),
                             int(variant))
    return None


_ROWS_CACHE = {}
# Fold only the partial rows a conv wrote (one per persistent workgroup on the halo kernel): the layer1 / stem
# BatchNorms take the one-launch wide fold.  Same-box step +0.55 % (profiles/r06/step_ab_partial_rows).
PARTIAL_ROWS = True


def _partial_rows(fn, *args):
    """mer_conv_fwd_rows / mer_conv_dgrad_rows: the partial rows the launch with these arguments wrote.  Cached on
    the shapes, the variant and the 16-byte alignment of the pointers (all the halo test reads of them)."""
    if not PARTIAL_ROWS:
        return None
    key = (fn,) + tuple(a % 16 == 0 if isinstance(a, int) and a > 1 << 20 else a for a in args)
    r = _ROWS_CACHE.get(key)
    if r is None:
        r = int(LIB.call_int(fn, *args))
        if r <= 0:
            raise MerKernelError(f"{fn}{args[:9]} failed: {r}")
        _ROWS_CACHE[key] = r
    return r


def conv_dgrad(dy, wt, dx, R, S, stride, pad, residual=None, mask=None, variant=-1, bnr=None, ds=None):
    """dx = conv-transpose(dy) (+ residual where mask > 0).  ``bnr``: optional fused BatchNorm-backward
    reduction of the BN the gradient flows into, ``(mask, x, ms, red[, x2, ms2, red2])`` with red(2)
    zeroed [BN_STAT_PARTS, C, 2] buffers (see mer_conv_dgrad_bnr).  ``ds``: ``(ds_dy, ds_wt)`` -- the input gradient
    of a 1x1 / stride-2 downsample of the same input, fused in (mer_conv_dgrad_ds)."""
    N, H, W, C = dx.shape
    Kc = dy.shape[-1]
    Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    if tuple(dy.shape) != (N, Ho, Wo, Kc) or tuple(wt.shape) != (C, R * S * Kc):
        raise ValueError(f"conv_dgrad shapes dy{tuple(dy.shape)} wt{tuple(wt.shape)} dx{tuple(dx.shape)}")
    b = list(bnr) + [None] * (7 - len(bnr)) if bnr is not None else [None] * 7
    for t in (b[0], b[1], b[4]):
        if t is not None and tuple(t.shape) != tuple(dx.shape):
            raise ValueError("conv_dgrad bnr tensors must match dx")
    for t in (b[3], b[6]):
        if t is not None and t.numel() != bn_red_rows(N * H * W) * C * 2:
            raise ValueError("conv_dgrad bnr red buffers must be zeroed [bn_red_rows(N*H*W), C, 2]")
    if ds is not None:
        ddy, dwt = ds
        Kd = ddy.shape[-1]
        if tuple(ddy.shape) != (N, Ho, Wo, Kd) or tuple(dwt.shape) != (C, Kd) or stride != 2 or R != 3 or pad != 1:
            raise ValueError("conv_dgrad ds: a 1x1 / stride-2 downsample gradient beside a 3x3 / stride-2 / pad-1 conv")
        _launch("conv_dgrad", (N, H, W, C, Kc, R, stride), "mer_conv_dgrad_ds", N, H, W, C, Kc, R, S, stride, pad,
                dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), _ptr(residual), _ptr(mask), *[_ptr(t) for t in b],
                ddy.data_ptr(), dwt.data_ptr(), Kd, int(variant), stream_ptr())
    else:
        _launch("conv_dgrad", (N, H, W, C, Kc, R, stride), "mer_conv_dgrad_bnr", N, H, W, C, Kc, R, S, stride, pad,
                dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), _ptr(residual), _ptr(mask), *[_ptr(t) for t in b],
                int(variant), stream_ptr())
    if bnr is None:
        return None
    return _partial_rows("mer_conv_dgrad_rows", N, H, W, C, Kc, R, S, stride, pad, dy.data_ptr(), wt.data_ptr(),
                         ds[0].data_ptr() if ds is not None else 0, int(variant))


def partials_sum(parts_buf, out, rows=None):
    """out[C,2] = fixed-order sum of the data rows of a [bn_red_rows(M), C, 2] fused-epilogue reduction
    buffer (its last 64 rows are the fold scratch).  ``rows``: the leading rows the producing conv_dgrad wrote (its
    return value; the rest are zero), else every data row."""
    P, C, _ = parts_buf.shape
    if P <= 64:
        raise ValueError("partials_sum expects a bn_red_rows(M) buffer (data rows + 64 scratch rows)")
    if rows is None:
        rows = P - 64
    if not 0 < rows <= P - 64:
        raise ValueError("partials_sum rows out of range")
    LIB("mer_partials_sum", C, int(rows), parts_buf.data_ptr(), out.data_ptr(), stream_ptr())
    return out


# Pixels per wgrad split, at least (tools/bench_conv.py on the ResNet18 layers, MI355X): 1024 in general -- more,
# shorter splits lose to the fold of their partial slabs -- but 256 for the tiny 1x1 downsample outputs (a K loop of
# 16 64-pixel steps per split was the whole time: 26 -> 19 us) and 512 where the output has so many tiles that
# 1024 leaves only 4 splits (layer4 3x3: 65 -> 58 us).
# Target workgroups per wgrad launch: 768 (256 / 384 / 512 lose 3.1 / 1.3 / 0.3 % of the step, 1024 loses 0.4 %).
_WGRAD_WGS = 768
# The trunk's default wgrad form for the stride-1 3x3 convs with K > 64 output channels (round 6): conv.hip variant 8,
# two K-groups of 8 waves per workgroup (in-workgroup split-K over the pixels).  A launch of it covers the pixels of two
# one-group splits: half the splits -- and half the fp32 slabs written and folded (~340 of the ~520 MB per step) -- for
# the same waves per CU, so it targets _WGRAD_WGS / 2 workgroups.  The others keep the one-group ring (4): the
# 64-channel stem / layer1 (its 48 KB blocks run three per CU, the 96 KB two-group block one: stem 78 -> 110 us
# standalone, profiles/r06/bench_wgrad_kg.txt), and the stride-2 / 1x1 wgrads, whose slabs are small and whose kernels
# ran 2-8 us slower each in the serialized trunk (profiles/r06/trunk_table_serial.txt).
WGRAD_VARIANT = 8


def _wgrad_min_pix(out_elems, tiles):
    return 256 if out_elems <= 65536 else (512 if tiles >= 96 else 1024)


def wgrad_split_count(P: int, splits: int) -> int:
    """The split count a wgrad launch asked for ``splits`` over P output pixels really uses (conv.hip
    conv_wgrad_impl): 64-pixel granules per split, every split non-empty."""
    splits = max(1, int(splits))
    pps = (-(-P // splits) + 63) // 64 * 64
    return -(-P // pps)


class WgradFolds:
    """Deferred split-K folds of one backward segment: conv_wgrad(..., defer=self) launches only the partial-slab
    pass and records (slabs, dw); flush() folds every record in ONE mer_wgrad_fold_batch launch on the current
    stream.  The slab tensors stay referenced until the flush is enqueued (stream order then protects them)."""

    MAX = 32

    def __init__(self):
        self.rows, self.keep = [], []

    def add(self, ws, dw, Kc, C, creal, RS, splits, map_=None):
        self.rows.append([ws.data_ptr(), dw.data_ptr(), _ptr(map_), Kc, C, creal, RS, splits])
        self.keep += [ws, dw, map_]

    def flush(self):
        import numpy as np
        for i in range(0, len(self.rows), self.MAX):
            tab = np.ascontiguousarray(np.array(self.rows[i:i + self.MAX], dtype=np.int64))
            _launch("wgrad_fold_batch", (len(tab),), "mer_wgrad_fold_batch", len(tab), tab.ctypes.data, stream_ptr())
        self.rows, self.keep = [], []


def conv_wgrad(x, dy, dw, R, S, stride, pad, creal=None, variant=-1, splits=None, defer=None, dw_map=None):
    """dw += weight gradient.  ``defer`` (a WgradFolds): leave the split-K slabs for its batched fold.  ``dw_map``
    (deferred only; int32 [R*S*C], -1 dropped): dw is any fp32 tensor, slab column j folds into dw[k].flat[map[j]]
    (the stem's space-to-depth gradient gathered straight into the 7x7 weight)."""
    N, H, W, C = x.shape
    Kc = dy.shape[-1]
    Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    creal = C if creal is None else creal
    if dw_map is not None:
        if defer is None or dw_map.dtype != torch.int32 or dw_map.numel() != R * S * C or not dw.is_contiguous():
            raise ValueError("conv_wgrad dw_map: deferred fold, int32 [R*S*C], contiguous dw")
        if dw.shape[0] != Kc or dw.dtype != torch.float32:
            raise ValueError("conv_wgrad shapes")
    elif tuple(dy.shape) != (N, Ho, Wo, Kc) or tuple(dw.shape) != (Kc, creal, R, S) or dw.dtype != torch.float32:
        raise ValueError("conv_wgrad shapes")
    if tuple(dy.shape) != (N, Ho, Wo, Kc):
        raise ValueError("conv_wgrad shapes")
    P = N * Ho * Wo
    tiles = ((Kc + 127) // 128) * ((R * S * C + 127) // 128)
    if variant == -1:
        variant = WGRAD_VARIANT if (Kc > 64 and stride == 1 and R * S > 1) else 4
    kg = 2 if variant == 8 else 1  # K-groups per workgroup
    if splits is None:  # ~768 groups of 8 waves (3 per CU), >= _wgrad_min_pix pixels each
        splits = int(max(1, min(-(-_WGRAD_WGS // (kg * tiles)), P // (kg * _wgrad_min_pix(Kc * R * S * C, tiles)))))
    ws = torch.empty(splits * Kc * R * S * C, device=x.device, dtype=torch.float32)
    if defer is not None:
        _launch("conv_wgrad", (N, H, W, C, Kc, R, stride), "mer_conv_wgrad_partials", N, H, W, C, Kc, R, S, stride,
                pad, x.data_ptr(), dy.data_ptr(), int(splits), ws.data_ptr(), int(variant), stream_ptr())
        defer.add(ws, dw, Kc, C, dw.numel() // Kc if dw_map is not None else creal, R * S,
                  wgrad_split_count(P, splits), dw_map)
        return
    _launch("conv_wgrad", (N, H, W, C, Kc, R, stride), "mer_conv_wgrad_ex", N, H, W, C, creal, Kc, R, S, stride, pad,
            x.data_ptr(), dy.data_ptr(), dw.data_ptr(), int(splits), ws.data_ptr(), int(variant), stream_ptr())


def pack_input_s2d(x, y):
    """fp32 NCHW frames -> space-to-depth bf16 [N][H/2+3][W/2+3][16] (the 4x4 stride-1 form of the stem conv)."""
    N, C, H, W = x.shape
    if tuple(y.shape) != (N, H // 2 + 3, W // 2 + 3, 16) or y.dtype != torch.bfloat16 or not y.is_contiguous():
        raise ValueError("pack_input_s2d shapes")
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError("pack_input_s2d reads contiguous fp32 NCHW frames")
    LIB("mer_pack_input_s2d", N, C, H, W, x.data_ptr(), y.data_ptr(), stream_ptr())


def pack_input_nhwc(x, y):
    N, C, H, W = x.shape
    LIB("mer_pack_input_nhwc", N, C, H, W, y.shape[-1], x.data_ptr(), y.data_ptr(), stream_ptr())


def pack_conv_weight(w, out, cp, transpose):
    Kc, C, R, S = w.shape
    LIB("mer_pack_conv_weight", Kc, C, R, S, cp, int(transpose), w.data_ptr(), out.data_ptr(), stream_ptr())


def pack_conv_weights(desc, blocks, flat=True):
    """Batched weight packing from a device int64 descriptor table [n, 9].  flat: one 1-D grid of ``blocks``
    blocks, column 8 of each record its first block (mer_pack_conv_weights_flat); otherwise the 2-D grid of
    mer_pack_conv_weights (``blocks`` is then the total element count and column 8 is ignored)."""
    if desc.dtype != torch.int64 or desc.dim() != 2 or desc.shape[1] != 9 or not desc.is_cuda:
        raise ValueError("pack descriptor table must be a device int64 [n, 9] tensor")
    name = "mer_pack_conv_weights_flat" if flat else "mer_pack_conv_weights"
    LIB(name, desc.shape[0], desc.data_ptr(), int(blocks), stream_ptr())


def bn_finalize(stats, M, eps, momentum, ms, rmean=None, rvar=None, nbt=None, rows=None):
    """``rows``: the leading statistics rows the producing conv_fwd wrote (its return value), else all of them."""
    C = ms.shape[0]
    if stats is not None and (stats.numel() != bn_stat_rows(int(M)) * C * 2 or not stats.is_contiguous()):
        raise ValueError("bn_finalize stats must be the conv_fwd float[bn_stat_rows(M)][C][2] buffer")
    if rows is None:
        rows = bn_stat_rows(int(M)) - 64
    LIB("mer_bn_finalize_rows", C, int(M), int(rows), _ptr(stats), float(eps), float(momentum), ms.data_ptr(),
        _ptr(rmean), _ptr(rvar), _ptr(nbt), stream_ptr())


def bn_finalize_pair(a, b, eps, momentum):
    """Two train-mode bn_finalize calls in one launch (mer_bn_finalize_rows2); a / b = (stats, M, ms, rmean, rvar,
    nbt, rows) with rows the conv_fwd return value (None: every row)."""
    args = []
    for stats, M, ms, rmean, rvar, nbt, rows in (a, b):
        C = ms.shape[0]
        if stats is None or stats.numel() != bn_stat_rows(int(M)) * C * 2 or not stats.is_contiguous():
            raise ValueError("bn_finalize_pair stats must be conv_fwd float[bn_stat_rows(M)][C][2] buffers")
        rows = bn_stat_rows(int(M)) - 64 if rows is None else rows
        args += [C, int(M), int(rows), stats.data_ptr(), ms.data_ptr(), _ptr(rmean), _ptr(rvar), _ptr(nbt)]
    LIB("mer_bn_finalize_rows2", *args, float(eps), float(momentum), stream_ptr())


def partials_sum_pair(buf_a, out_a, buf_b, out_b, rows=None):
    """partials_sum of two same-shape buffers in one launch (mer_partials_sum2)."""
    P, C, _ = buf_a.shape
    if tuple(buf_b.shape) != (P, C, 2) or P <= 64:
        raise ValueError("partials_sum_pair expects two bn_red_rows(M) buffers of one shape")
    rows = P - 64 if rows is None else rows
    if not 0 < rows <= P - 64:
        raise ValueError("partials_sum_pair rows out of range")
    LIB("mer_partials_sum2", C, int(rows), buf_a.data_ptr(), out_a.data_ptr(), buf_b.data_ptr(), out_b.data_ptr(),
        stream_ptr())
    return out_a, out_b


def bn_apply(x, ms, gamma, beta, y, relu, res=None, ms2=None, gamma2=None, beta2=None):
    C = x.shape[-1]
    M = x.numel() // C
    LIB("mer_bn_apply", M, C, x.data_ptr(), ms.data_ptr(), gamma.data_ptr(), beta.data_ptr(), _ptr(res), _ptr(ms2),
        _ptr(gamma2), _ptr(beta2), int(relu), y.data_ptr(), stream_ptr())


def bn_bwd_reduce(dy, mask, x, ms, red, workspace=None):
    """red[C,2] = (sum g, sum g*xhat) (written); workspace: float[BN_RED_WS_ROWS * C * 2] or None."""
    C = x.shape[-1]
    if workspace is None:
        workspace = torch.empty(BN_RED_WS_ROWS * C * 2, device=x.device, dtype=torch.float32)
    if workspace.numel() < BN_RED_WS_ROWS * C * 2:
        raise ValueError("bn_bwd_reduce workspace too small")
    LIB("mer_bn_bwd_reduce", x.numel() // C, C, dy.data_ptr(), _ptr(mask), x.data_ptr(), ms.data_ptr(),
        red.data_ptr(), workspace.data_ptr(), stream_ptr())


def bn_bwd_apply(dy, mask, x, ms, gamma, red, dx, dgamma, dbeta, batch_stats=True):
    C = x.shape[-1]
    LIB("mer_bn_bwd_apply", x.numel() // C, C, dy.data_ptr(), _ptr(mask), x.data_ptr(), ms.data_ptr(),
        gamma.data_ptr(), red.data_ptr(), int(batch_stats), dx.data_ptr(), _ptr(dgamma), _ptr(dbeta), stream_ptr())


def bn_bwd_apply2(dy, mask, x, ms, gamma, red, dx, dgamma, dbeta, x2, ms2, gamma2, red2, dx2, dgamma2, dbeta2,
                  batch_stats=True):
    """Two bn_bwd_apply passes sharing dy and the (non-None) mask in one launch (mer_bn_bwd_apply2)."""
    C = x.shape[-1]
    for t in (dy, mask, x2, dx, dx2):
        if tuple(t.shape) != tuple(x.shape):
            raise ValueError("bn_bwd_apply2 tensors must share one shape")
    LIB("mer_bn_bwd_apply2", x.numel() // C, C, dy.data_ptr(), mask.data_ptr(), x.data_ptr(), ms.data_ptr(),
        gamma.data_ptr(), red.data_ptr(), x2.data_ptr(), ms2.data_ptr(), gamma2.data_ptr(), red2.data_ptr(),
        int(batch_stats), dx.data_ptr(), dx2.data_ptr(), _ptr(dgamma), _ptr(dbeta), _ptr(dgamma2), _ptr(dbeta2),
        stream_ptr())


def maxpool_fwd(x, y, arg):
    N, H, W, C = x.shape
    LIB("mer_maxpool_fwd", N, H, W, C, x.data_ptr(), y.data_ptr(), arg.data_ptr(), stream_ptr())


def stem_bnrelu_maxpool(x, ms, gamma, beta, y, arg):
    """Fused stem tail: y/arg = maxpool3x3s2p1(relu(bn(x))) without storing the activation."""
    N, H, W, C = x.shape
    LIB("mer_stem_bnrelu_maxpool_fwd", N, H, W, C, x.data_ptr(), ms.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
        y.data_ptr(), arg.data_ptr(), stream_ptr())


def stem_pool_bn_bwd(dy, arg, x, ms, gamma, beta, red, dx, dgamma, dbeta, batch_stats=True, workspace=None):
    """Backward of stem_bnrelu_maxpool to the conv output x (red: float[C][2] written; workspace as
    bn_bwd_reduce)."""
    N, H, W, C = x.shape
    if workspace is None:
        workspace = torch.empty(BN_RED_WS_ROWS * C * 2, device=x.device, dtype=torch.float32)
    if workspace.numel() < BN_RED_WS_ROWS * C * 2:
        raise ValueError("stem_pool_bn_bwd workspace too small")
    LIB("mer_stem_pool_bn_bwd", N, H, W, C, dy.data_ptr(), arg.data_ptr(), x.data_ptr(), ms.data_ptr(),
        gamma.data_ptr(), beta.data_ptr(), red.data_ptr(), int(batch_stats), dx.data_ptr(), _ptr(dgamma),
        _ptr(dbeta), workspace.data_ptr(), stream_ptr())


def maxpool_bwd(dy, arg, dx):
    N, H, W, C = dx.shape
    LIB("mer_maxpool_bwd", N, H, W, C, dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), stream_ptr())


def avgpool_fwd(x, y):
    N, H, W, C = x.shape
    LIB("mer_avgpool_fwd", N, H * W, C, x.data_ptr(), y.data_ptr(), stream_ptr())


def avgpool_bwd(dy, dx):
    N, H, W, C = dx.shape
    LIB("mer_avgpool_bwd", N, H * W, C, dy.data_ptr(), dx.data_ptr(), stream_ptr())


def softmax_avg_fwd(za, zv, out, pa, pv):
    B, C = za.shape
    LIB("mer_softmax_avg_fwd", B, C, za.data_ptr(), zv.data_ptr(), out.data_ptr(), pa.data_ptr(), pv.data_ptr(),
        stream_ptr())


def softmax_avg_bwd(pa, pv, dout, da, dv):
    B, C = pa.shape
    LIB("mer_softmax_avg_bwd", B, C, pa.data_ptr(), pv.data_ptr(), dout.data_ptr(), da.data_ptr(), dv.data_ptr(),
        stream_ptr())


# ---- dynamic INT8 Linear (TorchModelRunner enable_dynamic_quant) ----
QP_PARTIAL = 2 * 512  # floats of min/max workspace for mer_quant_params_f32


def quant_params(x, partial, qparams, mode):
    """qparams[4] = {scale, 1/scale, zero_point, 0} from min/max over all of x (mode 0 act, 1 weight)."""
    _check_dev(x, partial, qparams)
    if not x.is_contiguous() or x.data_ptr() % 16:
        raise ValueError("quant_params needs a contiguous 16-byte aligned tensor")
    LIB("mer_quant_params", x.numel(), x.data_ptr(), _dt(x), partial.data_ptr(), int(mode), qparams.data_ptr(),
        stream_ptr())


def quantize_weight_s8(w, qparams, qw, colsum):
    N, K = w.shape
    if qw.shape[0] != N or qw.shape[1] < K or qw.shape[1] % 16 or qw.dtype != torch.int8:
        raise ValueError("qw must be int8 [N, ldq>=K], ldq % 16 == 0")
    LIB("mer_quantize_weight_s8", N, K, w.data_ptr(), w.stride(0), qparams.data_ptr(), qw.data_ptr(), qw.stride(0),
        colsum.data_ptr(), stream_ptr())


def gemm_i8dyn(x2d, x_qparams, qw, w_qparams, colsum, bias, out, act="none"):
    _check_dev(x2d, qw, out)
    M, K = x2d.shape
    N = qw.shape[0]
    if x2d.stride(1) != 1 or x2d.stride(0) % 8 or K % 16 or out.shape != (M, N) or x2d.data_ptr() % 16:
        raise ValueError(f"gemm_i8dyn: bad operands x{tuple(x2d.shape)} qw{tuple(qw.shape)} out{tuple(out.shape)}")
    _launch("gemm_i8dyn", (M, N, K), "mer_gemm_i8dyn", M, N, K, x2d.data_ptr(), _dt(x2d), x2d.stride(0), x_qparams.data_ptr(),
            qw.data_ptr(), qw.stride(0), w_qparams.data_ptr(), colsum.data_ptr(), _ptr(bias), ACT[act], out.data_ptr(),
            out.stride(0), stream_ptr())
    return out


# ---------------------------------------------------------------------------------------------------
# WavLM stage-2 fine-tuning (backward of the unfrozen last layers, csrc/wavlm_train.hip)
def _ptr0(t):
    return 0 if t is None else t.data_ptr()


def fold_rows(part, parts, n, ldp, out, offset=0):
    """out[k] += sum_p part[offset + p*ldp + k] (fixed order)."""
    if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() != n:
        raise ValueError("fold_rows: out must be contiguous fp32 of n elements")
    if offset + (parts - 1) * ldp + n > part.numel():
        raise ValueError("fold_rows: partial rows out of range")
    ws = _workspace(64 * n, out.device) if parts > 64 else None
    LIB("mer_fold_rows", int(parts), int(n), part.data_ptr() + 4 * offset, int(ldp), out.data_ptr(), _ptr0(ws),
        stream_ptr())


def ln_bwd(dy_a, x, gamma, eps, dy_b=None, dy_c=None, dx32=None, dx16=None):
    """LayerNorm backward on rows of x (fp32 pre-LN input).  Returns the partial-row buffer
    [ceil(rows/16)][3][d] (dgamma | dbeta | sum dx) for fold_rows."""
    rows, d = x.shape
    for t in (dy_a, dy_b, dy_c, dx32):
        if t is not None and (t.dtype != torch.float32 or tuple(t.shape) != (rows, d) or not t.is_contiguous()):
            raise ValueError("ln_bwd: fp32 [rows, d] contiguous operands expected")
    if dx16 is not None and (dx16.dtype != torch.bfloat16 or tuple(dx16.shape) != (rows, d)):
        raise ValueError("ln_bwd: dx16 must be bf16 [rows, d]")
    if x.dtype != torch.float32 or not x.is_contiguous() or d % 256 or d > 1024:
        raise ValueError("ln_bwd: x must be contiguous fp32 with d % 256 == 0, d <= 1024")
    part = _workspace(((rows + 15) // 16) * 3 * d, x.device)
    LIB("mer_ln_bwd", rows, d, dy_a.data_ptr(), _ptr0(dy_b), _ptr0(dy_c), x.data_ptr(), gamma.data_ptr(), float(eps),
        _ptr0(dx32), _ptr0(dx16), part.data_ptr(), stream_ptr())
    return part


def ln_bwd_fold(part, rows, d, dgamma=None, dbeta=None, dbias=None):
    parts = (rows + 15) // 16
    for i, out in enumerate((dgamma, dbeta, dbias)):
        if out is not None:
            fold_rows(part, parts, d, 3 * d, out, offset=i * d)


def colsum_into(x2d, out, col0=0, ncols=None):
    """out += colsum(x2d[:, col0:col0+ncols]) (deterministic, fixed order)."""
    rows, cols = x2d.shape
    part = _workspace(((rows + 63) // 64) * cols, x2d.device)
    LIB("mer_colpart", rows, cols, x2d.data_ptr(), _dt(x2d), x2d.stride(0), part.data_ptr(), stream_ptr())
    ncols = cols - col0 if ncols is None else ncols
    fold_rows(part, (rows + 63) // 64, ncols, cols, out, offset=col0)


def gelu_bf16(z, f):
    if z.dtype != torch.bfloat16 or f.dtype != torch.bfloat16 or z.numel() != f.numel() or z.numel() % 8:
        raise ValueError("gelu_bf16: bf16 operands of equal size (multiple of 8)")
    LIB("mer_gelu_bf16", z.numel(), z.data_ptr(), f.data_ptr(), stream_ptr())


def gelu_bwd(df, z, dz, dbias):
    """dz = df * gelu'(z) (bf16); dbias += colsum(dz)."""
    rows, cols = z.shape
    if df.dtype != torch.float32 or tuple(df.shape) != (rows, cols) or dz.dtype != torch.bfloat16:
        raise ValueError("gelu_bwd shapes")
    part = _workspace(((rows + 63) // 64) * cols, z.device)
    LIB("mer_gelu_bwd", rows, cols, df.data_ptr(), z.data_ptr(), dz.data_ptr(), part.data_ptr(), stream_ptr())
    fold_rows(part, (rows + 63) // 64, cols, cols, dbias)


def linear_wgrad(x, dy, dw, col0=0):
    """dw[N,K] += dy[:, col0:col0+N]^T x (bf16 MFMA); x bf16 [M,K] contiguous, dy bf16 [M, >= col0+N]."""
    M, Kin = x.shape
    N = dw.shape[0]
    if (x.dtype != torch.bfloat16 or dy.dtype != torch.bfloat16 or dw.dtype != torch.float32 or not x.is_contiguous()
            or tuple(dw.shape) != (N, Kin) or dy.shape[0] != M or dy.shape[1] < col0 + N or dy.stride(1) != 1
            or Kin % 8 or N % 8 or col0 % 8 or dy.stride(0) % 8):
        raise ValueError("linear_wgrad shapes")
    tiles = ((N + 127) // 128) * ((Kin + 127) // 128)
    splits = int(max(1, min(-(-512 // tiles), M // 512)))
    ws = _workspace(splits * N * Kin, x.device)
    LIB("mer_linear_wgrad", M, N, Kin, x.data_ptr(), dy.data_ptr() + 2 * col0, dy.stride(0), dw.data_ptr(), splits,
        ws.data_ptr(), stream_ptr())


def _attn_bwd_kp(L):
    """mer_wavlm_attention_bwd_kp: padded key count of the attention-backward scratch (16 * 4/8/10/12)."""
    nt = -(-L // 16)
    return 16 * (4 if nt <= 4 else 8 if nt <= 8 else 10 if nt <= 10 else 12)


def wavlm_attention_bwd(qkv, x, dout, gate_w, gate_b, gate_const, tbl, B, L, H, scale, dqkv, dx_gate=None,
                        drop_p=0.0, rng=None, site=0):
    """Backward of wavlm_attention (per-head table form; ``drop_p`` / ``rng`` / ``site``: the forward's attention-
    probability dropout, its mask regenerated).  Returns the gate partial rows [B*H*ceil(L/64)][8*64 + 8 + H] for
    fold_rows."""
    M = B * L
    if L > 192 or tuple(qkv.shape) != (M, 3 * H * 64) or tuple(dqkv.shape) != (M, 3 * H * 64) or dout.shape[0] != M:
        raise ValueError("wavlm_attention_bwd shapes")
    if qkv.dtype != torch.bfloat16 or dout.dtype != torch.float32 or dqkv.dtype != torch.bfloat16:
        raise ValueError("wavlm_attention_bwd expects bf16 qkv / dqkv and fp32 dout")
    if tuple(tbl.shape) != (H, 2 * L - 1) or tbl.dtype != torch.float32:
        raise ValueError("wavlm_attention_bwd: bias table [H, 2L-1] fp32")
    kp = _attn_bwd_kp(L)
    scratch = torch.empty(B * H * kp * (3 * kp + 64), device=qkv.device, dtype=torch.bfloat16)
    nrb = (L + 63) // 64  # AB_ROWS query rows per block (csrc/wavlm_train.hip)
    gpart = _workspace(B * H * nrb * (8 * 64 + 8 + H), qkv.device)
    tr = _train_args(drop_p, rng, site, None, 0)[:3]
    LIB("mer_wavlm_attention_bwd_tr", B, L, H, qkv.data_ptr(), qkv.stride(0), x.data_ptr(), x.stride(0),
        dout.data_ptr(), dout.stride(0), gate_w.data_ptr(), gate_b.data_ptr(), gate_const.data_ptr(), tbl.data_ptr(),
        float(scale), scratch.data_ptr(), dqkv.data_ptr(), dqkv.stride(0), _ptr0(dx_gate),
        dx_gate.stride(0) if dx_gate is not None else 0, gpart.data_ptr(), *tr, stream_ptr())
    return gpart, B * H * nrb


def dropout_rows(x, drop_p, rng, site, y32=None, y16=None):
    """y = x * mask / (1 - p) for dropout call site ``site`` (mask index row * cols + col, as the GEMM-epilogue
    dropout), fp32 and / or bf16 outputs (in place allowed when the dtypes match)."""
    rows, cols = x.shape
    for y in (y32, y16):
        if y is not None and tuple(y.shape) != (rows, cols):
            raise ValueError("dropout_rows output shape")
    if (y32 is not None and y32.dtype != torch.float32) or (y16 is not None and y16.dtype != torch.bfloat16):
        raise ValueError("dropout_rows: y32 fp32, y16 bf16")
    tr = _train_args(drop_p, rng, site, None, 0)[:3]
    LIB("mer_dropout_rows", rows, cols, x.data_ptr(), _dt(x), x.stride(0), _ptr0(y32),
        y32.stride(0) if y32 is not None else 0, _ptr0(y16), y16.stride(0) if y16 is not None else 0, *tr, stream_ptr())


def transpose_bf16(src, dst):
    rows, cols = src.shape
    if src.dtype != torch.bfloat16 or dst.dtype != torch.bfloat16 or tuple(dst.shape) != (cols, rows):
        raise ValueError("transpose_bf16 shapes")
    LIB("mer_transpose_bf16", rows, cols, src.data_ptr(), src.stride(0), dst.data_ptr(), dst.stride(0), stream_ptr())


# ---------------------------------------------------------------------------------------------------
# CLIP-style alignment loss (csrc/align.hip)
def clip_align_fwd(a, v, log_scale, an, vn, norms, logits, loss):
    B, D = a.shape
    for t in (a, v, an, vn):
        if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != (B, D):
            raise ValueError("clip_align_fwd: contiguous fp32 [B, D] operands expected")
    if norms.numel() != 2 * B or logits.numel() != B * B or loss.numel() != 1 or log_scale.numel() != 1:
        raise ValueError("clip_align_fwd: norms [2B], logits [B, B], loss [1], log_scale [1]")
    _check_dev(a, v, log_scale, an, vn, norms, logits, loss)
    LIB("mer_clip_align_fwd", B, D, a.data_ptr(), v.data_ptr(), log_scale.data_ptr(), an.data_ptr(), vn.data_ptr(),
        norms.data_ptr(), logits.data_ptr(), loss.data_ptr(), stream_ptr())


def clip_align_bwd(an, vn, norms, logits, log_scale, dloss, da, dv, dlog_scale=None):
    B, D = an.shape
    if tuple(da.shape) != (B, D) or tuple(dv.shape) != (B, D) or not (da.is_contiguous() and dv.is_contiguous()):
        raise ValueError("clip_align_bwd: da / dv must be contiguous [B, D]")
    ws = _workspace(B * B, an.device)
    LIB("mer_clip_align_bwd", B, D, an.data_ptr(), vn.data_ptr(), norms.data_ptr(), logits.data_ptr(),
        log_scale.data_ptr(), dloss.data_ptr(), ws.data_ptr(), da.data_ptr(), dv.data_ptr(), _ptr(dlog_scale),
        stream_ptr())


def add_scaled_scalar(x, y, w, out):
    LIB("mer_add_scaled_scalar", x.data_ptr(), y.data_ptr(), float(w), out.data_ptr(), stream_ptr())


def concat_prior_rows(tok, prior, out, L):
    """out[b*L + l] = [tok[b*L + l], prior[b], 0 ...] (INT8 token-bias input rows)."""
    rows, d = tok.shape
    B, pd = prior.shape
    if rows != B * L or out.shape[0] != rows or out.shape[1] < d + pd or not out.is_contiguous():
        raise ValueError("concat_prior_rows shapes")
    LIB("mer_concat_prior_rows", B, L, d, pd, out.shape[1], tok.contiguous().data_ptr(), prior.contiguous().data_ptr(),
        out.data_ptr(), stream_ptr())
    return out


def softmax_dropout_fwd(S, scale, P, Pd, h, p=0.0, rng=None, site=0):
    B, H, Lq, Lk = P.shape
    LIB("mer_softmax_dropout_fwd", B, H, int(h), Lq, Lk, S.data_ptr(), float(scale), P.data_ptr(), Pd.data_ptr(),
        float(p), rng_ptr(rng), int(site), stream_ptr())


def mha_bwd_lds_bytes(Lq: int, Lk: int, dh: int) -> int:
    import ctypes
    out = ctypes.c_long(0)
    LIB("mer_mha_bwd_lds_bytes", int(Lq), int(Lk), int(dh), ctypes.addressof(out))
    return int(out.value)


# ---------------------------------------------------------------------------------------------------
# fused xattn head forward (csrc/xattn_fused.hip)
def xh_split(desc):
    if desc.dtype != torch.int64 or desc.dim() != 2 or desc.shape[1] != 7 or not desc.is_cuda:
        raise ValueError("split descriptor table must be a device int64 [n, 7] tensor")
    LIB("mer_xh_split", desc.shape[0], desc.data_ptr(), stream_ptr())


def _planes(w):
    hi, lo = w
    return hi.data_ptr(), lo.data_ptr()


def _f32c(*ts):
    for t in ts:
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda):
            raise ValueError("fused head: contiguous fp32 device tensors expected")


def xh_audio_fwd(af, Ws, bs, Wa, ba, Wc, bq2, bkv1, a_s, a, q2, kv1, vf, Wv, bv, Wq1, bq1, v, q1):
    M, S = af.shape
    Mv, vdim = vf.shape
    if af.stride(1) != 1 or Ws[0].shape != (128, S) or Wc[0].shape != (384, 128) or Wv[0].shape != (128, vdim) \
            or tuple(v.shape) != (Mv, 128) or tuple(q1.shape) != (Mv, 128):
        raise ValueError("xh_audio_fwd shapes")
    _f32c(a_s, a, q2, kv1, vf, v, q1)
    _launch("xh_audio_fwd", (M, S), "mer_xh_audio_fwd", M, S, af.data_ptr(), _dt(af), af.stride(0), *_planes(Ws),
            bs.data_ptr(), *_planes(Wa), ba.data_ptr(), *_planes(Wc), bq2.data_ptr(), bkv1.data_ptr(), a_s.data_ptr(),
            a.data_ptr(), q2.data_ptr(), kv1.data_ptr(), Mv, vdim, vf.data_ptr(), *_planes(Wv), bv.data_ptr(),
            *_planes(Wq1), bq1.data_ptr(), v.data_ptr(), q1.data_ptr(), stream_ptr())


def xh_audio_fwd_pair(pair, bs, Wa, ba, Wc, bq2, bkv1, a_s, a, q2, kv1, vf, Wv, bv, Wq1, bq1, v, q1):
    """F1 after the first product ran as one bf16 GEMM: ``pair`` = [aseq Ws_hi^T | aseq Ws_lo^T] fp32 [M, 256].
    Equal to ``xh_audio_fwd`` up to fp32 rounding (its halves are summed after the K loop, not per k step)."""
    M = pair.shape[0]
    Mv, vdim = vf.shape
    if pair.shape[1] != 256 or pair.stride(1) != 1 or Wc[0].shape != (384, 128) or Wv[0].shape != (128, vdim) \
            or tuple(v.shape) != (Mv, 128) or tuple(q1.shape) != (Mv, 128):
        raise ValueError("xh_audio_fwd_pair shapes")
    _f32c(pair, a_s, a, q2, kv1, vf, v, q1)
    _launch("xh_audio_fwd", (M, 256), "mer_xh_audio_fwd_pair", M, pair.data_ptr(), pair.stride(0), bs.data_ptr(),
            *_planes(Wa), ba.data_ptr(), *_planes(Wc), bq2.data_ptr(), bkv1.data_ptr(), a_s.data_ptr(), a.data_ptr(),
            q2.data_ptr(), kv1.data_ptr(), Mv, vdim, vf.data_ptr(), *_planes(Wv), bv.data_ptr(), *_planes(Wq1),
            bq1.data_ptr(), v.data_ptr(), q1.data_ptr(), stream_ptr())


def xh_v2a_fwd(B, T, Ta, v, q1, kv1, Wo1, bo1, gamma, beta, Wkv2, bkv2, attn_p, path_p, rng, site_attn, site_path,
               scale, P1, o1, s_v, mu_v, rs_v, v1, kv2, emb, bias=None):
    if tuple(v.shape) != (B * T, 128) or tuple(q1.shape) != (B * T, 128) or tuple(kv1.shape) != (B * Ta, 256) \
            or (bias is not None and bias.numel() != B * T * Ta):
        raise ValueError("xh_v2a_fwd shapes")
    _f32c(v, q1, kv1, P1, o1, s_v, mu_v, rs_v, v1, kv2, emb, bias)
    _launch("xh_v2a_fwd", (B, T, Ta), "mer_xh_v2a_fwd", B, T, Ta, v.data_ptr(), q1.data_ptr(), kv1.data_ptr(),
            *_planes(Wo1), bo1.data_ptr(), gamma.data_ptr(), beta.data_ptr(), *_planes(Wkv2), bkv2.data_ptr(),
            float(attn_p), float(path_p), rng_ptr(rng), int(site_attn), int(site_path), float(scale), P1.data_ptr(),
            o1.data_ptr(), s_v.data_ptr(), mu_v.data_ptr(), rs_v.data_ptr(), v1.data_ptr(), kv2.data_ptr(),
            emb.data_ptr(), emb.stride(0), _ptr(bias), stream_ptr())


def xh_a2v_fwd(B, T, Ta, q2, kv2, a, Wo2, bo2, gamma, beta, attn_p, path_p, rng, site_attn, site_path, scale, P2, o2,
               s_a, mu_a, rs_a, part, bias=None):
    if tuple(q2.shape) != (B * Ta, 128) or tuple(kv2.shape) != (B * T, 256) or part.numel() != B * ((Ta + 15) // 16) * 128 \
            or (bias is not None and bias.numel() != B * T * Ta):
        raise ValueError("xh_a2v_fwd shapes")
    _f32c(q2, kv2, a, P2, o2, s_a, mu_a, rs_a, part, bias)
    _launch("xh_a2v_fwd", (B, T, Ta), "mer_xh_a2v_fwd", B, T, Ta, q2.data_ptr(), kv2.data_ptr(), a.data_ptr(),
            *_planes(Wo2), bo2.data_ptr(), gamma.data_ptr(), beta.data_ptr(), float(attn_p), float(path_p),
            rng_ptr(rng), int(site_attn), int(site_path), float(scale), P2.data_ptr(), o2.data_ptr(), s_a.data_ptr(),
            mu_a.data_ptr(), rs_a.data_ptr(), part.data_ptr(), _ptr(bias), stream_ptr())


def xh_mlp_fwd(B, Ta, gated, part, emb, W0, b0, W3, b3, Wc, bc, mlp_p, rng, site, h, g, fused, logits):
    H1, C = W0.shape[0], logits.shape[1]
    if W0.shape[1] != 256 or tuple(emb.shape) != (B, 256) or (gated and (W3.shape[0] != 1 or Wc is None)):
        raise ValueError("xh_mlp_fwd shapes")
    _f32c(part, emb, W0, b0, W3, b3, h, logits)
    LIB("mer_xh_mlp_fwd", B, Ta, int(bool(gated)), H1, C, part.data_ptr(), emb.data_ptr(), W0.data_ptr(), b0.data_ptr(),
        W3.data_ptr(), b3.data_ptr(), _ptr(Wc), _ptr(bc), float(mlp_p), rng_ptr(rng) if mlp_p > 0 else 0, int(site),
        h.data_ptr(), _ptr(g), _ptr(fused), logits.data_ptr(), stream_ptr())


def xh_prior_fwd(B, T, Ta, v, a, W0, b0, W3, b3, heads, scale, drop_p, rng, site, pg, h1, prior, tt, tp, v2a_bias,
                 a2v_bias):
    """The emotion-prior adapter forward in one launch (csrc/prior.hip): ``heads`` = [(weight [1, d + PD], bias [1])]
    of the v_query, a_key, a_query, v_key token-bias Linears; ``tt`` / ``tp`` = their 4 token / prior halves."""
    d, H1, PD = v.shape[1], W0.shape[0], W3.shape[0]
    if tuple(v.shape) != (B * T, d) or tuple(a.shape) != (B * Ta, d) or W0.shape[1] != 2 * d or W3.shape[1] != H1 \
            or any(w.numel() != d + PD or bb.numel() != 1 for w, bb in heads) or len(tt) != 4 or len(tp) != 4 \
            or tuple(v2a_bias.shape) != (B, T, Ta) or tuple(a2v_bias.shape) != (B, Ta, T):
        raise ValueError("xh_prior_fwd shapes")
    _f32c(v, a, W0, b0, W3, b3, pg, h1, prior, v2a_bias, a2v_bias, *tt, *tp, *[w for w, _ in heads])
    hw = [x.data_ptr() for wb in heads for x in wb]
    LIB("mer_xh_prior_fwd", B, T, Ta, d, H1, PD, v.data_ptr(), a.data_ptr(), W0.data_ptr(), b0.data_ptr(), W3.data_ptr(),
        b3.data_ptr(), *hw, scale.data_ptr(), float(drop_p), rng_ptr(rng) if drop_p > 0 else 0, int(site),
        pg.data_ptr(), h1.data_ptr(), prior.data_ptr(), *[t.data_ptr() for t in tt], *[t.data_ptr() for t in tp],
        v2a_bias.data_ptr(), a2v_bias.data_ptr(), stream_ptr())


def xh_prior_bwd(B, T, Ta, dbias_v2a, dbias_a2v, tt, tp, scale, head_w, W0, W3, h1, drop_p, rng, site, dtt, dtp,
                 dprior, dh1, dscale_part, dv, da):
    """Its backward (csrc/prior.hip): dtt / dtp / dprior / dh1 / dscale_part out, token gradients ADDED into dv, da."""
    d, H1, PD = dv.shape[1], W0.shape[0], W3.shape[0]
    if tuple(dbias_v2a.shape) != (B, T, Ta) or tuple(dbias_a2v.shape) != (B, Ta, T) or tuple(dv.shape) != (B * T, d) \
            or tuple(da.shape) != (B * Ta, d) or dscale_part.numel() != B or len(head_w) != 4:
        raise ValueError("xh_prior_bwd shapes")
    _f32c(dbias_v2a, dbias_a2v, W0, W3, h1, dprior, dh1, dscale_part, dv, da, *tt, *tp, *dtt, *dtp, *head_w)
    LIB("mer_xh_prior_bwd", B, T, Ta, d, H1, PD, dbias_v2a.data_ptr(), dbias_a2v.data_ptr(),
        *[t.data_ptr() for t in tt], *[t.data_ptr() for t in tp], scale.data_ptr(), *[w.data_ptr() for w in head_w],
        W0.data_ptr(), W3.data_ptr(), h1.data_ptr(), float(drop_p), rng_ptr(rng) if drop_p > 0 else 0, int(site),
        *[t.data_ptr() for t in dtt], *[t.data_ptr() for t in dtp], dprior.data_ptr(), dh1.data_ptr(),
        dscale_part.data_ptr(), dv.data_ptr(), da.data_ptr(), stream_ptr())


# ---------------------------------------------------------------------------------------------------
# fused xattn head backward (csrc/xattn_fused_bwd.hip); W*T arguments are transposed (hi, lo) planes
def xh_mlp_bwd(B, gated, dlogits, emb, h, g, W0, W3, Wc, mlp_p, rng, site, dh, dz, demb):
    """G4: the classifier head's data gradients -> dh [B, H1], dz [B] (gated), demb [B, 256]."""
    H1, C = W0.shape[0], dlogits.shape[1]
    if W0.shape[1] != 256 or tuple(emb.shape) != (B, 256) or tuple(demb.shape) != (B, 256) or tuple(h.shape) != (B, H1) \
            or tuple(dh.shape) != (B, H1) or (gated and (dz is None or dz.numel() != B)):
        raise ValueError("xh_mlp_bwd shapes")
    _f32c(dlogits, emb, h, g, W0, W3, Wc, dh, dz, demb)
    _launch("xh_mlp_bwd", (B,), "mer_xh_mlp_bwd", B, C, H1, int(bool(gated)), dlogits.data_ptr(), emb.data_ptr(),
            h.data_ptr(), _ptr(g), W0.data_ptr(), W3.data_ptr(), _ptr(Wc), float(mlp_p),
            rng_ptr(rng) if mlp_p > 0 else 0, int(site), dh.data_ptr(), _ptr(dz), demb.data_ptr(), stream_ptr())


def xh_a2v_bwd(B, T, Ta, demb, s_a, mu_a, rs_a, gamma, P2, kv2, q2, WoT2, attn_p, path_p, rng, site_attn, site_path,
               scale, da, da2, dqkv, dkv2_part, ln_part, dbias=None):
    nt = (Ta + 15) // 16
    if tuple(q2.shape) != (B * Ta, 128) or tuple(kv2.shape) != (B * T, 256) or tuple(dqkv.shape) != (B * Ta, 384) \
            or dkv2_part.numel() != B * nt * 16 * 256 or ln_part.numel() != B * nt * 256 or WoT2[0].shape != (128, 128):
        raise ValueError("xh_a2v_bwd shapes")
    _f32c(demb, s_a, mu_a, rs_a, gamma, P2, kv2, q2, da, da2, dqkv, dkv2_part, ln_part, dbias)
    if dbias is not None and dbias.numel() != B * Ta * T:
        raise ValueError("xh_a2v_bwd dbias shape")
    _launch("xh_a2v_bwd", (B, T, Ta), "mer_xh_a2v_bwd", B, T, Ta, demb.data_ptr(), s_a.data_ptr(), mu_a.data_ptr(),
            rs_a.data_ptr(), gamma.data_ptr(), P2.data_ptr(), kv2.data_ptr(), q2.data_ptr(), *_planes(WoT2),
            float(attn_p), float(path_p), rng_ptr(rng) if (attn_p > 0 or path_p > 0) else 0, int(site_attn),
            int(site_path), float(scale), da.data_ptr(), da2.data_ptr(), dqkv.data_ptr(), dkv2_part.data_ptr(),
            ln_part.data_ptr(), _ptr(dbias), stream_ptr())


def xh_v2a_bwd(B, T, Ta, dkv2_part, WkvT2, demb, s_v, mu_v, rs_v, gamma, WoT1, P1, kv1, q1, attn_p, path_p, rng,
               site_attn, site_path, scale, dkv2, dv2, dq1, dv, dqkv, ln_part, dbias=None):
    if tuple(kv1.shape) != (B * Ta, 256) or tuple(q1.shape) != (B * T, 128) or tuple(dkv2.shape) != (B * T, 256) \
            or WkvT2[0].shape != (128, 256) or ln_part.numel() != B * 256 or tuple(dv.shape) != (B * T, 128) \
            or dkv2_part.numel() != B * ((Ta + 15) // 16) * 16 * 256:
        raise ValueError("xh_v2a_bwd shapes")
    _f32c(dkv2_part, demb, s_v, mu_v, rs_v, gamma, P1, kv1, q1, dkv2, dv2, dq1, dv, dqkv, ln_part, dbias)
    if dbias is not None and dbias.numel() != B * T * Ta:
        raise ValueError("xh_v2a_bwd dbias shape")
    dev = dv.device
    do1 = torch.empty(B * T, 128, device=dev, dtype=torch.float32)  # G2a -> G2b hand-off
    dsh = torch.empty(B, 4, T, Ta, device=dev, dtype=torch.float32) if dbias is not None else None
    _launch("xh_v2a_bwd", (B, T, Ta), "mer_xh_v2a_bwd", B, T, Ta, dkv2_part.data_ptr(), *_planes(WkvT2),
            demb.data_ptr(), s_v.data_ptr(), mu_v.data_ptr(), rs_v.data_ptr(), gamma.data_ptr(), *_planes(WoT1),
            P1.data_ptr(), kv1.data_ptr(), q1.data_ptr(), float(attn_p), float(path_p),
            rng_ptr(rng) if (attn_p > 0 or path_p > 0) else 0, int(site_attn), int(site_path), float(scale),
            dkv2.data_ptr(), dv2.data_ptr(), dq1.data_ptr(), dv.data_ptr(), dqkv.data_ptr(), ln_part.data_ptr(),
            do1.data_ptr(), _ptr(dsh), _ptr(dbias), stream_ptr())


def xh_audio_bwd(dqkv, WcT, WaT, da, da_s, dq1, WqT1, WvT, dv, dvfeat):
    M, Mv = dqkv.shape[0], dq1.shape[0]
    vdim = WvT[0].shape[0]
    if tuple(dqkv.shape) != (M, 384) or WcT[0].shape != (128, 384) or WaT[0].shape != (128, 128) \
            or tuple(da.shape) != (M, 128) or tuple(da_s.shape) != (M, 128) or tuple(dq1.shape) != (Mv, 128) \
            or tuple(dv.shape) != (Mv, 128) or WqT1[0].shape != (128, 128) or WvT[0].shape != (vdim, 128) \
            or (dvfeat is not None and tuple(dvfeat.shape) != (Mv, vdim)):
        raise ValueError("xh_audio_bwd shapes")
    _f32c(dqkv, da, da_s, dq1, dv, dvfeat)
    _launch("xh_audio_bwd", (M,), "mer_xh_audio_bwd", M, dqkv.data_ptr(), *_planes(WcT), *_planes(WaT), da.data_ptr(),
            da_s.data_ptr(), Mv, vdim, dq1.data_ptr(), *_planes(WqT1), *_planes(WvT), dv.data_ptr(), _ptr(dvfeat),
            stream_ptr())


class WGradTable:
    """Problem table of mer_xh_wgrad (grouped weight gradients): add(dY, X, dW, db, splits) per Linear, then
    ``ws_floats()`` for the workspace and ``run(ws)``.  Rows live in a host int64 array (the launch copies them
    into its kernel arguments, so a captured graph keeps them)."""

    COLS = 11

    def __init__(self):
        self.rows = []
        self.keep = []  # the tensors whose addresses the rows hold

    def add(self, dY, X, dW, db, splits=1):
        M, N = dY.shape
        if dY.dtype != torch.float32 or dY.stride(1) != 1:
            raise ValueError("wgrad dY: fp32 rows with unit column stride")
        if X is not None and (X.shape[0] != M or X.stride(1) != 1 or tuple(dW.shape) != (N, X.shape[1])):
            raise ValueError("wgrad X / dW shapes")
        for t in (dW, db):
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
                raise ValueError("wgrad outputs: contiguous fp32")
        if db is not None and db.numel() != N:
            raise ValueError("wgrad db shape")
        K = 0 if X is None else X.shape[1]
        splits = max(1, min(int(splits), M))
        self.rows.append([dY.data_ptr(), dY.stride(0), _ptr(X), 0 if X is None else X.stride(0),
                          BF16 if (X is not None and X.dtype == torch.bfloat16) else F32, M, N, K, splits, _ptr(dW),
                          _ptr(db)])
        self.keep += [dY, X, dW, db]
        return self

    def _table(self):
        import numpy as np
        if len(self.rows) > 32:
            raise ValueError("mer_xh_wgrad takes at most 32 problems")
        return np.ascontiguousarray(np.array(self.rows, dtype=np.int64))

    def ws_floats(self) -> int:
        import ctypes
        tab = self._table()
        out = ctypes.c_longlong(0)
        LIB("mer_xh_wgrad_ws_floats", len(self.rows), tab.ctypes.data, ctypes.addressof(out))
        return int(out.value)

    def run(self, ws):
        tab = self._table()
        if ws.dtype != torch.float32 or not ws.is_cuda:
            raise ValueError("wgrad workspace: fp32 device tensor")
        _launch("xh_wgrad", (len(self.rows),), "mer_xh_wgrad", len(self.rows), tab.ctypes.data, ws.data_ptr(),
                ws.numel(), stream_ptr())
