"""Shared test helpers: golden loading and oracle-parameter construction."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from oracle import fusion_ref, params

GOLDEN = Path(__file__).resolve().parent / "golden"


def golden(name: str):
    return np.load(GOLDEN / name, allow_pickle=False)


def torch_state(named_shapes, seed: int = 0):
    return {k: torch.from_numpy(v) for k, v in params.init_state(named_shapes, seed).items()}


def xattn_params(xattn_head="concat", use_prior=False, **kw):
    p = torch_state(fusion_ref.xattn_head_param_shapes(xattn_head=xattn_head, use_prior=use_prior, **kw))
    fusion_ref.gated_bias_init(p, xattn_head)
    return p


def clip_head_params(mode: str):
    """Parameters of FusionModel(mode, fusion_align_mode="clip") outside the encoders, numpy-seeded like
    tools/gen_golden.py (logit_scale = log(1/0.07); gated: both gate biases -1)."""
    d_al, cd = 256, 256
    shapes = [("semantic_alignment.logit_scale", ()), ("semantic_alignment.audio_proj.weight", (d_al, 768)),
              ("semantic_alignment.audio_proj.bias", (d_al,)), ("semantic_alignment.video_proj.weight", (d_al, 512)),
              ("semantic_alignment.video_proj.bias", (d_al,)), ("audio_proj.weight", (cd, d_al)),
              ("audio_proj.bias", (cd,)), ("video_proj.weight", (cd, d_al)), ("video_proj.bias", (cd,))]
    if mode == "concat":
        shapes += [("fusion.0.weight", (cd, 2 * cd)), ("fusion.0.bias", (cd,)), ("fusion.3.weight", (8, cd)),
                   ("fusion.3.bias", (8,))]
    else:
        shapes += [("gate.0.weight", (cd, 2 * cd)), ("gate.0.bias", (cd,)), ("gate.3.weight", (1, cd)),
                   ("gate.3.bias", (1,)), ("classifier.weight", (8, cd)), ("classifier.bias", (8,))]
    p = torch_state(shapes)
    p["semantic_alignment.logit_scale"] = torch.tensor(float(np.log(1.0 / 0.07)), dtype=torch.float32)
    if mode == "gated":
        p["gate.0.bias"].fill_(-1.0)
        p["gate.3.bias"].fill_(-1.0)
    return p


def check_grad(g, key: str, grad, atol: float):
    """Compare a gradient with a golden stored whole (``grad.<key>``) or trimmed (head rows + row/col sums)."""
    grad = grad.detach().cpu().numpy() if hasattr(grad, "detach") else np.asarray(grad)
    if "grad." + key in g.files:
        ref = g["grad." + key]
        np.testing.assert_allclose(grad, ref, atol=atol * max(1.0, float(np.abs(ref).max())), err_msg=key)
        return
    head = g["grad." + key + ".head"]
    atol = atol * max(1.0, float(np.abs(head).max()))
    np.testing.assert_allclose(grad[:head.shape[0]], head, atol=atol, err_msg=key)
    scale = max(1.0, float(np.sqrt(grad.shape[0] * grad.shape[1])))
    np.testing.assert_allclose(grad.sum(0), g["grad." + key + ".colsum"], atol=atol * scale, err_msg=key + " colsum")
    np.testing.assert_allclose(grad.sum(1), g["grad." + key + ".rowsum"], atol=atol * scale, err_msg=key + " rowsum")


# ---- restatement of the kernels' counter-based dropout RNG (csrc/common.h mer_hash / mer_site_seed /
# dropout_scale), so masks can be checked bit-exactly on the host ----
_M64 = (1 << 64) - 1


def site_seed(base: int, site: int) -> int:
    return (base * 0x100000001B3 + site * 0x9E3779B97F4A7C15 + 1) & _M64


def hash_u32(seed: int, idx: np.ndarray) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint64)
    u32 = np.uint32
    with np.errstate(over="ignore"):
        s = u32(seed & 0xFFFFFFFF) ^ (u32(seed >> 32) * u32(0x85EBCA6B))
        lo = (idx & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (idx >> np.uint64(32)).astype(np.uint32)
        x = (lo ^ (hi * u32(0xC2B2AE35))) * u32(0x9E3779B9) + s
        x ^= x >> u32(16)
        x *= u32(0x7FEB352D)
        x ^= x >> u32(15)
        x *= u32(0x846CA68B)
        x ^= x >> u32(16)
    return x.astype(np.uint32)


def dropout_keep(base: int, site: int, idx: np.ndarray, p: float) -> np.ndarray:
    """Boolean keep mask of the kernels' dropout_scale for element indices ``idx`` (the xattn head's sites)."""
    u = (hash_u32(site_seed(base, site), idx) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return u >= np.float32(p)


def dropout_keep_pair(base: int, site: int, idx: np.ndarray, p: float) -> np.ndarray:
    """Boolean keep mask of dropout_scale_pair (csrc/common.h; the WavLM encoder's sites): one hash word per index
    pair idx >> 1, its low 16 bits for the even index and the high 16 bits for the odd one, kept when >= ceil(p 2^16)."""
    idx = np.asarray(idx, dtype=np.uint64)
    h = hash_u32(site_seed(base, site), idx >> np.uint64(1))
    half = np.where((idx & np.uint64(1)) == 1, h >> np.uint32(16), h & np.uint32(0xFFFF))
    thr = np.uint32(np.ceil(np.float32(p) * np.float32(65536.0)))
    return half >= thr


def attention_mask_index(B: int, H: int, L: int) -> np.ndarray:
    """Mask indices of the WavLM attention-probability dropout for [B, H, L, L]: ((b*H + h)*L + i)*LE + j with the
    row stride LE = L rounded up to even (so a row's keys pair up)."""
    le = L + (L & 1)
    rows = np.arange(B * H * L, dtype=np.uint64)[:, None] * np.uint64(le)
    return (rows + np.arange(L, dtype=np.uint64)[None, :]).reshape(-1)
