"""Fused xattn head forward (csrc/xattn_fused.hip): the xattn branch after the encoders
(``src/models/fusion.py:372-411``) in four launches on split-bf16 MFMA, instead of the ~20 forward
launches of ``xattn_head.head_forward``.

Scope of the fused path: d_model 128 with 4 heads (the reference's defaults, fusion.py:199-200), mean temporal
pooling (the fusion default), concat or gated head, no emotion prior, audio features that need no gradient
(bf16 from the frozen WavLM, or fp32), T <= 16 frames and Ta <= 160 audio frames (3 s clips: 8 and 149).  Everything else -- and INT8
inference -- runs the unfused schedule, which is the parity reference of this path.  The saved activations
have the unfused schedule's names and layouts, so ``xattn_head.head_backward`` runs unchanged on them.
"""
from __future__ import annotations

import os
from typing import Dict

import torch

from . import kernels as K

ENABLED = os.environ.get("MER_XATTN_FUSED", "1") != "0"

# (weight name, row slice) for each split plane; rows are contiguous slices of the reference's parameters
_PLANES = {
    "Ws": [("audio_seq_proj.weight", None)],
    "Wa": [("a_in_proj.weight", None)],
    "Wc": [("a2v_attn.in_proj_weight", (0, 1)), ("v2a_attn.in_proj_weight", (1, 3))],  # [q2 | k1 v1]
    "Wv": [("v_in_proj.weight", None)],
    "Wq1": [("v2a_attn.in_proj_weight", (0, 1))],
    "Wo1": [("v2a_attn.out_proj.weight", None)],
    "Wkv2": [("a2v_attn.in_proj_weight", (1, 3))],
    "Wo2": [("a2v_attn.out_proj.weight", None)],
}


def supported(cfg, p: Dict[str, torch.Tensor], v_feat: torch.Tensor, a_seq: torch.Tensor, qlin) -> bool:
    if not ENABLED or qlin is not None or cfg.use_prior or cfg.temporal_pooling != "mean":
        return False
    if cfg.num_heads != 4 or p["v_in_proj.weight"].shape[0] != 128 or cfg.xattn_head not in ("concat", "gated"):
        return False
    B, T, vd = v_feat.shape
    _, Ta, sd = a_seq.shape
    if a_seq.dtype not in (torch.bfloat16, torch.float32) or v_feat.dtype != torch.float32 or T > 16 or Ta > 160 \
            or vd % 32 or sd % 32:
        return False
    if a_seq.requires_grad:  # the fused forward has no audio-feature gradient path (stage 2 runs unfused)
        return False
    return p["audio_seq_proj.weight"].shape == (128, sd) and p["v_in_proj.weight"].shape == (128, vd)


class SplitPlanes:
    """bf16 hi / lo planes of the head weights the fused kernels read, refreshed by ONE mer_xh_split launch per
    forward (inside the captured head graph, so every replay splits the current Adam-updated weights)."""

    def __init__(self, p: Dict[str, torch.Tensor]):
        dev = p["v_in_proj.weight"].device
        rows = []
        self.planes = {}
        for key, parts in _PLANES.items():
            srcs = []
            for name, sl in parts:
                w = p[name]
                if sl is not None:  # rows [sl0 * d, sl1 * d) of a packed [3d, d] in_proj weight
                    w = w[sl[0] * w.shape[1]:sl[1] * w.shape[1]]
                srcs.append(w)
            n_rows = sum(s.shape[0] for s in srcs)
            k = srcs[0].shape[1]
            hi = torch.empty(n_rows, k, device=dev, dtype=torch.bfloat16)
            lo = torch.empty(n_rows, k, device=dev, dtype=torch.bfloat16)
            off = 0
            for s in srcs:
                if not s.is_contiguous():
                    raise ValueError("split planes need contiguous weight rows")
                n = s.numel()
                rows.append([s.data_ptr(), hi.data_ptr() + 2 * off, lo.data_ptr() + 2 * off, n])
                off += n
            self.planes[key] = (hi, lo)
        self.desc = torch.tensor(rows, dtype=torch.int64).to(dev)
        self.key = tuple(r[0] for r in rows)

    def refresh(self):
        K.xh_split(self.desc)

    def __getitem__(self, key):
        return self.planes[key]


_CACHE: Dict[tuple, SplitPlanes] = {}


def planes_for(p: Dict[str, torch.Tensor]) -> SplitPlanes:
    key = tuple(p[n].data_ptr() for n in ("audio_seq_proj.weight", "a_in_proj.weight", "a2v_attn.in_proj_weight",
                                          "v2a_attn.in_proj_weight", "v_in_proj.weight", "v2a_attn.out_proj.weight",
                                          "a2v_attn.out_proj.weight"))
    sp = _CACHE.get(key)
    if sp is None:
        if len(_CACHE) > 8:
            _CACHE.clear()
        sp = _CACHE[key] = SplitPlanes(p)
    return sp


def fused_forward(p, cfg, v_feat, a_seq, training, rng, ctx, sites):
    """Fill ``ctx`` (xattn_head.HeadCtx) exactly as head_forward does and return the logits."""
    B, T, vd = v_feat.shape
    _, Ta, sd = a_seq.shape
    d, H = 128, 4
    dev = v_feat.device
    f32 = torch.float32
    e = lambda *shape: torch.empty(shape, device=dev, dtype=f32)  # noqa: E731
    dp_attn = cfg.attn_dropout if training else 0.0
    dp_path = cfg.drop_path if training else 0.0
    dp_mlp = cfg.mlp_dropout if training else 0.0
    site_prior, site_v2a, site_vpath, site_a2v, site_apath, site_mlp = sites
    seed = rng if (training and rng is not None) else None
    if training and (dp_attn > 0 or dp_path > 0 or dp_mlp > 0) and seed is None:
        raise ValueError("train-mode dropout needs the step's RNG base")
    sp = planes_for(p)
    sp.refresh()
    vf = v_feat.reshape(B * T, vd).contiguous()
    af = a_seq.reshape(B * Ta, sd).contiguous()
    a_s, a, q2, kv1 = e(B * Ta, d), e(B * Ta, d), e(B * Ta, d), e(B * Ta, 2 * d)
    K.xh_audio_fwd(af, sp["Ws"], p["audio_seq_proj.bias"], sp["Wa"], p["a_in_proj.bias"], sp["Wc"],
                   p["a2v_attn.in_proj_bias"][:d], p["v2a_attn.in_proj_bias"][d:], a_s, a, q2, kv1)
    v, q1, o1 = e(B * T, d), e(B * T, d), e(B * T, d)
    P1 = e(B, H, T, Ta)
    s_v, mu_v, rs_v, v1, kv2 = e(B * T, d), e(B * T), e(B * T), e(B * T, d), e(B * T, 2 * d)
    emb = e(B, 2 * d)
    scale = (d // H) ** -0.5
    K.xh_v2a_fwd(B, T, Ta, vf, sp["Wv"], p["v_in_proj.bias"], sp["Wq1"], p["v2a_attn.in_proj_bias"][:d], kv1,
                 sp["Wo1"], p["v2a_attn.out_proj.bias"], p["v_norm.weight"], p["v_norm.bias"], sp["Wkv2"],
                 p["a2v_attn.in_proj_bias"][d:], dp_attn, dp_path, seed, site_v2a, site_vpath, scale, v, q1, P1, o1,
                 s_v, mu_v, rs_v, v1, kv2, emb)
    o2, P2 = e(B * Ta, d), e(B, H, Ta, T)
    s_a, mu_a, rs_a = e(B * Ta, d), e(B * Ta), e(B * Ta)
    part = e(B, (Ta + 15) // 16, d)
    K.xh_a2v_fwd(B, T, Ta, q2, kv2, a, sp["Wo2"], p["a2v_attn.out_proj.bias"], p["a_norm.weight"], p["a_norm.bias"],
                 dp_attn, dp_path, seed, site_a2v, site_apath, scale, P2, o2, s_a, mu_a, rs_a, part)
    sv = ctx.saved
    sv.update(vf=vf, af=af, v=v, a_s=a_s, a=a, q1=q1, kv1=kv1, o1=o1, P1=P1, v1=v1, s_v=s_v, mu_v=mu_v, rs_v=rs_v,
              q2=q2, kv2=kv2, o2=o2, P2=P2, s_a=s_a, mu_a=mu_a, rs_a=rs_a, emb=emb)
    if cfg.xattn_head == "concat":
        W0, b0 = p["xattn_mlp.0.weight"], p["xattn_mlp.0.bias"]
        W3, b3 = p["xattn_mlp.3.weight"], p["xattn_mlp.3.bias"]
        h = e(B, W0.shape[0])
        logits = e(B, W3.shape[0])
        K.xh_mlp_fwd(B, Ta, False, part, emb, W0, b0, W3, b3, None, None, dp_mlp, seed, site_mlp, h, None, None, logits)
        sv["h"] = h
    else:
        W0, b0 = p["xattn_gate.0.weight"], p["xattn_gate.0.bias"]
        W3, b3 = p["xattn_gate.3.weight"], p["xattn_gate.3.bias"]
        Wc, bc = p["xattn_classifier.weight"], p["xattn_classifier.bias"]
        h, g, fused = e(B, W0.shape[0]), e(B), e(B, d)
        logits = e(B, Wc.shape[0])
        K.xh_mlp_fwd(B, Ta, True, part, emb, W0, b0, W3, b3, Wc, bc, dp_mlp, seed, site_mlp, h, g, fused, logits)
        sv.update(h=h, g=g, fused=fused)
    ctx.cfg = cfg
    ctx.drops = (dp_attn, dp_path, dp_mlp, 0.0)
    return logits
