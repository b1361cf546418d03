"""Fused xattn head forward (csrc/xattn_fused.hip): the xattn branch after the encoders
(``src/models/fusion.py:372-411``) in four launches on split-bf16 MFMA, instead of the ~20 forward
launches of ``xattn_head.head_forward``.

Scope of the fused path: d_model 128 with 4 heads (the reference's defaults, fusion.py:199-200), mean temporal
pooling (the fusion default), concat or gated head, with or without the emotion-prior attention bias (the bias
enters F2 / F3 / G2 / G3; the adapter itself -- pooled means, prior_net, the four token-bias Linears -- is ONE launch
each way, csrc/prior.hip, its weight gradients problems of the grouped W launch; fusion.py:153-184,390-394), audio features
that need no gradient (bf16 from the frozen WavLM, or fp32), T <= 16 frames and Ta <= 160 audio frames (3 s clips: 8
and 149).  Everything else -- and INT8 inference -- runs the unfused schedule, which is the parity reference of this path.  The saved activations
have the unfused schedule's names and layouts, so ``xattn_head.head_backward`` runs unchanged on them.
"""
from __future__ import annotations

import os
from typing import Dict

import torch

from . import kernels as K

ENABLED = os.environ.get("MER_XATTN_FUSED", "1") != "0"
BWD_ENABLED = os.environ.get("MER_XATTN_FUSED_BWD", "1") != "0"
WGRAD_ROWS = 256  # rows of dY / X per weight-gradient workgroup (M is split over the grid)
PRIOR = "emotion_prior_bias."
PRIOR_HEADS = ("v_query_bias", "a_key_bias", "a_query_bias", "v_key_bias")  # mer_xh_prior_fwd's head order
F1_PAIR = True  # bf16 features: the first product as a bf16 GEMM + mer_xh_audio_fwd_pair (tools A/B only)

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
    if not ENABLED or qlin is not None or cfg.temporal_pooling != "mean":
        return False
    if cfg.num_heads != 4 or p["v_in_proj.weight"].shape[0] != 128 or cfg.xattn_head not in ("concat", "gated"):
        return False
    B, T, vd = v_feat.shape
    _, Ta, sd = a_seq.shape
    if a_seq.dtype not in (torch.bfloat16, torch.float32) or v_feat.dtype != torch.float32 or T > 16 or Ta > 160 \
            or vd % 32 or vd > 512 or sd % 64:
        return False
    if a_seq.requires_grad:  # the fused forward has no audio-feature gradient path (stage 2 runs unfused)
        return False
    # the classifier kernels' staging bounds (xh_mlp_fwd: H1 <= 256 hidden units, 4 * C <= 256 class rows;
    # xh_mlp_bwd: C <= 32): wider heads take the unfused schedule instead of failing the launch
    n0 = "xattn_mlp.0.weight" if cfg.xattn_head == "concat" else "xattn_gate.0.weight"
    C = (p["xattn_mlp.3.weight"] if cfg.xattn_head == "concat" else p["xattn_classifier.weight"]).shape[0]
    if p[n0].shape[0] > 256 or C > 32:
        return False
    return p["audio_seq_proj.weight"].shape == (128, sd) and p["v_in_proj.weight"].shape == (128, vd)


# transposed ([in][out]) planes of the backward's data-gradient products: (weight name, row slice) parts laid
# side by side as column blocks of the transposed plane
_TPLANES = {
    "WcT": _PLANES["Wc"],  # [128][384]: da += [dq2 | dK1 dV1] . [Wq2 ; Wkv1]
    "WaT": _PLANES["Wa"],
    "WoT2": _PLANES["Wo2"],
    "WkvT2": _PLANES["Wkv2"],  # [128][256]
    "WoT1": _PLANES["Wo1"],
    "WqT1": _PLANES["Wq1"],
    "WvT": _PLANES["Wv"],  # [vdim][128]
}


def _parts(p, parts):
    srcs = []
    for name, sl in parts:
        w = p[name]
        if sl is not None:  # rows [sl0 * d, sl1 * d) of a packed [3d, d] in_proj weight
            w = w[sl[0] * w.shape[1]:sl[1] * w.shape[1]]
        if not w.is_contiguous():
            raise ValueError("split planes need contiguous weight rows")
        srcs.append(w)
    return srcs


class SplitPlanes:
    """bf16 hi / lo planes of the head weights the fused kernels read, refreshed by ONE mer_xh_split launch per
    forward (inside the captured head graph, so every replay splits the current Adam-updated weights) and, for
    the transposed planes of the backward, one more per backward."""

    def __init__(self, p: Dict[str, torch.Tensor]):
        dev = p["v_in_proj.weight"].device
        self.planes = {}
        rows = []
        self.stacked = {}  # key -> [hi; lo] as one [2 * rows][k] bf16 matrix (the GEMM operand of F1's first product)
        for key, parts in _PLANES.items():
            srcs = _parts(p, parts)
            n_rows, k = sum(s.shape[0] for s in srcs), srcs[0].shape[1]
            both = torch.empty(2, n_rows, k, device=dev, dtype=torch.bfloat16)
            hi, lo = both[0], both[1]
            self.stacked[key] = both.view(2 * n_rows, k)
            off = 0
            for s in srcs:
                rows.append([s.data_ptr(), hi.data_ptr() + 2 * off, lo.data_ptr() + 2 * off, s.shape[0], s.shape[1], 0,
                             s.shape[1]])
                off += s.numel()
            self.planes[key] = (hi, lo)
        trows = []
        for key, parts in _TPLANES.items():
            srcs = _parts(p, parts)
            n_rows, k = sum(s.shape[0] for s in srcs), srcs[0].shape[1]
            hi = torch.empty(k, n_rows, device=dev, dtype=torch.bfloat16)
            lo = torch.empty(k, n_rows, device=dev, dtype=torch.bfloat16)
            col = 0
            for s in srcs:
                trows.append([s.data_ptr(), hi.data_ptr() + 2 * col, lo.data_ptr() + 2 * col, s.shape[0], s.shape[1], 1,
                              n_rows])
                col += s.shape[0]
            self.planes[key] = (hi, lo)
        self.desc = torch.tensor(rows, dtype=torch.int64).to(dev)
        self.desc_t = torch.tensor(trows, dtype=torch.int64).to(dev)
        self.desc_both = torch.tensor(rows + trows, dtype=torch.int64).to(dev)
        self.key = tuple(r[0] for r in rows)
        self.gen = 0  # forward refreshes so far (host-side; frozen into a captured graph like the launches)
        self.t_gen = -1  # the refresh that last wrote the transposed planes

    def refresh(self, transposed: bool = False):
        """One launch: the forward planes, plus the backward's transposed planes when a backward will follow."""
        self.gen += 1
        K.xh_split(self.desc_both if transposed else self.desc)
        if transposed:
            self.t_gen = self.gen

    def refresh_transposed(self):
        K.xh_split(self.desc_t)
        self.t_gen = self.gen

    def __getitem__(self, key):
        return self.planes[key]


_CACHE: Dict[tuple, SplitPlanes] = {}


def planes_for(p: Dict[str, torch.Tensor]) -> SplitPlanes:
    key = tuple((p[n].data_ptr(), tuple(p[n].shape)) for n in (
        "audio_seq_proj.weight", "a_in_proj.weight", "a2v_attn.in_proj_weight", "v2a_attn.in_proj_weight",
        "v_in_proj.weight", "v2a_attn.out_proj.weight", "a2v_attn.out_proj.weight"))
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
    dp_prior = cfg.prior_dropout if (training and cfg.use_prior) else 0.0
    seed = rng if (training and rng is not None) else None
    if training and (dp_attn > 0 or dp_path > 0 or dp_mlp > 0 or dp_prior > 0) and seed is None:
        raise ValueError("train-mode dropout needs the step's RNG base")
    sp = planes_for(p)
    sp.refresh(transposed=training)  # a training forward is followed by the fused backward
    ctx.planes_gen = sp.gen
    ctx.planes = sp  # a captured graph writes through sp's descriptors: keep them alive as long as the context
    vf = v_feat.reshape(B * T, vd).contiguous()
    af = a_seq.reshape(B * Ta, sd).contiguous()
    a_s, a, q2, kv1 = e(B * Ta, d), e(B * Ta, d), e(B * Ta, d), e(B * Ta, 2 * d)
    v, q1, o1 = e(B * T, d), e(B * T, d), e(B * T, d)
    if af.dtype == torch.bfloat16 and F1_PAIR:
        # the 768-deep first product as ONE pipelined bf16 GEMM against the stacked [hi; lo] planes (128 x 64 tiles:
        # 152 workgroups), F1 then sums the two halves: the product inside F1 was L2-latency-bound (~34 us)
        pair = e(B * Ta, 2 * d)
        K.gemm_bf16(af, sp.stacked["Ws"], pair, variant=7)
        K.xh_audio_fwd_pair(pair, p["audio_seq_proj.bias"], sp["Wa"], p["a_in_proj.bias"], sp["Wc"],
                            p["a2v_attn.in_proj_bias"][:d], p["v2a_attn.in_proj_bias"][d:], a_s, a, q2, kv1, vf, sp["Wv"],
                            p["v_in_proj.bias"], sp["Wq1"], p["v2a_attn.in_proj_bias"][:d], v, q1)
    else:
        K.xh_audio_fwd(af, sp["Ws"], p["audio_seq_proj.bias"], sp["Wa"], p["a_in_proj.bias"], sp["Wc"],
                       p["a2v_attn.in_proj_bias"][:d], p["v2a_attn.in_proj_bias"][d:], a_s, a, q2, kv1, vf, sp["Wv"],
                       p["v_in_proj.bias"], sp["Wq1"], p["v2a_attn.in_proj_bias"][:d], v, q1)
    sv = ctx.saved
    v2a_bias = a2v_bias = None
    if cfg.use_prior:  # the emotion-prior attention biases from the pre-attention tokens (fusion.py:390-391): one launch
        n = PRIOR
        H1, PD = p[n + "prior_net.0.weight"].shape[0], p[n + "prior_net.3.weight"].shape[0]
        pg, h1, prior = e(B, 2 * d), e(B, H1), e(B, PD)
        tt = [e(B * L, 1) for L in (T, Ta, Ta, T)]
        tp = [e(B, 1) for _ in PRIOR_HEADS]
        v2a_bias, a2v_bias = e(B, T, Ta), e(B, Ta, T)
        K.xh_prior_fwd(B, T, Ta, v, a, p[n + "prior_net.0.weight"], p[n + "prior_net.0.bias"],
                       p[n + "prior_net.3.weight"], p[n + "prior_net.3.bias"],
                       [(p[n + h + ".weight"], p[n + h + ".bias"]) for h in PRIOR_HEADS], p[n + "bias_scale"],
                       dp_prior, seed, site_prior, pg, h1, prior, tt, tp, v2a_bias, a2v_bias)
        sv.update(v=v, a=a, pg=pg, h1=h1, prior=prior)  # the unfused schedule's names (prior_backward reads them)
        for h, t_, p_ in zip(PRIOR_HEADS, tt, tp):
            sv["tt_" + h], sv["tp_" + h] = t_, p_
    P1 = e(B, H, T, Ta)
    s_v, mu_v, rs_v, v1, kv2 = e(B * T, d), e(B * T), e(B * T), e(B * T, d), e(B * T, 2 * d)
    emb = e(B, 2 * d)
    scale = (d // H) ** -0.5
    K.xh_v2a_fwd(B, T, Ta, v, q1, kv1, sp["Wo1"], p["v2a_attn.out_proj.bias"], p["v_norm.weight"], p["v_norm.bias"],
                 sp["Wkv2"], p["a2v_attn.in_proj_bias"][d:], dp_attn, dp_path, seed, site_v2a, site_vpath, scale, P1,
                 o1, s_v, mu_v, rs_v, v1, kv2, emb, bias=v2a_bias)
    o2, P2 = e(B * Ta, d), e(B, H, Ta, T)
    s_a, mu_a, rs_a = e(B * Ta, d), e(B * Ta), e(B * Ta)
    part = e(B, (Ta + 15) // 16, d)
    K.xh_a2v_fwd(B, T, Ta, q2, kv2, a, sp["Wo2"], p["a2v_attn.out_proj.bias"], p["a_norm.weight"], p["a_norm.bias"],
                 dp_attn, dp_path, seed, site_a2v, site_apath, scale, P2, o2, s_a, mu_a, rs_a, part, bias=a2v_bias)
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
    ctx.drops = (dp_attn, dp_path, dp_mlp, dp_prior)
    ctx.fused = True
    return logits


def backward_supported(ctx, p, need_da_seq: bool) -> bool:
    """The fused backward runs on a context the fused forward filled, unless the audio features need a gradient
    (stage 2 -- which the fused forward already excludes)."""
    if not BWD_ENABLED or not getattr(ctx, "fused", False) or need_da_seq:
        return False
    n0 = "xattn_mlp.0.weight" if ctx.cfg.xattn_head == "concat" else "xattn_gate.0.weight"
    C = (p["xattn_mlp.3.weight"] if ctx.cfg.xattn_head == "concat" else p["xattn_classifier.weight"]).shape[0]
    return C <= 32 and p[n0].shape[0] <= 256  # mer_xh_mlp_bwd's bounds


def _splits(M: int) -> int:
    """Row splits of one weight-gradient problem: WGRAD_ROWS rows (WGRAD_ROWS / 32 pipelined chunks) per workgroup."""
    return max(1, min(-(-M // WGRAD_ROWS), 64))


def fused_backward(p, ctx, dlogits, grads, need_dv_feat=True):
    """The fused backward (csrc/xattn_fused_bwd.hip) of a fused-forward context: the gradients head_backward
    would write (accumulated into ``grads``), returns dv_feat [B, T, vd] (or None)."""
    cfg = ctx.cfg
    sv = ctx.saved
    B, T, Ta, d, H = ctx.dims
    rng = ctx.rng
    dp_attn, dp_path, dp_mlp, _ = ctx.drops
    dev = dlogits.device
    f32 = torch.float32
    e = lambda *shape: torch.empty(shape, device=dev, dtype=f32)  # noqa: E731
    from .xattn_head import SITE_A2V, SITE_APATH, SITE_MLP, SITE_PRIOR, SITE_V2A, SITE_VPATH
    sp = getattr(ctx, "planes", None) or planes_for(p)
    if sp.t_gen != getattr(ctx, "planes_gen", None):  # the forward did not split them (eval-mode forward)
        sp.refresh_transposed()
    dlogits = dlogits.contiguous()
    demb = e(B, 2 * d)
    if cfg.xattn_head == "concat":
        n0, n3 = "xattn_mlp.0.", "xattn_mlp.3."
        dh, dz = e(B, p[n0 + "weight"].shape[0]), None
        K.xh_mlp_bwd(B, False, dlogits, sv["emb"], sv["h"], None, p[n0 + "weight"], p[n3 + "weight"], None, dp_mlp,
                     rng, SITE_MLP, dh, None, demb)
        # the classifier's weight gradients: problems of the grouped W launch below
        head_w = ((dh, sv["emb"], grads[n0 + "weight"], grads[n0 + "bias"]),
                  (dlogits, sv["h"], grads[n3 + "weight"], grads[n3 + "bias"]))
    else:
        n0, n3, nc = "xattn_gate.0.", "xattn_gate.3.", "xattn_classifier."
        dh, dz = e(B, p[n0 + "weight"].shape[0]), e(B, 1)
        K.xh_mlp_bwd(B, True, dlogits, sv["emb"], sv["h"], sv["g"], p[n0 + "weight"], p[n3 + "weight"],
                     p[nc + "weight"], dp_mlp, rng, SITE_MLP, dh, dz, demb)
        head_w = ((dh, sv["emb"], grads[n0 + "weight"], grads[n0 + "bias"]),
                  (dz, sv["h"], grads[n3 + "weight"], grads[n3 + "bias"]),
                  (dlogits, sv["fused"], grads[nc + "weight"], grads[nc + "bias"]))
    nt = (Ta + 15) // 16
    scale = (d // H) ** -0.5
    da, da2, dqkv = e(B * Ta, d), e(B * Ta, d), e(B * Ta, 3 * d)
    dkv2_part, lnp_a = e(B, nt, 16, 2 * d), e(B * nt, 2 * d)
    prior = cfg.use_prior
    dbias_a2v, dbias_v2a = (e(B, Ta, T), e(B, T, Ta)) if prior else (None, None)
    K.xh_a2v_bwd(B, T, Ta, demb, sv["s_a"], sv["mu_a"], sv["rs_a"], p["a_norm.weight"], sv["P2"], sv["kv2"], sv["q2"],
                 sp["WoT2"], dp_attn, dp_path, rng, SITE_A2V, SITE_APATH, scale, da, da2, dqkv, dkv2_part, lnp_a,
                 dbias=dbias_a2v)
    vf = sv["vf"]
    dkv2, dv2, dq1, dv = e(B * T, 2 * d), e(B * T, d), e(B * T, d), e(B * T, d)
    dvfeat = e(B * T, vf.shape[1]) if need_dv_feat else None
    lnp_v = e(B, 2 * d)
    K.xh_v2a_bwd(B, T, Ta, dkv2_part, sp["WkvT2"], demb, sv["s_v"], sv["mu_v"], sv["rs_v"], p["v_norm.weight"],
                 sp["WoT1"], sv["P1"], sv["kv1"], sv["q1"], dp_attn, dp_path, rng, SITE_V2A, SITE_VPATH, scale, dkv2,
                 dv2, dq1, dv, dqkv, lnp_v, dbias=dbias_v2a)
    prior_w = ()
    if prior:  # one launch: the prior's data gradients; its token gradients join da / dv before G1 reads them
        n = PRIOR
        dtt = [e(B * L, 1) for L in (T, Ta, Ta, T)]
        dtp = [e(B, 1) for _ in PRIOR_HEADS]
        dprior, dh1, dsc = e(B, sv["prior"].shape[1]), e(B, sv["h1"].shape[1]), e(B, 1)
        K.xh_prior_bwd(B, T, Ta, dbias_v2a, dbias_a2v, [sv["tt_" + h] for h in PRIOR_HEADS],
                       [sv["tp_" + h] for h in PRIOR_HEADS], p[n + "bias_scale"], [p[n + h + ".weight"] for h in PRIOR_HEADS],
                       p[n + "prior_net.0.weight"], p[n + "prior_net.3.weight"], sv["h1"], ctx.drops[3], rng, SITE_PRIOR,
                       dtt, dtp, dprior, dh1, dsc, dv, da)
        # its weight gradients: problems of the grouped launch below (token-bias weights split [token | prior] columns)
        prior_w = [(dh1, sv["pg"], grads[n + "prior_net.0.weight"], grads[n + "prior_net.0.bias"]),
                   (dprior, sv["h1"], grads[n + "prior_net.3.weight"], grads[n + "prior_net.3.bias"]),
                   (dsc, None, None, grads[n + "bias_scale"])]
        for h, dt, dq, toks in zip(PRIOR_HEADS, dtt, dtp, (sv["v"], sv["a"], sv["a"], sv["v"])):
            gw = grads[n + h + ".weight"]
            prior_w += [(dt, toks, gw[:, :d], None), (dq, sv["prior"], gw[:, d:], grads[n + h + ".bias"])]
    da_s = e(B * Ta, d)
    K.xh_audio_bwd(dqkv, sp["WcT"], sp["WaT"], da, da_s, dq1, sp["WqT1"], sp["WvT"], dv, dvfeat)
    gw1, gb1 = grads["v2a_attn.in_proj_weight"], grads["v2a_attn.in_proj_bias"]
    gw2, gb2 = grads["a2v_attn.in_proj_weight"], grads["a2v_attn.in_proj_bias"]
    Ma, Mv, af = B * Ta, B * T, sv["af"]
    W = K.WGradTable()
    for dY, X, dW, db in ((da_s, af, grads["audio_seq_proj.weight"], grads["audio_seq_proj.bias"]),
                          (da, sv["a_s"], grads["a_in_proj.weight"], grads["a_in_proj.bias"]),
                          (dqkv[:, :d], sv["a"], gw2[:d], gb2[:d]),
                          (dqkv[:, d:], sv["a"], gw1[d:], gb1[d:]),
                          (da2, sv["o2"], grads["a2v_attn.out_proj.weight"], grads["a2v_attn.out_proj.bias"]),
                          (dkv2, sv["v1"], gw2[d:], gb2[d:]),
                          (dv2, sv["o1"], grads["v2a_attn.out_proj.weight"], grads["v2a_attn.out_proj.bias"]),
                          (dq1, sv["v"], gw1[:d], gb1[:d]),
                          (dv, vf, grads["v_in_proj.weight"], grads["v_in_proj.bias"]),
                          (lnp_a[:, :d], None, None, grads["a_norm.weight"]),
                          (lnp_a[:, d:], None, None, grads["a_norm.bias"]),
                          (lnp_v[:, :d], None, None, grads["v_norm.weight"]),
                          (lnp_v[:, d:], None, None, grads["v_norm.bias"])) + head_w + tuple(prior_w):
        W.add(dY, X, dW, db, _splits(dY.shape[0]))
    ws = e(W.ws_floats())
    W.run(ws)
    return dvfeat.view(B, T, -1) if dvfeat is not None else None
