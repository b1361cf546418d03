"""Explicit forward/backward schedule of the xattn fusion head on the HIP kernels.

Reference: ``src/models/fusion.py:366-411`` (xattn branch after the encoders) with
``EmotionPriorBiasAdapter`` (fusion.py:153-184), ``StochasticDepth`` (11-26), the two
``nn.MultiheadAttention`` blocks (TORCH:6576-6606), mean ``TemporalPooler``
(temporal.py:108-109) and the concat / gated heads (fusion.py:311-327).

All head math is fp32 (parity bar: logits within 1e-3 of the CPU reference).  The
schedule is written out by hand -- no autograd tape inside: ``forward`` returns the
logits plus a context of saved buffers, ``backward`` walks the graph in reverse and
writes parameter gradients straight into caller-provided (flat) buffers.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

from . import kernels as K
from . import temporal_hip as TH
from . import xattn_fused as XF

# Dropout / drop-path sites: the step's RNG base is a device int64 [1] tensor (``rng``) mixed with a
# constant site id in-kernel (mer_site_seed), so the masks are regenerated in backward from (base, site)
# and a captured graph draws fresh masks every replay.
SITE_PRIOR, SITE_V2A, SITE_VPATH, SITE_A2V, SITE_APATH, SITE_MLP = 1, 2, 3, 4, 5, 6
SITE_VPOOL, SITE_APOOL = 100, 300  # + 8 per transformer layer (temporal_hip.py)


@dataclass
class HeadConfig:
    num_heads: int = 4
    xattn_head: str = "concat"
    use_prior: bool = False
    attn_dropout: float = 0.1
    drop_path: float = 0.1
    mlp_dropout: float = 0.2
    prior_dropout: float = 0.1
    temporal_pooling: str = "mean"
    temporal_num_heads: int = 4
    temporal_num_layers: int = 1
    temporal_dropout: float = 0.1


@dataclass
class HeadCtx:
    saved: Dict[str, torch.Tensor] = field(default_factory=dict)
    dims: tuple = ()
    rng: Optional[torch.Tensor] = None
    training: bool = False


def _e(shape, like, dtype=torch.float32):
    return torch.empty(shape, device=like.device, dtype=dtype)


def linear_runner(p: Dict[str, torch.Tensor], qlin: Optional[dict] = None):
    """``lin(name, x, out, act)`` for the Linear called ``name``: fp32 GEMM, or its dynamic-INT8 image
    when ``qlin`` (int8.quantize_dynamic_hip) holds one."""

    def lin(name, x, out, act="none"):
        if qlin is not None and name in qlin:
            return qlin[name](x, out, act)
        return K.linear_fwd(x, p[name + ".weight"], p[name + ".bias"], out, act=act)

    return lin


def head_forward(p: Dict[str, torch.Tensor], cfg: HeadConfig, v_feat: torch.Tensor, a_seq: torch.Tensor,
                 training: bool, rng: Optional[torch.Tensor] = None, qlin: Optional[dict] = None):
    """Returns (logits [B, C], ctx).  ``rng``: the step's device RNG base (training dropout), ``qlin``: INT8
    images of the plain Linears (inference only)."""
    B, T, vd = v_feat.shape
    _, Ta, sd = a_seq.shape
    d = p["v_in_proj.weight"].shape[0]
    H = cfg.num_heads
    ctx = HeadCtx(dims=(B, T, Ta, d, H), rng=rng, training=training)
    if XF.supported(cfg, p, v_feat, a_seq, qlin):  # four fused launches (csrc/xattn_fused.hip)
        logits = XF.fused_forward(p, cfg, v_feat, a_seq, training, rng, ctx,
                                  (SITE_PRIOR, SITE_V2A, SITE_VPATH, SITE_A2V, SITE_APATH, SITE_MLP))
        return logits, ctx
    sv = ctx.saved
    dp_attn = cfg.attn_dropout if training else 0.0
    dp_path = cfg.drop_path if training else 0.0
    dp_mlp = cfg.mlp_dropout if training else 0.0
    dp_prior = cfg.prior_dropout if training else 0.0
    vf = v_feat.reshape(B * T, vd)
    af = a_seq.reshape(B * Ta, sd)
    sv["vf"], sv["af"] = vf, af

    lin = linear_runner(p, qlin)
    v = lin("v_in_proj", vf, _e((B * T, d), vf))
    a_s = lin("audio_seq_proj", af, _e((B * Ta, d), af))
    a = lin("a_in_proj", a_s, _e((B * Ta, d), af))
    sv["v"], sv["a_s"], sv["a"] = v, a_s, a

    v2a_bias = a2v_bias = None
    if cfg.use_prior:
        v2a_bias, a2v_bias = prior_forward(p, v, a, B, T, Ta, dp_prior, rng, sv, lin, qlin)

    # ---- v2a: v2 = MHA(q=v, k=a, v=a)  (fusion.py:394) ----
    w1, b1 = p["v2a_attn.in_proj_weight"], p["v2a_attn.in_proj_bias"]
    q1 = K.linear_fwd(v, w1[:d], b1[:d], _e((B * T, d), v))
    kv1 = K.linear_fwd(a, w1[d:], b1[d:], _e((B * Ta, 2 * d), v))
    o1 = _e((B * T, d), v)
    P1 = _e((B, H, T, Ta), v)
    K.mha_fwd(q1, kv1[:, :d], kv1[:, d:], v2a_bias, o1, P1, B, H, T, Ta, dp_attn, rng, SITE_V2A)
    v2 = K.linear_fwd(o1, p["v2a_attn.out_proj.weight"], p["v2a_attn.out_proj.bias"], _e((B * T, d), v))
    v1, s_v, mu_v, rs_v = _e((B * T, d), v), _e((B * T, d), v), _e((B * T,), v), _e((B * T,), v)
    K.add_ln_fwd(v, v2, p["v_norm.weight"], p["v_norm.bias"], v1, s_v, mu_v, rs_v, T, dp_path, rng, SITE_VPATH)
    sv.update(q1=q1, kv1=kv1, o1=o1, P1=P1, v1=v1, s_v=s_v, mu_v=mu_v, rs_v=rs_v)

    # ---- a2v: a2 = MHA(q=a, k=v_new, v=v_new)  (fusion.py:398) ----
    w2, b2 = p["a2v_attn.in_proj_weight"], p["a2v_attn.in_proj_bias"]
    q2 = K.linear_fwd(a, w2[:d], b2[:d], _e((B * Ta, d), v))
    kv2 = K.linear_fwd(v1, w2[d:], b2[d:], _e((B * T, 2 * d), v))
    o2 = _e((B * Ta, d), v)
    P2 = _e((B, H, Ta, T), v)
    K.mha_fwd(q2, kv2[:, :d], kv2[:, d:], a2v_bias, o2, P2, B, H, Ta, T, dp_attn, rng, SITE_A2V)
    a2 = K.linear_fwd(o2, p["a2v_attn.out_proj.weight"], p["a2v_attn.out_proj.bias"], _e((B * Ta, d), v))
    a1, s_a, mu_a, rs_a = _e((B * Ta, d), v), _e((B * Ta, d), v), _e((B * Ta,), v), _e((B * Ta,), v)
    K.add_ln_fwd(a, a2, p["a_norm.weight"], p["a_norm.bias"], a1, s_a, mu_a, rs_a, Ta, dp_path, rng, SITE_APATH)
    sv.update(q2=q2, kv2=kv2, o2=o2, P2=P2, a1=a1, s_a=s_a, mu_a=mu_a, rs_a=rs_a)

    # ---- temporal pooling -> emb = [v_emb ; a_emb]  (fusion.py:401-406, temporal.py:105-110) ----
    emb = _e((B, 2 * d), v)
    if cfg.temporal_pooling == "mean":
        K.mean_pool_fwd(v1.view(B, T, d), emb[:, :d], ldy=2 * d)
        K.mean_pool_fwd(a1.view(B, Ta, d), emb[:, d:], ldy=2 * d)
    else:
        dp_t = cfg.temporal_dropout if training else 0.0
        kw = dict(num_heads=cfg.temporal_num_heads, num_layers=cfg.temporal_num_layers, dropout=dp_t, rng=rng)
        sv["vpool"] = TH.pool_forward(p, "v_temporal_pool.pool", cfg.temporal_pooling, v1.view(B, T, d), emb[:, :d],
                                      2 * d, site0=SITE_VPOOL, **kw)
        sv["apool"] = TH.pool_forward(p, "a_temporal_pool.pool", cfg.temporal_pooling, a1.view(B, Ta, d),
                                      emb[:, d:], 2 * d, site0=SITE_APOOL, **kw)
    sv["emb"] = emb

    if cfg.xattn_head == "concat":
        w0 = p["xattn_mlp.0.weight"]
        h = lin("xattn_mlp.0", emb, _e((B, w0.shape[0]), v), act="relu")
        K.dropout_(h, dp_mlp, rng, SITE_MLP)
        w3 = p["xattn_mlp.3.weight"]
        logits = lin("xattn_mlp.3", h, _e((B, w3.shape[0]), v))
        sv["h"] = h
    elif cfg.xattn_head == "gated":
        w0 = p["xattn_gate.0.weight"]
        h = lin("xattn_gate.0", emb, _e((B, w0.shape[0]), v), act="relu")
        K.dropout_(h, dp_mlp, rng, SITE_MLP)
        z = lin("xattn_gate.3", h, _e((B, 1), v))
        fused, g = _e((B, d), v), _e((B,), v)
        K.gate_mix_fwd(z, emb[:, :d], emb[:, d:], fused, g)
        wc = p["xattn_classifier.weight"]
        logits = lin("xattn_classifier", fused, _e((B, wc.shape[0]), v))
        sv.update(h=h, g=g, fused=fused)
    else:
        raise ValueError(f"Unknown xattn head: {cfg.xattn_head}")
    ctx.cfg = cfg
    ctx.drops = (dp_attn, dp_path, dp_mlp, dp_prior)
    return logits, ctx


def head_backward(p: Dict[str, torch.Tensor], ctx: HeadCtx, dlogits: torch.Tensor, grads: Dict[str, torch.Tensor],
                  need_dv_feat: bool = True, need_da_seq: bool = False, fused: Optional[bool] = None):
    """Reverse schedule.  ``grads[name]`` must be zero-initialised fp32 buffers (accumulated into).

    A context from the fused forward takes the fused backward (xattn_fused.fused_backward) unless ``fused`` is
    False; the unfused schedule below reads the same saved activations.
    Returns (dv_feat [B,T,vd] fp32 or None, da_seq or None).
    """
    if fused is not False and XF.backward_supported(ctx, p, need_da_seq):
        return XF.fused_backward(p, ctx, dlogits, grads, need_dv_feat), None
    cfg: HeadConfig = ctx.cfg
    sv = ctx.saved
    B, T, Ta, d, H = ctx.dims
    rng = ctx.rng
    dp_attn, dp_path, dp_mlp, dp_prior = ctx.drops
    z = lambda *shape: torch.zeros(shape, device=dlogits.device, dtype=torch.float32)  # noqa: E731
    e = lambda *shape: torch.empty(shape, device=dlogits.device, dtype=torch.float32)  # noqa: E731
    emb = sv["emb"]
    demb = e(B, 2 * d)

    if cfg.xattn_head == "concat":
        h = sv["h"]
        dh = e(B, h.shape[1])
        K.linear_bwd(h, p["xattn_mlp.3.weight"], dlogits, dx=dh, dw=grads["xattn_mlp.3.weight"], db=grads["xattn_mlp.3.bias"])
        K.relu_dropout_bwd_(dh, h, dp_mlp, rng, SITE_MLP)
        K.linear_bwd(emb, p["xattn_mlp.0.weight"], dh, dx=demb, dw=grads["xattn_mlp.0.weight"], db=grads["xattn_mlp.0.bias"])
    else:
        h, g, fused = sv["h"], sv["g"], sv["fused"]
        dfused = e(B, d)
        K.linear_bwd(fused, p["xattn_classifier.weight"], dlogits, dx=dfused, dw=grads["xattn_classifier.weight"],
                     db=grads["xattn_classifier.bias"])
        demb.zero_()
        dz = e(B, 1)
        K.gate_mix_bwd(g, emb[:, :d], emb[:, d:], dfused, dz, demb[:, :d], demb[:, d:])
        dh = e(B, h.shape[1])
        K.linear_bwd(h, p["xattn_gate.3.weight"], dz, dx=dh, dw=grads["xattn_gate.3.weight"], db=grads["xattn_gate.3.bias"])
        K.relu_dropout_bwd_(dh, h, dp_mlp, rng, SITE_MLP)
        K.linear_bwd(emb, p["xattn_gate.0.weight"], dh, dx=demb, dw=grads["xattn_gate.0.weight"],
                     db=grads["xattn_gate.0.bias"], dx_beta=1)

    # pooling backward
    if cfg.temporal_pooling == "mean":
        dv1 = e(B * T, d)
        da1 = e(B * Ta, d)
        K.mean_pool_bwd(demb[:, :d], dv1.view(B, T, d))
        K.mean_pool_bwd(demb[:, d:], da1.view(B, Ta, d))
    else:
        dv1 = TH.pool_backward(p, "v_temporal_pool.pool", sv["vpool"], demb[:, :d], grads).view(B * T, d)
        da1 = TH.pool_backward(p, "a_temporal_pool.pool", sv["apool"], demb[:, d:], grads).view(B * Ta, d)

    # ---- a2v backward ----
    da = e(B * Ta, d)
    da2 = e(B * Ta, d)
    K.add_ln_bwd(da1, sv["s_a"], sv["mu_a"], sv["rs_a"], p["a_norm.weight"], da, da2, grads["a_norm.weight"],
                 grads["a_norm.bias"], Ta, dp_path, rng, SITE_APATH)
    do2 = e(B * Ta, d)
    K.linear_bwd(sv["o2"], p["a2v_attn.out_proj.weight"], da2, dx=do2, dw=grads["a2v_attn.out_proj.weight"],
                 db=grads["a2v_attn.out_proj.bias"])
    dq2, dkv2 = e(B * Ta, d), e(B * T, 2 * d)
    dbias_a2v = e(B, Ta, T) if cfg.use_prior else None
    K.mha_bwd(sv["q2"], sv["kv2"][:, :d], sv["kv2"][:, d:], sv["P2"], do2, dq2, dkv2[:, :d], dkv2[:, d:], dbias_a2v,
              B, H, Ta, T, dp_attn, rng, SITE_A2V)
    w2 = p["a2v_attn.in_proj_weight"]
    gw2, gb2 = grads["a2v_attn.in_proj_weight"], grads["a2v_attn.in_proj_bias"]
    K.linear_bwd(sv["a"], w2[:d], dq2, dx=da, dw=gw2[:d], db=gb2[:d], dx_beta=1)
    K.linear_bwd(sv["v1"], w2[d:], dkv2, dx=dv1, dw=gw2[d:], db=gb2[d:], dx_beta=1)

    # ---- v2a backward ----
    dv = e(B * T, d)
    dv2 = e(B * T, d)
    K.add_ln_bwd(dv1, sv["s_v"], sv["mu_v"], sv["rs_v"], p["v_norm.weight"], dv, dv2, grads["v_norm.weight"],
                 grads["v_norm.bias"], T, dp_path, rng, SITE_VPATH)
    do1 = e(B * T, d)
    K.linear_bwd(sv["o1"], p["v2a_attn.out_proj.weight"], dv2, dx=do1, dw=grads["v2a_attn.out_proj.weight"],
                 db=grads["v2a_attn.out_proj.bias"])
    dq1, dkv1 = e(B * T, d), e(B * Ta, 2 * d)
    dbias_v2a = e(B, T, Ta) if cfg.use_prior else None
    K.mha_bwd(sv["q1"], sv["kv1"][:, :d], sv["kv1"][:, d:], sv["P1"], do1, dq1, dkv1[:, :d], dkv1[:, d:], dbias_v2a,
              B, H, T, Ta, dp_attn, rng, SITE_V2A)
    w1 = p["v2a_attn.in_proj_weight"]
    gw1, gb1 = grads["v2a_attn.in_proj_weight"], grads["v2a_attn.in_proj_bias"]
    K.linear_bwd(sv["v"], w1[:d], dq1, dx=dv, dw=gw1[:d], db=gb1[:d], dx_beta=1)
    K.linear_bwd(sv["a"], w1[d:], dkv1, dx=da, dw=gw1[d:], db=gb1[d:], dx_beta=1)

    # ---- emotion prior backward (fusion.py:170-184) ----
    if cfg.use_prior:
        prior_backward(p, sv, dbias_v2a, dbias_a2v, dv, da, grads, B, T, Ta, dp_prior, rng)

    # ---- input projections ----
    da_s = e(B * Ta, d)
    K.linear_bwd(sv["a_s"], p["a_in_proj.weight"], da, dx=da_s, dw=grads["a_in_proj.weight"], db=grads["a_in_proj.bias"])
    da_seq = None
    if need_da_seq:
        da_seq = e(B * Ta, sv["af"].shape[1])
    K.linear_bwd(sv["af"], p["audio_seq_proj.weight"], da_s, dx=da_seq, dw=grads["audio_seq_proj.weight"],
                 db=grads["audio_seq_proj.bias"])
    dv_feat = None
    if need_dv_feat:
        dv_feat = e(B * T, sv["vf"].shape[1])
    K.linear_bwd(sv["vf"], p["v_in_proj.weight"], dv, dx=dv_feat, dw=grads["v_in_proj.weight"], db=grads["v_in_proj.bias"])
    return (dv_feat.view(B, T, -1) if dv_feat is not None else None,
            da_seq.view(B, Ta, -1) if da_seq is not None else None)


def prior_forward(p, v, a, B, T, Ta, dp_prior, rng, sv, lin, qlin=None):
    """``EmotionPriorBiasAdapter.forward`` (fusion.py:178-184) on the pre-attention tokens v [B*T, d], a [B*Ta, d]:
    pooled means -> prior_net (256 -> 64 ReLU Dropout -> 8) -> the four token-bias Linears over cat([token, prior])
    -> (v2a_bias [B, T, Ta], a2v_bias [B, Ta, T]) = tanh(q + k) * bias_scale.  Saves what prior_backward reads."""
    n = "emotion_prior_bias."
    d = v.shape[1]
    pg = _e((B, 2 * d), v)
    K.mean_pool_fwd(v.view(B, T, d), pg[:, :d], ldy=2 * d)
    K.mean_pool_fwd(a.view(B, Ta, d), pg[:, d:], ldy=2 * d)
    h1 = lin(n + "prior_net.0", pg, _e((B, p[n + "prior_net.0.weight"].shape[0]), v), act="relu")
    K.dropout_(h1, dp_prior, rng, SITE_PRIOR)
    prior = lin(n + "prior_net.3", h1, _e((B, p[n + "prior_net.3.weight"].shape[0]), v))
    sv["pg"], sv["h1"], sv["prior"] = pg, h1, prior
    tok = {}
    for head, toks, L in (("v_query_bias", v, T), ("a_key_bias", a, Ta), ("a_query_bias", a, Ta), ("v_key_bias", v, T)):
        w = p[n + head + ".weight"]  # [1, d + pd]
        if qlin is not None and n + head in qlin:
            # INT8 (inference): the Linear sees cat([token, prior]) (fusion.py:171-174), quantized as ONE tensor
            ql = qlin[n + head]
            rows = K.concat_prior_rows(toks, prior, _e((toks.shape[0], ql.in_padded), v), L)
            tt = ql(rows, _e((toks.shape[0], 1), v))
            tp = torch.zeros(B, 1, device=v.device, dtype=torch.float32)
        else:
            tt = K.gemm(toks, w[:, :d], _e((toks.shape[0], 1), v), trans_b=True)
            tp = K.gemm(prior, w[:, d:], _e((B, 1), v), trans_b=True, bias=p[n + head + ".bias"])
        tok[head] = (tt, tp)
        sv["tt_" + head], sv["tp_" + head] = tt, tp
    v2a_bias = _e((B, T, Ta), v)
    K.token_bias_fwd(tok["v_query_bias"][0], tok["v_query_bias"][1], tok["a_key_bias"][0], tok["a_key_bias"][1],
                     p[n + "bias_scale"], v2a_bias)
    a2v_bias = _e((B, Ta, T), v)
    K.token_bias_fwd(tok["a_query_bias"][0], tok["a_query_bias"][1], tok["v_key_bias"][0], tok["v_key_bias"][1],
                     p[n + "bias_scale"], a2v_bias)
    return v2a_bias, a2v_bias


def prior_backward(p, sv, dbias_v2a, dbias_a2v, dv, da, grads, B, T, Ta, dp_prior, rng):
    """Backward of prior_forward (fusion.py:170-184): the prior weights' gradients (accumulated into ``grads``) and the
    token gradients ADDED into dv [B*T, d] and da [B*Ta, d] (token-bias Linears + the pooled means)."""
    n = "emotion_prior_bias."
    d = dv.shape[1]
    prior = sv["prior"]
    pd_ = prior.shape[1]
    dev = dv.device
    e = lambda *shape: torch.empty(shape, device=dev, dtype=torch.float32)  # noqa: E731
    dprior = torch.zeros(B, pd_, device=dev, dtype=torch.float32)
    dscale_part = e(2, B)
    spec = ((dbias_v2a, "v_query_bias", "a_key_bias", T, Ta, sv["v"], sv["a"], 0),
            (dbias_a2v, "a_query_bias", "v_key_bias", Ta, T, sv["a"], sv["v"], 1))
    for dbias, qh, kh, Lq, Lk, qtok, ktok, idx in spec:
        dqt, dkt, dqp, dkp = e(B * Lq, 1), e(B * Lk, 1), e(B, 1), e(B, 1)
        K.token_bias_bwd(sv["tt_" + qh], sv["tp_" + qh], sv["tt_" + kh], sv["tp_" + kh], p[n + "bias_scale"],
                         dbias, dqt, dkt, dqp, dkp, dscale_part[idx])
        for head, dtt, dtp, toks, dtoks in ((qh, dqt, dqp, qtok, dv if qtok is sv["v"] else da),
                                            (kh, dkt, dkp, ktok, dv if ktok is sv["v"] else da)):
            w = p[n + head + ".weight"]
            gw = grads[n + head + ".weight"]
            # tt = toks @ w[:, :d]^T  ;  tp = prior @ w[:, d:]^T + b
            K.linear_bwd(toks, w[:, :d], dtt, dx=dtoks, dw=gw[:, :d], dx_beta=1)
            K.linear_bwd(prior, w[:, d:], dtp, dx=dprior, dw=gw[:, d:], db=grads[n + head + ".bias"], dx_beta=1)
    K.vec_sum(dscale_part, grads[n + "bias_scale"], accumulate=True)
    dh1 = e(B, sv["h1"].shape[1])
    K.linear_bwd(sv["h1"], p[n + "prior_net.3.weight"], dprior, dx=dh1, dw=grads[n + "prior_net.3.weight"],
                 db=grads[n + "prior_net.3.bias"])
    K.relu_dropout_bwd_(dh1, sv["h1"], dp_prior, rng, SITE_PRIOR)
    dpg = e(B, 2 * d)
    K.linear_bwd(sv["pg"], p[n + "prior_net.0.weight"], dh1, dx=dpg, dw=grads[n + "prior_net.0.weight"],
                 db=grads[n + "prior_net.0.bias"])
    K.mean_pool_bwd(dpg[:, :d], dv.view(B, T, d), accumulate=True)
    K.mean_pool_bwd(dpg[:, d:], da.view(B, Ta, d), accumulate=True)


def used_param_names(cfg: HeadConfig):
    """Head parameters that receive a gradient (audio_time_conv is dead on the WavLM path, fusion.py:273)."""
    names = ["v_in_proj.weight", "v_in_proj.bias", "a_in_proj.weight", "a_in_proj.bias", "audio_seq_proj.weight",
             "audio_seq_proj.bias"]
    for m in ("v2a_attn", "a2v_attn"):
        names += [f"{m}.in_proj_weight", f"{m}.in_proj_bias", f"{m}.out_proj.weight", f"{m}.out_proj.bias"]
    names += ["v_norm.weight", "v_norm.bias", "a_norm.weight", "a_norm.bias"]
    if cfg.use_prior:
        n = "emotion_prior_bias."
        names += [n + "bias_scale", n + "prior_net.0.weight", n + "prior_net.0.bias", n + "prior_net.3.weight",
                  n + "prior_net.3.bias"]
        for hname in ("v_query_bias", "a_key_bias", "a_query_bias", "v_key_bias"):
            names += [n + hname + ".weight", n + hname + ".bias"]
    if cfg.temporal_pooling != "mean":
        for pool in ("v_temporal_pool.pool", "a_temporal_pool.pool"):
            names += TH.param_names(pool, cfg.temporal_pooling, cfg.temporal_num_layers)
    if cfg.xattn_head == "concat":
        names += ["xattn_mlp.0.weight", "xattn_mlp.0.bias", "xattn_mlp.3.weight", "xattn_mlp.3.bias"]
    else:
        names += ["xattn_gate.0.weight", "xattn_gate.0.bias", "xattn_gate.3.weight", "xattn_gate.3.bias",
                  "xattn_classifier.weight", "xattn_classifier.bias"]
    return names
