"""The fused xattn head forward (csrc/xattn_fused.hip, four launches on split-bf16 MFMA) against the unfused
schedule (xattn_head.head_forward, exact-f32 MFMA -- itself pinned to the reference goldens at 1e-4) on the C2
feature shapes (B=32, T=8, Ta=149), eval and train mode, with and without the emotion-prior bias (fusion.py:153-184,
390-398: the fused F2 / F3 add it to the scores, G2 / G3 return its gradient): the dropout / drop-path masks use the same indices,
so the same RNG base must give the same logits and saved activations in both paths (fp32-class agreement,
1e-5 relative), and the unchanged backward then gives the same gradients.  The C1 / C2 golden tests of
tests/test_head_gpu.py run through the fused path too (it is the default)."""
import numpy as np
import pytest
import torch

from tests.gpu_helpers import feats, head_model

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


@pytest.mark.parametrize("prior", [False, True])
@pytest.mark.parametrize("head", ["concat", "gated"])
@pytest.mark.parametrize("training", [False, True])
def test_fused_forward_matches_unfused(head, training, prior):
    from multimodalemotionrecognition_amd import xattn_fused as XF
    from multimodalemotionrecognition_amd import xattn_head as XH
    from multimodalemotionrecognition_amd.fusion import _head_grads

    m = head_model(head, prior).train(training)
    names, params = m.head_params()
    p = dict(zip(names, params))
    cfg = m.head_config()
    v, a = feats(32, 8, 149, seed=7)
    a = a.to(torch.bfloat16)  # the frozen WavLM's features
    rng = torch.full((1,), 4242, dtype=torch.int64, device="cuda")
    assert XF.supported(cfg, p, v, a, None)
    out = {}
    for fused in (False, True):
        XF.ENABLED = fused
        try:
            logits, ctx = XH.head_forward(p, cfg, v, a, training, rng)
            # (copies: the unfused backward leaves dS in P when the prior bias wants its gradient)
            saved = {k: t.clone() for k, t in ctx.saved.items() if isinstance(t, torch.Tensor)}
            dl = torch.from_numpy(np.random.default_rng(1).standard_normal(tuple(logits.shape)).astype(np.float32)).cuda()
            grads = _head_grads(p, set(XH.used_param_names(cfg)))
            grads = {n: torch.zeros_like(t) for n, t in grads.items()}
            dv, _ = XH.head_backward(p, ctx, dl, grads, need_dv_feat=True)
            out[fused] = (logits, saved, grads, dv)
        finally:
            XF.ENABLED = True
    (l0, s0, g0, dv0), (l1, s1, g1, dv1) = out[False], out[True]
    print(head, training, prior, "logits rel", _rel(l1, l0))
    assert _rel(l1, l0) < 1e-5
    keys = ("v", "a_s", "a", "q1", "kv1", "o1", "P1", "v1", "s_v", "q2", "kv2", "o2", "P2", "s_a", "emb", "h")
    keys += ("pg", "h1", "prior", "tt_v_query_bias", "tt_a_key_bias") if prior else ()
    # split-bf16 products (~2^-16 per term) vs exact-f32: measured up to 2.03e-5 max-abs relative (o2, train)
    for k in keys:
        assert _rel(s1[k], s0[k]) < 3e-5, (k, _rel(s1[k], s0[k]))
    for k in ("mu_v", "rs_v", "mu_a", "rs_a"):
        assert _rel(s1[k], s0[k]) < 3e-5, k
    for n in g0:
        # the prior's token-bias Linears: their bias gradient is ONE sum over every token's dS (positive and negative
        # terms cancel), so the ~1e-5 forward-level differences reach it amplified (measured 1.2e-4); likewise any
        # single-scalar gradient (the gate's output bias: one sum over the batch, 1.4e-4 with the fused prior)
        bar = 5e-4 if (n.startswith("emotion_prior_bias.") or g0[n].numel() == 1) else 1e-4
        assert _rel(g1[n], g0[n]) < bar, (n, _rel(g1[n], g0[n]))
    assert _rel(dv1, dv0) < 1e-4


@pytest.mark.parametrize("prior", [False, True])
@pytest.mark.parametrize("head", ["concat", "gated"])
@pytest.mark.parametrize("training", [False, True])
def test_fused_backward_matches_unfused(head, training, prior):
    """csrc/xattn_fused_bwd.hip against the unfused backward schedule on the SAME fused-forward context: every
    parameter gradient and dv_feat within 2e-5 (max-abs relative; split-bf16 products, ~2^-16 per term; measured
    <= 9.2e-6)."""
    from multimodalemotionrecognition_amd import xattn_head as XH
    from multimodalemotionrecognition_amd.fusion import _head_grads

    m = head_model(head, prior).train(training)
    names, params = m.head_params()
    p = dict(zip(names, params))
    cfg = m.head_config()
    v, a = feats(32, 8, 149, seed=11)
    a = a.to(torch.bfloat16)
    rng = torch.full((1,), 977, dtype=torch.int64, device="cuda")
    logits, ctx = XH.head_forward(p, cfg, v, a, training, rng)
    assert getattr(ctx, "fused", False)
    dl = torch.from_numpy(np.random.default_rng(3).standard_normal(tuple(logits.shape)).astype(np.float32)).cuda()
    out = {}
    probs = {k: ctx.saved[k].clone() for k in ("P1", "P2")}  # the unfused backward leaves dS in P (prior)

    def restore():
        for k, t in probs.items():
            ctx.saved[k].copy_(t)

    for fused in (False, True):
        restore()
        grads = {n: torch.zeros_like(t) for n, t in _head_grads(p, set(XH.used_param_names(cfg))).items()}
        dv, _ = XH.head_backward(p, ctx, dl, grads, need_dv_feat=True, fused=fused)
        out[fused] = (grads, dv)
    (g0, dv0), (g1, dv1) = out[False], out[True]
    worst = max((_rel(g1[n], g0[n]), n) for n in g0)
    print(head, training, prior, "worst grad rel", worst, "dv rel", _rel(dv1, dv0))
    for n in g0:
        assert _rel(g1[n], g0[n]) < 2e-5, (n, _rel(g1[n], g0[n]))
    assert _rel(dv1, dv0) < 2e-5
    # accumulation: a second fused backward into the same buffers doubles every gradient
    g2 = {n: t.clone() for n, t in g1.items()}
    restore()
    XH.head_backward(p, ctx, dl, g2, need_dv_feat=False, fused=True)
    for n in g1:
        assert _rel(g2[n], 2 * g1[n]) < 1e-6, n


@pytest.mark.parametrize("training", [False, True])
def test_f1_pair_matches_in_kernel(training):
    """F1's first product as one bf16 GEMM against stacked hi / lo planes + mer_xh_audio_fwd_pair (the default,
    ``xattn_fused.F1_PAIR``) against the in-kernel product of mer_xh_audio_fwd, which folds hi and lo into one running
    sum per k step: the two round differently, so they agree to fp32 rounding (a_s), which the next split-bf16
    products carry on (measured 2.3e-6 max-abs relative on a), and both forward paths give the same logits within the
    fused-vs-unfused bar."""
    from multimodalemotionrecognition_amd import xattn_fused as XF
    from multimodalemotionrecognition_amd import xattn_head as XH

    m = head_model("concat", False).train(training)
    names, params = m.head_params()
    p = dict(zip(names, params))
    cfg = m.head_config()
    v, a = feats(32, 8, 149, seed=7)
    a = a.to(torch.bfloat16)
    rng = torch.full((1,), 4242, dtype=torch.int64, device="cuda")
    out = {}
    prev = XF.F1_PAIR
    try:
        for pair in (False, True):
            XF.F1_PAIR = pair
            logits, ctx = XH.head_forward(p, cfg, v, a, training, rng)
            out[pair] = (logits.clone(), {k: ctx.saved[k].clone() for k in ("a_s", "a", "q2", "kv1")})
    finally:
        XF.F1_PAIR = prev
    (l0, s0), (l1, s1) = out[False], out[True]
    for k in s0:
        assert _rel(s1[k], s0[k]) < 1e-5, (k, _rel(s1[k], s0[k]))
    assert _rel(l1, l0) < 1e-5
