"""concat / gated / late fusion heads (fusion.py:358-363, 413-435) on the HIP kernels.

Inputs are the encoders' pooled embeddings (``audio_model.encode`` -> [B, Da],
``video_model.encode`` -> [B, Dv]).  fp32 math; one autograd node per head.
"""
from __future__ import annotations

import torch

from . import kernels as K
from .xattn_head import linear_runner

SITE_EMB_MLP = 11


def _grad_buf(p):
    from .fusion import grad_buffer
    return grad_buffer(p)


class _EmbHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a_emb, v_emb, mode, dp, rng, drop_a, drop_v, qlin, names, *params):
        p = dict(zip(names, params))
        lin = linear_runner(p, qlin)
        B = a_emb.shape[0]
        dev = a_emb.device
        e = lambda *s: torch.empty(s, device=dev, dtype=torch.float32)  # noqa: E731
        cd = p["audio_proj.weight"].shape[0]
        cat = e(B, 2 * cd)
        a, v = cat[:, :cd], cat[:, cd:]
        lin("audio_proj", a_emb, a)
        lin("video_proj", v_emb, v)
        if drop_a:
            a.zero_()
        if drop_v:
            v.zero_()
        sv = {"cat": cat}
        if mode == "concat":
            w0 = p["fusion.0.weight"]
            h = lin("fusion.0", cat, e(B, w0.shape[0]), act="relu")
            K.dropout_(h, dp, rng, SITE_EMB_MLP)
            w3 = p["fusion.3.weight"]
            out = lin("fusion.3", h, e(B, w3.shape[0]))
            sv["h"] = h
        else:
            w0 = p["gate.0.weight"]
            h = lin("gate.0", cat, e(B, w0.shape[0]), act="relu")
            K.dropout_(h, dp, rng, SITE_EMB_MLP)
            z = lin("gate.3", h, e(B, 1))
            fused, g = e(B, cd), e(B)
            K.gate_mix_fwd(z, a, v, fused, g)  # g*a + (1-g)*v  (fusion.py:434)
            wc = p["classifier.weight"]
            out = lin("classifier", fused, e(B, wc.shape[0]))
            sv.update(h=h, g=g, fused=fused)
        ctx.sv, ctx.p, ctx.names, ctx.params = sv, p, names, params
        ctx.mode, ctx.dp, ctx.rng, ctx.drops = mode, dp, rng, (drop_a, drop_v)
        ctx.a_emb, ctx.v_emb = a_emb, v_emb
        return out

    @staticmethod
    def backward(ctx, dout):
        p, sv = ctx.p, ctx.sv
        dout = dout.contiguous().float()
        B = dout.shape[0]
        dev = dout.device
        e = lambda *s: torch.empty(s, device=dev, dtype=torch.float32)  # noqa: E731
        used = ["audio_proj.weight", "audio_proj.bias", "video_proj.weight", "video_proj.bias"]
        used += (["fusion.0.weight", "fusion.0.bias", "fusion.3.weight", "fusion.3.bias"] if ctx.mode == "concat" else
                 ["gate.0.weight", "gate.0.bias", "gate.3.weight", "gate.3.bias", "classifier.weight", "classifier.bias"])
        drop_a, drop_v = ctx.drops
        # a dropped modality's projection output was replaced by zeros (fusion.py:47-53 zeros_like): it and its
        # encoder get no gradient at all (None, not zeros), so torch Adam's skip rule applies to them
        if drop_a:
            used = [n for n in used if not n.startswith("audio_proj.")]
        if drop_v:
            used = [n for n in used if not n.startswith("video_proj.")]
        grads = {n: _grad_buf(p[n]) for n in used}
        cat = sv["cat"]
        cd = cat.shape[1] // 2
        dcat = e(B, 2 * cd)
        if ctx.mode == "concat":
            h = sv["h"]
            dh = e(B, h.shape[1])
            K.linear_bwd(h, p["fusion.3.weight"], dout, dx=dh, dw=grads["fusion.3.weight"], db=grads["fusion.3.bias"])
            K.relu_dropout_bwd_(dh, h, ctx.dp, ctx.rng, SITE_EMB_MLP)
            K.linear_bwd(cat, p["fusion.0.weight"], dh, dx=dcat, dw=grads["fusion.0.weight"], db=grads["fusion.0.bias"])
        else:
            h, g, fused = sv["h"], sv["g"], sv["fused"]
            dfused = e(B, cd)
            K.linear_bwd(fused, p["classifier.weight"], dout, dx=dfused, dw=grads["classifier.weight"],
                         db=grads["classifier.bias"])
            dcat.zero_()
            dz = e(B, 1)
            K.gate_mix_bwd(g, cat[:, :cd], cat[:, cd:], dfused, dz, dcat[:, :cd], dcat[:, cd:])
            dh = e(B, h.shape[1])
            K.linear_bwd(h, p["gate.3.weight"], dz, dx=dh, dw=grads["gate.3.weight"], db=grads["gate.3.bias"])
            K.relu_dropout_bwd_(dh, h, ctx.dp, ctx.rng, SITE_EMB_MLP)
            K.linear_bwd(cat, p["gate.0.weight"], dh, dx=dcat, dw=grads["gate.0.weight"], db=grads["gate.0.bias"],
                         dx_beta=1)
        need_a, need_v = ctx.needs_input_grad[0] and not drop_a, ctx.needs_input_grad[1] and not drop_v
        da = e(*ctx.a_emb.shape) if need_a else None
        dv = e(*ctx.v_emb.shape) if need_v else None
        if not drop_a:
            K.linear_bwd(ctx.a_emb, p["audio_proj.weight"], dcat[:, :cd], dx=da, dw=grads["audio_proj.weight"],
                         db=grads["audio_proj.bias"])
        if not drop_v:
            K.linear_bwd(ctx.v_emb, p["video_proj.weight"], dcat[:, cd:], dx=dv, dw=grads["video_proj.weight"],
                         db=grads["video_proj.bias"])
        out = [grads.get(n) if (n in grads and t.requires_grad) else None for n, t in zip(ctx.names, ctx.params)]
        return (da, dv, None, None, None, None, None, None, None, *out)


def embedding_head(model, a_emb, v_emb, drop_a=False, drop_v=False):
    names, params = [], []
    for n, q in model.named_parameters():
        if n.startswith(("audio_model.", "video_model.")):
            continue
        names.append(n)
        params.append(q)
    rng = model.step_rng(a_emb.device) if model.training else None
    # a dropped modality is cut from the autograd graph (its encoder's backward never runs, as in the reference)
    a_in = a_emb.detach() if drop_a else a_emb
    v_in = v_emb.detach() if drop_v else v_emb
    # the nn.Dropout(0.2) of fusion / gate (fusion.py:256-262), active in train mode only
    dp = float((model.fusion if model.mode == "concat" else model.gate)[2].p) if model.training else 0.0
    return _EmbHeadFn.apply(a_in.contiguous(), v_in.contiguous(), model.mode, dp, rng,
                            bool(drop_a), bool(drop_v), int8_images(model), tuple(names), *params)


def int8_images(model):
    """The model's INT8 Linear images (int8.quantize_dynamic_hip) -- used in eval mode only."""
    return None if model.training else getattr(model, "_mer_int8", None)


class _LateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a_logits, v_logits):
        a_logits = a_logits.contiguous().float()
        v_logits = v_logits.contiguous().float()
        out = torch.empty_like(a_logits)
        pa, pv = torch.empty_like(a_logits), torch.empty_like(v_logits)
        K.softmax_avg_fwd(a_logits, v_logits, out, pa, pv)
        ctx.save_for_backward(pa, pv)
        return out

    @staticmethod
    def backward(ctx, dout):
        pa, pv = ctx.saved_tensors
        da, dv = torch.empty_like(pa), torch.empty_like(pv)
        K.softmax_avg_bwd(pa, pv, dout.contiguous().float(), da, dv)
        return da, dv


def late_probs(a_logits, v_logits):
    """late mode (fusion.py:358-363): (softmax(a) + softmax(v)) / 2 -- probabilities."""
    return _LateFn.apply(a_logits, v_logits)
