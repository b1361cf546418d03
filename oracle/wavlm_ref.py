"""fp32 CPU restatement of WavLM-base forward (eval semantics).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Follows transformers' ``modeling_wavlm.py`` (installed 5.15.0; the reference pins
5.1.0 in ``uv.lock``), cited as TF:<line>, as reached from the reference's
``WavLMAudioEncoder.encode_sequence`` (``src/models/wavlm_audio.py:165-183``).
Parameter names are the HF state-dict names under ``audio_model.wavlm.``.
Train-mode stochastic parts (SpecAugment TF:985-1030, dropout, LayerDrop TF:414-419)
are not part of the pinned semantics; see DESIGN.md.
"""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

CONV_KERNEL = (10, 3, 3, 3, 3, 2, 2)
CONV_STRIDE = (5, 2, 2, 2, 2, 2, 2)
HIDDEN = 768
HEADS = 12
LAYERS = 12
NUM_BUCKETS = 320
MAX_DISTANCE = 800
POS_K = 128
POS_GROUPS = 16


def feature_extractor(p: Dict[str, Tensor], wav: Tensor, prefix: str = "") -> Tensor:
    """TF:723-782: conv0 + GroupNorm(512,512) + GELU, then 6x (conv + GELU). Returns [B, L, 512]."""
    x = wav[:, None]
    for i, (k, s) in enumerate(zip(CONV_KERNEL, CONV_STRIDE)):
        x = F.conv1d(x, p[f"{prefix}feature_extractor.conv_layers.{i}.conv.weight"], stride=s)
        if i == 0:
            x = F.group_norm(x, x.shape[1], p[f"{prefix}feature_extractor.conv_layers.0.layer_norm.weight"],
                             p[f"{prefix}feature_extractor.conv_layers.0.layer_norm.bias"], 1e-5)
        x = F.gelu(x)
    return x.transpose(1, 2)


def pos_conv_weight(p: Dict[str, Tensor], prefix: str = "") -> Tensor:
    """weight_norm(dim=2) of the positional conv (TF:48-80): w = g * v / ||v||_{dims 0,1}."""
    g = p[f"{prefix}encoder.pos_conv_embed.conv.parametrizations.weight.original0"]
    v = p[f"{prefix}encoder.pos_conv_embed.conv.parametrizations.weight.original1"]
    return torch._weight_norm(v, g, 2)


def relative_position_bucket(rel: Tensor) -> Tensor:
    """TF:253-271."""
    nb = NUM_BUCKETS // 2
    buckets = (rel > 0).to(torch.long) * nb
    rel = torch.abs(rel)
    max_exact = nb // 2
    is_small = rel < max_exact
    large = torch.log(rel.float() / max_exact) / math.log(MAX_DISTANCE / max_exact) * (nb - max_exact)
    large = (max_exact + large).to(torch.long)
    large = torch.min(large, torch.full_like(large, nb - 1))
    return buckets + torch.where(is_small, rel, large)


def position_bias(p: Dict[str, Tensor], length: int, prefix: str = "") -> Tensor:
    """TF:243-251: ``[H, L, L]`` from layer 0's ``rel_attn_embed``."""
    ctx = torch.arange(length)[:, None]
    mem = torch.arange(length)[None, :]
    b = relative_position_bucket(mem - ctx)
    emb = p[f"{prefix}encoder.layers.0.attention.rel_attn_embed.weight"]
    return emb[b].permute(2, 0, 1)


def attention(p: Dict[str, Tensor], x: Tensor, pos_bias: Tensor, li: int, prefix: str = "") -> Tensor:
    """TF:147-186 + F.multi_head_attention_forward with separate q/k/v weights."""
    n = f"{prefix}encoder.layers.{li}.attention."
    bsz, length, d = x.shape
    dh = d // HEADS
    # gated relative position bias (TF:163-177): gate from the layer input, per head
    gx = x.view(bsz, length, HEADS, dh).permute(0, 2, 1, 3)
    proj = gx @ p[n + "gru_rel_pos_linear.weight"].t() + p[n + "gru_rel_pos_linear.bias"]
    proj = proj.view(bsz, HEADS, length, 2, 4).sum(-1)
    gate_a, gate_b = torch.sigmoid(proj).chunk(2, dim=-1)
    const = p[n + "gru_rel_pos_const"].view(1, HEADS, 1, 1)
    gate = gate_a * (gate_b * const - 1.0) + 2.0  # [B,H,L,1]
    bias = gate * pos_bias[None]  # [B,H,L,L]

    q = x @ p[n + "q_proj.weight"].t() + p[n + "q_proj.bias"]
    k = x @ p[n + "k_proj.weight"].t() + p[n + "k_proj.bias"]
    v = x @ p[n + "v_proj.weight"].t() + p[n + "v_proj.bias"]
    q = q.view(bsz, length, HEADS, dh).transpose(1, 2)
    k = k.view(bsz, length, HEADS, dh).transpose(1, 2)
    v = v.view(bsz, length, HEADS, dh).transpose(1, 2)
    s = (q * (1.0 / math.sqrt(dh))) @ k.transpose(-1, -2) + bias
    o = torch.softmax(s, dim=-1) @ v
    o = o.transpose(1, 2).reshape(bsz, length, d)
    return o @ p[n + "out_proj.weight"].t() + p[n + "out_proj.bias"]


def encoder_layer(p: Dict[str, Tensor], x: Tensor, pos_bias: Tensor, li: int, prefix: str = "") -> Tensor:
    """Post-LN ``WavLMEncoderLayer`` (TF:314-336)."""
    n = f"{prefix}encoder.layers.{li}."
    x = x + attention(p, x, pos_bias, li, prefix)
    x = F.layer_norm(x, (HIDDEN,), p[n + "layer_norm.weight"], p[n + "layer_norm.bias"], 1e-5)
    h = F.gelu(x @ p[n + "feed_forward.intermediate_dense.weight"].t() + p[n + "feed_forward.intermediate_dense.bias"])
    h = h @ p[n + "feed_forward.output_dense.weight"].t() + p[n + "feed_forward.output_dense.bias"]
    x = x + h
    return F.layer_norm(x, (HIDDEN,), p[n + "final_layer_norm.weight"], p[n + "final_layer_norm.bias"], 1e-5)


def wavlm_forward(p: Dict[str, Tensor], wav: Tensor, prefix: str = "", num_layers: int = LAYERS,
                  return_intermediates: bool = False):
    """``WavLMModel.forward`` (TF:1032-1085), eval mode. ``wav`` is [B, S] or [B, 1, S]."""
    if wav.dim() == 3:
        wav = wav.squeeze(1)
    inter = {}
    feats = feature_extractor(p, wav, prefix)
    inter["extract_conv"] = feats
    x = F.layer_norm(feats, (feats.shape[-1],), p[f"{prefix}feature_projection.layer_norm.weight"],
                     p[f"{prefix}feature_projection.layer_norm.bias"], 1e-5)
    x = x @ p[f"{prefix}feature_projection.projection.weight"].t() + p[f"{prefix}feature_projection.projection.bias"]
    inter["projected"] = x
    # WavLMEncoder.forward (TF:388-447)
    w = pos_conv_weight(p, prefix)
    pc = F.conv1d(x.transpose(1, 2), w, p[f"{prefix}encoder.pos_conv_embed.conv.bias"],
                  padding=POS_K // 2, groups=POS_GROUPS)
    pc = F.gelu(pc[:, :, :-1]).transpose(1, 2)
    x = x + pc
    x = F.layer_norm(x, (HIDDEN,), p[f"{prefix}encoder.layer_norm.weight"], p[f"{prefix}encoder.layer_norm.bias"], 1e-5)
    inter["encoder_in"] = x
    pb = position_bias(p, x.shape[1], prefix)
    for li in range(num_layers):
        x = encoder_layer(p, x, pb, li, prefix)
        if li == 0:
            inter["layer0"] = x
    return (x, inter) if return_intermediates else x


def wavlm_param_shapes(num_layers: int = LAYERS):
    """Names/shapes of ``WavLMModel(WavLMConfig())`` parameters (conv_bias=False)."""
    out = []
    cin = 1
    for i, k in enumerate(CONV_KERNEL):
        out.append((f"feature_extractor.conv_layers.{i}.conv.weight", (512, cin, k)))
        cin = 512
    out += [("feature_extractor.conv_layers.0.layer_norm.weight", (512,)),
            ("feature_extractor.conv_layers.0.layer_norm.bias", (512,)),
            ("feature_projection.layer_norm.weight", (512,)),
            ("feature_projection.layer_norm.bias", (512,)),
            ("feature_projection.projection.weight", (HIDDEN, 512)),
            ("feature_projection.projection.bias", (HIDDEN,)),
            ("masked_spec_embed", (HIDDEN,)),
            ("encoder.pos_conv_embed.conv.bias", (HIDDEN,)),
            ("encoder.pos_conv_embed.conv.parametrizations.weight.original0", (1, 1, POS_K)),
            ("encoder.pos_conv_embed.conv.parametrizations.weight.original1", (HIDDEN, HIDDEN // POS_GROUPS, POS_K)),
            ("encoder.layer_norm.weight", (HIDDEN,)),
            ("encoder.layer_norm.bias", (HIDDEN,))]
    for li in range(num_layers):
        n = f"encoder.layers.{li}."
        for proj in ("k_proj", "v_proj", "q_proj", "out_proj"):
            out += [(n + f"attention.{proj}.weight", (HIDDEN, HIDDEN)), (n + f"attention.{proj}.bias", (HIDDEN,))]
        out += [(n + "attention.gru_rel_pos_const", (1, HEADS, 1, 1)),
                (n + "attention.gru_rel_pos_linear.weight", (8, HIDDEN // HEADS)),
                (n + "attention.gru_rel_pos_linear.bias", (8,))]
        if li == 0:
            out.append((n + "attention.rel_attn_embed.weight", (NUM_BUCKETS, HEADS)))
        out += [(n + "layer_norm.weight", (HIDDEN,)), (n + "layer_norm.bias", (HIDDEN,)),
                (n + "feed_forward.intermediate_dense.weight", (3072, HIDDEN)),
                (n + "feed_forward.intermediate_dense.bias", (3072,)),
                (n + "feed_forward.output_dense.weight", (HIDDEN, 3072)),
                (n + "feed_forward.output_dense.bias", (HIDDEN,)),
                (n + "final_layer_norm.weight", (HIDDEN,)), (n + "final_layer_norm.bias", (HIDDEN,))]
    return out
