"""fp32 CPU restatement of the fusion head (xattn / concat / gated / late) and temporal pooling.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Every function is a functional restatement over a flat ``{state_dict_name: tensor}``
dict whose keys are the reference's own state-dict names (``fusion.py`` module
attribute names), so a reference checkpoint's head can be fed straight in.
Dropout / drop-path are treated as identity (eval mode, or train mode with p=0),
which is what the golden vectors pin.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
Params = Dict[str, Tensor]


def linear(x: Tensor, p: Params, name: str) -> Tensor:
    """nn.Linear: ``x W^T + b`` (dynamic INT8 when ``int8_ref.quantize_params`` marked it)."""
    if name + "._qweight" in p:
        from .int8_ref import linear_int8_torch

        return linear_int8_torch(x, p, name)
    y = x @ p[name + ".weight"].t()
    b = p.get(name + ".bias")
    return y + b if b is not None else y


def layer_norm(x: Tensor, p: Params, name: str, eps: float = 1e-5) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)


def mha(query: Tensor, kv: Tensor, p: Params, name: str, num_heads: int,
        attn_bias: Optional[Tensor] = None) -> Tensor:
    """``nn.MultiheadAttention(batch_first=True)`` explicit path, TORCH:6576-6606.

    ``attn_bias`` is the per-sample additive float mask ``[B, Lq, Lk]``; the reference
    ``repeat_interleave``s it over heads (``fusion.py:351-354``) so head h of sample b
    sees ``attn_bias[b]``.
    """
    w = p[name + ".in_proj_weight"]
    b = p[name + ".in_proj_bias"]
    d = w.shape[1]
    q = query @ w[:d].t() + b[:d]
    k = kv @ w[d:2 * d].t() + b[d:2 * d]
    v = kv @ w[2 * d:].t() + b[2 * d:]
    bsz, lq, _ = q.shape
    lk = k.shape[1]
    dh = d // num_heads
    q = q.view(bsz, lq, num_heads, dh).transpose(1, 2)
    k = k.view(bsz, lk, num_heads, dh).transpose(1, 2)
    v = v.view(bsz, lk, num_heads, dh).transpose(1, 2)
    s = (q * math.sqrt(1.0 / dh)) @ k.transpose(-1, -2)
    if attn_bias is not None:
        s = s + attn_bias[:, None]
    pr = torch.softmax(s, dim=-1)
    o = (pr @ v).transpose(1, 2).reshape(bsz, lq, d)
    return linear(o, p, name + ".out_proj")


def emotion_prior_bias(v: Tensor, a: Tensor, p: Params, name: str = "emotion_prior_bias"):
    """``EmotionPriorBiasAdapter.forward`` (fusion.py:170-184)."""
    vg = v.mean(dim=1)
    ag = a.mean(dim=1)
    h = torch.relu(linear(torch.cat([vg, ag], dim=-1), p, name + ".prior_net.0"))
    prior = linear(h, p, name + ".prior_net.3")

    def token_bias(qt, kt, qh, kh):
        qp = prior[:, None, :].expand(-1, qt.shape[1], -1)
        kp = prior[:, None, :].expand(-1, kt.shape[1], -1)
        qs = linear(torch.cat([qt, qp], dim=-1), p, name + "." + qh).squeeze(-1)
        ks = linear(torch.cat([kt, kp], dim=-1), p, name + "." + kh).squeeze(-1)
        return torch.tanh(qs[:, :, None] + ks[:, None, :]) * p[name + ".bias_scale"]

    v2a = token_bias(v, a, "v_query_bias", "a_key_bias")
    a2v = token_bias(a, v, "a_query_bias", "v_key_bias")
    return prior, v2a, a2v


def sinusoidal_pe(length: int, dim: int) -> Tensor:
    """``SinusoidalPositionalEncoding`` (temporal.py:29-43)."""
    position = torch.arange(length).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, dim, 2) * (-math.log(10000.0) / max(1, dim)))
    pe = torch.zeros(length, dim)
    pe[:, 0::2] = torch.sin(position * div_term)
    if dim > 1:
        pe[:, 1::2] = torch.cos(position * div_term[: pe[:, 1::2].shape[1]])
    return pe


def attn_pool(x: Tensor, p: Params, name: str) -> Tensor:
    """``TemporalAttentionPooling`` (temporal.py:9-26)."""
    h = layer_norm(x, p, name + ".score.0")
    h = F.gelu(linear(h, p, name + ".score.1"))
    logits = linear(h, p, name + ".score.4").squeeze(-1)
    w = torch.softmax(logits, dim=1).unsqueeze(-1)
    return torch.sum(x * w, dim=1)


def transformer_pool(x: Tensor, p: Params, name: str, num_heads: int, num_layers: int) -> Tensor:
    """``TemporalTransformerPooling`` (temporal.py:46-75): PE, pre-LN encoder layers, attention pool."""
    x = x + sinusoidal_pe(x.shape[1], x.shape[2]).to(x.dtype)
    for i in range(num_layers):
        ln = f"{name}.encoder.layers.{i}"
        h = layer_norm(x, p, ln + ".norm1")
        w = p[ln + ".self_attn.in_proj_weight"]
        x = x + mha(h, h, p, ln + ".self_attn", num_heads)
        h = layer_norm(x, p, ln + ".norm2")
        h = linear(F.gelu(linear(h, p, ln + ".linear1")), p, ln + ".linear2")
        x = x + h
        del w
    return attn_pool(x, p, name + ".pool")


def temporal_pool(x: Tensor, p: Params, name: str, mode: str, num_heads: int = 4, num_layers: int = 1) -> Tensor:
    """``TemporalPooler.forward`` (temporal.py:105-110)."""
    if x.ndim != 3:
        raise ValueError(f"TemporalPooler expects [B, T, D], got shape={tuple(x.shape)}")
    if mode == "mean":
        return x.mean(dim=1)
    if mode == "attn":
        return attn_pool(x, p, name + ".pool")
    if mode == "transformer":
        return transformer_pool(x, p, name + ".pool", num_heads, num_layers)
    raise ValueError(f"Unsupported temporal pooling mode: {mode}")


def xattn_forward(p: Params, v_feat: Tensor, a_seq: Tensor, *, num_heads: int = 4,
                  xattn_head: str = "concat", use_prior: bool = False,
                  temporal_pooling: str = "mean", temporal_num_heads: int = 4,
                  temporal_num_layers: int = 1):
    """xattn branch of ``FusionModel.forward`` after the encoders (fusion.py:372-411).

    ``v_feat`` = ``video_model.backbone(...)`` reshaped ``[B,T,v_dim]`` (fusion.py:370);
    ``a_seq`` = ``audio_model.encode_sequence(audio)`` ``[B,Ta,seq_dim]`` (fusion.py:377).
    Returns ``(logits, intermediates)``.
    """
    inter = {}
    v = linear(v_feat, p, "v_in_proj")
    a = linear(linear(a_seq, p, "audio_seq_proj"), p, "a_in_proj")
    inter["v0"], inter["a0"] = v, a
    v2a_bias = a2v_bias = None
    if use_prior:
        prior, v2a_bias, a2v_bias = emotion_prior_bias(v, a, p)
        inter["prior"], inter["v2a_bias"], inter["a2v_bias"] = prior, v2a_bias, a2v_bias
    v2 = mha(v, a, p, "v2a_attn", num_heads, v2a_bias)
    v = layer_norm(v + v2, p, "v_norm")
    a2 = mha(a, v, p, "a2v_attn", num_heads, a2v_bias)
    a = layer_norm(a + a2, p, "a_norm")
    inter["v1"], inter["a1"] = v, a
    v_emb = temporal_pool(v, p, "v_temporal_pool", temporal_pooling, temporal_num_heads, temporal_num_layers)
    a_emb = temporal_pool(a, p, "a_temporal_pool", temporal_pooling, temporal_num_heads, temporal_num_layers)
    inter["v_emb"], inter["a_emb"] = v_emb, a_emb
    if xattn_head == "concat":
        h = torch.relu(linear(torch.cat([v_emb, a_emb], dim=1), p, "xattn_mlp.0"))
        logits = linear(h, p, "xattn_mlp.3")
    elif xattn_head == "gated":
        h = torch.relu(linear(torch.cat([v_emb, a_emb], dim=1), p, "xattn_gate.0"))
        g = torch.sigmoid(linear(h, p, "xattn_gate.3"))
        logits = linear(g * v_emb + (1 - g) * a_emb, p, "xattn_classifier")
    else:
        raise ValueError(f"Unknown xattn head: {xattn_head}")
    return logits, inter


def clip_alignment(p: Params, a_emb: Tensor, v_emb: Tensor, name: str = "semantic_alignment"):
    """``ClipStyleAlignment.forward`` (fusion.py:137-150) -> (a_aligned, v_aligned, loss)."""
    a_al = linear(a_emb, p, name + ".audio_proj")
    v_al = linear(v_emb, p, name + ".video_proj")
    a_n = F.normalize(a_al, dim=-1)
    v_n = F.normalize(v_al, dim=-1)
    scale = p[name + ".logit_scale"].exp().clamp(max=100.0)
    logits = scale * (a_n @ v_n.t())
    t = torch.arange(logits.shape[0])
    loss = 0.5 * (F.cross_entropy(logits, t) + F.cross_entropy(logits.t(), t))
    return a_al, v_al, loss


def embedding_fusion_forward(p: Params, mode: str, a_emb: Tensor, v_emb: Tensor, align: bool = False):
    """Non-xattn ``concat`` / ``gated`` branch (fusion.py:413-435) after ``encode``.  ``align``: the
    ``fusion_align_mode="clip"`` variant (fusion.py:417-418); returns (out, alignment loss) then."""
    align_loss = None
    if align:
        a_emb, v_emb, align_loss = clip_alignment(p, a_emb, v_emb)
    out = _embedding_head(p, mode, a_emb, v_emb)
    return (out, align_loss) if align else out


def _embedding_head(p: Params, mode: str, a_emb: Tensor, v_emb: Tensor):
    a = linear(a_emb, p, "audio_proj")
    v = linear(v_emb, p, "video_proj")
    if mode == "concat":
        h = torch.relu(linear(torch.cat([a, v], dim=1), p, "fusion.0"))
        return linear(h, p, "fusion.3")
    if mode == "gated":
        h = torch.relu(linear(torch.cat([a, v], dim=1), p, "gate.0"))
        g = torch.sigmoid(linear(h, p, "gate.3"))
        return linear(g * a + (1 - g) * v, p, "classifier")
    raise ValueError(f"Unknown fusion mode: {mode}")


def late_forward(a_logits: Tensor, v_logits: Tensor) -> Tensor:
    """``late`` mode (fusion.py:358-363): mean of the two softmaxes (probabilities, not logits)."""
    return (torch.softmax(a_logits, dim=1) + torch.softmax(v_logits, dim=1)) / 2.0


def cross_entropy(logits: Tensor, labels: Tensor, label_smoothing: float = 0.0) -> Tensor:
    """``nn.CrossEntropyLoss(label_smoothing)`` (train.py:1033), mean reduction."""
    return F.cross_entropy(logits, labels, label_smoothing=label_smoothing)


def late_nll(probs: Tensor, labels: Tensor) -> Tensor:
    """late-mode loss ``NLLLoss(log(p + 1e-8))`` (train.py:212-214)."""
    return F.nll_loss(torch.log(probs + 1e-8), labels)


def _lin(n, o, i, bias=True):
    return [(n + ".weight", (o, i))] + ([(n + ".bias", (o,))] if bias else [])


def _mha(n, d):
    return [(n + ".in_proj_weight", (3 * d, d)), (n + ".in_proj_bias", (3 * d,))] + _lin(n + ".out_proj", d, d)


def _ln(n, d):
    return [(n + ".weight", (d,)), (n + ".bias", (d,))]


def _pool_shapes(n, d, mode, num_layers):
    if mode == "mean":
        return []
    if mode == "attn":
        h = max(1, d // 2)
        return _ln(n + ".pool.score.0", d) + _lin(n + ".pool.score.1", h, d) + _lin(n + ".pool.score.4", 1, h)
    out = []
    ffn = max(d * 2, int(d * 4.0))
    for i in range(num_layers):
        ln = f"{n}.pool.encoder.layers.{i}"
        out += _mha(ln + ".self_attn", d) + _lin(ln + ".linear1", ffn, d) + _lin(ln + ".linear2", d, ffn)
        out += _ln(ln + ".norm1", d) + _ln(ln + ".norm2", d)
    h = max(1, d // 2)
    out += _ln(n + ".pool.pool.score.0", d) + _lin(n + ".pool.pool.score.1", h, d) + _lin(n + ".pool.pool.score.4", 1, h)
    return out


def xattn_head_param_shapes(v_dim=512, seq_dim=768, d_model=128, num_classes=8, common_dim=256,
                            audio_n_mels=768, xattn_head="concat", use_prior=False, prior_dim=8,
                            prior_hidden=64, temporal_pooling="mean", temporal_num_layers=1):
    """Names/shapes of ``FusionModel(mode='xattn')``'s own parameters (fusion.py:263-327), in module order."""
    d = d_model
    out = _lin("v_in_proj", d, v_dim) + _lin("a_in_proj", d, d)
    out += [("audio_time_conv.weight", (d, audio_n_mels, 3)), ("audio_time_conv.bias", (d,))]
    out += _lin("audio_seq_proj", d, seq_dim)
    out += _mha("v2a_attn", d) + _mha("a2v_attn", d) + _ln("v_norm", d) + _ln("a_norm", d)
    if use_prior:
        n = "emotion_prior_bias"
        out += [(n + ".bias_scale", ())]  # module-own params precede submodules in state_dict order
        out += _lin(n + ".prior_net.0", prior_hidden, 2 * d) + _lin(n + ".prior_net.3", prior_dim, prior_hidden)
        for hname in ("v_query_bias", "a_key_bias", "a_query_bias", "v_key_bias"):
            out += _lin(f"{n}.{hname}", 1, d + prior_dim)
    out += _pool_shapes("v_temporal_pool", d, temporal_pooling, temporal_num_layers)
    out += _pool_shapes("a_temporal_pool", d, temporal_pooling, temporal_num_layers)
    if xattn_head == "concat":
        out += _lin("xattn_mlp.0", common_dim, 2 * d) + _lin("xattn_mlp.3", num_classes, common_dim)
    else:
        out += _lin("xattn_gate.0", d, 2 * d) + _lin("xattn_gate.3", 1, d) + _lin("xattn_classifier", num_classes, d)
    return out


def gated_bias_init(p: Params, xattn_head: str = "concat") -> None:
    """``_init_xattn_gated_bias`` (fusion.py:338-344): BOTH gate Linear biases are filled with -1
    (the ``layer != self.xattn_gate[-1]`` test compares against the Sigmoid)."""
    if xattn_head == "gated":
        p["xattn_gate.0.bias"].fill_(-1.0)
        p["xattn_gate.3.bias"].fill_(-1.0)
