"""``WavLMAudioEncoder`` mirror (``src/models/wavlm_audio.py``) with a WavLM-base forward on HIP kernels.

The module tree reproduces transformers' ``WavLMModel`` attribute names, so state-dict keys are
identical (``audio_model.wavlm.encoder.layers.3.attention.q_proj.weight``, the positional conv's
``parametrizations.weight.original0/1`` ...) and reference checkpoints load unchanged.  The model
is built offline from the WavLM-base config (the reference's ``from_pretrained`` network fetch has
its own offline fallback to exactly this, wavlm_audio.py:35-41).

Forward (``encode_sequence``, wavlm_audio.py:165-183 -> TF:1032-1085), all bf16 activations with
fp32 accumulation:
  conv0 + GroupNorm + GELU (two-pass, deterministic) -> conv1..6 (Conv1d-as-GEMM, GELU epilogue)
  -> LayerNorm(512) -> projection GEMM -> grouped pos-conv GEMM (+GELU +residual) -> LayerNorm
  -> 12 x [fused QKV GEMM -> gated-rel-pos attention -> out-proj GEMM (+residual) -> LN
           -> FFN GEMM (+GELU) -> FFN GEMM (+residual) -> LN]
Frozen by default (no backward).  Stage 2 (``unfreeze_backbone(n)``, wavlm_audio.py:70-88) runs the frozen
prefix as above and the last n layers as one autograd node (``forward_train`` / ``tail_backward``,
csrc/wavlm_train.hip), eval semantics (no dropout / LayerDrop).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
from torch import nn

from . import graphs as G
from . import kernels as K
from .nn_ops import draw_seed, hip_dropout, hip_linear
from .optim import weight_version
from .temporal import TemporalPooler

CONV_DIM = 512
CONV_KERNEL = (10, 3, 3, 3, 3, 2, 2)
CONV_STRIDE = (5, 2, 2, 2, 2, 2, 2)


class WavLMConfigLite:
    """The WavLM-base hyper-parameters used by ``WavLMModel(WavLMConfig())`` (TF config defaults)."""

    hidden_size = 768
    num_attention_heads = 12
    num_hidden_layers = 12
    intermediate_size = 3072
    num_buckets = 320
    max_bucket_distance = 800
    num_conv_pos_embeddings = 128
    num_conv_pos_embedding_groups = 16
    layer_norm_eps = 1e-5
    # train-mode regularisers (WavLMConfig defaults; active whenever the module is in train mode, as in the
    # reference, which keeps the frozen WavLM in train mode under no_grad: train.py:194, wavlm_audio.py:177-182)
    hidden_dropout = 0.1
    attention_dropout = 0.1
    activation_dropout = 0.1
    feat_proj_dropout = 0.0
    layerdrop = 0.1
    mask_time_prob = 0.05
    mask_time_length = 10
    mask_time_min_masks = 2


# dropout call sites of the WavLM forward (mixed with the forward's RNG base, csrc/common.h mer_site_seed)
SITE_TIME_MASK, SITE_ENC_DROPOUT = 1000, 1001


def _gemm_pick(ctl) -> int:
    """GEMM tile rule of a frozen forward (csrc/gemm_bf16.hip pick_variant): the train-mode forward (``ctl`` set)
    is the one the train step prefetches on its side stream beside the trunk, where the step is bound by the two
    streams' summed CU-time, so its GEMMs take the CU-time pick (-2: every shape on the 256^2 split ring); eval /
    inference and the stage-2 tail run alone and keep the wall-time pick (-1)."""
    return -2 if ctl is not None else -1


def _layer_sites(li: int):
    """(attention probs, attention output, FFN activation, FFN output) dropout sites of encoder layer li."""
    b = 1100 + 8 * li
    return b, b + 1, b + 2, b + 3


class TrainCtl:
    """Host-drawn randomness of one train-mode WavLM forward: the dropout / SpecAugment RNG base and the LayerDrop
    bitmask (bit i set = layer i skipped; TF:417-419 draws torch.rand([]) per layer, layer 0 never skipped).
    ``rng`` / ``skip`` are device int64 scalars the kernels read (graph-capturable)."""

    def __init__(self, seed: int, mask: int, rng: torch.Tensor, skip: torch.Tensor):
        self.seed, self.mask, self.rng, self.skip = seed, mask, rng, skip

    def executed(self, num_layers: int) -> int:
        return sum(1 for i in range(num_layers) if not (self.mask >> i) & 1)


class _ConvLayer(nn.Module):
    def __init__(self, layer_id: int):
        super().__init__()
        cin = 1 if layer_id == 0 else CONV_DIM
        self.conv = nn.Conv1d(cin, CONV_DIM, CONV_KERNEL[layer_id], stride=CONV_STRIDE[layer_id], bias=False)
        if layer_id == 0:
            self.layer_norm = nn.GroupNorm(CONV_DIM, CONV_DIM, affine=True)


class _FeatureExtractor(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv_layers = nn.ModuleList([_ConvLayer(i) for i in range(len(CONV_KERNEL))])


class _FeatureProjection(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layer_norm = nn.LayerNorm(CONV_DIM, eps=cfg.layer_norm_eps)
        self.projection = nn.Linear(CONV_DIM, cfg.hidden_size)


class _PosConv(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        conv = nn.Conv1d(cfg.hidden_size, cfg.hidden_size, cfg.num_conv_pos_embeddings,
                         padding=cfg.num_conv_pos_embeddings // 2, groups=cfg.num_conv_pos_embedding_groups)
        self.conv = nn.utils.parametrizations.weight_norm(conv, name="weight", dim=2)


class _Attention(nn.Module):
    def __init__(self, cfg, has_bias: bool):
        super().__init__()
        d, h = cfg.hidden_size, cfg.num_attention_heads
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.q_proj = nn.Linear(d, d)
        self.out_proj = nn.Linear(d, d)
        self.gru_rel_pos_const = nn.Parameter(torch.ones(1, h, 1, 1))
        self.gru_rel_pos_linear = nn.Linear(d // h, 8)
        if has_bias:
            self.rel_attn_embed = nn.Embedding(cfg.num_buckets, h)


class _FeedForward(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.intermediate_dense = nn.Linear(cfg.hidden_size, cfg.intermediate_size)
        self.output_dense = nn.Linear(cfg.intermediate_size, cfg.hidden_size)


class _EncoderLayer(nn.Module):
    def __init__(self, cfg, has_bias):
        super().__init__()
        self.attention = _Attention(cfg, has_bias)
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.feed_forward = _FeedForward(cfg)
        self.final_layer_norm = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.pos_conv_embed = _PosConv(cfg)
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.layers = nn.ModuleList([_EncoderLayer(cfg, i == 0) for i in range(cfg.num_hidden_layers)])


def relative_position_buckets(length: int, num_buckets: int = 320, max_distance: int = 800) -> np.ndarray:
    """Bucket of every relative position j - i in [-(L-1), L-1] (TF:253-271), int32 [2L-1]."""
    rel = np.arange(-(length - 1), length, dtype=np.int64)
    nb = num_buckets // 2
    buckets = (rel > 0).astype(np.int64) * nb
    r = np.abs(rel)
    max_exact = nb // 2
    with np.errstate(divide="ignore"):
        large = np.log(np.maximum(r, 1).astype(np.float32) / max_exact) / math.log(max_distance / max_exact) * (nb - max_exact)
    large = np.minimum((max_exact + large).astype(np.int64), nb - 1)
    return (buckets + np.where(r < max_exact, r, large)).astype(np.int32)


class WavLMBackbone(nn.Module):
    """Parameter container named like transformers' ``WavLMModel`` + the HIP forward schedule."""

    def __init__(self, cfg: Optional[WavLMConfigLite] = None):
        super().__init__()
        self.config = cfg or WavLMConfigLite()
        self.feature_extractor = _FeatureExtractor()
        self.feature_projection = _FeatureProjection(self.config)
        self.masked_spec_embed = nn.Parameter(torch.empty(self.config.hidden_size).uniform_())
        self.encoder = _Encoder(self.config)
        self._packed = None
        self._packed_key = None
        self._buckets: Dict[tuple, torch.Tensor] = {}
        self._graphs = G.GraphCache()
        # reference semantics: train mode = dropout + LayerDrop + SpecAugment; False runs train mode with eval
        # semantics (deterministic parity tests against the fp32 oracle)
        self.train_semantics = True
        self.executed_layers = 0  # encoder layers actually run by train-mode forwards (bench.py's FLOP count)
        self.train_forwards = 0

    # ---- train-mode randomness ----
    def train_active(self) -> bool:
        return self.training and self.train_semantics

    def draw_train(self, num_layers: Optional[int] = None):
        """(seed, LayerDrop mask) for one train-mode forward, from the host generators (torch.manual_seed
        reproduces them); None in eval semantics."""
        if not self.train_active():
            return None
        cfg = self.config
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        r = torch.rand(cfg.num_hidden_layers)
        mask = 0
        for i in range(1, cfg.num_hidden_layers):
            if float(r[i]) < cfg.layerdrop:
                mask |= 1 << i
        nl = cfg.num_hidden_layers if num_layers is None else num_layers
        self.executed_layers += sum(1 for i in range(nl) if not (mask >> i) & 1)
        self.train_forwards += 1
        return seed, mask

    @staticmethod
    def train_ctl(draw, device, rng=None, skip=None) -> Optional[TrainCtl]:
        """Device scalars of a draw (fresh, or refilled static graph buffers)."""
        if draw is None:
            return None
        seed, mask = draw
        if rng is None:
            rng = torch.full((1,), seed, dtype=torch.int64, device=device)
            skip = torch.full((1,), mask, dtype=torch.int64, device=device)
        else:
            rng.fill_(seed)
            skip.fill_(mask)
        return TrainCtl(seed, mask, rng, skip)

    # ---- frozen-weight preparation (runs once per weight version, on the GPU kernels) ----
    def _param_list(self):
        lst = self.__dict__.get("_mer_params")
        if lst is None:
            lst = self.__dict__["_mer_params"] = list(self.parameters())
        return lst

    def _weights_key(self):
        return tuple(weight_version(q) for q in self._param_list())

    def _prefix_param_count(self, first_layer: int) -> int:
        """Number of entries of _param_list() (module order) before encoder layer ``first_layer``."""
        first = next(iter(self.encoder.layers[first_layer].parameters()))
        return next(i for i, q in enumerate(self._param_list()) if q is first)

    def trainable(self) -> bool:
        return any(q.requires_grad for q in self._param_list())

    @torch.no_grad()
    def packed_weights(self):
        key = self._weights_key()
        if self._packed is not None and self._packed_key == key:
            return self._packed
        limit = self.__dict__.get("_pack_limit")  # stage-2 prefix call: only layers < limit are used
        if limit is not None and self._packed is not None:
            n = self._prefix_param_count(limit)
            if self._packed_key[:n] == key[:n]:
                return self._packed
        dev = self.masked_spec_embed.device
        cfg = self.config
        pk = {"conv": []}
        fe = self.feature_extractor.conv_layers
        pk["conv0_w"] = fe[0].conv.weight.detach().reshape(CONV_DIM, CONV_KERNEL[0]).contiguous()
        for i in range(1, len(CONV_KERNEL)):
            w = fe[i].conv.weight.detach()  # [Cout, Cin, k] -> [Cout, k, Cin]
            k = CONV_KERNEL[i]
            dst = torch.empty(CONV_DIM, k, CONV_DIM, device=dev, dtype=torch.bfloat16)
            K.permute3_bf16(w.contiguous(), (CONV_DIM, k, CONV_DIM), (CONV_DIM * k, 1, k), dst)
            pk["conv"].append(dst.view(CONV_DIM, k * CONV_DIM))
        pk["proj_w"] = self._bf16(self.feature_projection.projection.weight)
        pc = self.encoder.pos_conv_embed.conv
        g = pc.parametrizations.weight.original0.detach().reshape(-1).contiguous()
        v = pc.parametrizations.weight.original1.detach().contiguous()  # [768, 48, 128]
        scale = torch.empty(cfg.num_conv_pos_embeddings, device=dev, dtype=torch.float32)
        K.weightnorm_scale(v, g, scale)
        taps, cg = cfg.num_conv_pos_embeddings, cfg.hidden_size // cfg.num_conv_pos_embedding_groups
        wp = torch.empty(cfg.hidden_size, taps, cg, device=dev, dtype=torch.bfloat16)  # [g*Cg+n][tap][c]
        K.permute3_bf16(v, (cfg.hidden_size, taps, cg), (cg * taps, 1, taps), wp, scale=scale)
        pk["posconv_w"] = wp
        layers = []
        for layer in self.encoder.layers:
            at = layer.attention
            qkv = torch.empty(3 * cfg.hidden_size, cfg.hidden_size, device=dev, dtype=torch.bfloat16)
            for j, lin in enumerate((at.q_proj, at.k_proj, at.v_proj)):
                K.cast_bf16(lin.weight.detach().contiguous(), qkv[j * cfg.hidden_size:(j + 1) * cfg.hidden_size])
            qkv_b = torch.cat([at.q_proj.bias, at.k_proj.bias, at.v_proj.bias]).detach().contiguous()
            layers.append(dict(qkv_w=qkv, qkv_b=qkv_b, out_w=self._bf16(at.out_proj.weight),
                               ff1_w=self._bf16(layer.feed_forward.intermediate_dense.weight),
                               ff2_w=self._bf16(layer.feed_forward.output_dense.weight),
                               gate_c=at.gru_rel_pos_const.detach().reshape(-1).contiguous()))
        pk["layers"] = layers
        pk["rel_emb"] = self.encoder.layers[0].attention.rel_attn_embed.weight.detach().contiguous()
        self._packed, self._packed_key = pk, key
        return pk

    @staticmethod
    def _bf16(w):
        dst = torch.empty(w.shape, device=w.device, dtype=torch.bfloat16)
        K.cast_bf16(w.detach().contiguous(), dst)
        return dst

    def buckets(self, length: int, device) -> torch.Tensor:
        key = (length, str(device))
        if key not in self._buckets:
            cfg = self.config
            self._buckets[key] = torch.from_numpy(relative_position_buckets(length, cfg.num_buckets,
                                                                            cfg.max_bucket_distance)).to(device)
        return self._buckets[key]

    @torch.no_grad()
    def forward_hip(self, wav: torch.Tensor, out_dtype=torch.bfloat16, num_layers: Optional[int] = None,
                    capture: Optional[dict] = None):
        """Raw waveform [B, S] fp32 -> last_hidden_state [B, L, 768] (bf16 or fp32).

        ``capture`` (tests): receives copies of 'extract_features' (post-LN conv features, what HF
        returns as ``extract_features``) and 'layer0' (output of encoder layer 0).  In train mode (reference
        semantics) the forward applies SpecAugment time masking, dropout and LayerDrop (``draw_train``).

        After one eager call per input shape the whole schedule (conv0 .. final LayerNorm) runs as one
        captured hipGraph (graphs.py); a train-mode graph re-reads its RNG base and LayerDrop mask from two
        device scalars refilled before each replay."""
        if not wav.is_cuda:
            raise RuntimeError("WavLM runs on the MI355X kernels; move the waveform to the GPU")
        wav = wav.contiguous().float()
        nl = None if num_layers is None or num_layers >= len(self.encoder.layers) else int(num_layers)
        draw = self.draw_train(nl)
        self.__dict__["_last_draw"] = draw
        if capture is None and not G.capturing():
            # a prefix run (stage 2) is keyed on the prefix's weights only: the trainable tail changes every step
            wkey = self._weights_key()
            key = (tuple(wav.shape), out_dtype, wav.device.index, nl, draw is not None,
                   wkey if nl is None else wkey[:self._prefix_param_count(nl)])
            if self._graphs.ready(key):
                return self._forward_graphed(wav, out_dtype, key, nl, draw)
        ctl = self.train_ctl(draw, wav.device)
        x, L = self._stage_a(wav)
        y = self._conv_layer(x, 1, L, pick=_gemm_pick(ctl))
        return self._stage_b(y, L, out_dtype, nl, capture, ctl)

    def _forward_graphed(self, wav, out_dtype, key, nl=None, draw=None):
        """One captured graph per key (the whole forward, conv0 .. final LayerNorm)."""
        g = self._graphs.get(key)
        if g is None:
            ctl = None
            if draw is not None:  # static RNG-base / LayerDrop-mask scalars the graph reads
                ctl = self.train_ctl(draw, wav.device)
            def run(w):
                x, L0 = self._stage_a(w)
                return self._stage_b(self._conv_layer(x, 1, L0, pick=_gemm_pick(ctl)), L0, out_dtype, nl, None, ctl)

            graph = G.StaticGraph(run, [wav])
            # the graph reads the packed weights captured with it: keep that pack alive (a later full repack,
            # e.g. after the stage-2 tail moved, replaces self._packed while a prefix key still matches)
            g = self._graphs.put(key, (graph, ctl, self._packed))
        graph, ctl, _ = g
        if draw is not None:
            self.train_ctl(draw, wav.device, ctl.rng, ctl.skip)
        return G.hand_out(graph.replay(wav))

    def _stage_a(self, wav):
        """conv0 -> GroupNorm + GELU (one fused deterministic kernel pair): [B, S] -> [B, L0, 512] bf16."""
        pk = self.packed_weights()
        B, S = wav.shape
        L = (S - CONV_KERNEL[0]) // CONV_STRIDE[0] + 1
        xg = torch.empty(B, L, CONV_DIM, device=wav.device, dtype=torch.bfloat16)
        gn = self.feature_extractor.conv_layers[0].layer_norm
        K.wavlm_conv0_gn_gelu(wav, pk["conv0_w"], gn.weight, gn.bias, xg, eps=gn.eps)
        return xg, L

    def _conv_layer(self, x, i, L, out=None, pick=-1):
        """Feature-extractor conv i >= 1 as an implicit GEMM with fused GELU (TF:723-782).  ``pick``: the GEMM
        tile rule (-1 wall time, -2 CU-time: see ``_gemm_pick``)."""
        k, s = CONV_KERNEL[i], CONV_STRIDE[i]
        B = x.shape[0]
        L_out = (L - k) // s + 1
        y = out if out is not None else torch.empty(B, L_out, CONV_DIM, device=x.device, dtype=torch.bfloat16)
        K.gemm_bf16(x, self.packed_weights()["conv"][i - 1], y, M=B * L_out, K=k * CONV_DIM,
                    rows=(L_out, s * CONV_DIM, L * CONV_DIM), act="gelu", variant=pick)
        return y

    def _stage_b(self, x, L0, out_dtype, num_layers, capture, ctl: Optional[TrainCtl] = None):
        """conv2..6 -> feature projection (-> SpecAugment) -> positional conv -> encoder LN (-> dropout) -> encoder
        layers (x = conv1 output).  ``ctl``: train-mode randomness (None = eval semantics)."""
        cfg = self.config
        pk = self.packed_weights()
        B = x.shape[0]
        dev = x.device
        bf = torch.bfloat16
        L = (L0 - CONV_KERNEL[1]) // CONV_STRIDE[1] + 1
        pick = _gemm_pick(ctl)
        for i in range(2, len(CONV_KERNEL)):
            x = self._conv_layer(x, i, L, pick=pick)
            L = x.shape[1]
        D = cfg.hidden_size
        fp = self.feature_projection
        xn = torch.empty(B * L, CONV_DIM, device=dev, dtype=bf)
        K.layernorm(x.view(B * L, CONV_DIM), fp.layer_norm.weight, fp.layer_norm.bias, xn, eps=fp.layer_norm.eps)
        if capture is not None:
            capture["extract_features"] = xn.view(B, L, CONV_DIM).clone()
        h = torch.empty(B * L, D, device=dev, dtype=bf)
        K.gemm_bf16(xn, pk["proj_w"], h, bias=fp.projection.bias, variant=pick)  # feat_proj_dropout = 0 (TF:98-104)
        tr = ctl is not None
        if tr and cfg.mask_time_prob > 0:  # SpecAugment on the projected features (TF:1063 -> 1006-1015)
            K.wavlm_time_mask(h, B, L, self.masked_spec_embed, cfg.mask_time_prob, cfg.mask_time_length,
                              cfg.mask_time_min_masks, ctl.rng, SITE_TIME_MASK,
                              mask_out=capture.get("mask_out") if capture is not None else None)
        # positional conv: h + gelu(posconv(h) + bias)  (TF:82-90, 414-416)
        pc = self.encoder.pos_conv_embed.conv
        hp = torch.empty(B * L, D, device=dev, dtype=bf)
        K.posconv_gemm_bf16(h, pk["posconv_w"], hp, B, L, D, cfg.num_conv_pos_embedding_groups,
                            cfg.num_conv_pos_embeddings, cfg.num_conv_pos_embeddings // 2, pc.bias, h, act="gelu")
        x = torch.empty(B * L, D, device=dev, dtype=bf)
        hd = cfg.hidden_dropout if tr else 0.0
        K.layernorm(hp, self.encoder.layer_norm.weight, self.encoder.layer_norm.bias, x, eps=cfg.layer_norm_eps,
                    drop_p=hd, rng=ctl.rng if tr else None, site=SITE_ENC_DROPOUT)
        H = cfg.num_attention_heads
        # the relative-position bias rows of every head, gathered once per packed-weight version and length
        # (layer 0's embedding serves all layers, TF:380-385): [H][2L-1], read directly by the attention kernel
        tbls = pk.setdefault("bias_tables", {})
        if L not in tbls:
            tbls[L] = pk["rel_emb"][self.buckets(L, dev).long()].t().contiguous()
        bias_tbl = tbls[L]
        scale = (D // H) ** -0.5
        nl = cfg.num_hidden_layers if num_layers is None else num_layers
        qkv = torch.empty(B * L, 3 * D, device=dev, dtype=bf)
        att = torch.empty(B * L, D, device=dev, dtype=bf)
        # the residual sums each post-LayerNorm normalises (x + out_proj(att), x1 + ffn): bf16, like every other
        # activation of the encoder -- half the bytes of the fp32 sums the two GEMM epilogues used to write and the
        # LayerNorms to read back (the statistics are taken in fp32 over the stored values)
        ysum = torch.empty(B * L, D, device=dev, dtype=bf)
        x1 = torch.empty(B * L, D, device=dev, dtype=bf)
        ff = torch.empty(B * L, cfg.intermediate_size, device=dev, dtype=bf)
        ad, acd = (cfg.attention_dropout, cfg.activation_dropout) if tr else (0.0, 0.0)
        rng = ctl.rng if tr else None
        for li in range(nl):
            layer = self.encoder.layers[li]
            lw = pk["layers"][li]
            at = layer.attention
            # LayerDrop (train): every launch of a skipped layer is a no-op, so x passes through unchanged
            sk = dict(skip=ctl.skip, skip_bit=li) if tr else {}
            s_att, s_out, s_act, s_ffn = _layer_sites(li)
            K.gemm_bf16(x, lw["qkv_w"], qkv, bias=lw["qkv_b"], variant=pick, **sk)
            K.wavlm_attention(qkv, x, at.gru_rel_pos_linear.weight, at.gru_rel_pos_linear.bias, lw["gate_c"],
                              bias_tbl, None, att, B, L, H, scale, drop_p=ad, rng=rng, site=s_att, **sk)
            K.gemm_bf16(att, lw["out_w"], ysum, bias=at.out_proj.bias, residual=x, drop_p=hd, rng=rng, site=s_out,
                        variant=pick, **sk)
            K.layernorm(ysum, layer.layer_norm.weight, layer.layer_norm.bias, x1, eps=cfg.layer_norm_eps, **sk)
            K.gemm_bf16(x1, lw["ff1_w"], ff, bias=layer.feed_forward.intermediate_dense.bias, act="gelu",
                        drop_p=acd, rng=rng, site=s_act, variant=pick, **sk)
            K.gemm_bf16(ff, lw["ff2_w"], ysum, bias=layer.feed_forward.output_dense.bias, residual=x1, drop_p=hd,
                        rng=rng, site=s_ffn, variant=pick, **sk)
            last = li == nl - 1
            # train mode writes every layer in place (a skipped last layer must leave x as the output)
            xo = torch.empty(B * L, D, device=dev, dtype=out_dtype) if (last and not tr) else x
            K.layernorm(ysum, layer.final_layer_norm.weight, layer.final_layer_norm.bias, xo, eps=cfg.layer_norm_eps,
                        **sk)
            x = xo
            if capture is not None and li == 0:
                capture["layer0"] = x.view(B, L, D).clone()
        if x.dtype != out_dtype:  # train mode (in-place layers) or an empty stack: the bf16 buffer -> out_dtype
            x = K.bf16_convert(x, torch.empty(B * L, D, device=dev, dtype=out_dtype))
        return x.view(B, L, D)

    # ---- stage-2 fine-tuning: backward through the unfrozen last layers ----
    def first_trainable_layer(self) -> int:
        """Index of the first encoder layer with trainable parameters.  Only a suffix of whole encoder layers
        may train (what ``_unfreeze_last_n_layers`` produces, wavlm_audio.py:70-88); layer 0 owns the shared
        relative-position embedding and the feature extractor / projection / pos-conv stay frozen."""
        layers = self.encoder.layers
        first = next((i for i, l in enumerate(layers) if any(q.requires_grad for q in l.parameters())), None)
        if first is None:
            raise RuntimeError("no trainable WavLM layer")
        outside = [n for n, q in self.named_parameters() if q.requires_grad and not n.startswith("encoder.layers.")]
        if first == 0 or outside or not all(all(q.requires_grad for q in l.parameters()) for l in layers[first:]):
            raise NotImplementedError("WavLM fine-tuning supports unfreezing whole last layers 1..11 "
                                      "(unfreeze_backbone(n), n <= 11); got a different trainable set")
        return first

    def forward_prefix(self, wav: torch.Tensor):
        """The frozen part of a stage-2 forward: conv stack + layers [0, first) -> (bf16 [B, L, D], bias table,
        LayerDrop mask of the forward -- its bits >= first decide the trainable layers).  Independent of the
        trainable weights, so it can run ahead (``FusionModel.prefetch_audio``)."""
        if not wav.is_cuda:
            raise RuntimeError("WavLM runs on the MI355X kernels; move the waveform to the GPU")
        first = self.first_trainable_layer()
        self.__dict__["_pack_limit"] = first  # the trainable layers' stale packs are not re-cast every step
        try:
            with torch.no_grad():
                x = self.forward_hip(wav.contiguous().float(), out_dtype=torch.bfloat16, num_layers=first)
                tbl = self.packed_weights()["bias_tables"][x.shape[1]]
                draw = self.__dict__.get("_last_draw")
        finally:
            self.__dict__["_pack_limit"] = None
        if draw is not None:  # the trainable layers' executions (the prefix counted its own)
            self.executed_layers += sum(1 for i in range(first, len(self.encoder.layers)) if not (draw[1] >> i) & 1)
        return x, tbl, (draw[1] if draw is not None else 0), (draw[0] if draw is not None else None)

    def forward_train(self, wav: torch.Tensor, prefix=None) -> torch.Tensor:
        """Stage-2 forward: frozen conv stack + layers [0, first) on the inference schedule (or ``prefix``, a
        ``forward_prefix`` result computed ahead), then layers [first, 12) saving their activations.  Returns
        fp32 [B, L, 768] tracked by autograd."""
        first = self.first_trainable_layer()
        x, tbl, mask, seed = prefix if prefix is not None else self.forward_prefix(wav)
        names, params = [], []
        for li in range(first, len(self.encoder.layers)):
            for n, q in self.encoder.layers[li].named_parameters():
                names.append((li, n))
                params.append(q)
        return _WavLMTailFn.apply(x, tbl, self, first, (mask, seed), tuple(names), *params)

    def tail_forward(self, x, tbl, first, mask: int = 0, seed: Optional[int] = None):
        """Layers [first, 12) on bf16 x [B, L, D]; returns (fp32 output [B*L, D], saved activations).  Layers
        whose bit is set in the LayerDrop ``mask`` (train mode, TF:417-419) are skipped: no activations are saved
        and their parameters get no gradient (torch Adam then leaves them alone, as in the reference).  ``seed``
        (train mode: the forward's RNG base, the prefix's draw) applies the reference's dropouts inside the layers
        -- attention probabilities, attention output, FFN activation, FFN output (TF:206-228, 286-294, 323), the
        same call sites and masks as the frozen train-mode forward -- and tail_backward regenerates them."""
        cfg = self.config
        B, L, D = x.shape
        H = cfg.num_attention_heads
        M = B * L
        dev = x.device
        bf = torch.bfloat16
        scale = (D // H) ** -0.5
        nl = len(self.encoder.layers)
        h = x.reshape(M, D)
        rng = torch.full((1,), int(seed), dtype=torch.int64, device=dev) if seed is not None else None
        hd, ad, acd = ((cfg.hidden_dropout, cfg.attention_dropout, cfg.activation_dropout) if rng is not None
                       else (0.0, 0.0, 0.0))
        saved = []
        for li in range(first, nl):
            if (mask >> li) & 1:
                saved.append(None)
                continue
            layer = self.encoder.layers[li]
            at = layer.attention
            lw = _pack_layer(layer, dev)
            s_att, s_out, s_act, s_ffn = _layer_sites(li)
            sv = dict(x=h, pack=lw, rng=rng, drop=(hd, ad, acd))
            qkv = torch.empty(M, 3 * D, device=dev, dtype=bf)
            K.gemm_bf16(h, lw["qkv_w"], qkv, bias=lw["qkv_b"])
            att = torch.empty(M, D, device=dev, dtype=bf)
            K.wavlm_attention(qkv, h, at.gru_rel_pos_linear.weight, at.gru_rel_pos_linear.bias, lw["gate_c"], tbl, None,
                              att, B, L, H, scale, drop_p=ad, rng=rng, site=s_att)
            y1 = torch.empty(M, D, device=dev, dtype=torch.float32)
            K.gemm_bf16(att, lw["out_w"], y1, bias=at.out_proj.bias, residual=h, drop_p=hd, rng=rng, site=s_out)
            x1 = torch.empty(M, D, device=dev, dtype=bf)
            K.layernorm(y1, layer.layer_norm.weight, layer.layer_norm.bias, x1, eps=cfg.layer_norm_eps)
            z = torch.empty(M, cfg.intermediate_size, device=dev, dtype=bf)
            K.gemm_bf16(x1, lw["ff1_w"], z, bias=layer.feed_forward.intermediate_dense.bias)
            f = torch.empty_like(z)
            K.gelu_bf16(z, f)
            if acd > 0:  # the frozen forward's act="gelu" GEMM epilogue dropout: same site, index row * FF + col
                K.dropout_rows(f, acd, rng, s_act, y16=f)
            y2 = torch.empty(M, D, device=dev, dtype=torch.float32)
            K.gemm_bf16(f, lw["ff2_w"], y2, bias=layer.feed_forward.output_dense.bias, residual=x1, drop_p=hd, rng=rng,
                        site=s_ffn)
            last = li == nl - 1
            out = torch.empty(M, D, device=dev, dtype=torch.float32 if last else bf)
            K.layernorm(y2, layer.final_layer_norm.weight, layer.final_layer_norm.bias, out, eps=cfg.layer_norm_eps)
            sv.update(qkv=qkv, att=att, y1=y1, x1=x1, z=z, f=f, y2=y2)
            saved.append(sv)
            h = out
        if h.dtype != torch.float32:  # the last layer(s) dropped: the output is the bf16 input of that layer
            h = K.bf16_convert(h.contiguous(), torch.empty(M, D, device=dev, dtype=torch.float32))
        return h, saved

    def tail_backward(self, dout, saved, tbl, first, B, L, grads):
        """Backward of tail_forward given dout fp32 [B*L, D]; accumulates into ``grads`` {param: buffer}."""
        cfg = self.config
        D, H, FF = cfg.hidden_size, cfg.num_attention_heads, cfg.intermediate_size
        M = B * L
        dev = dout.device
        bf, f32 = torch.bfloat16, torch.float32
        eps = cfg.layer_norm_eps
        scale = (D // H) ** -0.5
        addends = (dout.reshape(M, D).contiguous(), None, None)
        for k in range(len(saved) - 1, -1, -1):
            li = first + k
            if saved[k] is None:  # LayerDrop: the layer was the identity
                continue
            sv, layer = saved[k], self.encoder.layers[li]
            cap = self.__dict__.get("_capture_upstream")
            if cap is not None:  # tests: the gradient arriving at this layer's output (sum of the addends)
                cap[li] = tuple(a.detach().clone() if a is not None else None for a in addends)
            at, ff = layer.attention, layer.feed_forward
            lw = sv["pack"]
            g = grads
            rng, (hd, ad, acd) = sv["rng"], sv["drop"]
            s_att, s_out, s_act, s_ffn = _layer_sites(li)
            # final LayerNorm; its sum-of-dx partials are the FFN output bias gradient (residual: dy2 -> x1 too)
            dy2, dy2h = torch.empty(M, D, device=dev, dtype=f32), torch.empty(M, D, device=dev, dtype=bf)
            part = K.ln_bwd(addends[0], sv["y2"], layer.final_layer_norm.weight, eps, dy_b=addends[1],
                            dy_c=addends[2], dx32=dy2, dx16=dy2h)
            K.ln_bwd_fold(part, M, D, g[layer.final_layer_norm.weight], g[layer.final_layer_norm.bias],
                          g[ff.output_dense.bias] if hd == 0 else None)
            gf = dy2h  # gradient of the FFN output branch: the residual keeps dy2, the branch sees its dropout mask
            if hd > 0:
                gf32, gf = torch.empty(M, D, device=dev, dtype=f32), torch.empty(M, D, device=dev, dtype=bf)
                K.dropout_rows(dy2, hd, rng, s_ffn, y32=gf32, y16=gf)
                K.colsum_into(gf32, g[ff.output_dense.bias])
            K.linear_wgrad(sv["f"], gf, g[ff.output_dense.weight])
            df = torch.empty(M, FF, device=dev, dtype=f32)
            K.gemm_bf16(gf, _transposed(lw, "ff2_w", dev), df)
            if acd > 0:
                K.dropout_rows(df, acd, rng, s_act, y32=df)
            dz = torch.empty(M, FF, device=dev, dtype=bf)
            K.gelu_bwd(df, sv["z"], dz, g[ff.intermediate_dense.bias])
            K.linear_wgrad(sv["x1"], dz, g[ff.intermediate_dense.weight])
            dx1 = torch.empty(M, D, device=dev, dtype=f32)
            K.gemm_bf16(dz, _transposed(lw, "ff1_w", dev), dx1)
            # attention LayerNorm (input y1 = x + out_proj(att)); residual gradient dy2 joins here
            dy1, dy1h = torch.empty(M, D, device=dev, dtype=f32), torch.empty(M, D, device=dev, dtype=bf)
            part = K.ln_bwd(dx1, sv["y1"], layer.layer_norm.weight, eps, dy_b=dy2, dx32=dy1, dx16=dy1h)
            K.ln_bwd_fold(part, M, D, g[layer.layer_norm.weight], g[layer.layer_norm.bias],
                          g[at.out_proj.bias] if hd == 0 else None)
            go, goh = dy1, dy1h  # gradient of the attention-output branch (dropout mask in train mode)
            if hd > 0:
                go, goh = torch.empty(M, D, device=dev, dtype=f32), torch.empty(M, D, device=dev, dtype=bf)
                K.dropout_rows(dy1, hd, rng, s_out, y32=go, y16=goh)
                K.colsum_into(go, g[at.out_proj.bias])
            K.linear_wgrad(sv["att"], goh, g[at.out_proj.weight])
            # gradient of the attention output in fp32 from fp32 operands (exact-f32 MFMA GEMM): the softmax
            # backward's dp_ij - sum_j p_ij dp_ij cancels for peaked rows, so bf16 operands here would cost
            # the score-path gradients (q/k/gate) ~10% (tests/test_wavlm_stage2_gpu.py)
            datt = torch.empty(M, D, device=dev, dtype=f32)
            K.gemm(go, at.out_proj.weight.detach(), datt)
            need_dx = k > 0
            dqkv = torch.empty(M, 3 * D, device=dev, dtype=bf)
            dxg = torch.empty(M, D, device=dev, dtype=f32) if need_dx else None
            gpart, nparts = K.wavlm_attention_bwd(sv["qkv"], sv["x"], datt, at.gru_rel_pos_linear.weight,
                                                  at.gru_rel_pos_linear.bias, lw["gate_c"], tbl, B, L, H, scale,
                                                  dqkv, dxg, drop_p=ad, rng=rng, site=s_att)
            ldp = 8 * 64 + 8 + H
            K.fold_rows(gpart, nparts, 8 * 64, ldp, g[at.gru_rel_pos_linear.weight], offset=0)
            K.fold_rows(gpart, nparts, 8, ldp, g[at.gru_rel_pos_linear.bias], offset=8 * 64)
            K.fold_rows(gpart, nparts, H, ldp, g[at.gru_rel_pos_const], offset=8 * 64 + 8)
            cpart = K._workspace(((M + 63) // 64) * 3 * D, dev)
            K.LIB("mer_colpart", M, 3 * D, dqkv.data_ptr(), K.BF16, dqkv.stride(0), cpart.data_ptr(), K.stream_ptr())
            for j, lin in enumerate((at.q_proj, at.k_proj, at.v_proj)):
                K.linear_wgrad(sv["x"], dqkv, g[lin.weight], col0=j * D)
                K.fold_rows(cpart, (M + 63) // 64, D, 3 * D, g[lin.bias], offset=j * D)
            if need_dx:
                dxq = torch.empty(M, D, device=dev, dtype=f32)
                K.gemm_bf16(dqkv, _transposed(lw, "qkv_w", dev), dxq)
                addends = (dxq, dy1, dxg)


def _pack_layer(layer, dev):
    """bf16 operands of one trainable encoder layer (re-cast every forward: the weights move each step)."""
    at = layer.attention
    D = at.q_proj.weight.shape[0]
    qkv = torch.empty(3 * D, D, device=dev, dtype=torch.bfloat16)
    for j, lin in enumerate((at.q_proj, at.k_proj, at.v_proj)):
        K.cast_bf16(lin.weight.detach().contiguous(), qkv[j * D:(j + 1) * D])
    qkv_b = torch.cat([at.q_proj.bias, at.k_proj.bias, at.v_proj.bias]).detach().contiguous()
    return dict(qkv_w=qkv, qkv_b=qkv_b, out_w=WavLMBackbone._bf16(at.out_proj.weight),
                ff1_w=WavLMBackbone._bf16(layer.feed_forward.intermediate_dense.weight),
                ff2_w=WavLMBackbone._bf16(layer.feed_forward.output_dense.weight),
                gate_c=at.gru_rel_pos_const.detach().reshape(-1))


def _transposed(lw, name, dev):
    """W^T (bf16) of a packed weight, built on first use in backward."""
    key = name + "_t"
    if key not in lw:
        w = lw[name]
        lw[key] = torch.empty(w.shape[1], w.shape[0], device=dev, dtype=torch.bfloat16)
        K.transpose_bf16(w, lw[key])
    return lw[key]


class _WavLMTailFn(torch.autograd.Function):
    """Autograd node of the unfrozen WavLM layers (stage 2): forward = tail_forward, backward =
    tail_backward writing each parameter gradient straight into its ``grad_buffer`` slot."""

    @staticmethod
    def forward(ctx, x, tbl, enc, first, draw, names, *params):
        out, saved = enc.tail_forward(x, tbl, first, draw[0], draw[1])
        B, L, D = x.shape
        ctx.enc, ctx.first, ctx.saved, ctx.tbl, ctx.shape = enc, first, saved, tbl, (B, L)
        ctx.params, ctx.names = params, names
        return out.view(B, L, D)

    @staticmethod
    def backward(ctx, dout):
        from .fusion import grad_buffer

        B, L = ctx.shape
        ran = {ctx.first + k for k, sv in enumerate(ctx.saved) if sv is not None}
        grads = {q: grad_buffer(q) for (li, _), q in zip(ctx.names, ctx.params) if li in ran}
        ctx.enc.tail_backward(dout.float().contiguous(), ctx.saved, ctx.tbl, ctx.first, B, L, grads)
        ctx.saved = None
        return (None, None, None, None, None, None) + tuple(
            grads[q] if (q.requires_grad and q in grads) else None for q in ctx.params)


class WavLMAudioEncoder(nn.Module):
    """wavlm_audio.py:13-183 -- same constructor, stage helpers and encode API."""

    def __init__(self, num_classes: int, embedding_dim: int = 768, model_name: str = "microsoft/wavlm-base",
                 temporal_pooling: str = "mean", temporal_num_heads: int = 4, temporal_num_layers: int = 1,
                 temporal_dropout: float = 0.1):
        super().__init__()
        self.num_classes = num_classes
        self.embedding_dim = embedding_dim
        self.model_name = model_name
        # offline build of the WavLM-base architecture (the reference's own fallback, wavlm_audio.py:35-41)
        self.wavlm = WavLMBackbone()
        actual_hidden_size = self.wavlm.config.hidden_size
        self.sequence_dim = actual_hidden_size
        self.temporal_pool = TemporalPooler(actual_hidden_size, temporal_pooling, temporal_num_heads,
                                            temporal_num_layers, temporal_dropout)
        self.classifier = nn.Sequential(nn.Linear(actual_hidden_size, embedding_dim), nn.ReLU(inplace=True),
                                        nn.Dropout(0.2), nn.Linear(embedding_dim, num_classes))
        self._freeze_backbone()

    def _freeze_backbone(self):
        for param in self.wavlm.parameters():
            param.requires_grad = False

    def _unfreeze_last_n_layers(self, n: int = 2):
        if n == 0:
            return
        num_layers = len(self.wavlm.encoder.layers)
        for i in range(max(0, num_layers - n), num_layers):
            for param in self.wavlm.encoder.layers[i].parameters():
                param.requires_grad = True

    def unfreeze_backbone(self, num_last_layers: int = 2):
        self._unfreeze_last_n_layers(num_last_layers)

    def get_stage1_params(self):
        return list(self.classifier.parameters())

    def get_stage2_params(self):
        backbone, head = [], []
        for name, param in self.named_parameters():
            if param.requires_grad:
                (head if ("classifier" in name or "head" in name) else backbone).append(param)
        return {"backbone": backbone, "head": head}

    def _wav(self, x):
        return x.squeeze(1) if x.dim() == 3 else x

    def encode_sequence(self, x: torch.Tensor, out_dtype=torch.bfloat16, prefix=None) -> torch.Tensor:
        """[B,1,S] or [B,S] -> [B, Ta, 768] hidden states (bf16 activations; wavlm_audio.py:165-183)."""
        if self.wavlm.trainable() and torch.is_grad_enabled():
            # stage 2 (wavlm_audio.py:70-88 unfreeze_backbone): frozen prefix forward, then the unfrozen last
            # layers as one autograd node whose backward runs csrc/wavlm_train.hip; fp32 output so the
            # head's audio-input gradient arrives in the dtype the node produced
            return self.wavlm.forward_train(self._wav(x), prefix=prefix)
        if prefix is not None:
            raise RuntimeError("a frozen-prefix result is only consumed by a stage-2 (trainable tail) forward")
        return self.wavlm.forward_hip(self._wav(x), out_dtype=out_dtype)

    def encode_prefix(self, x: torch.Tensor):
        """The frozen part of a stage-2 ``encode_sequence`` (prefetchable; see WavLMBackbone.forward_prefix)."""
        return self.wavlm.forward_prefix(self._wav(x))

    def encode(self, x: torch.Tensor, hidden: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``hidden``: this clip batch's ``encode_sequence(x, fp32)`` computed ahead (FusionModel.prefetch_audio)."""
        hidden = self.encode_sequence(x, out_dtype=torch.float32) if hidden is None else hidden
        a_emb = self.temporal_pool(hidden)
        if a_emb.size(-1) != self.embedding_dim:
            a_emb = hip_linear(a_emb, self.classifier[0])
        return a_emb

    def draw_dropout_seed(self) -> Optional[int]:
        """The classifier dropout's host seed drawn ahead of ``forward`` (None when the dropout is off): the late
        fusion's early prefetch draws it before starting the next batch's encoder, keeping the inline RNG order."""
        return draw_seed(float(self.classifier[2].p), self.training)

    def forward(self, x: torch.Tensor, hidden: Optional[torch.Tensor] = None,
                drop_seed: Optional[int] = None) -> torch.Tensor:
        hidden = self.encode_sequence(x, out_dtype=torch.float32) if hidden is None else hidden
        a_emb = self.temporal_pool(hidden)
        h = hip_linear(a_emb, self.classifier[0], act="relu")
        # the nn.Dropout(0.2) of wavlm_audio.py:58
        h = hip_dropout(h, float(self.classifier[2].p), self.training, seed=drop_seed)
        return hip_linear(h, self.classifier[3])
