"""CPU restatement of the reference's dynamic INT8 ``nn.Linear`` (optimized_runtime.py:95-96:
``torch.quantization.quantize_dynamic(model, {nn.Linear}, dtype=torch.qint8)`` on the x86/fbgemm engine).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

The algorithm lives in PyTorch's quantization stack (torch 2.10 here, fbgemm backend), not in the
reference tree; restated from its published behaviour and pinned bit-exactly against
``torch.ao.quantization.quantize_dynamic`` on this image (tools/gen_golden.py ``int8_head_b64`` and
tests/test_oracle_golden.py):

* weight: per-tensor symmetric qint8 (``MinMaxObserver(qint8, per_tensor_symmetric)``):
  ``ws = max(amax(|W|) / 127.5, eps_f32)`` in fp32, ``qw = clamp(rint(W * (1/ws)), -128, 127)``;
* activation, per call: per-TENSOR min/max over the whole (flattened) input, fbgemm
  ``ChooseQuantizationParams(min, max, 0, 255, reduce_range=True)`` -> qmin 0, qmax 127, zero point
  nudged to an integer, ``qx = clamp(rint(fma(x, 1/xs, zp)), 0, 255)`` (the AVX2 fmadd+round path);
* int32 accumulation ``acc = sum_k qx*qw - zp * sum_k qw``;
* output ``y = fma(float(acc), float(xs*ws), bias)`` in fp32.
"""
from __future__ import annotations

from typing import Dict, Iterable

import numpy as np
import torch

_SMALL_SCALE = 6.1e-5
_F32_EPS = np.float32(np.finfo(np.float32).eps)


def choose_qparams(xmin: float, xmax: float, qmin: int = 0, qmax: int = 127):
    """fbgemm ChooseQuantizationParams (preserve_sparsity=False, no power-of-two scale)."""
    xmin = min(float(np.float32(xmin)), 0.0)
    xmax = max(float(np.float32(xmax)), 0.0)
    scale = (xmax - xmin) / (qmax - qmin)
    if np.float32(scale) == 0 or np.isinf(np.float32(1.0) / np.float32(scale)):
        scale = 0.1
    if scale < _SMALL_SCALE:
        org = scale
        scale = _SMALL_SCALE
        if xmin == 0.0:
            xmax = _SMALL_SCALE * (qmax - qmin)
        elif xmax == 0.0:
            xmin = -_SMALL_SCALE * (qmax - qmin)
        else:
            amp = float(np.float32(_SMALL_SCALE / org))
            xmin, xmax = xmin * amp, xmax * amp
    z_from_min = qmin - xmin / scale
    z_from_max = qmax - xmax / scale
    e_min = abs(qmin) - abs(xmin / scale)
    e_max = abs(qmax) - abs(xmax / scale)
    z0 = z_from_min if e_min < e_max else z_from_max
    if z0 < qmin:
        zp = qmin
    elif z0 > qmax:
        zp = qmax
    else:
        zp = int(np.rint(z0))
    return np.float32(scale), zp


def quantize_weight(w: np.ndarray):
    w = np.asarray(w, dtype=np.float32)
    amax = np.float32(max(-float(w.min()), float(w.max()), 0.0))
    ws = np.float32(amax / np.float32(127.5))
    ws = max(ws, _F32_EPS)
    qw = np.clip(np.rint(w * (np.float32(1.0) / ws)), -128, 127).astype(np.int8)
    return qw, np.float32(ws)


def quantize_activation(x: np.ndarray):
    x = np.asarray(x, dtype=np.float32)
    xs, zp = choose_qparams(float(x.min()), float(x.max()))
    inv = np.float64(np.float32(1.0) / xs)
    t = (x.astype(np.float64) * inv + zp).astype(np.float32)  # single-rounding fma
    return np.clip(np.rint(t), 0, 255).astype(np.int64), xs, zp


def int8_linear(x: np.ndarray, qw: np.ndarray, ws: np.float32, bias: np.ndarray) -> np.ndarray:
    """Dynamic-quant Linear on [..., K] input; returns fp32 [..., N]."""
    lead = x.shape[:-1]
    x2 = np.asarray(x, dtype=np.float32).reshape(-1, x.shape[-1])
    qx, xs, zp = quantize_activation(x2)
    qw64 = qw.astype(np.int64)
    acc = qx @ qw64.T - zp * qw64.sum(1)[None, :]
    s = np.float64(np.float32(xs * ws))
    b = np.zeros(qw.shape[0]) if bias is None else np.asarray(bias, dtype=np.float32).astype(np.float64)
    y = (acc.astype(np.float32).astype(np.float64) * s + b[None, :]).astype(np.float32)
    return y.reshape(*lead, qw.shape[0])


def quantize_params(p: Dict[str, torch.Tensor], names: Iterable[str]) -> Dict[str, torch.Tensor]:
    """Copy of ``p`` whose listed Linears carry ``<name>._qweight`` / ``<name>._wscale``; the oracle's
    ``fusion_ref.linear`` then routes them through :func:`int8_linear`."""
    q = dict(p)
    for n in names:
        qw, ws = quantize_weight(p[n + ".weight"].detach().cpu().numpy())
        q[n + "._qweight"] = torch.from_numpy(qw)
        q[n + "._wscale"] = torch.tensor(float(ws), dtype=torch.float32)
    return q


def linear_int8_torch(x: torch.Tensor, p: Dict[str, torch.Tensor], name: str) -> torch.Tensor:
    b = p.get(name + ".bias")
    y = int8_linear(x.detach().cpu().numpy(), p[name + "._qweight"].numpy(), np.float32(p[name + "._wscale"].item()),
                    None if b is None else b.detach().cpu().numpy())
    return torch.from_numpy(y)


# Linears the reference's quantize_dynamic converts in each head (exact-type match on nn.Linear:
# the MHA out_proj is a NonDynamicallyQuantizableLinear and stays fp32).
XATTN_INT8 = {"concat": ("v_in_proj", "audio_seq_proj", "a_in_proj", "xattn_mlp.0", "xattn_mlp.3"),
              "gated": ("v_in_proj", "audio_seq_proj", "a_in_proj", "xattn_gate.0", "xattn_gate.3", "xattn_classifier")}
EMB_INT8 = {"concat": ("audio_proj", "video_proj", "fusion.0", "fusion.3"),
            "gated": ("audio_proj", "video_proj", "gate.0", "gate.3", "classifier")}

# With the emotion-prior adapter (fusion.py:153-184) quantize_dynamic also converts prior_net.0/3 and the four
# token-bias Linear(d + prior_dim, 1) (their input is the concatenated [token; prior] row tensor).
PRIOR_INT8 = tuple("emotion_prior_bias." + n for n in ("prior_net.0", "prior_net.3", "v_query_bias", "a_key_bias",
                                                        "a_query_bias", "v_key_bias"))
