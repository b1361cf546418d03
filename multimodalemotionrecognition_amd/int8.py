"""Dynamic INT8 Linear layers for inference -- ``TorchModelRunner(enable_dynamic_quant=True)``.

The reference (optimized_runtime.py:95-96) applies ``torch.quantization.quantize_dynamic(model,
{nn.Linear}, qint8)`` on CPU only; here the same arithmetic (int8 weights, per-call per-tensor int8
activations, int32 accumulation, fp32 dequant -- oracle/int8_ref.py) runs on ``v_mfma_i32_16x16x64_i8``.

Which Linears are quantized follows the reference's exact-type rule: every plain ``nn.Linear`` of the
fusion head (``nn.MultiheadAttention.out_proj`` is a ``NonDynamicallyQuantizableLinear`` and stays fp32).
The WavLM encoder stays bf16: the reference's quantize_dynamic crashes on it (its attention reads
``q_proj.weight`` as a tensor, TF:213,225-227), so no reference INT8 WavLM exists to match.
"""
from __future__ import annotations

from typing import Dict

import torch
from torch import nn

from . import kernels as K


class QuantizedLinear:
    """Device-resident int8 image of one ``nn.Linear`` (weights quantized once, at conversion)."""

    def __init__(self, lin: nn.Linear):
        w = lin.weight.detach().float().contiguous()
        if not w.is_cuda:
            raise RuntimeError("quantize on the device: move the model to 'cuda' first")
        N, Kd = w.shape
        dev = w.device
        self.in_features, self.out_features = Kd, N
        # K padded to the i8 MFMA's multiple of 16 with zero weights; callers with in_features % 16 != 0 pass
        # zero-padded input rows of width in_padded (the emotion-prior token-bias Linears, K = 136)
        self.in_padded = (Kd + 15) // 16 * 16
        self.wqp = torch.empty(4, device=dev)
        self.qw = torch.empty(N, self.in_padded, device=dev, dtype=torch.int8)
        self.colsum = torch.empty(N, device=dev, dtype=torch.int32)
        self._part = torch.empty(K.QP_PARTIAL, device=dev)
        self.xqp = torch.empty(4, device=dev)
        K.quant_params(w, self._part, self.wqp, mode=1)
        K.quantize_weight_s8(w, self.wqp, self.qw, self.colsum)
        self.bias = None if lin.bias is None else lin.bias.detach().float().contiguous()

    def __call__(self, x2d: torch.Tensor, out: torch.Tensor, act: str = "none") -> torch.Tensor:
        x2d = x2d.contiguous()
        if x2d.shape[1] != self.in_padded:
            raise ValueError(f"INT8 Linear expects rows of {self.in_padded} (zero-padded) features, got {x2d.shape[1]}")
        K.quant_params(x2d, self._part, self.xqp, mode=0)
        return K.gemm_i8dyn(x2d, self.xqp, self.qw, self.wqp, self.colsum, self.bias, out, act=act)

    def weight_scale(self) -> float:
        return float(self.wqp[0].item())


def quantizable_linears(model: nn.Module) -> Dict[str, nn.Linear]:
    """Plain nn.Linear modules of the fusion head (exact type, as quantize_dynamic matches them)."""
    return {n: m for n, m in model.named_modules()
            if type(m) is nn.Linear and not n.startswith(("audio_model.", "video_model."))}


def quantize_dynamic_hip(model: nn.Module) -> Dict[str, QuantizedLinear]:
    """Attach int8 images of the head's Linears to ``model`` (``model._mer_int8``); returns them.  With the
    emotion-prior adapter this includes ``prior_net.0/3`` and the four token-bias Linears (their concatenated
    [token; prior] input is quantized as one tensor, as quantize_dynamic does)."""
    q = {n: QuantizedLinear(m) for n, m in quantizable_linears(model).items()}
    model._mer_int8 = q
    return q
