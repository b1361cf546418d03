"""Batch-inference runtime mirroring ``src/optimized_runtime.py`` (TorchModelRunner) and the tensor path
of ``src/inference_worker.py:_process_batch`` (stack -> predict_probs -> per-row top-1).

Checkpoints use the reference's format ``{"model": state_dict, "val_f1", "config"}`` and its state-dict
key names, so a checkpoint written by the reference's train.py loads unchanged.  Loading is
``torch.load(weights_only=True)`` (tensors + plain containers only).
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Dict, List, Optional

import torch
from .train import build_model

FOUR_CLASS_LABELS = ["neutral_calm", "happy", "negative", "surprised"]
EIGHT_CLASS_LABELS = ["neutral", "calm", "happy", "sad", "angry", "fearful", "disgust", "surprised"]
FUSION_MODES = {"audio", "video", "late", "concat", "gated", "xattn", "xattn_concat", "xattn_gated"}


def labels_for_num_classes(num_classes: int) -> List[str]:
    return EIGHT_CLASS_LABELS if num_classes == 8 else FOUR_CLASS_LABELS


# (state-dict prefix that must be present, fusion mode, xattn head) in the precedence order of
# optimized_runtime.py:22-37; fusion checkpoints carry both encoders, single-encoder ones one of them.
_FUSION_SIGNATURES = (("xattn_gate.", "xattn", "gated"), ("xattn_mlp.", "xattn", "concat"),
                      ("fusion.", "concat", "concat"), ("gate.", "gated", "gated"))
_SINGLE_SIGNATURES = ((("encoder.", "wavlm."), "audio"), (("backbone.",), "video"))
# config key -> build_model keyword default (the runner reads these from checkpoint["config"])
_CONFIG_DEFAULTS = dict(
    xattn_d_model=128, xattn_heads=4, xattn_attn_dropout=0.1, xattn_stochastic_depth=0.1,
    xattn_use_emotion_prior=False, xattn_emotion_prior_dim=8, xattn_emotion_prior_hidden_dim=64,
    xattn_emotion_prior_dropout=0.1, temporal_pooling="mean", temporal_num_heads=4, temporal_num_layers=1,
    temporal_dropout=0.1, audio_n_mels=64, use_resnet_audio=True, fusion_align_mode="none", fusion_align_dim=256,
    fusion_align_temperature=0.07)


def _has_prefix(keys, *prefixes) -> bool:
    return any(k.startswith(prefixes) for k in keys)


def infer_model_signature(state_dict: Dict[str, torch.Tensor]):
    """(fusion mode, xattn head) from the checkpoint's key prefixes -- optimized_runtime.py:22-37."""
    keys = list(state_dict)
    if _has_prefix(keys, "audio_model.") and _has_prefix(keys, "video_model."):
        for prefix, mode, head in _FUSION_SIGNATURES:
            if _has_prefix(keys, prefix):
                return mode, head
        return "late", "concat"
    for prefixes, mode in _SINGLE_SIGNATURES:
        if _has_prefix(keys, *prefixes):
            return mode, "concat"
    raise RuntimeError("Unable to infer model type from checkpoint state_dict keys.")


def checkpoint_uses_wavlm(state_dict: Dict[str, torch.Tensor]) -> bool:
    """optimized_runtime.py:40-41."""
    return _has_prefix(list(state_dict), "audio_model.wavlm.", "wavlm.")


class TorchModelRunner:
    """optimized_runtime.py:44-108 on the MI355X kernels.

    ``enable_dynamic_quant`` selects the INT8 linear path (per-tensor symmetric int8 weights, dynamic
    per-row int8 activations, int32 MFMA accumulation) that mirrors ``quantize_dynamic({nn.Linear})``;
    in the reference it is CPU-only (optimized_runtime.py:95-96), here it runs on the GPU.
    """

    def __init__(self, checkpoint_path: Optional[str] = None, device: str = "cuda", fallback_fusion: str = "xattn",
                 enable_dynamic_quant: bool = False, checkpoint: Optional[Dict[str, Any]] = None):
        self.device = torch.device(device)
        if checkpoint is None:
            checkpoint = torch.load(Path(checkpoint_path).expanduser(), map_location="cpu", weights_only=True)
        if not isinstance(checkpoint, dict) or "model" not in checkpoint:
            raise RuntimeError("Checkpoint format not supported. Expected {'model': state_dict, 'config': ...}.")
        self.config = checkpoint.get("config", {}) or {}
        state_dict = checkpoint["model"]
        if "fusion" in self.config:
            self.fusion_mode = str(self.config.get("fusion", fallback_fusion))
            xattn_head = str(self.config.get("xattn_head", "concat"))
        else:
            self.fusion_mode, xattn_head = infer_model_signature(state_dict)
        if self.fusion_mode not in FUSION_MODES:
            raise ValueError(f"Unsupported fusion mode: {self.fusion_mode}")
        self.num_classes = int(self.config.get("num_classes", 8))
        self.use_wavlm = bool(self.config.get("use_wavlm", checkpoint_uses_wavlm(state_dict)))
        self.labels = labels_for_num_classes(self.num_classes)
        kw = {k: self.config.get(k, d) for k, d in _CONFIG_DEFAULTS.items()}
        model = build_model(num_classes=self.num_classes, fusion=self.fusion_mode, pretrained_video=False,
                            xattn_head=xattn_head, use_wavlm=self.use_wavlm, **kw)
        missing, unexpected = model.load_state_dict(state_dict, strict=False)
        if unexpected:
            raise RuntimeError(f"Unexpected checkpoint keys ({len(unexpected)}): {unexpected[:8]}")
        if len(missing) > 32:
            raise RuntimeError(f"Too many missing keys when loading checkpoint ({len(missing)}). "
                               "Checkpoint architecture does not match the inferred runtime model.")
        self.model = model.to(self.device).eval()
        self.int8 = bool(enable_dynamic_quant)
        if self.int8:
            from .int8 import quantize_dynamic_hip
            quantize_dynamic_hip(self.model)

    def predict_probs(self, videos: torch.Tensor, audios: torch.Tensor) -> torch.Tensor:
        """optimized_runtime.py:99-108: softmax probabilities (late mode already returns probabilities)."""
        with torch.inference_mode():
            videos = videos.to(self.device, non_blocking=True)
            audios = audios.to(self.device, non_blocking=True)
            if self.fusion_mode == "audio":
                outputs = self.model(audios)
            elif self.fusion_mode == "video":
                outputs = self.model(videos)
            else:
                outputs = self.model(videos, audios)
            probs = outputs if self.fusion_mode == "late" else _softmax(outputs)
        return probs.detach().cpu()


def _softmax(x: torch.Tensor) -> torch.Tensor:
    from . import kernels as K

    x = x.contiguous().float()
    out = torch.empty_like(x)
    pa = torch.empty_like(x)
    K.softmax_avg_fwd(x, x, out, pa, torch.empty_like(x))  # (softmax + softmax) / 2 == softmax
    return out


def process_batch(runner: TorchModelRunner, videos: List[torch.Tensor], audios: List[torch.Tensor]):
    """Tensor path of inference_worker.py:_process_batch (131-147): stack, predict, per-row top-1."""
    v = torch.stack(videos, dim=0)
    a = torch.stack(audios, dim=0)
    probs = runner.predict_probs(v, a)
    out = []
    for row in probs:
        top = int(row.argmax().item())
        out.append({"labels": runner.labels, "probs": [round(float(p), 6) for p in row.tolist()],
                    "top1": {"label": runner.labels[top], "prob": round(float(row[top].item()), 6)}})
    return out
