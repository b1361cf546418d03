"""Clip assembly on the MI355X (first step): the arithmetic of ``src/data/ravdess.py``'s
``load_video_frames`` after decode and ``load_audio_wav`` after ``librosa.load``, run on the device so only
decoded uint8 frames / raw waveforms cross PCIe and the batch is assembled in HBM.

* ``preprocess_frames`` -- decoded RGB uint8 frames ``[N, H, W, 3]`` -> ``[N, 3, size, size]`` fp32:
  ``cv2.resize(..., INTER_LINEAR)`` (ravdess.py:352), ``/ 255`` (:363), ImageNet normalisation (:386-389).
* ``video_clip_batch`` -- ``B`` clips of ``T`` such frames -> the model's ``[B, T, 3, size, size]`` input.
* ``pad_crop_waveforms`` -- a ragged list of mono waveforms -> ``[B, 1, sample_rate * duration]``
  (ravdess.py:505-513).

Decoding (cv2.VideoCapture / librosa), face detection / crop and the augmentations stay on the host
(DESIGN.md section 7).  Kernels: ``csrc/clips.hip``; CPU restatement: ``oracle/clips_ref.py``.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from . import kernels as K

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess_frames(frames: torch.Tensor, size: int = 112) -> torch.Tensor:
    """``[N, H, W, 3]`` uint8 RGB on the GPU -> ``[N, 3, size, size]`` fp32, normalised."""
    if not frames.is_cuda:
        raise RuntimeError("preprocess_frames runs on the MI355X kernels; move the frames to the GPU")
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError("frames must be uint8 [N, H, W, 3] (RGB)")
    frames = frames.contiguous()
    N, H, W, _ = frames.shape
    out = torch.empty(N, 3, size, size, device=frames.device, dtype=torch.float32)
    K.LIB("mer_frames_resize_normalize", N, H, W, frames.data_ptr(), H * W * 3, size, *IMAGENET_MEAN, *IMAGENET_STD,
          out.data_ptr(), K.stream_ptr())
    return out


def video_clip_batch(frames: torch.Tensor, size: int = 112) -> torch.Tensor:
    """``[B, T, H, W, 3]`` uint8 -> ``[B, T, 3, size, size]`` fp32 (the FusionModel video input)."""
    B, T = frames.shape[:2]
    return preprocess_frames(frames.reshape(B * T, *frames.shape[2:]), size).view(B, T, 3, size, size)


def _h2d(t: torch.Tensor, dev) -> torch.Tensor:
    """Asynchronous host-to-device copy from a PINNED staging copy: the caching host allocator keeps the pinned
    block alive until the copy has executed.  (An asynchronous copy straight from a pageable temporary may still be
    in flight when the temporary is freed and its memory reused -- the device then reads whatever is there.)"""
    return t.pin_memory().to(dev, non_blocking=True)


def pad_crop_waveforms(wavs: Sequence[torch.Tensor], sample_rate: int = 16000, duration_sec: float = 3.0,
                       device=None) -> torch.Tensor:
    """Ragged mono waveforms (1-D fp32, host or device) -> ``[B, 1, target]`` on the GPU, zero-padded at the end or
    cropped to ``target = int(sample_rate * duration_sec)`` (ravdess.py:505-513)."""
    if not wavs:
        raise ValueError("empty waveform batch")
    target = int(sample_rate * duration_sec)
    dev = torch.device(device) if device is not None else next((w.device for w in wavs if w.is_cuda), None)
    if dev is None or dev.type != "cuda":
        raise RuntimeError("pad_crop_waveforms assembles the batch on the MI355X; pass device='cuda'")
    flat: List[torch.Tensor] = [w.reshape(-1).to(torch.float32) for w in wavs]
    lengths = [int(w.numel()) for w in flat]
    offsets = [0]
    for n in lengths[:-1]:
        offsets.append(offsets[-1] + n)
    if not sum(lengths):
        packed = torch.zeros(1, device=dev)
    elif all(not w.is_cuda for w in flat):  # decoded on the host: one contiguous PINNED host buffer, one H2D copy
        packed = _h2d(torch.cat(flat), dev)
    else:
        packed = torch.cat([w.to(dev) if w.is_cuda else _h2d(w, dev) for w in flat])
    meta = _h2d(torch.tensor([offsets, lengths], dtype=torch.int64), dev)
    out = torch.empty(len(flat), 1, target, device=dev, dtype=torch.float32)
    K.LIB("mer_wav_pad_crop", len(flat), target, packed.data_ptr(), meta[0].data_ptr(), meta[1].data_ptr(),
          out.data_ptr(), K.stream_ptr())
    return out
