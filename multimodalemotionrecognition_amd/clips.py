"""Clip assembly on the MI355X (first step): the arithmetic of ``src/data/ravdess.py``'s
``load_video_frames`` after decode and ``load_audio_wav`` after ``librosa.load``, run on the device so only
decoded uint8 frames / raw waveforms cross PCIe and the batch is assembled in HBM.

* ``preprocess_frames`` -- decoded RGB uint8 frames ``[N, H, W, 3]`` -> ``[N, 3, size, size]`` fp32:
  ``cv2.resize(..., INTER_LINEAR)`` (ravdess.py:352), ``/ 255`` (:363), ImageNet normalisation (:386-389).
* ``video_clip_batch`` -- ``B`` clips of ``T`` such frames -> the model's ``[B, T, 3, size, size]`` input.
* ``augment_clips`` -- the train-split video augmentation (ravdess.py:366-384: uint8 round trip,
  ``cv2.GaussianBlur(k, 0)``, darken, Gaussian noise, clip) + normalisation of ``B`` clips, per-clip draws from
  ``draw_video_augment``.
* ``pad_crop_waveforms`` -- a ragged list of mono waveforms -> ``[B, 1, sample_rate * duration]``
  (ravdess.py:505-513).

Decoding (cv2.VideoCapture / librosa), face detection / crop and the audio augmentation stay on the host
(DESIGN.md section 4c).  Kernels: ``csrc/clips.hip``; CPU restatement: ``oracle/clips_ref.py``.
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


NORMAL_TABLE_BITS = 16


def normal_table() -> torch.Tensor:
    """fp32 [65536]: the standard normal inverse CDF at (i + 0.5) / 65536 (float64, then rounded) -- the
    augmentation noise draws z = table[hash >> 16] (a 16-bit-resolution Gaussian, |z| <= 4.17)."""
    n = 1 << NORMAL_TABLE_BITS
    u = (torch.arange(n, dtype=torch.float64) + 0.5) / n
    return torch.special.ndtri(u).to(torch.float32)


_ZTABLES = {}


def _ztable(dev) -> torch.Tensor:
    t = _ZTABLES.get(dev)
    if t is None:
        t = _ZTABLES[dev] = normal_table().to(dev)
    return t


def draw_video_augment(rng) -> tuple:
    """One clip's draws of ravdess.py:368-372 from a numpy Generator, in the reference's order: brightness factor
    U(0.2, 0.6), noise scale U(0, 5e-4), blur ksize from {3, 5, 7} -- plus the 63-bit seed of the clip's noise."""
    factor = float(rng.uniform(0.2, 0.6))
    noise_scale = float(rng.uniform(0.0, 0.0005))
    ksize = int(rng.choice([3, 5, 7]))
    if ksize % 2 == 0:
        ksize += 1
    return factor, noise_scale, ksize, int(rng.integers(0, 2 ** 63 - 1))


def resize_frames_u8(frames: torch.Tensor, size: int = 112, out: torch.Tensor = None) -> torch.Tensor:
    """``[N, H, W, 3]`` uint8 on the GPU -> ``[N, size, size, 3]`` uint8 (cv2.resize INTER_LINEAR, ravdess.py:352)."""
    if not frames.is_cuda or frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError("frames must be uint8 [N, H, W, 3] (RGB) on the GPU")
    frames = frames.contiguous()
    N, H, W, _ = frames.shape
    if out is None:
        out = torch.empty(N, size, size, 3, device=frames.device, dtype=torch.uint8)
    K.LIB("mer_frames_resize_u8", N, H, W, frames.data_ptr(), H * W * 3, size, out.data_ptr(), K.stream_ptr())
    return out


def augment_clips(frames_u8: torch.Tensor, params: Sequence[tuple]) -> torch.Tensor:
    """Resized clips ``[B, T, S, S, 3]`` uint8 on the GPU + one ``draw_video_augment`` tuple per clip ->
    ``[B, T, 3, S, S]`` fp32: the augmentation of ravdess.py:366-384 then the ImageNet normalisation (:386-389)."""
    if not frames_u8.is_cuda:
        raise RuntimeError("augment_clips runs on the MI355X kernels; move the frames to the GPU")
    if frames_u8.dtype != torch.uint8 or frames_u8.dim() != 5 or frames_u8.shape[-1] != 3 \
            or frames_u8.shape[2] != frames_u8.shape[3]:
        raise ValueError("frames must be uint8 [B, T, S, S, 3]")
    B, T, S = frames_u8.shape[:3]
    if len(params) != B:
        raise ValueError(f"{len(params)} augmentation draws for {B} clips")
    for _, _, k, _ in params:
        if k not in (1, 3, 5, 7):
            raise ValueError(f"blur ksize {k}: the device blur implements cv2's sigma-0 kernels of size <= 7")
    dev = frames_u8.device
    fp = _h2d(torch.tensor([[f, n, float(k)] for f, n, k, _ in params], dtype=torch.float32), dev)
    seeds = _h2d(torch.tensor([sd for _, _, _, sd in params], dtype=torch.int64), dev)
    out = torch.empty(B, T, 3, S, S, device=dev, dtype=torch.float32)
    K.LIB("mer_frames_augment_normalize", B * T, S, T, frames_u8.contiguous().data_ptr(), fp.data_ptr(),
          seeds.data_ptr(), _ztable(dev).data_ptr(), *IMAGENET_MEAN, *IMAGENET_STD, out.data_ptr(), K.stream_ptr())
    return out


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
