"""CPU restatement of the reference's clip preprocessing after decode (numpy, integer arithmetic where the
reference is integer).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

* ``resize_linear_u8`` -- ``cv2.resize(frame, (size, size), interpolation=cv2.INTER_LINEAR)`` on an RGB uint8
  frame (``src/data/ravdess.py:352``), restated from OpenCV's published scalar fixed-point path
  (``modules/imgproc/src/resize.cpp``: coefficient tables with INTER_RESIZE_COEF_BITS = 11, horizontal pass
  into int, vertical pass with ``FixedPtCast<int, uchar, 22>``; an exact 2x downscale switches to the
  INTER_AREA 2x2 average).  opencv-python is not installed here (cv2 import fails), so this is
  **parity unpinned** against cv2 itself: OpenCV's SIMD vertical pass rounds intermediates differently and
  can differ from its scalar path by 1 LSB on some pixels.
* ``normalize_frames`` -- ``/255`` then ImageNet ``(x - mean) / std`` and HWC -> CHW
  (``ravdess.py:363,386-389``), float32 like the reference's numpy code.
* ``augment_clip`` -- the train-split video augmentation (``ravdess.py:366-384``) given the clip's draws:
  ``(frames * 255).astype(uint8)``, ``cv2.GaussianBlur(img, (k, k), 0)``, ``/ 255``, ``* factor``, ``+ noise``,
  ``clip(0, 1)``.  The blur is restated from OpenCV's published 8U path (``modules/imgproc/src/smooth.dispatch.cpp``
  ``getGaussianKernelBitExact``: for sigma <= 0 and ksize 3 / 5 / 7 the fixed table {1,2,1}/4, {1,4,6,4,1}/16,
  {2,7,14,18,14,7,2}/64 -- NOT the sigma = 0.3((k-1)/2 - 1) + 0.8 formula, which applies to larger kernels; the
  fixed-point separable filter is exact for these weights and its uint8 cast rounds half up; BORDER_REFLECT_101).
  cv2 is not installed: **parity against cv2 itself is unpinned**.  The noise is this build's own draw
  (``np.random.normal`` on the reference's unseeded global RNG cannot be reproduced by anyone): z from a
  65,536-entry inverse-normal table indexed by the high 16 bits of ``mer_hash(clip seed, element)``, restated below
  bit for bit.
* ``pad_crop_wav`` -- zero-pad or crop to ``sample_rate * duration`` samples (``ravdess.py:505-513``).
"""
from __future__ import annotations

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS
MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def _coeffs(src: int, dst: int):
    """Per destination index: (source index, weight0, weight1, single-tap flag) of OpenCV's linear table."""
    scale = 1.0 / (float(dst) / float(src))  # cv::resize: scale_x = 1 / inv_scale_x
    ofs = np.empty(dst, np.int64)
    a0 = np.empty(dst, np.int64)
    a1 = np.empty(dst, np.int64)
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0.0), 0
        if s >= src - 1:
            f, s = np.float32(0.0), src - 1
        c0 = np.float32(np.float32(1.0) - f) * np.float32(COEF_SCALE)
        c1 = f * np.float32(COEF_SCALE)
        ofs[d] = s
        a0[d] = int(np.rint(c0))
        a1[d] = int(np.rint(c1))
    return ofs, a0, a1


def resize_linear_u8(frame: np.ndarray, size: int) -> np.ndarray:
    """[H, W, C] uint8 -> [size, size, C] uint8, cv2.INTER_LINEAR semantics (scalar fixed-point path)."""
    H, W, C = frame.shape
    src = frame.astype(np.int64)
    if H == 2 * size and W == 2 * size:  # exact 2x: INTER_AREA fast path, (sum of 2x2 + 2) >> 2
        s = src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    xo, xa0, xa1 = _coeffs(W, size)
    yo, yb0, yb1 = _coeffs(H, size)
    x1 = np.minimum(xo + 1, W - 1)
    # horizontal pass on every needed source row
    hor = src[:, xo, :] * xa0[None, :, None] + src[:, x1, :] * xa1[None, :, None]  # [H, size, C]
    y1 = np.minimum(yo + 1, H - 1)
    v = hor[yo] * yb0[:, None, None] + hor[y1] * yb1[:, None, None]
    out = (v + (1 << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS)
    return np.clip(out, 0, 255).astype(np.uint8)


def normalize_frames(frames_u8: np.ndarray) -> np.ndarray:
    """[T, S, S, 3] uint8 -> [T, 3, S, S] float32: /255, (x - mean) / std (ravdess.py:363,386-389)."""
    f = frames_u8.astype(np.float32) / np.float32(255.0)
    f = (f - MEAN) / STD
    return np.ascontiguousarray(f.transpose(0, 3, 1, 2))


def preprocess_frames(frames_u8: np.ndarray, size: int = 112) -> np.ndarray:
    """Decoded RGB frames [T, H, W, 3] uint8 -> model input [T, 3, size, size] float32."""
    return normalize_frames(np.stack([resize_linear_u8(f, size) for f in frames_u8]))


_BLUR = {1: ([1], 0), 3: ([1, 2, 1], 2), 5: ([1, 4, 6, 4, 1], 4), 7: ([2, 7, 14, 18, 14, 7, 2], 6)}


def blur_u8(img: np.ndarray, k: int) -> np.ndarray:
    """cv2.GaussianBlur(img, (k, k), 0) on [H, W, C] uint8, k in {1, 3, 5, 7}: exact integer form of OpenCV's
    bit-exact 8U path, BORDER_REFLECT_101."""
    w, m = _BLUR[k]
    r = k // 2
    H, W, _ = img.shape

    def refl(n):  # cv::borderInterpolate(p, n, BORDER_REFLECT_101)
        out = []
        for p in range(-r, n + r):
            while n > 1 and (p < 0 or p >= n):
                p = -p if p < 0 else 2 * n - 2 - p
            out.append(p if n > 1 else 0)
        return np.array(out)

    src = img.astype(np.int64)
    ry, rx = refl(H), refl(W)
    hor = sum(w[i] * src[:, rx[i:i + W], :] for i in range(k))  # [H, W, C]
    acc = sum(w[i] * hor[ry[i:i + H], :, :] for i in range(k))
    if m == 0:
        return acc.astype(np.uint8)
    return ((acc + (1 << (2 * m - 1))) >> (2 * m)).astype(np.uint8)


def _mer_hash(seed: int, idx: np.ndarray) -> np.ndarray:
    """common.h mer_hash(seed, idx) for idx < 2^32 (uint32 arithmetic, wrapping)."""
    M = np.uint64(0xFFFFFFFF)
    seed = np.uint64(seed)
    s = (seed & M) ^ (((seed >> np.uint64(32)) * np.uint64(0x85EBCA6B)) & M)
    x = idx.astype(np.uint64) & M
    x = (x * np.uint64(0x9E3779B9) + s) & M
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M
    x ^= x >> np.uint64(16)
    return x


def augment_clip(frames_u8: np.ndarray, factor: float, noise_scale: float, ksize: int, seed: int,
                 ztable: np.ndarray) -> np.ndarray:
    """[T, S, S, 3] uint8 resized frames -> [T, 3, S, S] float32: ravdess.py:363-389 with augment=True."""
    T, S, _, C = frames_u8.shape
    f = frames_u8.astype(np.float32) / np.float32(255.0)
    q = (f * np.float32(255.0)).astype(np.uint8)  # ravdess.py:374 (truncating cast; the identity on 0..255)
    fac, sig = np.float32(factor), np.float32(noise_scale)
    out = np.empty((T, S, S, C), np.float32)
    for t in range(T):
        img = blur_u8(q[t], ksize).astype(np.float32) / np.float32(255.0)
        img = img * fac
        if sig > 0:
            e = np.arange(t * S * S * C, (t + 1) * S * S * C, dtype=np.uint64)
            z = ztable[(_mer_hash(seed, e) >> np.uint64(16)).astype(np.int64)].reshape(S, S, C)
            img = img + sig * z
        out[t] = np.clip(img, np.float32(0.0), np.float32(1.0))
    out = (out - MEAN) / STD
    return np.ascontiguousarray(out.transpose(0, 3, 1, 2))


def pad_crop_wav(wav: np.ndarray, target_len: int) -> np.ndarray:
    """[n] float32 -> [1, target_len]: zero-pad at the end or crop (ravdess.py:505-513)."""
    out = np.zeros(target_len, np.float32)
    n = min(len(wav), target_len)
    out[:n] = wav[:n]
    return out[None]
