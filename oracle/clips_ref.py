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


def pad_crop_wav(wav: np.ndarray, target_len: int) -> np.ndarray:
    """[n] float32 -> [1, target_len]: zero-pad at the end or crop (ravdess.py:505-513)."""
    out = np.zeros(target_len, np.float32)
    n = min(len(wav), target_len)
    out[:n] = wav[:n]
    return out[None]
