"""Deterministic, machine-independent parameter and input generators.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Everything is drawn from numpy's PCG64 so that the build container (which
generates the golden vectors from the imported reference) and the GPU box
(which regenerates the same weights/inputs to feed the HIP path) agree bit for
bit.  Each tensor gets its own stream keyed by ``crc32(name)`` so the value of a
parameter never depends on which other parameters exist.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

IMAGENET_MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
IMAGENET_STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(name.encode())]))


def init_tensor(name: str, shape: Tuple[int, ...], seed: int = 0) -> np.ndarray:
    """Name-driven init that keeps activations O(1) through every layer."""
    arr = _init_tensor(name, shape, seed)
    return np.array(np.asarray(arr).reshape(tuple(int(s) for s in shape)), order="C")


def _init_tensor(name: str, shape: Tuple[int, ...], seed: int = 0):
    rng = _rng(seed, name)
    shape = tuple(int(s) for s in shape)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "running_mean":
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if leaf == "running_var":
        return (1.0 + 0.2 * rng.random(shape)).astype(np.float32)
    if leaf == "masked_spec_embed":
        return rng.random(shape).astype(np.float32)
    if leaf in ("bias_scale", "gru_rel_pos_const"):
        return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    if leaf == "original0":  # weight-norm magnitude g of the WavLM positional conv
        return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    if "rel_attn_embed" in name:
        return (0.5 * rng.standard_normal(shape)).astype(np.float32)
    if len(shape) <= 1:
        is_norm = any(t in name for t in ("norm", "bn", "downsample.1", "backbone.1.")) or (
            name.startswith("backbone.1") or ".bn" in name
        )
        if leaf == "weight" and is_norm:
            return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
        if leaf == "weight":  # e.g. GroupNorm affine
            return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
        return (0.05 * rng.standard_normal(shape)).astype(np.float32)
    fan_in = int(np.prod(shape[1:]))
    return (rng.standard_normal(shape) / np.sqrt(max(fan_in, 1))).astype(np.float32)


def init_state(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 0) -> Dict[str, np.ndarray]:
    return {name: init_tensor(name, shape, seed) for name, shape in named_shapes}


def feature_inputs(batch: int, t: int, ta: int, v_dim: int = 512, a_dim: int = 768,
                   seed: int = 20261015) -> Tuple[np.ndarray, np.ndarray]:
    """C1-style feature-level inputs: video feats N(0,1) [B,T,v_dim], audio feats N(0,1) [B,Ta,a_dim]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    v = rng.standard_normal((batch, t, v_dim)).astype(np.float32)
    a = rng.standard_normal((batch, ta, a_dim)).astype(np.float32)
    return v, a


def clip_inputs(batch: int, frames: int = 8, size: int = 112, samples: int = 48000,
                num_classes: int = 8, seed: int = 20261015):
    """Synthetic 3 s clips laid out like ``ravdess.py:386-389,505-513``.

    video = (U[0,1) - mean_c) / std_c -> [B,T,3,H,W]; audio = clip(N(0, 0.1^2), -1, 1) -> [B,1,S];
    labels uniform in [0, num_classes).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    video = rng.random((batch, frames, 3, size, size), dtype=np.float32)
    video = (video - IMAGENET_MEAN[None, None, :, None, None]) / IMAGENET_STD[None, None, :, None, None]
    audio = np.clip(0.1 * rng.standard_normal((batch, 1, samples)), -1.0, 1.0).astype(np.float32)
    labels = rng.integers(0, num_classes, size=(batch,), dtype=np.int64)
    return video.astype(np.float32), audio, labels
