"""oracle/clips_ref.py (cv2 INTER_LINEAR fixed-point restatement, ravdess.py:352-389,505-513) sanity checks.
cv2 is not installed, so the restatement is checked against the geometry it must share with an independent
float bilinear (torch F.interpolate, align_corners=False, no antialias): within 1 LSB of uint8 everywhere."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import clips_ref


@pytest.mark.parametrize("shape", [(720, 1280), (90, 160), (112, 112), (50, 70), (300, 200), (1, 1)])
def test_resize_matches_float_bilinear_within_one_lsb(shape):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(*shape, 3), dtype=np.uint8)
    ours = clips_ref.resize_linear_u8(img, 112).astype(np.int32)
    t = torch.from_numpy(img).permute(2, 0, 1)[None].double()
    ref = F.interpolate(t, size=(112, 112), mode="bilinear", align_corners=False)[0].permute(1, 2, 0).numpy()
    assert np.abs(ours - ref).max() <= 1.0 + 1e-9


def test_exact_2x_is_area_average():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, size=(224, 224, 3), dtype=np.uint8)
    ours = clips_ref.resize_linear_u8(img, 112).astype(np.int32)
    s = img.astype(np.int32).reshape(112, 2, 112, 2, 3).sum(axis=(1, 3))
    assert np.array_equal(ours, (s + 2) >> 2)


def test_identity_size_is_copy_and_normalisation_order():
    rng = np.random.default_rng(5)
    frames = rng.integers(0, 256, size=(2, 112, 112, 3), dtype=np.uint8)
    out = clips_ref.preprocess_frames(frames)
    assert out.shape == (2, 3, 112, 112) and out.dtype == np.float32
    ref = ((frames.astype(np.float32) / 255.0 - clips_ref.MEAN) / clips_ref.STD).transpose(0, 3, 1, 2)
    assert np.array_equal(out, ref)


def test_pad_crop_matches_reference_semantics():
    for n in (0, 10, 48000, 50000):
        w = np.arange(n, dtype=np.float32)
        ref = torch.from_numpy(w)[None]
        ref = F.pad(ref, (0, 48000 - n)) if n < 48000 else ref[:, :48000]
        assert np.array_equal(clips_ref.pad_crop_wav(w, 48000), ref.numpy())
