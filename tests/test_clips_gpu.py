"""Device clip assembly (csrc/clips.hip) vs oracle/clips_ref.py: bit-exact (integer resize, IEEE fp32
normalisation in the reference's operation order), ragged waveform batches exact."""
import numpy as np
import pytest
import torch

from oracle import clips_ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(720, 1280), (90, 160), (224, 224), (112, 112), (50, 70), (300, 200), (1, 1)])
def test_preprocess_frames_bit_exact(shape):
    from multimodalemotionrecognition_amd.clips import preprocess_frames

    rng = np.random.default_rng(hash(shape) % 1000)
    frames = rng.integers(0, 256, size=(3, *shape, 3), dtype=np.uint8)
    got = preprocess_frames(torch.from_numpy(frames).cuda()).cpu().numpy()
    ref = clips_ref.preprocess_frames(frames)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), float(np.abs(got - ref).max())


def test_video_clip_batch_layout():
    from multimodalemotionrecognition_amd.clips import video_clip_batch

    rng = np.random.default_rng(9)
    frames = rng.integers(0, 256, size=(2, 8, 96, 128, 3), dtype=np.uint8)
    got = video_clip_batch(torch.from_numpy(frames).cuda())
    assert tuple(got.shape) == (2, 8, 3, 112, 112)
    ref = clips_ref.preprocess_frames(frames.reshape(16, 96, 128, 3)).reshape(2, 8, 3, 112, 112)
    assert np.array_equal(got.cpu().numpy(), ref)


def test_pad_crop_waveforms_ragged():
    from multimodalemotionrecognition_amd.clips import pad_crop_waveforms

    rng = np.random.default_rng(10)
    lens = [0, 17, 48000, 61234, 30000]
    wavs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)) for n in lens]
    got = pad_crop_waveforms(wavs, device="cuda").cpu().numpy()
    assert got.shape == (5, 1, 48000)
    for i, w in enumerate(wavs):
        assert np.array_equal(got[i], clips_ref.pad_crop_wav(w.numpy(), 48000)), i
