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


@pytest.mark.parametrize("shape", [(720, 1280), (90, 160), (224, 224), (112, 112), (50, 70), (300, 200), (1, 1)])
def test_augment_clips_bit_exact(shape):
    """Train-split video augmentation (ravdess.py:366-384) on the device vs oracle/clips_ref.augment_clip: resize to
    uint8, blur k = 3 / 5 / 7, darken, table-Gaussian noise (and none), clip, normalise -- bit-exact."""
    from multimodalemotionrecognition_amd import clips

    rng = np.random.default_rng(hash(shape) % 977)
    B, T = 4, 3
    frames = rng.integers(0, 256, size=(B, T, *shape, 3), dtype=np.uint8)
    params = [clips.draw_video_augment(rng) for _ in range(B)]
    params[1] = (params[1][0], params[1][1], 3, params[1][3])
    params[2] = (params[2][0], 0.0, 7, params[2][3])  # noise_scale 0: no noise term
    params[3] = (params[3][0], params[3][1], 5, params[3][3])
    dev = torch.from_numpy(frames.reshape(B * T, *shape, 3)).cuda()
    u8 = clips.resize_frames_u8(dev).view(B, T, 112, 112, 3)
    got = clips.augment_clips(u8, params).cpu().numpy()
    zt = clips.normal_table().numpy()
    for b in range(B):
        r8 = np.stack([clips_ref.resize_linear_u8(f, 112) for f in frames[b]])
        assert np.array_equal(u8[b].cpu().numpy(), r8)
        ref = clips_ref.augment_clip(r8, *params[b], zt)
        assert np.array_equal(got[b], ref), (b, params[b], float(np.abs(got[b] - ref).max()))


def test_clip_loader_augment_bit_exact(tmp_path):
    """ClipLoader(augment=True): the video tensor equals the oracle's augmentation with the loader's own draws
    (per (seed, epoch, item) generator, video drawn before audio as ravdess.py:639-645 loads them)."""
    from multimodalemotionrecognition_amd import clips
    from multimodalemotionrecognition_amd.data import ClipLoader, select_frames
    from oracle.io_ref import write_wav

    rng = np.random.default_rng(4)
    items = []
    for i in range(4):
        fr = rng.integers(0, 256, size=(10, 60 + 8 * i, 80, 3), dtype=np.uint8)
        wav = tmp_path / f"{i}.wav"
        write_wav(str(wav), (rng.standard_normal(16000) * 0.1).astype(np.float32), 16000)
        items.append((fr, str(wav), i % 8))
    loader = ClipLoader(items, batch_size=2, workers=2, device="cuda", shuffle=True, seed=11, augment=True)
    zt = clips.normal_table().numpy()
    from multimodalemotionrecognition_amd.data import shard_indices
    order = shard_indices(4, 0, 1, True, 11, 0)
    seen = 0
    for bi, (video, audio, labels, meta) in enumerate(loader):
        for j in range(video.shape[0]):
            gi = int(order[bi * 2 + j])
            assert int(meta["index"][j]) == gi
            g = np.random.default_rng([11, 0, gi])
            prm = clips.draw_video_augment(g)
            sel = select_frames(items[gi][0], 8, None)
            r8 = np.stack([clips_ref.resize_linear_u8(f, 112) for f in sel])
            ref = clips_ref.augment_clip(r8, *prm, zt)
            assert np.array_equal(video[j].cpu().numpy(), ref), gi
            seen += 1
    assert seen == 4
