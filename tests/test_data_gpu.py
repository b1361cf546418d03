"""The clip loader (data.ClipLoader) on the MI355X: host decode in libmer_io.so worker threads, device crop /
resize / normalise / pad-crop (csrc/clips.hip).  Each batch is checked against the oracle restatements
(oracle/io_ref.py, oracle/clips_ref.py) of ravdess.py:280-578 on the same files; rank sharding is disjoint."""
import numpy as np
import pytest
import torch

from multimodalemotionrecognition_amd import data as D
from oracle import clips_ref as CR
from oracle import io_ref as R

pytestmark = pytest.mark.gpu


def _items(tmp_path, n=6):
    rng = np.random.default_rng(11)
    items = []
    for i in range(n):
        T, H, W = int(rng.integers(5, 40)), int(rng.integers(90, 200)), int(rng.integers(90, 200))
        frames = rng.integers(0, 256, (T, H, W, 3), dtype=np.uint8)
        fp = tmp_path / f"f{i}.npy"
        np.save(fp, frames)
        secs = float(rng.uniform(1.5, 4.0))
        wp = tmp_path / f"a{i}.wav"
        R.write_wav(wp, rng.uniform(-0.6, 0.6, (int(48000 * secs), 2)), 48000, "pcm16")
        bbox = (int(W * 0.2), int(H * 0.15), int(W * 0.7), int(H * 0.8)) if i % 2 else None
        items.append((str(fp), str(wp), i % 8, bbox))
    return items


def test_clip_loader_batches_match_oracle(tmp_path):
    items = _items(tmp_path)
    loader = D.ClipLoader(items, batch_size=3, workers=3)
    batches = list(loader)
    assert len(batches) == 2
    for bi, (video, audio, labels, meta) in enumerate(batches):
        assert tuple(video.shape) == (3, 8, 3, 112, 112) and tuple(audio.shape) == (3, 1, 48000)
        assert meta["index"].tolist() == list(range(3 * bi, 3 * bi + 3))
        assert video.is_cuda and audio.is_cuda and labels.tolist() == [it[2] for it in items[3 * bi:3 * bi + 3]]
        for j in range(3):
            fp, wp, _, bbox = items[3 * bi + j]
            sel = D.select_frames(np.load(fp), 8, bbox)
            ref_v = CR.preprocess_frames(sel, 112)
            assert float(np.abs(video[j].cpu().numpy() - ref_v).max()) < 1e-4
            mono, _ = R.read_wav_mono_ref(wp)
            ref_a = CR.pad_crop_wav(R.resample_ref(mono, 48000, 16000), 48000)
            assert float(np.abs(audio[j, 0].cpu().numpy() - ref_a).max()) < 1e-5


def test_clip_loader_rank_shards(tmp_path):
    items = _items(tmp_path, 4)
    seen = []
    for rank in range(2):
        for _, _, labels, _ in D.ClipLoader(items, batch_size=2, rank=rank, world=2, workers=2):
            seen += labels.tolist()
    assert sorted(seen) == sorted(it[2] for it in items)


def test_load_video_frames_device(tmp_path):
    rng = np.random.default_rng(2)
    frames = rng.integers(0, 256, (30, 120, 160, 3), dtype=np.uint8)
    out = D.load_video_frames(frames, 8, 112, bbox=(20, 10, 120, 100))
    ref = CR.preprocess_frames(D.select_frames(frames, 8, (20, 10, 120, 100)), 112)
    assert out.is_cuda and float(np.abs(out.cpu().numpy() - ref).max()) < 1e-4
