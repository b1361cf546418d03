"""Host input pipeline (libmer_io.so, include/mer_io.h) against the numpy / scipy restatement in oracle/io_ref.py:
WAV decode of every sample format the reference's soundfile path reads (bit-exact), channel mean, the
resample_poly restatement (1e-5 abs), ravdess.py's frame-index sampling and face-box geometry (exact) and the
bar-noise mix (1e-6).  CPU only."""
import numpy as np
import pytest

from multimodalemotionrecognition_amd import data as D
from oracle import io_ref as R


@pytest.fixture(scope="module", autouse=True)
def _built():
    if not D._LIB_PATH.exists():
        pytest.skip("libmer_io.so not built")


@pytest.mark.parametrize("fmt", ["pcm8", "pcm16", "pcm24", "pcm32", "float32", "float64"])
@pytest.mark.parametrize("ch", [1, 2])
def test_wav_decode_matches_reference_scaling(tmp_path, fmt, ch):
    rng = np.random.default_rng(3)
    x = rng.uniform(-0.9, 0.9, (1001, ch))
    p = tmp_path / f"a_{fmt}_{ch}.wav"
    R.write_wav(p, x, 48000, fmt, extensible=(fmt == "pcm24"))
    got, sr = D.read_wav_mono(p)
    ref, rsr = R.read_wav_mono_ref(p)
    assert sr == rsr == 48000 and got.dtype == np.float32 and got.shape == ref.shape
    assert np.array_equal(got, ref), float(np.abs(got - ref).max())
    info = D.wav_info(p)
    assert info["channels"] == ch and info["frames"] == 1001


def test_wav_errors(tmp_path):
    p = tmp_path / "bad.wav"
    p.write_bytes(b"RIFX0000WAVE")
    with pytest.raises(D.MerIOError):
        D.read_wav_mono(p)
    with pytest.raises(D.MerIOError):
        D.read_wav_mono(tmp_path / "missing.wav")


@pytest.mark.parametrize("sr_in,sr_out", [(48000, 16000), (44100, 16000), (22050, 16000), (8000, 16000),
                                          (16000, 16000), (32000, 16000)])
def test_resample_matches_resample_poly(sr_in, sr_out):
    rng = np.random.default_rng(sr_in)
    x = (rng.standard_normal(sr_in // 3) * 0.2).astype(np.float32)
    got = D.resample(x, sr_in, sr_out)
    ref = R.resample_ref(x, sr_in, sr_out)
    assert got.shape == ref.shape
    assert float(np.abs(got - ref).max()) < 1e-5


@pytest.mark.parametrize("total", [0, 1, 5, 8, 9, 30, 87, 100, 151, 1000])
@pytest.mark.parametrize("num", [1, 8, 16])
def test_uniform_indices(total, num):
    assert D.uniform_indices(total, num) == R.uniform_indices_ref(total, num)


def test_face_crop_box():
    rng = np.random.default_rng(5)
    for _ in range(200):
        h, w = int(rng.integers(50, 800)), int(rng.integers(50, 800))
        x1, y1 = int(rng.integers(-20, w)), int(rng.integers(-20, h))
        x2, y2 = x1 + int(rng.integers(1, 300)), y1 + int(rng.integers(1, 300))
        for pr in (0.0, 0.3, 0.55):
            assert D.face_crop_box(h, w, (x1, y1, x2, y2), pr) == R.face_crop_box_ref(h, w, (x1, y1, x2, y2), pr)


def test_mix_noise_and_audio_pipeline(tmp_path):
    rng = np.random.default_rng(9)
    wav = (rng.standard_normal(48000) * 0.3).astype(np.float32)
    noise = (rng.standard_normal(20000) * 0.1).astype(np.float32)
    for start, snr in ((0, 20.0), (1234, 5.0), (19999, 10.0)):
        got = D.mix_noise(wav, noise, start, snr)
        assert float(np.abs(got - R.mix_noise_ref(wav, noise, start, snr)).max()) < 1e-6
    # load_audio_wav: decode 48 kHz stereo -> 16 kHz mono -> 3 s pad / crop
    for secs in (2.0, 4.0):
        x = rng.uniform(-0.5, 0.5, (int(48000 * secs), 2))
        p = tmp_path / f"clip{secs}.wav"
        R.write_wav(p, x, 48000, "pcm16")
        out = D.load_audio_wav(p)
        mono, _ = R.read_wav_mono_ref(p)
        ref = R.resample_ref(mono, 48000, 16000)
        ref = np.pad(ref, (0, max(0, 48000 - ref.size)))[:48000]
        assert tuple(out.shape) == (1, 48000)
        assert float(np.abs(out[0].numpy() - ref).max()) < 1e-5


def test_select_frames_crop_and_padding():
    frames = np.arange(20 * 60 * 80 * 3, dtype=np.int64).reshape(20, 60, 80, 3).astype(np.uint8)
    sel = D.select_frames(frames, 8, bbox=(10, 5, 40, 35))
    idx = R.uniform_indices_ref(20, 8)
    x1, y1, x2, y2 = R.face_crop_box_ref(60, 80, (10, 5, 40, 35))
    assert np.array_equal(sel, frames[idx][:, y1:y2, x1:x2])
    short = D.select_frames(frames[:3], 8)
    assert np.array_equal(short, frames[[0, 1, 2, 2, 2, 2, 2, 2]])
