"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): numpy / scipy restatement of the host input
pipeline of src/data/ravdess.py and src/utils/face_crop.py, against which libmer_io.so (include/mer_io.h) is
tested.  Parity notes: the reference decodes with librosa.load -> soundfile and resamples with soxr_hq; neither is
installed here, so the decode scaling restates soundfile's documented float conversion and the resampler is
scipy.signal.resample_poly (the algorithm mer_resample implements) -- parity with soxr is unpinned."""
from __future__ import annotations

import struct

import numpy as np


def write_wav(path, data: np.ndarray, rate: int, fmt: str = "pcm16", extensible: bool = False):
    """data [frames, channels] in [-1, 1] -> a RIFF/WAVE file (test fixture writer)."""
    data = np.asarray(data, dtype=np.float64)
    if data.ndim == 1:
        data = data[:, None]
    frames, ch = data.shape
    if fmt == "pcm8":
        raw, tag, bits = np.clip(np.round(data * 128 + 128), 0, 255).astype(np.uint8).tobytes(), 1, 8
    elif fmt == "pcm16":
        raw, tag, bits = np.clip(np.round(data * 32768), -32768, 32767).astype("<i2").tobytes(), 1, 16
    elif fmt == "pcm24":
        v = np.clip(np.round(data * 8388608), -8388608, 8388607).astype("<i4").reshape(-1)
        b = v.view(np.uint8).reshape(-1, 4)[:, :3]
        raw, tag, bits = b.tobytes(), 1, 24
    elif fmt == "pcm32":
        raw, tag, bits = np.clip(np.round(data * 2147483648.0), -2147483648, 2147483647).astype("<i4").tobytes(), 1, 32
    elif fmt == "float32":
        raw, tag, bits = data.astype("<f4").tobytes(), 3, 32
    elif fmt == "float64":
        raw, tag, bits = data.astype("<f8").tobytes(), 3, 64
    else:
        raise ValueError(fmt)
    block = ch * bits // 8
    if extensible:
        guid = struct.pack("<H", tag) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
        fmt_chunk = struct.pack("<HHIIHHHHI", 0xFFFE, ch, rate, rate * block, block, bits, 22, bits, 0) + guid
    else:
        fmt_chunk = struct.pack("<HHIIHH", tag, ch, rate, rate * block, block, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt_chunk)) + fmt_chunk
    body += b"LIST" + struct.pack("<I", 4) + b"INFO"  # an extra chunk the reader must skip
    body += b"data" + struct.pack("<I", len(raw)) + raw + (b"\x00" if len(raw) & 1 else b"")
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def read_wav_mono_ref(path):
    """soundfile.read(dtype='float32') + librosa.to_mono (mean over channels) -> (samples, rate)."""
    b = open(path, "rb").read()
    assert b[:4] == b"RIFF" and b[8:12] == b"WAVE"
    pos, fmt = 12, None
    while pos + 8 <= len(b):
        cid, size = b[pos:pos + 4], struct.unpack("<I", b[pos + 4:pos + 8])[0]
        body = b[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, rate, _, block, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE:
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, rate, block, bits)
        elif cid == b"data":
            tag, ch, rate, block, bits = fmt
            n = len(body) // block
            if tag == 3:
                x = np.frombuffer(body[:n * block], dtype="<f4" if bits == 32 else "<f8").astype(np.float64)
            elif bits == 8:
                x = (np.frombuffer(body[:n * block], dtype=np.uint8).astype(np.float64) - 128) / 128.0
            elif bits == 16:
                x = np.frombuffer(body[:n * block], dtype="<i2") / 32768.0
            elif bits == 24:
                u = np.frombuffer(body[:n * block], dtype=np.uint8).reshape(-1, 3).astype(np.int32)
                v = (u[:, 0] << 8 | u[:, 1] << 16 | u[:, 2] << 24) >> 8
                x = v / 8388608.0
            else:
                x = np.frombuffer(body[:n * block], dtype="<i4") / 2147483648.0
            x = x.astype(np.float32).reshape(n, ch)
            return (x[:, 0] if ch == 1 else x.mean(axis=1, dtype=np.float32)), rate
        pos += 8 + size + (size & 1)
    raise ValueError("no data chunk")


def resample_ref(x, sr_in, sr_out):
    from math import gcd

    from scipy.signal import resample_poly
    g = gcd(sr_in, sr_out)
    return resample_poly(np.asarray(x, dtype=np.float32), sr_out // g, sr_in // g)


def uniform_indices_ref(total, num):
    """ravdess.py:272-277 verbatim semantics."""
    if total <= 0:
        return [0] * num
    if total >= num:
        return np.linspace(0, total - 1, num=num).round().astype(int).tolist()
    return list(range(total)) + [total - 1] * (num - total)


def face_crop_box_ref(h, w, bbox, pad_ratio=0.3):
    x1, y1, x2, y2 = bbox
    pad_x, pad_y = int((x2 - x1) * pad_ratio), int((y2 - y1) * pad_ratio)
    return max(0, x1 - pad_x), max(0, y1 - pad_y), min(w, x2 + pad_x), min(h, y2 + pad_y)


def mix_noise_ref(wav, noise, start, snr_db):
    """ravdess.py:543-566 (float64 powers)."""
    n = wav.size
    seg = noise[(start + np.arange(n)) % noise.size].astype(np.float64)
    ps, pn = np.mean(wav.astype(np.float64) ** 2), np.mean(seg ** 2)
    target = ps / max(10 ** (snr_db / 10.0), 1e-8)
    s = np.float32(np.sqrt(target / pn)) if pn > 1e-8 else np.float32(1.0)
    return np.clip(wav.astype(np.float32) + noise[(start + np.arange(n)) % noise.size].astype(np.float32) * s, -1, 1)
