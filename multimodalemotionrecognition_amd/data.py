"""Real input pipeline: ``src/data/ravdess.py``'s clip loading with the host work in native
code (``host/mer_io.cpp`` -> ``libmer_io.so``, C-ABI ``include/mer_io.h``) and the batch assembly on the MI355X
(``clips.py`` -> ``csrc/clips.hip``).

* ``load_audio_wav`` -- ravdess.py:488-578: WAV decode + mono mix + resample to 16 kHz (native), pad / crop to
  3 s, bar-noise augmentation at a drawn SNR (native mix).  librosa's soxr_hq resampler is absent from this image:
  the native resampler restates ``scipy.signal.resample_poly`` (parity with soxr unpinned; pinned against scipy).
* ``uniform_indices`` -- ravdess.py:272-277, the frame sampling of ``load_video_frames``.
* ``face_crop_box`` -- face_crop.py:151-190 (``crop_with_padding``'s box, pad 0.3).
* ``load_video_frames`` -- ravdess.py:280-390 after decode: index sampling, face-box crop, resize + /255 +
  ImageNet normalisation on the device.  Video DECODING (cv2.VideoCapture) and face DETECTION (MediaPipe) need
  libraries this image does not have: the caller supplies decoded RGB uint8 frames (any decoder) and, optionally,
  the detected bbox; without one the full frame is used -- the reference's own fallback when MediaPipe is missing
  (ravdess.py:300-304).
* ``ClipLoader`` -- the DataLoader of train.py for the GPU path: worker threads decode clips (the native calls
  release the GIL), each rank takes a disjoint shard (DP), and batches land in HBM as
  ``[B, 8, 3, 112, 112]`` / ``[B, 1, 48000]`` / labels.
"""
from __future__ import annotations

import ctypes
import queue
import threading
from pathlib import Path
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import clips

_LIB_PATH = Path(__file__).resolve().parent / "libmer_io.so"
_lib = None
_lock = threading.Lock()

IO_ERRORS = {-1: "cannot open / read the file", -2: "not a RIFF/WAVE file or unsupported sample format",
             -3: "bad argument"}


class MerIOError(RuntimeError):
    pass


def _io():
    global _lib
    with _lock:
        if _lib is None:
            if not _LIB_PATH.exists():
                raise MerIOError(f"host input library not built: {_LIB_PATH} is missing (make -C "
                                 "multimodalemotionrecognition_amd/host, or __graft_entry__.build())")
            lib = ctypes.CDLL(str(_LIB_PATH))
            P, I, LL, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float
            sig = {
                "mer_wav_info": (I, [ctypes.c_char_p, P, P, P, P, P]),
                "mer_wav_read_mono": (I, [ctypes.c_char_p, P, LL, P]),
                "mer_resample_len": (LL, [LL, I, I]),
                "mer_resample": (I, [P, LL, I, I, P, LL, P]),
                "mer_uniform_indices": (I, [I, I, P]),
                "mer_face_crop_box": (I, [I, I, I, I, I, I, F, P]),
                "mer_mix_noise": (I, [P, LL, P, LL, LL, F]),
            }
            for name, (res, args) in sig.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            _lib = lib
    return _lib


def _check(rc, what):
    if rc != 0:
        raise MerIOError(f"{what}: {IO_ERRORS.get(rc, rc)}")


def wav_info(path) -> dict:
    sr, ch, fr, fmt, bits = ctypes.c_int(), ctypes.c_int(), ctypes.c_longlong(), ctypes.c_int(), ctypes.c_int()
    _check(_io().mer_wav_info(str(path).encode(), ctypes.byref(sr), ctypes.byref(ch), ctypes.byref(fr),
                              ctypes.byref(fmt), ctypes.byref(bits)), f"wav_info({path})")
    return {"sample_rate": sr.value, "channels": ch.value, "frames": fr.value, "format": fmt.value, "bits": bits.value}


def read_wav_mono(path) -> Tuple[np.ndarray, int]:
    """(float32 mono samples, native sample rate) -- soundfile scaling, channel mean (librosa.load with sr=None)."""
    info = wav_info(path)
    out = np.empty(max(1, info["frames"]), dtype=np.float32)
    n = ctypes.c_longlong()
    _check(_io().mer_wav_read_mono(str(path).encode(), out.ctypes.data, out.size, ctypes.byref(n)), f"read({path})")
    return out[:n.value], info["sample_rate"]


def resample(x: np.ndarray, sr_in: int, sr_out: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = _io().mer_resample_len(x.size, sr_in, sr_out)
    if n < 0:
        raise MerIOError("resample: bad rates")
    out = np.empty(max(1, n), dtype=np.float32)
    got = ctypes.c_longlong()
    _check(_io().mer_resample(x.ctypes.data, x.size, sr_in, sr_out, out.ctypes.data, out.size, ctypes.byref(got)),
           "resample")
    return out[:got.value]


def uniform_indices(total: int, num: int) -> List[int]:
    out = np.empty(max(1, num), dtype=np.int32)
    _check(_io().mer_uniform_indices(int(total), int(num), out.ctypes.data), "uniform_indices")
    return out[:num].tolist()


def face_crop_box(h: int, w: int, bbox, pad_ratio: float = 0.3) -> Tuple[int, int, int, int]:
    out = np.empty(4, dtype=np.int32)
    x1, y1, x2, y2 = (int(v) for v in bbox)
    _check(_io().mer_face_crop_box(int(h), int(w), x1, y1, x2, y2, float(pad_ratio), out.ctypes.data), "crop box")
    return tuple(int(v) for v in out)


def mix_noise(wav: np.ndarray, noise: np.ndarray, start: int, snr_db: float) -> np.ndarray:
    """In place on a float32 copy; returns it (ravdess.py:543-566)."""
    w = np.array(wav, dtype=np.float32, copy=True)
    nz = np.ascontiguousarray(noise, dtype=np.float32).reshape(-1)
    _check(_io().mer_mix_noise(w.ctypes.data, w.size, nz.ctypes.data, nz.size, int(start), float(snr_db)), "mix")
    return w


def load_audio_wav(audio_path, sample_rate: int = 16000, duration_sec: float = 3.0, augment: bool = False,
                   bar_noise: Optional[np.ndarray] = None, rng: Optional[np.random.Generator] = None) -> torch.Tensor:
    """ravdess.py:488-578 -> host float32 ``[1, int(sample_rate * duration_sec)]``.  ``bar_noise``: the 16 kHz bar
    noise track (the reference's ``_load_bar_noise``); without one, augmentation falls back to Gaussian noise at
    the drawn SNR as the reference does."""
    wav, sr = read_wav_mono(audio_path)
    if sr != sample_rate:
        wav = resample(wav, sr, sample_rate)
    target = int(sample_rate * duration_sec)
    if wav.size < target:
        wav = np.pad(wav, (0, target - wav.size))
    else:
        wav = wav[:target]
    if augment:
        rng = rng if rng is not None else np.random.default_rng()
        level = rng.uniform(0.0, 1.0)
        if level >= 0.5:
            snr_db = float(rng.choice([20.0, 15.0, 10.0])) if level < 0.9 else 5.0
            if bar_noise is not None and bar_noise.size:
                n = bar_noise.size
                tiled = n if n >= target else n * (target // n + 1)
                max_start = max(0, tiled - target)
                start = int(rng.integers(0, max_start + 1)) if max_start > 0 else 0
                wav = mix_noise(wav, bar_noise, start, snr_db)
            else:
                p = float(np.mean(wav.astype(np.float32) ** 2))
                noise = rng.normal(0, np.sqrt(p / max(10 ** (snr_db / 10.0), 1e-8)), wav.shape).astype(np.float32)
                wav = np.clip(wav + noise, -1.0, 1.0)
    return torch.from_numpy(np.ascontiguousarray(wav, dtype=np.float32)).unsqueeze(0)


FrameSource = Union[np.ndarray, torch.Tensor, Callable[[], np.ndarray], str, Path]


def _frames(src: FrameSource) -> np.ndarray:
    """Decoded RGB uint8 frames [T, H, W, 3]: an array, a ``.npy`` file or a decoder callable."""
    if callable(src):
        src = src()
    if isinstance(src, (str, Path)):
        src = np.load(str(src), allow_pickle=False)
    if isinstance(src, torch.Tensor):
        src = src.cpu().numpy()
    a = np.asarray(src)
    if a.dtype != np.uint8 or a.ndim != 4 or a.shape[-1] != 3:
        raise ValueError("decoded frames must be uint8 [T, H, W, 3] RGB")
    return a


def select_frames(frames: np.ndarray, num_frames: int = 8, bbox=None, pad_ratio: float = 0.3) -> np.ndarray:
    """The host half of load_video_frames: uniform sampling, face-box crop (one box for every frame, as the
    reference reuses the first frame's detection), padding by repeating the last frame -> [num_frames, h, w, 3]."""
    T, H, W, _ = frames.shape
    if T == 0:
        return np.zeros((num_frames, 1, 1, 3), dtype=np.uint8)
    idx = [min(i, T - 1) for i in uniform_indices(T, num_frames)]
    sel = frames[idx]
    if bbox is not None:
        x1, y1, x2, y2 = face_crop_box(H, W, bbox, pad_ratio)
        if x2 > x1 and y2 > y1:
            sel = sel[:, y1:y2, x1:x2]
    return np.ascontiguousarray(sel)


def load_video_frames(src: FrameSource, num_frames: int = 8, size: int = 112, bbox=None,
                      device="cuda") -> torch.Tensor:
    """ravdess.py:280-390 after decode -> ``[num_frames, 3, size, size]`` fp32 on the device."""
    sel = select_frames(_frames(src), num_frames, bbox)
    dev_frames = torch.from_numpy(sel).to(device, non_blocking=False)
    return clips.preprocess_frames(dev_frames, size)


def _collate_meta(metas: List[dict]) -> dict:
    """default_collate of the reference's per-clip meta dicts (ravdess.py:608-615): one list per key (ints as a
    tensor, as torch's collate does)."""
    keys = []
    for m in metas:
        keys += [k for k in m if k not in keys]
    out = {}
    for k in keys:
        vals = [m.get(k) for m in metas]
        out[k] = torch.tensor(vals) if all(isinstance(v, int) and not isinstance(v, bool) for v in vals) else vals
    return out


def shard_indices(n: int, rank: int, world: int, shuffle: bool, seed: int, epoch: int) -> np.ndarray:
    """``torch.utils.data.DistributedSampler`` order (drop_last=False): one permutation of ALL items drawn by
    ``torch.randperm`` from a CPU generator seeded with (seed + epoch) on every rank -- the sampler's own draw, so
    the shuffled order is the reference pipeline's --, padded by wrapping to a multiple of ``world``, then every
    ``world``-th index from ``rank``: every rank sees the same number of items and, across epochs, different clips."""
    if shuffle:
        order = torch.randperm(n, generator=torch.Generator().manual_seed(int(seed) + int(epoch))).numpy()
    else:
        order = np.arange(n)
    total = -(-n // world) * world if n else 0
    if total > n:
        reps = -(-(total - n) // n)
        order = np.concatenate([order] + [order] * reps)[:total]
    return order[rank:total:world]


class ClipLoader:
    """Batches of ``(video [B, 8, 3, 112, 112], audio [B, 1, 48000], labels [B], meta)`` assembled on the GPU --
    the 4-tuples of the reference's datasets (ravdess.py:616, 654) that ``train_one_epoch`` unpacks
    (train.py:200).

    ``items``: ``(frames source, wav path, label[, bbox-or-None[, meta dict]])`` per clip.  Data parallelism:
    rank ``rank`` of ``world`` takes a ``DistributedSampler``-style shard of one global permutation
    (``shard_indices``), so all ranks run the same number of steps (a rank with an extra step would block in the
    gradient all-reduce).  ``workers`` threads decode ahead (``prefetch`` batches).  ``augment``: the reference's
    train-split audio augmentation (ravdess.py:519-578, bar noise at a drawn SNR; ``bar_noise`` is the 16 kHz
    track, else Gaussian noise), drawn from a generator seeded per (seed, epoch, item) so the draws do not depend
    on thread scheduling.  ``augment`` also applies the reference's train-split video augmentation
    (cv2.GaussianBlur(k, 0) + darken + Gaussian noise on the uint8 frames, ravdess.py:366-384) on the device, one
    ``clips.augment_clips`` launch per batch with per-clip draws from the same generator; it is bit-exact against
    the restatement in ``oracle/clips_ref.py``, and parity against cv2 itself is unpinned (cv2 is absent here)."""

    def __init__(self, items: Sequence[Tuple], batch_size: int = 32, num_frames: int = 8, size: int = 112,
                 sample_rate: int = 16000, duration_sec: float = 3.0, rank: int = 0, world: int = 1,
                 workers: int = 8, prefetch: int = 2, device="cuda", shuffle: bool = False, seed: int = 0,
                 drop_last: bool = True, augment: bool = False, bar_noise: Optional[np.ndarray] = None):
        self.all_items = list(items)
        self.rank, self.world = int(rank), max(1, int(world))
        if not 0 <= self.rank < self.world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.B, self.T, self.size = batch_size, num_frames, size
        self.sr, self.dur = sample_rate, duration_sec
        self.workers, self.prefetch = max(1, workers), max(1, prefetch)
        self.device = torch.device(device)
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.augment, self.bar_noise = bool(augment), bar_noise
        self.epoch = 0

    @property
    def items(self):
        """This rank's items in epoch-0 order."""
        return [self.all_items[i] for i in shard_indices(len(self.all_items), self.rank, self.world, False, 0, 0)]

    def num_samples(self) -> int:
        return -(-len(self.all_items) // self.world) if self.all_items else 0

    def __len__(self):
        n = self.num_samples()
        return n // self.B if self.drop_last else -(-n // self.B)

    def _assemble(self, decoded):
        # frames of one batch may differ in size (per-clip crops): resize each clip's frames on the device
        if self.augment:  # resized uint8 clips, then ONE augmentation + normalisation launch with per-clip draws
            u8 = torch.empty(len(decoded), self.T, self.size, self.size, 3, device=self.device, dtype=torch.uint8)
            for i, (f, _, _, _, _) in enumerate(decoded):
                clips.resize_frames_u8(torch.from_numpy(f).to(self.device), self.size, out=u8[i])
            video = clips.augment_clips(u8, [va for _, _, _, _, va in decoded])
        else:
            vids = [clips.preprocess_frames(torch.from_numpy(f).to(self.device), self.size) for f, _, _, _, _ in decoded]
            video = torch.stack(vids).contiguous()
        audio = clips.pad_crop_waveforms([torch.from_numpy(w) for _, w, _, _, _ in decoded], self.sr, self.dur,
                                         device=self.device)
        labels = torch.tensor([lab for _, _, lab, _, _ in decoded], dtype=torch.long).to(self.device)
        return video, audio, labels, _collate_meta([m for _, _, _, m, _ in decoded])

    def __iter__(self):
        order = shard_indices(len(self.all_items), self.rank, self.world, self.shuffle, self.seed, self.epoch)
        epoch = self.epoch
        self.epoch += 1
        nb = len(self)
        batches = [order[i * self.B:(i + 1) * self.B] for i in range(nb)]
        out_q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()

        def produce():
            from concurrent.futures import ThreadPoolExecutor
            try:
                with ThreadPoolExecutor(self.workers) as ex:
                    for b in batches:
                        if stop.is_set():
                            return
                        decoded = list(ex.map(self._decode_epoch(epoch), [(int(i), self.all_items[i]) for i in b]))
                        out_q.put(("ok", decoded))
            except BaseException as e:  # surfaced to the consumer
                out_q.put(("err", e))
            out_q.put(("end", None))

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        try:
            while True:
                kind, val = out_q.get()
                if kind == "end":
                    return
                if kind == "err":
                    raise val
                yield self._assemble(val)
        finally:
            stop.set()

    def _decode_epoch(self, epoch):
        def fn(job):
            gi, item = job
            src, wav_path, label = item[0], item[1], item[2]
            bbox = item[3] if len(item) > 3 else None
            meta = dict(item[4]) if len(item) > 4 and item[4] is not None else {}
            meta.setdefault("index", int(gi))
            frames = select_frames(_frames(src), self.T, bbox)
            rng = np.random.default_rng([self.seed, epoch, int(gi)]) if self.augment else None
            # the reference loads (and augments) the video before the audio (ravdess.py:639-645): same draw order
            vaug = clips.draw_video_augment(rng) if self.augment else None
            wav = load_audio_wav(wav_path, self.sr, self.dur, augment=self.augment, bar_noise=self.bar_noise,
                                 rng=rng)[0].numpy()
            return frames, wav, int(label), meta, vaug
        return fn
