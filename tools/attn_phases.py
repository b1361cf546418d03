"""Phase timing of the WavLM attention kernel: builds multimodalemotionrecognition_amd/libmer_hip_at.so (the library
with -DMER_ATTN_TIMING, see AT() in csrc/wavlm.hip), runs one B=32 launch (eval, then train) and prints, over the
workgroups (thread 0 = wave 0), the median / max of each phase's duration and of the start / end offsets from the
first workgroup's start (us at the 100 MHz wall clock).
    python tools/attn_phases.py build      (here: hipcc, no GPU)
    python tools/attn_phases.py run        (GPU box)"""
import ctypes
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodalemotionrecognition_amd"
AT_LIB = PKG / "libmer_hip_at.so"
PHASES = ["start->loads back", "LDS store + sync", "gate", "QK^T + max", "exp + sum (+mask)", "PV + store"]


def build():
    csrc = PKG / "csrc"
    out = csrc / "build" / "at"
    out.mkdir(parents=True, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-DMER_ATTN_TIMING", f"-I{ROOT / 'include'}",
             "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
    o = out / "wavlm.o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", str(csrc / "wavlm.hip"), "-o", str(o)])
    objs = [str(p) for p in sorted((csrc / "build").glob("*.o")) if p.name != "wavlm.o"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", str(o), *objs, "-o",
                           str(AT_LIB)])


def run():
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalemotionrecognition_amd import _lib
    _lib._LIB_PATH = AT_LIB
    from multimodalemotionrecognition_amd import kernels as K

    B, L, H, D = 32, 149, 12, 768
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B * L, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    x = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
    gw = torch.randn(8, 64, device="cuda", generator=g) * 0.1
    gb, gc = torch.zeros(8, device="cuda"), torch.ones(H, device="cuda")
    tbl = torch.randn(H, 2 * L - 1, device="cuda", generator=g)
    out = torch.empty(B * L, D, device="cuda", dtype=torch.bfloat16)
    rng = torch.full((1,), 77, dtype=torch.int64, device="cuda")
    for mode, p in (("eval", 0.0), ("train", 0.1)):
        for _ in range(5):
            K.wavlm_attention(qkv, x, gw, gb, gc, tbl, None, out, B, L, H, 0.125, drop_p=p, rng=rng if p else None)
        torch.cuda.synchronize()
        buf = np.zeros((2048, 8), dtype=np.int64)
        assert _lib.LIB._dll.mer_at_read(ctypes.c_void_p(buf.ctypes.data)) == 0
        nb = B * H * 2
        t = buf[:nb, :7].astype(np.float64) / 100.0  # 100 MHz -> us
        t0 = t[:, 0].min()
        print(f"{mode}: {nb} workgroups, kernel span {t[:, 6].max() - t0:.2f} us; block start offsets "
              f"median {np.median(t[:, 0] - t0):.2f} max {np.max(t[:, 0] - t0):.2f}; block durations median "
              f"{np.median(t[:, 6] - t[:, 0]):.2f} max {np.max(t[:, 6] - t[:, 0]):.2f}", flush=True)
        late = (t[:, 0] - t0) > 3.0
        hw = buf[:nb, 7]
        cu = ((hw >> 32) & 0xF) * 1000 + ((hw >> 13) & 0x7) * 100 + ((hw >> 8) & 0xF)  # xcc, se, cu
        u, c = np.unique(cu[~late], return_counts=True)
        print(f"   {late.sum()} workgroups start > 3 us after the first; first-round workgroups per CU: "
              f"{dict(zip(*np.unique(c, return_counts=True)))} over {len(u)} CUs", flush=True)
        for k, name in enumerate(PHASES):
            d = t[:, k + 1] - t[:, k]
            print(f"   {name:22s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f}",
                  flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
