"""Phase timing of the fused head kernels: builds multimodalemotionrecognition_amd/libmer_hip_xt.so (the kernel
library with -DMER_XH_TIMING, see XT() in csrc/xattn_common.h), runs one fused head forward + backward through
it and prints, per instrumented kernel, the median over workgroups of each phase's duration (us, wall clock).
    python tools/xt_phases.py build      (here: hipcc, no GPU)
    python tools/xt_phases.py run        (GPU box)"""
import ctypes
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodalemotionrecognition_amd"
XT_LIB = PKG / "libmer_hip_xt.so"
NAMES = {0: "G1 audio_bwd", 1: "W wgrad", 2: "F1 audio_fwd", 3: "F2 v2a_fwd"}


def build():
    csrc = PKG / "csrc"
    out = csrc / "build" / "xt"
    out.mkdir(parents=True, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-DMER_XH_TIMING", f"-I{ROOT / 'include'}",
             "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
    xt_objs = []
    for name in ("xattn_fused", "xattn_fused_bwd"):
        o = out / f"{name}.o"
        subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", str(csrc / f"{name}.hip"), "-o", str(o)])
        xt_objs.append(str(o))
    objs = [str(o) for o in sorted((csrc / "build").glob("*.o")) if not o.name.startswith("xattn_fused")]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *xt_objs, *objs, "-o",
                           str(XT_LIB)])


def run():
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalemotionrecognition_amd import _lib
    _lib._LIB_PATH = XT_LIB  # the instrumented library (this tool only)
    sys.path.insert(0, str(ROOT))
    from multimodalemotionrecognition_amd import xattn_head as XH
    from multimodalemotionrecognition_amd.fusion import _head_grads
    from tests.gpu_helpers import feats, head_model
    from multimodalemotionrecognition_amd import xattn_fused as XF
    XF.F1_PAIR = "nopair" not in sys.argv[2:]
    m = head_model("concat", False).train(True)
    names, params = m.head_params()
    p = dict(zip(names, params))
    cfg = m.head_config()
    v, a = feats(32, 8, 149, seed=7)
    a = a.to(torch.bfloat16)
    rng = torch.full((1,), 4242, dtype=torch.int64, device="cuda")
    grads = {n: torch.zeros_like(t) for n, t in _head_grads(p, set(XH.used_param_names(cfg))).items()}
    dl = torch.randn(32, 8, device="cuda")
    for _ in range(5):
        logits, ctx = XH.head_forward(p, cfg, v, a, True, rng)
        XH.head_backward(p, ctx, dl, grads, need_dv_feat=True)
    torch.cuda.synchronize()
    buf = np.zeros((4, 512, 16), dtype=np.int64)
    fwd = np.zeros((4, 512, 16), dtype=np.int64)
    assert _lib.LIB._dll.mer_xt_read_bwd(ctypes.c_void_p(buf.ctypes.data)) == 0
    assert _lib.LIB._dll.mer_xt_read_fwd(ctypes.c_void_p(fwd.ctypes.data)) == 0
    buf[2] = fwd[2]
    buf[3] = fwd[3]
    tick_us = 0.01  # wall_clock64: 100 MHz
    for slot, name in NAMES.items():
        t = buf[slot]
        for k0, sub in ((0, ""), (8, " (k 8+)")):  # F1: audio blocks stamp 0-3, video blocks 8-10
            used = [b for b in range(512) if t[b, k0] != 0]
            if not used:
                continue
            nph = max(k for k in range(k0, 16) if t[used[0], k] != 0)
            rows = []
            for k in range(k0 + 1, nph + 1):
                d = [(t[b, k] - t[b, k - 1]) * tick_us for b in used if t[b, k] and t[b, k - 1]]
                rows.append(f"p{k} {np.median(d):6.2f}")
            tot = [(t[b, nph] - t[b, k0]) * tick_us for b in used]
            span = (max(t[b, nph] for b in used) - min(t[b, k0] for b in used)) * tick_us
            print(f"{name + sub:22s} blocks {len(used):4d}  " + "  ".join(rows)
                  + f"  | block total {np.median(tot):6.2f} max {np.max(tot):6.2f}  span {span:6.2f} us")

if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
