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
NAMES_FWD = {1: "F3 a2v_fwd", 2: "F1 audio_fwd", 3: "F2a v2a_attn"}
NAMES_BWD = {0: "G1 audio_bwd", 1: "W wgrad", 2: "G2b v2a_attn_bwd", 3: "G3 a2v_bwd"}
TICK_US = 0.01  # wall_clock64: 100 MHz


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
    def step():
        logits, ctx = XH.head_forward(p, cfg, v, a, True, rng)
        XH.head_backward(p, ctx, dl, grads, need_dv_feat=True)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    if "graph" in sys.argv[2:]:  # the stamps of a captured-graph replay (no host work between the launches)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    bwd = np.zeros((4, 512, 16), dtype=np.int64)
    fwd = np.zeros((4, 512, 16), dtype=np.int64)
    assert _lib.LIB._dll.mer_xt_read_bwd(ctypes.c_void_p(bwd.ctypes.data)) == 0
    assert _lib.LIB._dll.mer_xt_read_fwd(ctypes.c_void_p(fwd.ctypes.data)) == 0
    tabs = {("fwd", k): fwd[k] for k in NAMES_FWD} | {("bwd", k): bwd[k] for k in NAMES_BWD}
    names = {("fwd", k): v for k, v in NAMES_FWD.items()} | {("bwd", k): v for k, v in NAMES_BWD.items()}
    for key, t in tabs.items():
        for k0, sub in ((0, ""), (8, " (k 8+)")):  # F1 / G1: audio blocks stamp 0.., video blocks 8..
            used = [b for b in range(512) if t[b, k0] != 0]
            if not used:
                continue
            nph = max(k for k in range(k0, 12) if t[used[0], k] != 0)
            rows = []
            for k in range(k0 + 1, nph + 1):
                d = [(t[b, k] - t[b, k - 1]) * TICK_US for b in used if t[b, k] and t[b, k - 1]]
                rows.append(f"p{k} {np.median(d):6.2f}")
            tot = [(t[b, nph] - t[b, k0]) * TICK_US for b in used]
            span = (max(t[b, nph] for b in used) - min(t[b, k0] for b in used)) * TICK_US
            print(f"{names[key] + sub:22s} blocks {len(used):4d}  " + "  ".join(rows)
                  + f"  | block total {np.median(tot):6.2f} max {np.max(tot):6.2f}  span {span:6.2f} us")
    if "core" in sys.argv[2:]:
        core(tabs, names)


# the attention cores (QK^T, softmax, PV and their backward) inside the fused head's kernels: (table, first
# stamp, last stamp) of the attention phase and the kernel's last stamp
CORE = {("fwd", 3): (0, 4, 4), ("fwd", 1): (0, 1, 2), ("bwd", 2): (0, 4, 4), ("bwd", 3): (1, 2, 3)}


def core(tabs, names):
    """roofline_head.core_attn: for each of the four kernels that hold an attention core, the attention phase's
    share of the median block time x the kernel's span (first block entry to last block end) in this replay;
    written to gpurun_out/core_attn.json (committed as profiles/r06/core_attn.json, which bench.py reports)"""
    import json
    import numpy as np
    out, total = {}, 0.0
    for key, (a0, a1, last) in CORE.items():
        t = tabs[key]
        used = [b for b in range(512) if t[b, 0] != 0 and t[b, last] != 0]
        attn = np.median([(t[b, a1] - t[b, a0]) * TICK_US for b in used])
        blk = np.median([(t[b, last] - t[b, 0]) * TICK_US for b in used])
        span = (max(t[b, last] for b in used) - min(t[b, 0] for b in used)) * TICK_US
        us = span * attn / blk
        total += us
        out[names[key]] = {"blocks": len(used), "attn_phase_us_median": round(float(attn), 3),
                           "block_us_median": round(float(blk), 3), "kernel_span_us": round(float(span), 3),
                           "core_us": round(float(us), 3)}
    res = {"core_attn_us": round(total, 3), "kernels": out,
           "method": "tools/xt_phases.py run pair graph core: wall_clock64 phase stamps (-DMER_XH_TIMING library) of "
                     "one captured-graph replay of the fused head fwd+bwd at B=32, T=8, Ta=149; per kernel the "
                     "attention phase's share of the median block time times the kernel's span"}
    print(json.dumps(res, indent=1))
    dst = ROOT / "gpurun_out" / "core_attn.json"  # (copied to profiles/r06/ by hand: only gpurun_out/ comes back)
    if "save" in sys.argv[2:]:
        dst.write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
