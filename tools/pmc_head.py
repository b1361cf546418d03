"""HBM traffic and MFMA utilisation of the fused xattn head (csrc/xattn_fused*.hip) from rocprofv3 --pmc passes.

    python tools/pmc_head.py run                    (GPU box, under rocprofv3 --pmc ...: ITERS eager fused
                                                     forward + backward steps at the C2 shapes, after 3 warm-ups)
    python tools/pmc_head.py summarize <pmc dir>    (here: per-step and per-kernel sums of every head kernel)

One pass per counter group (rocprofv3 does not split counters over passes): FETCH_SIZE; WRITE_SIZE;
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE.  HBM bytes = 1024 * (2 * FETCH_SIZE + WRITE_SIZE) (FETCH doubled: the
gfx950 correction of MI355X_MICROARCH.md 'HBM'); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x
GRBM_GUI_ACTIVE / 8), per kernel."""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
ITERS = 5
HEAD_KERNELS = ("xh_", "ce_kernel", "gemm_pipe_kernel")  # (the head's F1 pair product is a bf16 GEMM)


def run():
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalemotionrecognition_amd import xattn_head as XH
    from multimodalemotionrecognition_amd.fusion import _head_grads
    from tests.gpu_helpers import feats, head_model

    m = head_model("concat", False).train(True)
    names, params = m.head_params()
    p = dict(zip(names, params))
    cfg = m.head_config()
    v, a = feats(32, 8, 149, seed=7)
    a = a.to(torch.bfloat16)
    rng = torch.full((1,), 4242, dtype=torch.int64, device="cuda")
    grads = {n: torch.zeros_like(t) for n, t in _head_grads(p, set(XH.used_param_names(cfg))).items()}
    dl = torch.from_numpy(np.random.default_rng(1).standard_normal((32, 8)).astype(np.float32)).cuda()
    for _ in range(3 + ITERS):
        logits, ctx = XH.head_forward(p, cfg, v, a, True, rng)
        XH.head_backward(p, ctx, dl, grads, need_dv_feat=True)
    torch.cuda.synchronize()
    print(f"ran {3 + ITERS} fused head steps", flush=True)


def kernel_key(full: str) -> str:
    """Kernel name without its argument list, return type and namespace: a demangled name can begin with
    "void (anonymous namespace)::...", whose FIRST "(" is the namespace's, not the argument list's -- cutting there
    dropped every anonymous-namespace kernel (F1's bf16 GEMM among them) from the sums."""
    name = full.replace("(anonymous namespace)::", "")
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):  # the argument list is the first "(" outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    name = name[:cut]
    return name[5:] if name.startswith("void ") else name


def summarize(root):
    per = defaultdict(lambda: defaultdict(float))   # kernel -> counter -> sum over dispatches
    disp = defaultdict(set)
    mfma = defaultdict(list)
    rows = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = kernel_key(r["Kernel_Name"])
            if not any(k in name for k in HEAD_KERNELS):
                continue
            rows[(r["Dispatch_Id"], name)][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add(r["Dispatch_Id"])
    for (d, name), c in rows.items():
        for k, v in c.items():
            per[name][k] += v
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            mfma[name].append(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * c["GRBM_GUI_ACTIVE"] / 8.0))
    steps = 3 + ITERS  # every dispatch of the run (warm-ups included: same work)
    out = {"steps": steps, "kernels": {}}
    tot_f = tot_w = 0.0
    for name, c in sorted(per.items()):
        f_kb, w_kb = c.get("FETCH_SIZE", 0.0) / steps, c.get("WRITE_SIZE", 0.0) / steps
        tot_f, tot_w = tot_f + f_kb, tot_w + w_kb
        out["kernels"][name] = {"hbm_bytes_per_step": int(1024 * (2 * f_kb + w_kb)),
                                "mfma_busy_frac": round(sum(mfma[name]) / len(mfma[name]), 4) if mfma[name] else None}
    out["fetch_kb_raw_per_step"] = tot_f
    out["write_kb_per_step"] = tot_w
    out["traffic_bytes_per_step"] = int(1024 * (2 * tot_f + tot_w))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2])
