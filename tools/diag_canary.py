"""Out-of-bounds write hunt for the fused xattn head: every torch.empty the head schedule allocates (eager, no graph)
gets PAD extra elements filled with a canary pattern; after the forward and after the backward each allocation's pad
must be intact.  Prints the allocation shape / call site of every damaged pad."""
import sys
import traceback
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from tests.gpu_helpers import feats, head_model  # noqa: E402
from multimodalemotionrecognition_amd import xattn_head as XH  # noqa: E402
from multimodalemotionrecognition_amd.fusion import _head_grads  # noqa: E402

PAD = 4096
_orig_empty = torch.empty
records = []


def _empty(*shape, device=None, dtype=None, **kw):
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    dt = dtype if dtype is not None else torch.float32
    n = 1
    for s in shape:
        n *= int(s)
    if device is None or torch.device(device).type != "cuda":
        return _orig_empty(*shape, device=device, dtype=dt, **kw)
    base = _orig_empty(n + PAD, device=device, dtype=dt)
    base[n:].fill_(-123456.75 if dt.is_floating_point else 0x5A)
    where = [f"{f.name}:{f.lineno}" for f in traceback.extract_stack()[-4:-1]]
    records.append((base, n, tuple(shape), where))
    return base[:n].view(*shape) if shape else base[:1].view(())


def check(tag):
    torch.cuda.synchronize()
    bad = 0
    for base, n, shape, where in records:
        pad = base[n:]
        ref = torch.full_like(pad, -123456.75 if pad.dtype.is_floating_point else 0x5A)
        if not torch.equal(pad, ref):
            k = int((pad != ref).nonzero()[0])
            print(f"{tag}: OOB write past {shape} {pad.dtype} (first damaged pad element {k}) allocated at {where}",
                  flush=True)
            bad += 1
    print(f"{tag}: {len(records)} allocations checked, {bad} damaged", flush=True)


for head in ("concat", "gated"):
    for prior in (False, True):
        m = head_model(head, prior).train(True)
        names, params = m.head_params()
        p = dict(zip(names, params))
        cfg = m.head_config()
        v, a = feats(32, 8, 149, seed=7)
        a = a.to(torch.bfloat16)
        rng = torch.full((1,), 4242, dtype=torch.int64, device="cuda")
        grads = {n: torch.zeros_like(t) for n, t in _head_grads(p, set(XH.used_param_names(cfg))).items()}
        torch.empty = _empty
        try:
            records.clear()
            logits, ctx = XH.head_forward(p, cfg, v, a, True, rng)
            check(f"{head} prior={prior} forward")
            dl = torch.from_numpy(np.random.default_rng(1).standard_normal(tuple(logits.shape)).astype(np.float32)).cuda()
            XH.head_backward(p, ctx, dl, grads, need_dv_feat=True)
            check(f"{head} prior={prior} forward+backward")
        finally:
            torch.empty = _orig_empty
