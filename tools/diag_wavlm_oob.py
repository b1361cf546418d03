"""Out-of-bounds READ hunt for the WavLM forward: every torch.empty the (eager) forward allocates gets PAD trailing
elements filled with NaN (bf16 / fp32); if any kernel reads past the end of a buffer and the value reaches an output,
the hidden states turn non-finite or differ from the normally allocated run.  Also checks the conv-stack and layer-0
intermediates."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import params as OP  # noqa: E402
from multimodalemotionrecognition_amd import graphs as G  # noqa: E402
from multimodalemotionrecognition_amd.wavlm_audio import WavLMAudioEncoder  # noqa: E402

G.ENABLED = False  # eager: every intermediate is a fresh (padded) allocation
PAD = 1 << 16
_orig_empty = torch.empty


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
    if dt.is_floating_point:
        base[n:].fill_(float("nan"))
    else:
        base[n:].fill_(-1)
    return base[:n].view(*shape) if shape else base[:1].view(())


torch.manual_seed(0)
enc = WavLMAudioEncoder(num_classes=8).cuda().train()
for sem in (False, True):
    enc.wavlm.train_semantics = sem
    _, a, _ = OP.clip_inputs(4, seed=9)
    a = torch.from_numpy(a).cuda()
    torch.manual_seed(5)
    cap0 = {}
    with torch.no_grad():
        ref = enc.wavlm.forward_hip(a.squeeze(1), out_dtype=torch.float32, capture=cap0).clone()
    torch.empty = _empty
    try:
        torch.manual_seed(5)
        cap1 = {}
        with torch.no_grad():
            out = enc.wavlm.forward_hip(a.squeeze(1), out_dtype=torch.float32, capture=cap1).clone()
    finally:
        torch.empty = _orig_empty
    torch.cuda.synchronize()
    print(f"train_semantics={sem}: output finite {bool(torch.isfinite(out).all())}, max|d| vs unpadded "
          f"{float((out - ref).abs().nan_to_num(1e30).max()):.3e}", flush=True)
    for k in cap0:
        d = (cap1[k].float() - cap0[k].float()).abs().nan_to_num(1e30).max()
        print(f"   {k}: finite {bool(torch.isfinite(cap1[k].float()).all())} max|d| {float(d):.3e}", flush=True)
