"""Localise a run-to-run difference of the late-prefetch schedule (TrainStep with next_audio, early prefetch off):
two identical 6-step runs; after every step the WavLM features the step consumed, the logits and every flat
gradient are compared; prints the first step / tensors that differ."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import params as OP  # noqa: E402
from multimodalemotionrecognition_amd import fusion as FU  # noqa: E402
from multimodalemotionrecognition_amd import train as T  # noqa: E402

import gc

B = 4
early = sys.argv[1] == "1" if len(sys.argv) > 1 else False
GC = sys.argv[2] if len(sys.argv) > 2 else "auto"   # auto | off | each (collect after every step)
if GC == "off":
    gc.disable()
T.EARLY_PREFETCH = early
batches = []
for i in range(6):
    v, a, y = OP.clip_inputs(B, seed=500 + i)
    batches.append((torch.from_numpy(v).cuda(), torch.from_numpy(a).cuda(), torch.from_numpy(y).cuda()))


from multimodalemotionrecognition_amd import graphs as G  # noqa: E402
import traceback  # noqa: E402

_CAP = {"step": -1}
_orig_init = G.StaticGraph.__init__


def _spy_init(self, fn, ex, stream=None):
    where = [f"{f.name}:{f.lineno}" for f in traceback.extract_stack()[-6:-1]]
    print(f"   capture at step {_CAP['step']}: {where}", flush=True)
    _orig_init(self, fn, ex, stream)


G.StaticGraph.__init__ = _spy_init

SERIAL = sys.argv[3] if len(sys.argv) > 3 else "none"   # none | after_prefetch (main waits for the WavLM)
if SERIAL == "after_prefetch":
    _orig_pf = FU.FusionModel.prefetch_audio

    def _pf(self, audio):
        r = _orig_pf(self, audio)
        torch.cuda.current_stream().wait_stream(FU._side_stream(audio.device))
        return r

    FU.FusionModel.prefetch_audio = _pf


def _wait_side():
    torch.cuda.current_stream().wait_stream(FU._side_stream(torch.device("cuda")))


if SERIAL == "before_adam":  # the WavLM overlaps the head + trunk backward only
    from multimodalemotionrecognition_amd import optim as OPT
    _orig_step = OPT.FusedAdam.step

    def _st(self, closure=None):
        _wait_side()
        return _orig_step(self, closure)

    OPT.FusedAdam.step = _st
if SERIAL == "before_trunk_bwd":  # the WavLM overlaps the head backward only
    from multimodalemotionrecognition_amd import video as VI
    _orig_tb = VI._TrunkGraphs.backward

    def _tb(self, dfeat, params):
        _wait_side()
        return _orig_tb(self, dfeat, params)

    VI._TrunkGraphs.backward = _tb
if SERIAL == "before_head_bwd":  # the WavLM overlaps the CE backward only
    _orig_hb = FU._HeadGraphs.backward

    def _hb(self, dlogits):
        _wait_side()
        return _orig_hb(self, dlogits)

    FU._HeadGraphs.backward = _hb


def run():
    torch.manual_seed(0)
    m = T.build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda()
    opt = T.build_optimizer(m)
    names = {id(q): n for n, q in m.named_parameters()}
    step = T.TrainStep(m, opt, T.make_loss("xattn"), "xattn")
    seen = []
    orig = FU.FusionModel.xattn_from_features

    def spy(self, v_feat, a_seq):
        seen.append((v_feat.detach().float().clone(), a_seq.detach().float().clone()))
        return orig(self, v_feat, a_seq)

    FU.FusionModel.xattn_from_features = spy
    torch.manual_seed(1)
    rec = []
    try:
        for i, (v, a, y) in enumerate(batches):
            _CAP["step"] = i
            nxt = batches[i + 1][1] if i + 1 < len(batches) else None
            loss, _ = step(v, a, y, next_audio=nxt)
            torch.cuda.synchronize()
            if GC == "each":
                n = gc.collect()
                print(f"   step {i}: gc collected {n}", flush=True)
            grads = {names[id(p)]: p.grad.detach().clone() for _, p, _, _ in opt.param_slices() if p.grad is not None}
            pf = m._prefetched[2].detach().float().clone() if m._prefetched is not None else None
            aud = [float(b[1].double().sum()) for b in batches]
            rec.append((float(loss), seen[-1], grads, [f.clone() for f in opt.flat_params()], pf, aud))
    finally:
        FU.FusionModel.xattn_from_features = orig
    return rec


r1, r2 = run(), run()
for i, (a, b) in enumerate(zip(r1, r2)):
    dv = float((a[1][0] - b[1][0]).abs().max())
    da = float((a[1][1] - b[1][1]).abs().max())
    dg = [n for n in a[2] if not torch.equal(a[2][n], b[2][n])]
    dp = [j for j, (x, y) in enumerate(zip(a[3], b[3])) if not torch.equal(x, y)]
    dpf = float((a[4] - b[4]).abs().max()) if a[4] is not None else -1
    print(f"step {i}: loss {a[0]} {b[0]}  |d v_feat| {dv:.3e} |d a_seq| {da:.3e}  grads differing {len(dg)} "
          f"{dg[:6]}  params differ {dp}  |d prefetched-at-end| {dpf:.3e}  audio sums equal {a[5] == b[5]}", flush=True)
# the prefetched features at the end of each step vs WavLM alone on that batch (same host draws are not
# reproducible here, so compare eval semantics only when train semantics are off)
