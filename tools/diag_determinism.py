"""Determinism probe: the explicit TrainStep loop over 6 distinct B=4 batches, run twice per configuration;
prints per-step losses so the first diverging step shows.  argv: B, then configs "early,prefetch,off" where off
is a '+'-list of graph caches to disable (wavlm, trunk, head) or '-'."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import params as OP  # noqa: E402
from multimodalemotionrecognition_amd import train as T  # noqa: E402

B = int(sys.argv[1])
batches = []
for i in range(6):
    v, a, y = OP.clip_inputs(B, seed=500 + i)
    batches.append((torch.from_numpy(v).cuda(), torch.from_numpy(a).cuda(), torch.from_numpy(y).cuda()))


def run(prefetch, off):
    torch.manual_seed(0)
    m = T.build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda()
    caches = {"wavlm": m.audio_model.wavlm._graphs, "trunk": m.video_model.backbone._graphs, "head": m._head_graphs}
    for name in off:
        caches[name].ready = lambda key: False
    opt = T.build_optimizer(m)
    step = T.TrainStep(m, opt, T.make_loss("xattn"), "xattn")
    torch.manual_seed(1)
    out = []
    for i, (v, a, y) in enumerate(batches):
        nxt = batches[i + 1][1] if (prefetch and i + 1 < len(batches)) else None
        loss, _ = step(v, a, y, next_audio=nxt)
        out.append(float(loss))
    return out


for cfg in sys.argv[2:]:
    early, prefetch, off = cfg.split(",")
    T.EARLY_PREFETCH = early == "1"
    offl = [] if off == "-" else off.split("+")
    r1, r2, r3 = run(prefetch == "1", offl), run(prefetch == "1", offl), run(prefetch == "1", offl)
    same = [x == y == z for x, y, z in zip(r1, r2, r3)]
    print(f"{cfg}: same={same}", flush=True)
    print("   ", r1, "\n   ", r2, "\n   ", r3, flush=True)
