"""Graph-vs-eager divergence hunt on one model: runs the trunk fwd/bwd twice eagerly and then graphed
on the same weights (no optimizer step), printing max differences per stage."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from multimodalemotionrecognition_amd import graphs as G  # noqa: E402
from multimodalemotionrecognition_amd.train import build_model, build_optimizer  # noqa: E402


def main():
    torch.manual_seed(7)
    m = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda()
    opt = build_optimizer(m)
    trunk = m.video_model.backbone
    video, audio, _ = bench.synthetic_batch(torch.device("cuda"), 5)
    x = video[:4].reshape(32, 3, 112, 112)
    res = []
    for it in range(4):
        G.ENABLED = it >= 2
        opt.zero_grad()
        # freeze BN running stats effects: eval-independent comparison of feats and grads
        f = trunk(x)
        g = torch.ones_like(f)
        f.backward(g)
        grads = {n: p.grad.detach().clone() for n, p in trunk.named_parameters() if p.grad is not None}
        res.append((f.detach().clone(), grads))
        torch.cuda.synchronize()
        print(it, "graphs" if G.ENABLED else "eager", "runners:", len(trunk._graphs.graphs), flush=True)
    f0, g0 = res[0]
    for it in range(1, 4):
        f, g = res[it]
        print(f"it{it}: feats max|d| {float((f - f0).abs().max()):.3e} (scale {float(f0.abs().max()):.3e})")
        worst = max(((float((g[n] - g0[n]).abs().max()) / max(1e-6, float(g0[n].abs().max())), n) for n in g0))
        print(f"it{it}: worst rel grad diff {worst[0]:.3e} at {worst[1]}  (missing: {set(g0) - set(g)})")
    a0 = m.audio_model.wavlm.forward_hip(audio[:4, 0])
    G.ENABLED = True
    for _ in range(3):
        a1 = m.audio_model.wavlm.forward_hip(audio[:4, 0])
    print("wavlm graph vs eager max|d|", float((a1.float() - a0.float()).abs().max()))
    # whole model forward, fixed weights: eager x2 then graphed x3 (fresh model: fresh graph caches)
    torch.manual_seed(7)
    m2 = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda()
    m2.attn_dropout = 0.0
    m2.v_drop_path.drop_prob = m2.a_drop_path.drop_prob = 0.0
    m2.xattn_mlp[2].p = 0.0
    outs = []
    for it in range(5):
        G.ENABLED = it >= 2
        with torch.no_grad():
            outs.append(m2(video[:4], audio[:4]).clone())
        torch.cuda.synchronize()
    for it in range(1, 5):
        print(f"model logits it{it} vs it0: max|d| {float((outs[it] - outs[0]).abs().max()):.3e}")


if __name__ == "__main__":
    main()
