"""Generate golden vectors by importing the REFERENCE implementation (build container only).

Run:  python tools/gen_golden.py   (needs /root/reference; never runs on the GPU box)

The reference's ``src/models/fusion.py`` / ``temporal.py`` are imported by path and
transformers' ``WavLMModel(WavLMConfig())`` is built offline (never ``from_pretrained``).
Weights and inputs come from ``oracle.params`` (numpy PCG64, name-keyed), so the GPU
box regenerates them bit-exactly without the reference.  Only inputs' seeds, the
expected outputs and selected intermediates are written to ``tests/golden/*.npz``.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch
from torch import nn

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
REF_SRC = Path("/root/reference/src")
sys.path.insert(0, str(REF_SRC))

from models.fusion import FusionModel  # noqa: E402  (reference)
from models.temporal import TemporalPooler  # noqa: E402  (reference)

from oracle import fusion_ref, params, wavlm_ref  # noqa: E402

OUT = ROOT / "tests" / "golden"
OUT.mkdir(parents=True, exist_ok=True)
torch.set_num_threads(8)


class IdentityBackbone(nn.Module):
    def forward(self, x):  # [N,512,1,1] -> [N,512,1,1]
        return x


class StubVideo(nn.Module):
    """Feature-level stand-in for VideoNet: backbone = identity, encode = identity on [B,512]."""

    def __init__(self, dim=512, num_classes=8):
        super().__init__()
        self.embedding_dim = dim
        self.backbone = IdentityBackbone()
        self.classifier = nn.Linear(dim, num_classes)

    def encode(self, x):
        return x

    def forward(self, x):
        return self.classifier(x)


class StubAudio(nn.Module):
    """Feature-level stand-in for WavLMAudioEncoder: encode_sequence / encode = identity."""

    def __init__(self, dim=768, num_classes=8):
        super().__init__()
        self.sequence_dim = dim
        self.embedding_dim = dim
        self.classifier = nn.Sequential(nn.Linear(dim, dim), nn.ReLU(inplace=True), nn.Dropout(0.2),
                                        nn.Linear(dim, num_classes))

    def encode_sequence(self, x):
        return x

    def encode(self, x):
        return x

    def forward(self, x):
        return self.classifier(x)


def load_numpy_init(module: nn.Module, seed: int = 0, fixups=None):
    sd = module.state_dict()
    new = {k: torch.from_numpy(params.init_tensor(k, tuple(v.shape), seed)) for k, v in sd.items()}
    if fixups:
        fixups(new)
    module.load_state_dict(new)
    return new


def head_names(model):
    return [(k, tuple(v.shape)) for k, v in model.state_dict().items()
            if not k.startswith(("audio_model.", "video_model."))]


def xattn_model(head="concat", prior=False, d_model=128, heads=4, v_dim=512, seq_dim=768, pooling="mean",
                t_heads=4, t_layers=1):
    m = FusionModel(StubAudio(seq_dim), StubVideo(v_dim), num_classes=8, mode="xattn", xattn_head=head,
                    d_model=d_model, num_heads=heads, audio_n_mels=768, xattn_use_emotion_prior=prior,
                    temporal_pooling=pooling, temporal_num_heads=t_heads, temporal_num_layers=t_layers,
                    temporal_dropout=0.0)
    return m


def gated_fix(head):
    def f(sd):
        if head == "gated":
            sd["xattn_gate.0.bias"].fill_(-1.0)
            sd["xattn_gate.3.bias"].fill_(-1.0)
    return f


def gen_xattn_c1():
    for head in ("concat", "gated"):
        for prior in (False, True):
            m = xattn_model(head, prior)
            expect = fusion_ref.xattn_head_param_shapes(xattn_head=head, use_prior=prior)
            got = head_names(m)
            assert got == expect, f"param listing mismatch: {set(got) ^ set(expect)}"
            load_numpy_init(m, 0, gated_fix(head))
            m.eval()
            v, a = params.feature_inputs(2, 8, 64)
            cap = {}
            m.v_norm.register_forward_hook(lambda mod, i, o: cap.__setitem__("v1", o.detach().clone()))
            m.a_norm.register_forward_hook(lambda mod, i, o: cap.__setitem__("a1", o.detach().clone()))
            with torch.no_grad():
                logits = m(torch.from_numpy(v)[..., None, None], torch.from_numpy(a))
            assert tuple(logits.shape) == (2, 8)
            np.savez_compressed(OUT / f"xattn_c1_{head}_prior{int(prior)}.npz", logits=logits.numpy(),
                                v1=cap["v1"].numpy(), a1=cap["a1"].numpy(), batch=2, t=8, ta=64,
                                seed=20261015)
            print("xattn c1", head, prior, logits[0, :3])


def gen_xattn_c2_grads():
    """C2-shape head (B=32, T=8, Ta=149): eval logits, CE-loss grads, one Adam step."""
    for head, prior in (("concat", False), ("concat", True), ("gated", False)):
        m = xattn_model(head, prior)
        load_numpy_init(m, 0, gated_fix(head))
        m.eval()
        v, a = params.feature_inputs(32, 8, 149, seed=7)
        labels = torch.from_numpy(np.random.Generator(np.random.PCG64(8)).integers(0, 8, 32))
        vt = torch.from_numpy(v)[..., None, None].requires_grad_(True)
        at = torch.from_numpy(a).requires_grad_(True)
        logits = m(vt, at)
        loss = nn.CrossEntropyLoss()(logits, labels)
        loss.backward()
        out = {"logits": logits.detach().numpy(), "loss": np.float32(loss.item()), "labels": labels.numpy(),
               "grad_v": vt.grad[:2, :, :, 0, 0].numpy(), "grad_a": at.grad[:2].numpy()}
        trainable = [(n, q) for n, q in m.named_parameters()
                     if q.grad is not None and not n.startswith(("audio_model.", "video_model."))]
        for n, q in trainable:
            out["grad." + n] = q.grad.numpy().copy()
        opt = torch.optim.Adam([q for _, q in trainable], lr=1e-3, weight_decay=1e-4)
        opt.step()
        for n, q in trainable:
            out["adam1." + n] = q.detach().numpy().copy()
        if head != "concat" or prior:  # keep fixture size small: full grads only for the default config
            out = {k: v for k, v in out.items() if not k.startswith(("grad", "adam1."))}
        np.savez_compressed(OUT / f"xattn_c2_{head}_prior{int(prior)}.npz", **out)
        print("xattn c2", head, prior, float(loss.detach()))


def gen_small_shapes():
    """Shapes of the reference's own tests (test_attention_integration.py:80-125): d_model=8, heads=2."""
    for pooling in ("mean", "attn", "transformer"):
        m = xattn_model("concat", False, d_model=8, heads=2, v_dim=16, seq_dim=8, pooling=pooling, t_heads=2)
        load_numpy_init(m, 0)
        m.eval()
        v, a = params.feature_inputs(2, 4, 12, v_dim=16, a_dim=8, seed=11)
        with torch.no_grad():
            logits = m(torch.from_numpy(v)[..., None, None], torch.from_numpy(a))
        assert tuple(logits.shape) == (2, 8)
        np.savez_compressed(OUT / f"xattn_small_{pooling}.npz", logits=logits.numpy())
    x = torch.from_numpy(params.feature_inputs(2, 5, 1, v_dim=8, seed=12)[0])
    for mode in ("mean", "attn", "transformer"):
        pool = TemporalPooler(dim=8, mode=mode, num_heads=2, num_layers=1, dropout=0.0)
        load_numpy_init(pool, 0)
        pool.eval()
        with torch.no_grad():
            y = pool(x)
        np.savez_compressed(OUT / f"temporal_{mode}.npz", x=x.numpy(), y=y.numpy(),
                            names=np.array([k for k in pool.state_dict().keys()]))


def gen_c4_heads():
    """late / concat / gated at feature level (fusion.py:358-363, 413-435)."""
    rng = np.random.Generator(np.random.PCG64(13))
    a_emb = rng.standard_normal((4, 768)).astype(np.float32)
    v_emb = rng.standard_normal((4, 512)).astype(np.float32)
    for mode in ("late", "concat", "gated"):
        m = FusionModel(StubAudio(), StubVideo(), num_classes=8, mode=mode)

        def fix(sd):
            if mode == "gated":
                sd["gate.0.bias"].fill_(-1.0)
                sd["gate.3.bias"].fill_(-1.0)
        load_numpy_init(m, 0, fix)
        m.eval()
        with torch.no_grad():
            out = m(torch.from_numpy(v_emb), torch.from_numpy(a_emb))
        np.savez_compressed(OUT / f"c4_{mode}.npz", a_emb=a_emb, v_emb=v_emb, out=out.numpy(),
                            names=np.array(list(m.state_dict().keys())))
        print("c4", mode, out[0, :3])


def gen_int8_head():
    """C5 reference: CPU dynamic INT8 (optimized_runtime.py:95-96) of the xattn head at B=64."""
    m = xattn_model("concat", False)
    load_numpy_init(m, 0)
    m.eval()
    v, a = params.feature_inputs(64, 8, 149, seed=21)
    vt, at = torch.from_numpy(v)[..., None, None], torch.from_numpy(a)
    with torch.no_grad():
        fp = m(vt, at)
    q = torch.ao.quantization.quantize_dynamic(m, {nn.Linear}, dtype=torch.qint8)
    with torch.no_grad():
        lq = q(vt, at)
    quantized = sorted(n for n, mod in q.named_modules() if type(mod).__name__ == "Linear" and "quantized" in type(mod).__module__)
    np.savez_compressed(OUT / "int8_head_b64.npz", logits_fp32=fp.numpy(), logits_int8=lq.numpy(),
                        quantized=np.array(quantized))
    print("int8", (fp - lq).abs().max().item(), (fp.argmax(1) == lq.argmax(1)).float().mean().item(), quantized)


def gen_wavlm():
    from transformers import WavLMConfig, WavLMModel
    m = WavLMModel(WavLMConfig())
    expect = wavlm_ref.wavlm_param_shapes()
    got = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    assert sorted(got) == sorted(expect), set(got) ^ set(expect)
    load_numpy_init(m, 0)
    m.eval()
    _, audio, _ = params.clip_inputs(2, seed=31)
    cap = {}
    m.encoder.layers[0].register_forward_hook(lambda mod, i, o: cap.__setitem__("layer0", o[0].detach().clone()))
    with torch.no_grad():
        out = m(torch.from_numpy(audio).squeeze(1))
    np.savez_compressed(OUT / "wavlm_b2.npz", last_hidden=out.last_hidden_state.numpy(),
                        extract_features=out.extract_features.numpy(), layer0=cap["layer0"].numpy())
    print("wavlm", out.last_hidden_state.shape, out.last_hidden_state[0, 0, :3])


def gen_c4_clip():
    """concat / gated with fusion_align_mode="clip" (fusion.py:127-150, 417-418) at feature level, eval mode
    (no dropout, no ModalityDropout): logits, the alignment loss and the gradients of
    CE(logits) + 0.5 * align_loss (train.py:221-225) w.r.t. every head parameter and both inputs."""
    rng = np.random.Generator(np.random.PCG64(41))
    a_emb = rng.standard_normal((6, 768)).astype(np.float32)
    v_emb = rng.standard_normal((6, 512)).astype(np.float32)
    labels = torch.from_numpy(rng.integers(0, 8, 6))
    for mode in ("concat", "gated"):
        m = FusionModel(StubAudio(), StubVideo(), num_classes=8, mode=mode, fusion_align_mode="clip",
                        fusion_align_dim=256, fusion_align_temperature=0.07)

        def fix(sd):
            sd["semantic_alignment.logit_scale"].fill_(float(np.log(1.0 / 0.07)))
            if mode == "gated":
                sd["gate.0.bias"].fill_(-1.0)
                sd["gate.3.bias"].fill_(-1.0)
        load_numpy_init(m, 0, fix)
        m.eval()
        at = torch.from_numpy(a_emb).requires_grad_(True)
        vt = torch.from_numpy(v_emb).requires_grad_(True)
        logits = m(vt, at)
        align = m.pop_alignment_loss()
        loss = nn.CrossEntropyLoss()(logits, labels) + 0.5 * align
        loss.backward()
        out = {"a_emb": a_emb, "v_emb": v_emb, "labels": labels.numpy(), "logits": logits.detach().numpy(),
               "align": np.float32(align.item()), "loss": np.float32(loss.item()),
               "grad_a": at.grad.numpy(), "grad_v": vt.grad.numpy(), "names": np.array(list(m.state_dict().keys()))}
        for n, q in m.named_parameters():
            if q.grad is not None and not n.startswith(("audio_model.", "video_model.")):
                out["grad." + n] = q.grad.numpy().copy()
        np.savez_compressed(OUT / f"c4_clip_{mode}.npz", **_trim(out))
        print("c4 clip", mode, float(align), float(loss))


def gen_int8_head_prior():
    """C5 INT8 with the emotion-prior adapter: quantize_dynamic({nn.Linear}) also quantizes prior_net and the
    four token-bias Linears (optimized_runtime.py:95-96)."""
    m = xattn_model("concat", True)
    load_numpy_init(m, 0)
    m.eval()
    v, a = params.feature_inputs(64, 8, 149, seed=22)
    vt, at = torch.from_numpy(v)[..., None, None], torch.from_numpy(a)
    with torch.no_grad():
        fp = m(vt, at)
    q = torch.ao.quantization.quantize_dynamic(m, {nn.Linear}, dtype=torch.qint8)
    with torch.no_grad():
        lq = q(vt, at)
    quantized = sorted(n for n, mod in q.named_modules() if type(mod).__name__ == "Linear" and "quantized" in type(mod).__module__)
    np.savez_compressed(OUT / "int8_head_prior_b64.npz", logits_fp32=fp.numpy(), logits_int8=lq.numpy(),
                        quantized=np.array(quantized))
    print("int8 prior", (fp - lq).abs().max().item(), (fp.argmax(1) == lq.argmax(1)).float().mean().item(), quantized)


def gen_encoder_transformer_pool():
    """TemporalPooler('transformer', num_heads=4) at the encoders' widths (train.py:357-443 passes
    temporal_pooling into both encoders): VideoNet.encode at 512 (head_dim 128) over T=8 frames and
    WavLMAudioEncoder.encode at 768 (head_dim 192) over Ta=149 frames; eval mode, plus input / parameter
    gradients of sum(y * w) for a fixed w."""
    for dim, length, seed in ((512, 8, 51), (768, 149, 52)):
        pool = TemporalPooler(dim=dim, mode="transformer", num_heads=4, num_layers=1, dropout=0.1)
        load_numpy_init(pool, 0)
        pool.eval()
        x = torch.from_numpy(params.feature_inputs(3, length, 1, v_dim=dim, seed=seed)[0]).requires_grad_(True)
        y = pool(x)
        w = torch.from_numpy(np.random.Generator(np.random.PCG64(seed + 100)).standard_normal(tuple(y.shape))
                             .astype(np.float32))
        (y * w).sum().backward()
        out = {"x": x.detach().numpy(), "y": y.detach().numpy(), "w": w.numpy(), "grad_x": x.grad.numpy(),
               "names": np.array(list(pool.state_dict().keys()))}
        for n, q in pool.named_parameters():
            out["grad." + n] = q.grad.numpy().copy()
        np.savez_compressed(OUT / f"temporal_transformer_d{dim}.npz", **_trim(out))
        print("transformer pool", dim, y[0, :3])


def _trim(out, limit=16384, rows=8):
    """Keep fixtures small: a gradient larger than ``limit`` elements is stored as its first ``rows`` rows plus
    its column sums and row sums (``<key>.head`` / ``.colsum`` / ``.rowsum``)."""
    res = {}
    for k, v in out.items():
        if k.startswith("grad.") and isinstance(v, np.ndarray) and v.size > limit and v.ndim == 2:
            res[k + ".head"] = v[:rows].copy()
            res[k + ".colsum"] = v.sum(0, dtype=np.float64).astype(np.float32)
            res[k + ".rowsum"] = v.sum(1, dtype=np.float64).astype(np.float32)
        else:
            res[k] = v
    return res


GENERATORS = dict(xattn_c1=gen_xattn_c1, xattn_c2=gen_xattn_c2_grads, small=gen_small_shapes, c4=gen_c4_heads,
                  int8=gen_int8_head, wavlm=gen_wavlm, c4_clip=gen_c4_clip, int8_prior=gen_int8_head_prior,
                  enc_transformer=gen_encoder_transformer_pool)

if __name__ == "__main__":
    for name in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[name]()
