"""Results must not depend on what runs beside a kernel on the other stream.

The train step runs the next batch's WavLM forward on a side stream while the main stream runs the trunk and the
fused xattn head.  With packed-fp32 VALU instructions in the library (v_pk_fma_f32 & co., which the compiler emitted
for the WavLM conv0 pass, GEMM epilogues, ...), the WavLM outputs changed whenever the head's kernels ran on the
same CUs (whole GroupNorm channels of conv0 shifted by up to 1.6; 17 of 20 replays of the conv-stack graph
differed); with the feature off (Makefile) every replay is bit-identical.  Bar: bit-identity,
eager launch by launch and for the captured graphs of a real train step."""
import pytest
import torch

from oracle import params as OP

pytestmark = pytest.mark.gpu


def _head_calls(m, B=4):
    """(fn, args, kwargs) of the fused head forward's F1 / F2 / F3 launches (xh_audio_fwd[_pair], xh_v2a_fwd, xh_a2v_fwd)."""
    from multimodalemotionrecognition_amd import kernels as K
    from multimodalemotionrecognition_amd import xattn_head as XH

    names, params = m.head_params()
    p = dict(zip(names, params))
    rec, orig = [], {}
    for n in ("xh_audio_fwd", "xh_audio_fwd_pair", "xh_v2a_fwd", "xh_a2v_fwd"):
        orig[n] = fn = getattr(K, n)

        def wrapped(*a, _fn=fn, **kw):
            rec.append((_fn, a, kw))
            return _fn(*a, **kw)
        setattr(K, n, wrapped)
    try:
        g = torch.Generator(device="cuda").manual_seed(3)
        v_feat = torch.randn(B, 8, 512, device="cuda", generator=g)
        a_seq = torch.randn(B, 149, 768, device="cuda", generator=g).to(torch.bfloat16)
        rng = torch.full((1,), 1234, dtype=torch.int64, device="cuda")
        with torch.no_grad():
            XH.head_forward(p, m.head_config(), v_feat, a_seq, True, rng)
    finally:
        for n, fn in orig.items():
            setattr(K, n, fn)
    torch.cuda.synchronize()
    return rec


def test_wavlm_launches_beside_head_kernels_bit_identical(monkeypatch):
    """Eager WavLM conv stack (0 encoder layers, train semantics): every launch synchronised and its tensor
    arguments kept; the disturbed run starts 4 head-kernel launches on another stream right before each WavLM
    launch.  Every launch's arguments must match the undisturbed run bit for bit."""
    from multimodalemotionrecognition_amd import graphs as G
    from multimodalemotionrecognition_amd import kernels as K
    from multimodalemotionrecognition_amd.train import build_model

    torch.manual_seed(0)
    m = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda().train()
    calls = _head_calls(m)
    side = torch.cuda.Stream()
    state = {"disturb": None, "rec": None}

    def wrap(fn):
        def w(*args, **kw):
            if state["disturb"] is not None:
                dfn, da, dkw = state["disturb"]
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(4):
                        dfn(*da, **dkw)
            r = fn(*args, **kw)
            torch.cuda.synchronize()
            state["rec"].append([t.clone() for t in list(args) + list(kw.values())
                                 if isinstance(t, torch.Tensor) and t.is_cuda])
            return r
        return w

    for n in ("gemm_bf16", "posconv_gemm_bf16", "wavlm_conv0_gn_gelu", "layernorm", "wavlm_time_mask", "bf16_convert"):
        monkeypatch.setattr(K, n, wrap(getattr(K, n)))
    monkeypatch.setattr(G, "ENABLED", False)
    _, a, _ = OP.clip_inputs(4, seed=9)
    wav = torch.from_numpy(a).cuda().squeeze(1)

    def run(disturb):
        state["disturb"], state["rec"] = disturb, []
        torch.manual_seed(5)
        with torch.no_grad():
            out = m.audio_model.wavlm.forward_hip(wav, out_dtype=torch.float32, num_layers=0).clone()
        torch.cuda.synchronize()
        return out, state["rec"]

    ref_out, ref = run(None)
    assert len(ref) >= 12
    for trial in range(3):
        for c in calls:
            out, rec = run(c)
            for i, (x, y) in enumerate(zip(ref, rec)):
                assert all(torch.equal(u, v) for u, v in zip(x, y)), (trial, i)
            assert torch.equal(out, ref_out)


def test_wavlm_graph_beside_head_graph_bit_identical():
    """The captured graphs of a real train step (late prefetch): the WavLM graph replayed on the side stream beside
    the head forward graph on the main stream equals its isolated replay, 12 times out of 12."""
    from multimodalemotionrecognition_amd import fusion as FU
    from multimodalemotionrecognition_amd import train as T

    early = T.EARLY_PREFETCH
    T.EARLY_PREFETCH = False
    try:
        B = 4
        batches = []
        for i in range(4):
            v, a, y = OP.clip_inputs(B, seed=500 + i)
            batches.append((torch.from_numpy(v).cuda(), torch.from_numpy(a).cuda(), torch.from_numpy(y).cuda()))
        torch.manual_seed(0)
        m = T.build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda()
        step = T.TrainStep(m, T.build_optimizer(m), T.make_loss("xattn"), "xattn")
        for i, (v, a, y) in enumerate(batches):
            step(v, a, y, next_audio=batches[(i + 1) % 4][1])
    finally:
        T.EARLY_PREFETCH = early
    torch.cuda.synchronize()
    wav = m.audio_model.wavlm
    w = batches[1][1].squeeze(1).contiguous()
    with torch.no_grad():
        for _ in range(2):  # eager warm-up, then capture: the 0-layer (conv stack) graph
            wav.forward_hip(w, num_layers=0)
    torch.cuda.synchronize()
    graphs = [g[0] for k, g in wav._graphs.graphs.items() if k[3] in (0, None)]
    hg = next(iter(m._head_graphs.graphs.values()))
    side = FU._side_stream(torch.device("cuda"))
    cur = torch.cuda.current_stream()
    assert len(graphs) == 2 and hg.fwd is not None
    for wg in graphs:
        wg.replay(wg.static_in[0])
        torch.cuda.synchronize()
        ref = wg.out.clone()
        bad = 0
        for _ in range(12):
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                wg.replay(wg.static_in[0])
            for _ in range(4):
                hg.fwd.replay(*hg.fwd.static_in)
            cur.wait_stream(side)
            torch.cuda.synchronize()
            bad += not torch.equal(wg.out, ref)
        assert bad == 0, bad
