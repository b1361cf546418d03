"""Pin the CPU oracle against golden vectors produced by the imported reference.

These run on CPU only (no GPU) and are the reason the oracle can be trusted as the
parity checker for the HIP path.  Goldens: ``tools/gen_golden.py``.
"""
import numpy as np
import pytest
import torch

from oracle import fusion_ref, params, resnet18_ref, wavlm_ref
from tests.helpers import check_grad, clip_head_params, golden, torch_state, xattn_params


@pytest.mark.parametrize("head", ["concat", "gated"])
@pytest.mark.parametrize("prior", [0, 1])
def test_xattn_c1_logits(head, prior):
    g = golden(f"xattn_c1_{head}_prior{prior}.npz")
    p = xattn_params(head, bool(prior))
    v, a = params.feature_inputs(2, 8, 64)
    logits, inter = fusion_ref.xattn_forward(p, torch.from_numpy(v), torch.from_numpy(a),
                                             xattn_head=head, use_prior=bool(prior))
    assert tuple(logits.shape) == (2, 8)
    np.testing.assert_allclose(logits.numpy(), g["logits"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(inter["v1"].numpy(), g["v1"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(inter["a1"].numpy(), g["a1"], rtol=0, atol=2e-5)


def test_xattn_c2_grads_and_adam():
    g = golden("xattn_c2_concat_prior0.npz")
    p = xattn_params("concat", False)
    v, a = params.feature_inputs(32, 8, 149, seed=7)
    vt = torch.from_numpy(v).requires_grad_(True)
    at = torch.from_numpy(a).requires_grad_(True)
    used = [k[len("grad."):] for k in g.files if k.startswith("grad.")]
    for k in used:
        p[k].requires_grad_(True)
    logits, _ = fusion_ref.xattn_forward(p, vt, at)
    loss = fusion_ref.cross_entropy(logits, torch.from_numpy(g["labels"]))
    loss.backward()
    np.testing.assert_allclose(logits.detach().numpy(), g["logits"], atol=3e-5)
    assert abs(float(loss.detach()) - float(g["loss"])) < 1e-5
    np.testing.assert_allclose(vt.grad[:2].numpy(), g["grad_v"], atol=1e-6)
    np.testing.assert_allclose(at.grad[:2].numpy(), g["grad_a"], atol=1e-6)
    for k in used:
        np.testing.assert_allclose(p[k].grad.numpy(), g["grad." + k], atol=2e-6, err_msg=k)
    # unused head params get no gradient, exactly like the reference (audio_time_conv is dead)
    assert "audio_time_conv.weight" not in used
    from oracle.train_ref import AdamRef
    opt = AdamRef([p[k] for k in used], lr=1e-3, weight_decay=1e-4)
    opt.step()
    for k in used:
        # first Adam step is ~lr*sign(g): elements with |g|~eps are sensitive to 1e-9 grad noise
        np.testing.assert_allclose(p[k].detach().numpy(), g["adam1." + k], atol=5e-5, err_msg=k)


@pytest.mark.parametrize("head,prior", [("concat", 1), ("gated", 0)])
def test_xattn_c2_variants(head, prior):
    g = golden(f"xattn_c2_{head}_prior{prior}.npz")
    p = xattn_params(head, bool(prior))
    v, a = params.feature_inputs(32, 8, 149, seed=7)
    logits, _ = fusion_ref.xattn_forward(p, torch.from_numpy(v), torch.from_numpy(a), xattn_head=head,
                                         use_prior=bool(prior))
    np.testing.assert_allclose(logits.numpy(), g["logits"], atol=3e-5)


@pytest.mark.parametrize("pooling", ["mean", "attn", "transformer"])
def test_small_shapes_reference_tests(pooling):
    """d_model=8, heads=2 as in test_attention_integration.py:80-125."""
    g = golden(f"xattn_small_{pooling}.npz")
    p = torch_state(fusion_ref.xattn_head_param_shapes(v_dim=16, seq_dim=8, d_model=8, temporal_pooling=pooling))
    v, a = params.feature_inputs(2, 4, 12, v_dim=16, a_dim=8, seed=11)
    logits, _ = fusion_ref.xattn_forward(p, torch.from_numpy(v), torch.from_numpy(a), num_heads=2,
                                         temporal_pooling=pooling, temporal_num_heads=2)
    assert tuple(logits.shape) == (2, 8)
    np.testing.assert_allclose(logits.numpy(), g["logits"], atol=2e-5)


@pytest.mark.parametrize("mode", ["mean", "attn", "transformer"])
def test_temporal_pooler(mode):
    g = golden(f"temporal_{mode}.npz")
    names = [str(n) for n in g["names"]] if "names" in g.files else []
    shapes = fusion_ref._pool_shapes("x", 8, mode, 1)
    # reference TemporalPooler's own state-dict names start at "pool."; ours are prefixed "x."
    p = {n: torch.from_numpy(params.init_tensor(n[2:], s)) for n, s in shapes}
    assert sorted(n[2:] for n, _ in shapes) == sorted(n for n in names if not n.endswith("pe"))
    y = fusion_ref.temporal_pool(torch.from_numpy(g["x"]), {k: v for k, v in p.items()}, "x", mode, 2, 1)
    np.testing.assert_allclose(y.numpy(), g["y"], atol=2e-5)


def test_temporal_pooler_rejects_non_3d():
    with pytest.raises(ValueError):
        fusion_ref.temporal_pool(torch.zeros(2, 3), {}, "x", "mean")


@pytest.mark.parametrize("mode", ["late", "concat", "gated"])
def test_c4_heads(mode):
    g = golden(f"c4_{mode}.npz")
    names = [str(n) for n in g["names"]]
    shapes = []
    # rebuild the state dict with the reference's own names (shapes from the oracle listing)
    shape_of = {"audio_proj.weight": (256, 768), "audio_proj.bias": (256,), "video_proj.weight": (256, 512),
                "video_proj.bias": (256,), "fusion.0.weight": (256, 512), "fusion.0.bias": (256,),
                "fusion.3.weight": (8, 256), "fusion.3.bias": (8,), "gate.0.weight": (256, 512),
                "gate.0.bias": (256,), "gate.3.weight": (1, 256), "gate.3.bias": (1,),
                "classifier.weight": (8, 256), "classifier.bias": (8,),
                "audio_model.classifier.0.weight": (768, 768), "audio_model.classifier.0.bias": (768,),
                "audio_model.classifier.3.weight": (8, 768), "audio_model.classifier.3.bias": (8,),
                "video_model.classifier.weight": (8, 512), "video_model.classifier.bias": (8,)}
    for n in names:
        shapes.append((n, shape_of[n]))
    p = torch_state(shapes)
    if mode == "gated":
        p["gate.0.bias"].fill_(-1.0)
        p["gate.3.bias"].fill_(-1.0)
    a, v = torch.from_numpy(g["a_emb"]), torch.from_numpy(g["v_emb"])
    if mode == "late":
        al = fusion_ref.linear(torch.relu(fusion_ref.linear(a, p, "audio_model.classifier.0")), p,
                               "audio_model.classifier.3")
        vl = fusion_ref.linear(v, p, "video_model.classifier")
        out = fusion_ref.late_forward(al, vl)
    else:
        out = fusion_ref.embedding_fusion_forward(p, mode, a, v)
    np.testing.assert_allclose(out.numpy(), g["out"], atol=2e-5)


def test_wavlm_b2():
    g = golden("wavlm_b2.npz")
    p = torch_state(wavlm_ref.wavlm_param_shapes())
    _, audio, _ = params.clip_inputs(2, seed=31)
    torch.set_num_threads(8)
    with torch.no_grad():
        out, inter = wavlm_ref.wavlm_forward(p, torch.from_numpy(audio), return_intermediates=True)
    ef = torch.nn.functional.layer_norm(inter["extract_conv"], (512,), p["feature_projection.layer_norm.weight"],
                                        p["feature_projection.layer_norm.bias"], 1e-5)
    np.testing.assert_allclose(ef.numpy(), g["extract_features"], atol=1e-4)
    np.testing.assert_allclose(inter["layer0"].numpy(), g["layer0"], atol=2e-4)
    np.testing.assert_allclose(out.numpy(), g["last_hidden"], atol=5e-4)


def test_resnet18_structure():
    """Parity UNPINNED (torchvision absent): structural checks only."""
    shapes = resnet18_ref.param_shapes()
    n = sum(int(np.prod(s)) for k, s in shapes if not k.endswith(("running_mean", "running_var", "num_batches_tracked")))
    assert n == 11_176_512
    p = torch_state(shapes)
    x = torch.randn(2, 3, 112, 112)
    y = resnet18_ref.resnet18_trunk(p, x, training=True)
    assert tuple(y.shape) == (2, 512, 1, 1)


def test_int8_head_c5():
    """Dynamic-INT8 xattn head at B=64 (C5) vs the reference's CPU quantize_dynamic output."""
    from oracle import int8_ref

    g = golden("int8_head_b64.npz")
    head_linears = sorted(n for n in g["quantized"] if not n.startswith(("audio_model.", "video_model.")))
    assert head_linears == sorted(int8_ref.XATTN_INT8["concat"])
    p = int8_ref.quantize_params(xattn_params("concat", False), head_linears)
    v, a = params.feature_inputs(64, 8, 149, seed=21)
    with torch.no_grad():
        fp, _ = fusion_ref.xattn_forward(xattn_params("concat", False), torch.from_numpy(v), torch.from_numpy(a))
        lq, _ = fusion_ref.xattn_forward(p, torch.from_numpy(v), torch.from_numpy(a))
    np.testing.assert_allclose(fp.numpy(), g["logits_fp32"], atol=2e-5)
    np.testing.assert_allclose(lq.numpy(), g["logits_int8"], atol=2e-5)
    assert (lq.argmax(1).numpy() == g["logits_int8"].argmax(1)).all()


def test_int8_qparams_edge_cases():
    from oracle import int8_ref

    # all-positive / all-negative / all-zero inputs (zero point pinned to the range ends; scale fallback)
    assert int8_ref.choose_qparams(0.5, 2.0)[1] == 0
    assert int8_ref.choose_qparams(-2.0, -0.5)[1] == 127
    assert float(int8_ref.choose_qparams(0.0, 0.0)[0]) == np.float32(0.1)
    s, _ = int8_ref.choose_qparams(-1e-6, 1e-6)
    assert float(s) == np.float32(6.1e-5)
    qw, ws = int8_ref.quantize_weight(np.array([[1.0, -2.0], [0.5, 0.0]], np.float32))
    assert qw.min() >= -128 and qw.max() <= 127 and float(ws) == np.float32(2.0 / 127.5)


@pytest.mark.parametrize("mode", ["concat", "gated"])
def test_c4_clip_alignment(mode):
    """fusion_align_mode="clip" (fusion.py:127-150, 417-418): logits, the CLIP loss and the gradients of
    CE + 0.5 * align (train.py:221-225) vs the imported reference."""
    g = golden(f"c4_clip_{mode}.npz")
    p = clip_head_params(mode)
    assert sorted(p) == sorted(str(n) for n in g["names"] if not str(n).startswith(("audio_model.", "video_model.")))
    for q in p.values():
        q.requires_grad_(True)
    a = torch.from_numpy(g["a_emb"]).requires_grad_(True)
    v = torch.from_numpy(g["v_emb"]).requires_grad_(True)
    out, align = fusion_ref.embedding_fusion_forward(p, mode, a, v, align=True)
    loss = fusion_ref.cross_entropy(out, torch.from_numpy(g["labels"])) + 0.5 * align
    loss.backward()
    np.testing.assert_allclose(out.detach().numpy(), g["logits"], atol=2e-5)
    assert abs(float(align) - float(g["align"])) < 2e-5 and abs(float(loss) - float(g["loss"])) < 2e-5
    np.testing.assert_allclose(a.grad.numpy(), g["grad_a"], atol=2e-6)
    np.testing.assert_allclose(v.grad.numpy(), g["grad_v"], atol=2e-6)
    for k, q in p.items():
        check_grad(g, k, q.grad, atol=2e-6)


def test_int8_head_prior_c5():
    """INT8 with the emotion-prior adapter: prior_net and the token-bias Linears are quantized too."""
    from oracle import int8_ref

    g = golden("int8_head_prior_b64.npz")
    head_linears = sorted(str(n) for n in g["quantized"] if not str(n).startswith(("audio_model.", "video_model.")))
    assert head_linears == sorted(int8_ref.XATTN_INT8["concat"] + int8_ref.PRIOR_INT8)
    p = int8_ref.quantize_params(xattn_params("concat", True), head_linears)
    v, a = params.feature_inputs(64, 8, 149, seed=22)
    with torch.no_grad():
        fp, _ = fusion_ref.xattn_forward(xattn_params("concat", True), torch.from_numpy(v), torch.from_numpy(a),
                                         use_prior=True)
        lq, _ = fusion_ref.xattn_forward(p, torch.from_numpy(v), torch.from_numpy(a), use_prior=True)
    np.testing.assert_allclose(fp.numpy(), g["logits_fp32"], atol=2e-5)
    np.testing.assert_allclose(lq.numpy(), g["logits_int8"], atol=1e-4)
    assert (lq.argmax(1).numpy() == g["logits_int8"].argmax(1)).all()


@pytest.mark.parametrize("dim", [512, 768])
def test_encoder_transformer_pool(dim):
    """TemporalPooler('transformer', 4 heads) at the encoders' widths (head_dim 128 / 192)."""
    g = golden(f"temporal_transformer_d{dim}.npz")
    shapes = fusion_ref._pool_shapes("tp", dim, "transformer", 1)
    p = torch_state([(k[len("tp."):], s) for k, s in shapes])
    assert sorted(p) == sorted(str(n) for n in g["names"] if not str(n).endswith("pe"))
    for q in p.values():
        q.requires_grad_(True)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    y = fusion_ref.transformer_pool(x, p, "pool", num_heads=4, num_layers=1)
    (y * torch.from_numpy(g["w"])).sum().backward()
    np.testing.assert_allclose(y.detach().numpy(), g["y"], atol=3e-5)
    np.testing.assert_allclose(x.grad.numpy(), g["grad_x"], atol=3e-6)
    for k, q in p.items():
        if k == "pool.pool.score.4.bias":  # softmax is shift-invariant: this gradient is 0 up to rounding noise
            assert abs(float(q.grad)) < 1e-4
            continue
        check_grad(g, k, q.grad, atol=5e-6)
