"""Dynamic-INT8 Linear kernels (C5, TorchModelRunner enable_dynamic_quant) vs the oracle restatement of
the reference's quantize_dynamic (oracle/int8_ref.py, itself pinned to the reference's output)."""
import numpy as np
import pytest
import torch

from oracle import fusion_ref, int8_ref, params
from tests.gpu_helpers import feats, head_model
from tests.helpers import golden, xattn_params

pytestmark = pytest.mark.gpu


def _qp(x, mode):
    from multimodalemotionrecognition_amd import kernels as K

    part = torch.empty(K.QP_PARTIAL, device="cuda")
    qp = torch.empty(4, device="cuda")
    K.quant_params(x, part, qp, mode)
    return qp.cpu().numpy()


@pytest.mark.parametrize("case", ["normal", "positive", "negative", "zeros", "tiny", "large", "odd_len"])
def test_activation_qparams_exact(case):
    rng = np.random.default_rng(3)
    x = {"normal": rng.normal(0.2, 1.3, (513, 77)), "positive": rng.random((64, 64)) + 0.5,
         "negative": -rng.random((64, 64)) - 0.25, "zeros": np.zeros((8, 16)), "tiny": rng.normal(0, 1e-6, (32, 32)),
         "large": rng.normal(0, 300.0, (1000, 768)), "odd_len": rng.normal(1.0, 2.0, (7,))}[case].astype(np.float32)
    qp = _qp(torch.from_numpy(x).cuda(), 0)
    s, zp = int8_ref.choose_qparams(float(x.min()), float(x.max()))
    assert qp[0] == s and qp[2] == zp and qp[1] == np.float32(1.0) / s


def test_weight_quantization_exact():
    from multimodalemotionrecognition_amd import kernels as K

    rng = np.random.default_rng(4)
    w = (rng.standard_normal((70, 96)) * 0.05).astype(np.float32)
    wd = torch.from_numpy(w).cuda()
    qp = _qp(wd, 1)
    qw_ref, ws_ref = int8_ref.quantize_weight(w)
    assert qp[0] == ws_ref
    qw = torch.empty(70, 112, dtype=torch.int8, device="cuda")  # padded leading dim
    cs = torch.empty(70, dtype=torch.int32, device="cuda")
    K.quantize_weight_s8(wd, torch.from_numpy(qp).cuda(), qw, cs)
    got = qw.cpu().numpy()
    assert np.array_equal(got[:, :96], qw_ref) and not got[:, 96:].any()
    assert np.array_equal(cs.cpu().numpy(), qw_ref.astype(np.int64).sum(1))


@pytest.mark.parametrize("M,N,K,act", [(37, 70, 48, "none"), (512, 128, 512, "relu"), (9536, 128, 768, "none"),
                                       (64, 8, 256, "none"), (1, 1, 16, "relu")])
def test_gemm_i8dyn_vs_oracle(M, N, K, act):
    from multimodalemotionrecognition_amd.int8 import QuantizedLinear

    torch.manual_seed(M + N + K)
    lin = torch.nn.Linear(K, N)
    x = torch.randn(M, K) * 1.7 + 0.3
    ql = QuantizedLinear(lin.cuda())
    out = torch.empty(M, N, device="cuda")
    ql(x.cuda(), out, act)
    qw, ws = int8_ref.quantize_weight(lin.weight.detach().cpu().numpy())
    ref = int8_ref.int8_linear(x.numpy(), qw, ws, lin.bias.detach().cpu().numpy())
    if act == "relu":
        ref = np.maximum(ref, 0)
    got = out.cpu().numpy()
    assert np.array_equal(ql.qw.cpu().numpy(), qw)
    # same integer arithmetic and the same single-rounding fma dequant: bit-exact
    assert np.abs(got - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())
    assert (got == ref).mean() > 0.999


def test_int8_head_c5_golden():
    """xattn head at B=64 with INT8 Linears vs the reference's quantize_dynamic logits."""
    from multimodalemotionrecognition_amd.int8 import quantize_dynamic_hip

    g = golden("int8_head_b64.npz")
    m = head_model("concat", False).eval()
    q = quantize_dynamic_hip(m)
    assert sorted(q) == sorted(int8_ref.XATTN_INT8["concat"])
    v, a = feats(64, 8, 149, seed=21)
    with torch.inference_mode():
        lq = m.xattn_from_features(v, a).cpu().numpy()
    # MHA / LayerNorm stay fp32 on both sides; a 1e-7 difference can move one activation across a
    # rounding tie in the next quantization (one quantum = ~1e-3 in a logit), hence 5e-3.
    diff = np.abs(lq - g["logits_int8"]).max()
    print("int8 head max|dlogit| vs reference:", diff)
    assert diff < 5e-3
    assert (lq.argmax(1) == g["logits_int8"].argmax(1)).mean() >= 63 / 64
    # and the oracle restatement agrees with the kernel path too
    p = int8_ref.quantize_params(xattn_params("concat", False), int8_ref.XATTN_INT8["concat"])
    vv, aa = params.feature_inputs(64, 8, 149, seed=21)
    lo, _ = fusion_ref.xattn_forward(p, torch.from_numpy(vv), torch.from_numpy(aa))
    assert np.abs(lq - lo.numpy()).max() < 5e-3


def test_int8_gated_head_and_training_uses_fp32():
    from multimodalemotionrecognition_amd.int8 import quantize_dynamic_hip

    m = head_model("gated", False).eval()
    quantize_dynamic_hip(m)
    v, a = feats(16, 8, 149, seed=5)
    with torch.inference_mode():
        lq = m.xattn_from_features(v, a).cpu()
    p = int8_ref.quantize_params(xattn_params("gated", False), int8_ref.XATTN_INT8["gated"])
    vv, aa = params.feature_inputs(16, 8, 149, seed=5)
    lo, _ = fusion_ref.xattn_forward(p, torch.from_numpy(vv), torch.from_numpy(aa), xattn_head="gated")
    assert float((lq - lo).abs().max()) < 5e-3
    # train mode ignores the INT8 images (quantize_dynamic is an inference transform)
    m.train()
    m.attn_dropout = 0.0
    m.v_drop_path.drop_prob = 0.0
    m.xattn_gate[2].p = 0.0
    lf = m.xattn_from_features(v, a).detach().cpu()
    ref, _ = fusion_ref.xattn_forward(xattn_params("gated", False), torch.from_numpy(vv), torch.from_numpy(aa),
                                      xattn_head="gated")
    assert float((lf - ref).abs().max()) < 1e-3
