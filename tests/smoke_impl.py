"""Body of __graft_entry__.smoke(): one tiny xattn-head forward+backward on cuda:0 vs the CPU oracle."""
import torch

from multimodalemotionrecognition_amd.losses import CrossEntropyLoss
from oracle import fusion_ref
from tests.gpu_helpers import feats, head_model, max_abs, oracle_head_params


def run_smoke():
    m = head_model("concat", True)
    m.eval()
    v, a = feats(2, 8, 64)
    labels = torch.tensor([1, 5], device="cuda")
    logits = m.xattn_from_features(v, a)
    loss = CrossEntropyLoss()(logits, labels)
    loss.backward()
    torch.cuda.synchronize()
    p = oracle_head_params("concat", True)
    for k in p:
        p[k].requires_grad_(True)
    ref, _ = fusion_ref.xattn_forward(p, v.cpu(), a.cpu(), use_prior=True)
    ref_loss = fusion_ref.cross_entropy(ref, labels.cpu())
    ref_loss.backward()
    err = max_abs(logits, ref)
    gerr = max_abs(m.v2a_attn.in_proj_weight.grad, p["v2a_attn.in_proj_weight"].grad)
    assert err < 1e-3, f"smoke logits mismatch {err}"
    assert gerr < 1e-4, f"smoke grad mismatch {gerr}"
    print(f"smoke ok: max|dlogit|={err:.2e} max|dgrad|={gerr:.2e}")
