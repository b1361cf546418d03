"""Shared test helpers: golden loading and oracle-parameter construction."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from oracle import fusion_ref, params

GOLDEN = Path(__file__).resolve().parent / "golden"


def golden(name: str):
    return np.load(GOLDEN / name, allow_pickle=False)


def torch_state(named_shapes, seed: int = 0):
    return {k: torch.from_numpy(v) for k, v in params.init_state(named_shapes, seed).items()}


def xattn_params(xattn_head="concat", use_prior=False, **kw):
    p = torch_state(fusion_ref.xattn_head_param_shapes(xattn_head=xattn_head, use_prior=use_prior, **kw))
    fusion_ref.gated_bias_init(p, xattn_head)
    return p
