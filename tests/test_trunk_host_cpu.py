"""Host-side logic of the trunk backward's deferred weight-gradient folds (no GPU): the stem's slab-column map and
the fold table the batched launch receives."""
import numpy as np
import pytest
import torch

from multimodalemotionrecognition_amd import kernels as K
from multimodalemotionrecognition_amd.video import S2D_CH, _stem_wgrad_index, _stem_wgrad_map


def test_stem_wgrad_map_inverts_the_gather_index():
    """map[j] = flat (c, r, s) of the 7x7 weight that slab column j (tap-major, space-to-depth channel minor) is,
    -1 for the padded taps / channels; it must be the exact inverse of the [16][4][4] gather index the immediate
    path uses (which reads the PyTorch-layout wgrad: channel-major)."""
    R = S = 7
    C = 3
    idx = _stem_wgrad_index(R, S, C, "cpu").tolist()  # flat (c, r, s) -> ch * 16 + ry * 4 + rx
    m = _stem_wgrad_map(R, S, C, "cpu")
    assert m.dtype == torch.int32 and m.numel() == 4 * 4 * S2D_CH
    used = {}
    for j, o in enumerate(m.tolist()):
        if o < 0:
            continue
        tap, ch = divmod(j, S2D_CH)
        used[o] = ch * 16 + tap  # the same element in the [ch][ry][rx] layout
    assert len(used) == C * R * S  # every weight element is covered exactly once
    assert [used[o] for o in range(C * R * S)] == idx


def test_wgrad_folds_table_and_split_count():
    """conv_wgrad(defer=...) records one row per launch with the kernel's effective split count (every split
    non-empty, 64-pixel granules) and flush() clears the record (no launch without rows)."""
    f = K.WgradFolds()
    f.flush()  # nothing recorded: no launch, no error
    ws = torch.zeros(4)
    dw = torch.zeros(2)
    f.add(ws, dw, 64, 64, 64, 9, 7)
    assert len(f.rows) == 1 and f.rows[0][3:] == [64, 64, 64, 9, 7]
    for P, splits in ((200704, 154), (4096, 6), (1000, 64), (100, 3), (64, 1), (65, 2)):
        eff = K.wgrad_split_count(P, splits)
        pps = (-(-P // splits) + 63) // 64 * 64  # pixels per split, a multiple of 64
        assert 1 <= eff <= splits and pps % 64 == 0 and (eff - 1) * pps < P <= eff * pps  # none empty, all covered
    assert K.wgrad_split_count(1000, 64) == 16  # 64 asked, 16-pixel splits rounded up to 64: 16 non-empty
    assert np.array(f.rows, dtype=np.int64).shape == (1, 8)


def test_stem_wgrad_table_built_outside_capture(monkeypatch):
    """the deferred fold's stem map is a pageable H2D copy, so prepare_backward builds it before any
    graph capture; inside a capture the prebuilt table is returned as is, and a missing one raises instead of
    copying inside the capture."""
    from multimodalemotionrecognition_amd import graphs as G
    from multimodalemotionrecognition_amd import video

    trunk = video.ResNet18Trunk()
    dev = torch.device("cpu")
    monkeypatch.setattr(G, "capturing", lambda: False)
    built = trunk.stem_wgrad_table(dev, True)  # what prepare_backward does for the default (deferred) folds
    monkeypatch.setattr(G, "capturing", lambda: True)
    assert trunk.stem_wgrad_table(dev, True) is built
    with pytest.raises(RuntimeError, match="prepare_backward"):
        trunk.stem_wgrad_table(dev, False)  # the immediate-fold index was never built
