"""Host-side logic of data.ClipLoader (no GPU): DistributedSampler-style sharding -- one global permutation per
epoch, padded so every rank gets the same number of items (a rank with an extra step would block forever in the
gradient all-reduce) -- and the reference's (video, audio, label, meta) batch contract (ravdess.py:616, 654)."""
import numpy as np
import pytest

from multimodalemotionrecognition_amd import data as D


@pytest.mark.parametrize("n,world", [(10, 3), (9, 3), (7, 4), (1, 2), (32, 8), (0, 2)])
def test_shard_indices_equal_lengths_and_cover(n, world):
    shards = [D.shard_indices(n, r, world, True, 5, 0) for r in range(world)]
    assert len({len(s) for s in shards}) == 1
    flat = np.concatenate(shards) if n else np.array([], dtype=int)
    assert set(flat.tolist()) == set(range(n))
    assert len(flat) == (-(-n // world) * world if n else 0)


def test_shard_indices_global_shuffle_changes_per_epoch():
    a = [D.shard_indices(64, 0, 2, True, 7, e) for e in range(3)]
    assert not np.array_equal(a[0], a[1]) and not np.array_equal(a[1], a[2])
    # the same epoch draws the same permutation on every rank: the union of one epoch is disjoint
    e0 = [set(D.shard_indices(64, r, 2, True, 7, 0).tolist()) for r in range(2)]
    assert not (e0[0] & e0[1])
    # across epochs a rank sees different clips (not a fixed subset)
    assert set(a[0].tolist()) != set(a[1].tolist())
    # unshuffled: rank::world over the list padded by wrapping (DistributedSampler)
    assert D.shard_indices(7, 1, 2, False, 0, 0).tolist() == [1, 3, 5, 0]


def test_clip_loader_len_equal_across_ranks():
    items = [(None, None, i) for i in range(13)]
    lens = [len(D.ClipLoader(items, batch_size=2, rank=r, world=4, device="cpu", drop_last=True)) for r in range(4)]
    assert lens == [2, 2, 2, 2]
    lens = [len(D.ClipLoader(items, batch_size=3, rank=r, world=4, device="cpu", drop_last=False)) for r in range(4)]
    assert lens == [2, 2, 2, 2]
    with pytest.raises(ValueError):
        D.ClipLoader(items, rank=4, world=4, device="cpu")


def test_collate_meta_like_default_collate():
    out = D._collate_meta([{"emotion": 3, "actor": "01", "index": 0}, {"emotion": 5, "actor": "02", "index": 1}])
    assert out["emotion"].tolist() == [3, 5] and out["actor"] == ["01", "02"] and out["index"].tolist() == [0, 1]


def test_train_one_epoch_rejects_bad_batches():
    import torch

    from multimodalemotionrecognition_amd.train import train_one_epoch

    class _Opt:
        def zero_grad(self):
            pass

    with pytest.raises(ValueError):
        train_one_epoch(torch.nn.Linear(1, 1), [(torch.zeros(1), torch.zeros(1))], _Opt(), torch.device("cpu"),
                        None, "xattn")
