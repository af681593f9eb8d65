"""m3d_topk_keys (ops.topk_keys): the hand-written radix-select top-k that
replaces torch.topk in the ProposalLayer (tf.nn.top_k(scores, k, sorted=True),
core/models.py:403-404).  Against a numpy sort of the same int64 keys:
values and positions bit-exact, for the ProposalLayer shapes (112 k anchors ->
15000 at 128^3, 4.2 M -> 15000 at 256^3), edge sizes (k = 1, k = n, n not a
multiple of the block), keys that share their top 32 / 53 bits (every digit
pass decides), negative keys (signed order), the slab merge's padded
candidates, the bitonic fallback above 32768 selected keys, and the k > n
InvalidArgument."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _np_topk(keys, k):
    # exact descending order of distinct int64 keys (no float conversion)
    order = np.argsort(keys, kind="stable")[::-1]
    return keys[order[:k]], order[:k]


def _distinct(rng, n, mode):
    if mode == "random":
        k = rng.choice(np.iinfo(np.int64).max // 2, size=n, replace=False).astype(np.int64)
        k[rng.random(n) < 0.5] *= -1
        return k
    if mode == "score_keys":
        # m3d_score_keys layout: (signed-orderable score << 32) | (0xFFFFFFFF - index), few distinct scores
        s = rng.integers(0, 50, n).astype(np.int64)
        return (s << 32) | (0xFFFFFFFF - np.arange(n, dtype=np.int64))
    if mode == "shared53":
        # identical top 53 bits except for a few: the last passes decide
        base = np.int64(0x123456789ABC) << 16
        return base + rng.permutation(n).astype(np.int64)
    raise ValueError(mode)


@pytest.mark.parametrize("n,k,mode", [
    (112_320, 15_000, "score_keys"),      # configs[1] ProposalLayer
    (4_194_304, 15_000, "score_keys"),    # configs[3] 256^3
    (1000, 1, "random"), (1000, 1000, "random"), (777, 333, "random"),
    (65_536, 2048, "shared53"), (300_000, 6000, "random"),
    (100_000, 40_000, "random"),          # > 32768 selected: bitonic permutation path
])
def test_topk_matches_sort(cuda, n, k, mode):
    from m3d import ops
    rng = np.random.default_rng(n + k)
    keys = _distinct(rng, n, mode)
    vals, pos = ops.topk_keys(torch.from_numpy(keys).to(cuda), k, positions=True)
    want_v, want_p = _np_topk(keys, k)
    assert np.array_equal(vals.cpu().numpy(), want_v)
    assert np.array_equal(pos.cpu().numpy(), want_p)


def test_topk_order_matches_torch_on_scores(cuda):
    """ops.topk_order (score keys of probs[:, 1]) equals tf.nn.top_k's order on
    ties (lower index first): the scores are rounded to 2 decimals, so most
    are tied."""
    from m3d import ops
    rng = np.random.default_rng(1)
    p1 = np.round(rng.uniform(size=50_000), 2).astype(np.float32)
    probs = torch.from_numpy(np.stack([1 - p1, p1], 1)).to(cuda)
    got = ops.topk_order(probs, 6000).cpu().numpy()
    want = np.lexsort((np.arange(p1.size), -p1))[:6000]
    assert np.array_equal(got, want)


def test_topk_rejects_k_above_n(cuda):
    from m3d import ops
    with pytest.raises(ValueError, match="at least k"):
        ops.topk_keys(torch.arange(10, device=cuda, dtype=torch.int64), 11)
