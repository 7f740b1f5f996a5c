"""bench.py's per-rank layouts (CPU): every global window is covered exactly once by the ranks'
slices, in rank order, 4-edge aligned under --merge prefilter (rank 0's share from
prefilter_share0; none at all when that is 0: rank 0 then only merges), and the strong layout's even split otherwise."""
import sys

import pytest

sys.argv = ["bench.py"]
import bench  # noqa: E402


class _A:
    edge_factor, scale, window_log2, scaling, share0 = 16, 26, 24, "strong", None


@pytest.mark.parametrize("world", [2, 3, 4, 5, 7, 8])
@pytest.mark.parametrize("share0", [None, 0.0, 0.3])
def test_prefilter_slices_tile_every_window(world, share0):
    a = _A()
    a.merge, a.share0 = "prefilter", share0
    rows = [bench.layout(a, world, r) for r in range(world)]
    W = rows[0][2]
    off = 0
    for r, (E_rank, W_rank, W_glob, nwin, E, o) in enumerate(rows):
        assert W_glob == W and o == off and E_rank == nwin * W_rank
        assert W_rank > 0 or (r == 0 and (share0 == 0.0 or bench.prefilter_share0(world) == 0.0))
        assert r == 0 or W_rank % 4 == 0
        off += W_rank
    assert off == W


def test_prefilter_share0_balances_rank0():
    assert bench.prefilter_share0(1) == 1.0
    assert 0.4 < bench.prefilter_share0(2) < 0.5
    assert bench.prefilter_share0(8) == 0.0                 # rank 0 folds no slice of its own


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_even_strong_layout(world):
    a = _A()
    a.merge = "allgather"
    rows = [bench.layout(a, world, r) for r in range(world)]
    assert [r[5] for r in rows] == [r * rows[0][1] for r in range(world)]
    assert sum(r[1] for r in rows) == rows[0][2]
