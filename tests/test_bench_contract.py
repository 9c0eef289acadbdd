"""bench.py's C5 sub-record: the fixed 512-instance sweep (BASELINE configs[4])
is split over the ranks with the same cluster-size mix on every rank, each
instance solved exactly once (no rank can be left with only the slow small-k
128-GPU configuration)."""
import collections
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import sw_synth as ss  # noqa: E402


def test_sweep_cycles_cluster_sizes():
    probs = ss.sweep_problems(8, N=12)
    assert [p.G for p in probs] == [32, 64, 128, 256] * 2
    assert all(p.T == 30 for p in probs)
    k = {p.G: p.k for p in probs}
    assert k == {32: 10.0, 64: 10.0, 128: 1e-3, 256: 1e5}


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c5_share_same_mix_every_rank(world):
    sizes = (32, 64, 128, 256)
    idx = list(range(bench.C5_INSTANCES))
    seen = []
    for rank in range(world):
        mine = bench.c5_share(idx, world, rank)
        seen += mine
        mix = collections.Counter(sizes[i % 4] for i in mine)
        assert mix == {G: bench.C5_INSTANCES // 4 // world for G in sizes}, (world, rank, mix)
    assert sorted(seen) == idx


def test_c5_order_puts_small_k_first_and_keeps_every_instance():
    probs = bench.c5_share(ss.sweep_problems(64, N=12), 2, 1)
    ordered = bench.c5_order(probs)
    assert sorted(id(p) for p in ordered) == sorted(id(p) for p in probs)
    ks = [p.k for p in ordered]
    assert ks == sorted(ks) and ks[0] == 1e-3
