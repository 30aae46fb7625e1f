"""Distributed runtime with GPU engines on one MI355X (ranks share the device; the
status/steal protocol runs over gloo, nodes leave and enter the device pools)."""
import pytest

from dist_gpu_accelerated_tree_search_amd.parallel.launch import spawn_local
from dist_gpu_accelerated_tree_search_amd.parallel.workers import solve_rank

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4])
def test_gpu_ranks_golden(world):
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "gpu", "comm": "gloo", "device": 0,
            "engine": {"ring_bytes": 1 << 28, "max_parents": 1 << 14},
            "dist": {"slice_min_s": 0.0001, "init_per_rank": 8}}
    res = spawn_local(world, solve_rank, (spec,), timeout=600)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == (2573652, 2648, 1377)


def test_gpu_ranks_queens():
    spec = {"problem": "nqueens", "N": 13, "backend": "gpu", "comm": "gloo", "device": 0,
            "engine": {"ring_bytes": 1 << 28, "max_parents": 1 << 12}, "dist": {"slice_min_s": 0.0001}}
    res = spawn_local(2, solve_rank, (spec,), timeout=600)
    assert (res[0]["tree"], res[0]["sol"]) == (4674889, 73712)
