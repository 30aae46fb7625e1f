"""Taillard generator: native C++ vs an independent Python oracle (ref c_taillard.c)."""
import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.utils import taillard as tl


def test_ta001_first_row_is_the_published_one():
    # first machine row of ta001 as printed in Taillard (1993)
    expect = [54, 83, 15, 71, 77, 36, 53, 38, 27, 87, 76, 91, 14, 29, 12, 77, 32, 87, 68, 94]
    assert tl.processing_times(1)[0].tolist() == expect
    assert ops.cpu().taillard_processing_times(1)[:20] == expect


@pytest.mark.parametrize("inst", list(range(1, 121, 7)) + [14, 21, 56, 120])
def test_native_matches_python(inst):
    C = ops.cpu()
    assert C.taillard_jobs(inst) == tl.jobs(inst)
    assert C.taillard_machines(inst) == tl.machines(inst)
    assert C.taillard_best_ub(inst) == tl.best_known(inst)
    p = np.asarray(C.taillard_processing_times(inst)).reshape(tl.machines(inst), tl.jobs(inst))
    assert np.array_equal(p, tl.processing_times(inst))
    assert p.min() >= 1 and p.max() <= 99


def test_class_geometry():
    shapes = {(tl.jobs(i), tl.machines(i)) for i in range(1, 121)}
    assert shapes == {(20, 5), (20, 10), (20, 20), (50, 5), (50, 10), (50, 20), (100, 5), (100, 10), (100, 20),
                      (200, 10), (200, 20), (500, 20)}
    with pytest.raises(ValueError):
        tl.jobs(0)
    with pytest.raises(Exception):
        ops.cpu().taillard_jobs(121)


def test_synthetic_matches():
    a = np.asarray(ops.cpu().synthetic_processing_times(30, 7, 12345)).reshape(7, 30)
    assert np.array_equal(a, tl.synthetic(30, 7, 12345))


def test_instance_tables():
    inst = ops.cpu().PfspInstance.taillard(14)
    p = np.asarray(inst.p).reshape(inst.machines, inst.jobs)
    # min heads: min over jobs of the time spent on machines < k
    heads = np.concatenate([[0], np.cumsum(p, axis=0)[:-1].min(axis=1)])
    tails = np.concatenate([np.cumsum(p[::-1], axis=0)[:-1][::-1].min(axis=1), [0]])
    assert inst.min_heads == heads.tolist()
    assert inst.min_tails == tails.tolist()
    assert inst.npairs == inst.machines * (inst.machines - 1) // 2
    lags = np.asarray(inst.lags).reshape(inst.npairs, inst.jobs)
    for q in range(inst.npairs):
        a, b = inst.pair_m0[q], inst.pair_m1[q]
        assert np.array_equal(lags[q], p[a + 1:b].sum(axis=0))
        order = inst.johnson[q * inst.jobs:(q + 1) * inst.jobs]
        assert sorted(order) == list(range(inst.jobs))
        # Johnson's rule: {a < b} by increasing a first, then the rest by decreasing b
        pa, pb = p[a] + lags[q], p[b] + lags[q]
        part = [0 if pa[j] < pb[j] else 1 for j in order]
        assert part == sorted(part)
        first = [pa[j] for j in order if pa[j] < pb[j]]
        second = [pb[j] for j in order if pa[j] >= pb[j]]
        assert first == sorted(first) and second == sorted(second, reverse=True)
