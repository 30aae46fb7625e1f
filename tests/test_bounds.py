"""Host lower bounds: LB1 == LB1_d, LB2 >= LB1, validity, early exit."""
import itertools

import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel
from dist_gpu_accelerated_tree_search_amd.utils import nodes as nd

INT_MAX = 2**31 - 1


def random_nodes(model, n, seed):
    rng = np.random.default_rng(seed)
    depths = rng.integers(0, model.jobs, size=n)
    perms = np.stack([rng.permutation(model.jobs) for _ in range(n)])
    return nd.pfsp_pack(depths, perms, model.jobs)


@pytest.mark.parametrize("inst", [1, 5, 11, 14, 21, 29, 31])
def test_lb1_equals_lb1_d(inst):
    m1 = PfspModel(inst, 1)
    m0 = PfspModel(inst, 0)
    nodes = random_nodes(m1, 200, inst)
    assert np.array_equal(m1.child_bounds_cpu(nodes), m0.child_bounds_cpu(nodes))


@pytest.mark.parametrize("inst", [3, 14, 21])
def test_lb2_dominates_lb1(inst):
    nodes = random_nodes(PfspModel(inst, 1), 150, inst + 100)
    b1 = PfspModel(inst, 1).child_bounds_cpu(nodes)
    b2 = PfspModel(inst, 2).child_bounds_cpu(nodes, INT_MAX)
    assert (b2 >= b1).all()


def test_lb2_early_exit_semantics():
    m = PfspModel(14, 2)
    nodes = random_nodes(m, 100, 7)
    full = m.child_bounds_cpu(nodes, INT_MAX)
    best = 1377
    cut = m.child_bounds_cpu(nodes, best)
    # same prune decision; exact value whenever the full bound does not exceed best
    assert np.array_equal(full < best, cut < best)
    keep = full <= best
    assert np.array_equal(full[keep], cut[keep])
    assert (cut[~keep] > best).all()


def _optimal_completion(inst, prefix):
    C = ops.cpu()
    rest = [j for j in range(inst.jobs) if j not in prefix]
    return min(C.makespan(inst, list(prefix) + list(p)) for p in itertools.permutations(rest))


def test_bounds_are_valid_on_a_small_instance():
    # 7 jobs x 4 machines: every bound must be <= the best completion of its prefix
    p = np.random.default_rng(3).integers(1, 100, size=(4, 7))
    C = ops.cpu()
    inst = C.PfspInstance.from_matrix(7, 4, p.reshape(-1).tolist())
    rng = np.random.default_rng(5)
    for _ in range(40):
        d = int(rng.integers(1, 6))
        perm = rng.permutation(7).tolist()
        opt = _optimal_completion(inst, perm[:d])
        assert C.lb1(inst, perm, d) <= opt
        assert C.lb2(inst, perm, d, INT_MAX) <= opt
    # a complete schedule's LB1 is at least its makespan
    perm = list(range(7))
    assert C.lb1(inst, perm, 7) >= C.makespan(inst, perm)


def test_lb1_children_indexing():
    C = ops.cpu()
    inst = C.PfspInstance.taillard(21)
    perm = list(np.random.default_rng(1).permutation(20))
    d = 6
    by_job = C.lb1_children(inst, perm, d)
    for k in range(d, 20):
        c = perm.copy()
        c[d], c[k] = c[k], c[d]
        assert by_job[perm[k]] == C.lb1(inst, c, d + 1)
