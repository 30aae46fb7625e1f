"""Golden trees on the host drivers (reference outputs measured with -u 1)."""
import pytest

from dist_gpu_accelerated_tree_search_amd import QueensModel, PfspModel, solve_cpu

# (inst, lb) -> (tree, sol, makespan)
GOLDEN = {
    (14, 0): (2573652, 2648, 1377),
    (14, 1): (2573652, 2648, 1377),
    (14, 2): (144639, 0, 1377),
    (2, 1): (30, 0, 1359),
    (2, 2): (7, 0, 1359),
    (3, 2): (80062, 0, 1081),
    (4, 2): (33283, 0, 1293),
    (7, 0): (271602, 28447, 1234),
    (9, 2): (58783, 0, 1230),
    (19, 1): (178, 0, 1593),
    (19, 2): (80, 0, 1593),
    (12, 0): (3913907, 18, 1659),
}
QUEENS = {8: (2056, 92), 10: (35538, 724), 12: (856188, 14200)}


@pytest.mark.parametrize("key", [(14, 0), (2, 1), (2, 2), (3, 2), (4, 2), (7, 0), (9, 2), (19, 1), (19, 2)])
def test_pfsp_sequential(key):
    r = solve_cpu(PfspModel(*key), ub=1, threads=0)
    assert (r.tree, r.sol, r.best) == GOLDEN[key]


@pytest.mark.parametrize("threads,ws", [(1, True), (3, True), (4, False), (8, True)])
def test_pfsp_multicore_same_tree(threads, ws):
    r = solve_cpu(PfspModel(14, 0), ub=1, threads=threads, ws=ws)
    assert (r.tree, r.sol, r.best) == GOLDEN[(14, 0)]
    assert len(r.workers) == threads
    assert sum(w.tree for w in r.workers) <= r.tree


def test_pfsp_multicore_lb1_and_lb2():
    assert (lambda r: (r.tree, r.sol, r.best))(solve_cpu(PfspModel(14, 1), threads=8)) == GOLDEN[(14, 1)]
    assert (lambda r: (r.tree, r.sol, r.best))(solve_cpu(PfspModel(3, 2), threads=4)) == GOLDEN[(3, 2)]


def _brute_force_optimum(model):
    import itertools

    from dist_gpu_accelerated_tree_search_amd import ops

    C = ops.cpu()
    return min(C.makespan(model.native, list(p)) for p in itertools.permutations(range(model.jobs)))


@pytest.mark.parametrize("lb", [0, 1, 2])
def test_pfsp_ub_inf_finds_optimum(lb):
    model = PfspModel.synthetic(8, 5, 2024 + lb, lb=lb)
    opt = _brute_force_optimum(model)
    assert solve_cpu(model, ub=0, threads=0).best == opt
    assert solve_cpu(model, ub=0, threads=3, m=2).best == opt


@pytest.mark.parametrize("N", [8, 10, 12])
def test_queens(N):
    assert (lambda r: (r.tree, r.sol))(solve_cpu(QueensModel(N))) == QUEENS[N]
    assert (lambda r: (r.tree, r.sol))(solve_cpu(QueensModel(N), threads=4, m=5)) == QUEENS[N]


def test_queens_g_does_not_change_counts():
    assert (lambda r: (r.tree, r.sol))(solve_cpu(QueensModel(10, 3))) == QUEENS[10]


@pytest.mark.slow
def test_queens_14_sequential():
    r = solve_cpu(QueensModel(14))
    assert (r.tree, r.sol) == (27358552, 365596)


@pytest.mark.parametrize("inst,beam", [(14, 32), (21, 32), (1, 8), (31, 8)])
def test_beam_dive_gives_a_real_schedule_makespan(inst, beam, monkeypatch):
    # opt-in (TTS_DIVE): -u 0 device searches start from the dive's makespan: a complete schedule's, so
    # never below the optimum (Taillard's best known for these solved instances), and
    # close to it (within 10 %)
    import itertools  # noqa: F401

    from dist_gpu_accelerated_tree_search_amd import ops
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel

    m = PfspModel(inst, 1)
    v = ops.cpu().pfsp_dive(m.native, beam)
    assert m.best_known <= v <= 1.25 * m.best_known, (v, m.best_known)
    h = ops.cpu().pfsp_neh(m.native, 2_000_000)  # NEH + iterated greedy: within 3 %
    assert m.best_known <= h <= 1.03 * m.best_known, (h, m.best_known)
    monkeypatch.setenv("TTS_DIVE", str(beam))
    assert m.search_best(0) == min(v, ops.cpu().pfsp_neh(m.native, 5_000_000))


def test_u0_starts_from_inf_by_default(monkeypatch):
    # the reference's -u 0 semantics: no heuristic incumbent unless asked for
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import INT_MAX, PfspModel

    monkeypatch.delenv("TTS_DIVE", raising=False)
    assert PfspModel(14, 1).search_best(0) == INT_MAX
    assert PfspModel(14, 1).search_best(1) == 1377


def test_beam_dive_exact_on_tiny_instances():
    import itertools

    import numpy as np

    from dist_gpu_accelerated_tree_search_amd import ops
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel

    m = PfspModel.synthetic(7, 4, seed=5, lb=1)
    p = np.asarray(m.native.p).reshape(4, 7)

    def cmax(perm):
        c = [0] * 4
        for j in perm:
            for k in range(4):
                c[k] = max(c[k], c[k - 1] if k else 0) + int(p[k, j])
        return c[-1]

    opt = min(cmax(q) for q in itertools.permutations(range(7)))
    assert ops.cpu().pfsp_dive(m.native, 5040) == opt  # a beam as wide as the tree is exact
    assert ops.cpu().pfsp_dive(m.native, 1) >= opt
    assert ops.cpu().pfsp_neh(m.native, 0) >= opt  # NEH + local search alone
    assert ops.cpu().pfsp_neh(m.native, 10_000_000) == opt
