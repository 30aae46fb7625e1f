"""Dynamic local DFS iterations of the LB1 / LB1_d front kernel (front_dyn): workgroups
step until a time budget, sharing pops through XCD-local queue slots. Every budget —
from a few microseconds (many iterations, queue blocks left over as output chunks) to
longer than the solve (one iteration carries the tree) — must give the golden -u 1
trees, and the probe records of the dynamic steps must match the host oracle."""
import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
from dist_gpu_accelerated_tree_search_amd.search import solve_engine, solve_gpu

pytestmark = pytest.mark.gpu

GOLDEN = {(14, 1): (2573652, 2648, 1377), (14, 0): (2573652, 2648, 1377), (3, 1): (2573133, 5689, 1081),
          (4, 1): (1163892, 941, 1293), (7, 0): (271602, 28447, 1234), (12, 0): (3913907, 18, 1659),
          (13, 1): (4052758, 15, 1496)}


def opts(dyn_us, **kw):
    return EngineOptions(max_parents=1 << 19, ring_bytes=1 << 30, dyn_us=dyn_us, **kw)


@pytest.mark.parametrize("dyn_us", [3, 20, 100, 5000])
def test_dyn_golden(dyn_us):
    for key, gold in GOLDEN.items():
        m = PfspModel(*key)
        eng = m.make_engine("gpu", 0, opts(dyn_us))
        for _ in range(2):  # the second solve replays the learned first graph
            r = solve_engine(m, eng, ub=1)
            assert (r.tree, r.sol, r.best) == gold, (key, dyn_us)
        del eng


@pytest.mark.parametrize("q", ["8", "16", "64"])
def test_dyn_small_queue(q, monkeypatch):
    # one / two / eight slots per XCD partition: donors find the queue full, thieves wait
    monkeypatch.setenv("TTS_DYN_Q", q)
    for key in ((14, 1), (12, 0)):
        r = solve_gpu(PfspModel(*key), ub=1, opts=opts(50))
        assert (r.tree, r.sol, r.best) == GOLDEN[key]


def test_dyn_bigger_tree_and_unknown_optimum():
    # ta008 LB1_d: 113,458,723 nodes over many budgets; ta014 -u 0 finds the optimum
    r = solve_gpu(PfspModel(8, 0), opts=opts(200))
    assert (r.tree, r.sol, r.best) == (113458723, 808498, 1206)
    r = solve_gpu(PfspModel(14, 1), ub=0, opts=opts(200))
    assert r.best == 1377 and r.tree >= GOLDEN[(14, 1)][0]


@pytest.mark.parametrize("dyn_us", [10, 1000])
def test_dyn_probe_records_match_host(dyn_us):
    model = PfspModel(14, 1)
    nodes, _, _, best = model.warmup(1377, 25)
    H = ops.require_gpu(0)
    r = H.pfsp_front_probe(model.jobs, model.machines, list(model.native.p), model.lb,
                           np.ascontiguousarray(nodes, dtype=np.uint8), best, max_parents=1 << 19, cap=1 << 25,
                           dyn_us=dyn_us)
    assert r["checked"] == r["records"] > 0
    assert r["bad_job"] == 0 and r["bad_remain"] == 0 and r["bad_lb"] == 0, r
    assert r["by_kind"]["dynamic"] > 0, r["by_kind"]
    tree, sol, _ = model.drain(best, nodes)
    assert (r["tree"], r["sol"]) == (tree, sol)


@pytest.mark.parametrize("world", [2, 8])
def test_dyn_in_graph_split(world):
    # an in-graph rank split (no dynamic iteration while armed), then dynamic rank shares
    m = PfspModel(14, 1)
    nodes, tree1, sol1, best = m.warmup(1377, 25)
    tree, sol = tree1, sol1
    for rank in range(world):
        eng = m.make_engine("gpu", 0, opts(50))
        eng.set_split(rank, world, 512 * world)
        eng.begin(nodes, best)
        eng.run()
        assert not eng.split_pending()
        st = eng.stats()
        tree += st["tree"]
        sol += st["sol"]
        del eng
    assert (tree, sol) == GOLDEN[(14, 1)][:2]
