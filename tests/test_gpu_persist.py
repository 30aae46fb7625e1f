"""Persistent iterations (csrc/hip/pfsp_kernels.hpp lb1_small_persist): the LB1 register
path explores a whole window inside one kernel, workgroups sharing work through
donations (opt-in: TTS_PERSIST_MIN). Every knob setting must give the golden trees:
the work-sharing protocol may neither lose nor duplicate a node."""
import pytest

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, solve_engine

pytestmark = pytest.mark.gpu

GOLDEN = {(14, 1): (2573652, 2648, 1377), (14, 0): (2573652, 2648, 1377), (7, 0): (271602, 28447, 1234),
          (13, 1): (4052758, 15, 1496), (3, 1): (2573133, 5689, 1081), (8, 0): (113458723, 808498, 1206)}
OPTS = EngineOptions(ring_bytes=1 << 30, max_parents=1 << 19)


def _env(monkeypatch, **kv):
    for k in ("MIN", "US", "WG", "DMIN", "WT"):
        monkeypatch.delenv(f"TTS_PERSIST_{k}", raising=False)
    for k, v in kv.items():
        monkeypatch.setenv(f"TTS_PERSIST_{k}", str(v))


@pytest.mark.parametrize("knobs", [
    dict(MIN=256),                       # from the warm-up frontier on
    dict(MIN=20000, DMIN=16),            # from a wide pool, eager donations
    dict(MIN=256, DMIN=512, WT=0),       # plain stores + L2 write-back before a wait
    dict(MIN=256, US=10),                # 10-us budget: stops mid-search, untaken slices put back
    dict(MIN=256, WG=96),                # few workgroups with deep stacks (21 chunk slots each)
])
def test_persist_goldens(knobs, monkeypatch):
    _env(monkeypatch, **knobs)
    for key in ((14, 1), (7, 0), (13, 1), (3, 1)):
        m = PfspModel(*key)
        eng = m.make_engine("gpu", 0, OPTS)
        for _ in range(2):  # twice on one engine: epochs, generations and records carry over
            r = solve_engine(m, eng)
            assert (r.tree, r.sol, r.best) == GOLDEN[key], (key, knobs)
        st = eng.stats()
        assert st["p_steps"] > 0 and st["p_waits"] > 0
        del eng


def test_persist_big_tree_and_off_switch(monkeypatch):
    _env(monkeypatch, MIN=256, US=300)
    m = PfspModel(8, 0)
    eng = m.make_engine("gpu", 0, OPTS)
    r = solve_engine(m, eng)
    assert (r.tree, r.sol, r.best) == GOLDEN[(8, 0)]
    assert eng.stats()["p_donations"] > 0
    del eng
    _env(monkeypatch)  # default: off
    m = PfspModel(14, 1)
    eng = m.make_engine("gpu", 0, OPTS)
    r = solve_engine(m, eng)
    assert (r.tree, r.sol, r.best) == GOLDEN[(14, 1)]
    assert eng.stats()["p_steps"] == 0


def test_persist_without_incumbent(monkeypatch):
    # -u 0: the incumbent falls during the search (read by the workgroups now and then)
    _env(monkeypatch, MIN=256)
    m = PfspModel(14, 1)
    eng = m.make_engine("gpu", 0, OPTS)
    r = solve_engine(m, eng, ub=0)
    assert r.best == 1377 and r.tree > GOLDEN[(14, 1)][0]


@pytest.mark.parametrize("world", [2, 4])
def test_persist_after_in_search_split(world, monkeypatch):
    # ranks run identical (non-persistent) iterations until the split, then each
    # explores its share persistently: the shares add up to the golden tree
    _env(monkeypatch, MIN=256)
    m = PfspModel(14, 1)
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    tree = sol = 0
    for r in range(world):
        e = m.make_engine("gpu", 0, OPTS)
        e.set_split(r, world, 4096)
        e.begin(nodes, best)
        e.run()
        assert not e.split_pending()
        st = e.stats()
        tree += st["tree"]
        sol += st["sol"]
        del e
    assert (tree + tree1, sol + sol1) == GOLDEN[(14, 1)][:2]
