"""Device pool transfers: stream-ordered export/import between engines and the
pinned, asynchronous spill/refill of the ring bottom (csrc/hip/engine.hpp,
csrc/hip/host_spill.hpp)."""
import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel
from dist_gpu_accelerated_tree_search_amd.search import solve_engine

pytestmark = pytest.mark.gpu
GOLD14 = (2573652, 2648, 1377)


@pytest.mark.parametrize("ub,frontier,window", [(1, 300_000, 1024), (1, 25, 1024), (0, 25, 1024), (1, 200_000, 256)])
def test_pinned_spill_and_refill_keep_the_tree(ub, frontier, window):
    # a ring (2^19 nodes) far too small for the pool: the bottom goes to pinned host
    # blocks (asynchronous D2H on the transfer stream) and comes back under the ring
    # bottom (H2D ahead of need); with -u 1 the tree is deterministic, so no node may
    # be lost or duplicated
    model = PfspModel(14, 1)
    # (window 256: a graph's growth is over half the ring, refills must leave room for it)
    eng = model.make_engine("gpu", 0, EngineOptions(max_parents=window, ring_bytes=1 << 20))
    r = solve_engine(model, eng, ub=ub, m=frontier)
    st = eng.stats()
    assert r.best == 1377
    if ub == 1:
        assert (r.tree, r.sol) == GOLD14[:2]
    if frontier > 25:
        assert st["spilled"] > 0 and st["refilled"] > 0 and st["pinned_bytes"] > 0, st
    assert st["host_nodes"] == 0 and st["device_nodes"] == 0


def test_trace_records_replays_and_pool_copies():
    # engine.set_trace / engine.trace (csrc/hip/engine.hpp): timing events around every
    # graph replay (kind 0), spill D2H (1) and refill H2D (2); the forced-spill solve
    # keeps the golden tree, and every interval is well-formed
    model = PfspModel(14, 1)
    eng = model.make_engine("gpu", 0, EngineOptions(max_parents=1024, ring_bytes=1 << 20))
    eng.set_trace(True)
    r = solve_engine(model, eng, ub=1, m=300_000)
    assert (r.tree, r.sol, r.best) == GOLD14
    tr = eng.trace()
    assert tr.ndim == 2 and tr.shape[1] == 3 and len(tr) > 0
    kinds = set(tr[:, 0].astype(int).tolist())
    assert {0, 2} <= kinds, kinds  # replays and refills (the frontier starts in pinned blocks)
    assert (tr[:, 2] >= tr[:, 1]).all() and (tr[:, 1] >= 0).all()
    eng.set_trace(False)
    r = solve_engine(model, eng, ub=1, m=25)
    assert (r.tree, r.sol, r.best) == GOLD14
    assert len(eng.trace()) == 0


def test_export_import_between_engines_keeps_the_tree():
    import torch

    model = PfspModel(14, 1)
    opts = EngineOptions(max_parents=1 << 12, ring_bytes=1 << 28)
    a, b = model.make_engine("gpu", 0, opts), model.make_engine("gpu", 0, opts)
    nodes, t1, s1, best = model.warmup(model.initial_best(1), 200)
    a.begin(nodes, int(best))
    b.begin(nodes[:0], int(best))
    a.run(max_launches=2)
    n = a.size() // 2
    buf = torch.empty(n * model.node_bytes, dtype=torch.uint8, device="cuda:0")
    assert a.transfer_stream != 0
    got = a.export_to(buf.data_ptr(), n)
    assert got == n
    a.fence()  # host-side handoff between two engines of one process
    b.import_from(buf.data_ptr(), n)
    assert b.size() == n
    a.run()
    b.run()
    sa, sb = a.stats(), b.stats()
    assert (t1 + sa["tree"] + sb["tree"], s1 + sa["sol"] + sb["sol"]) == GOLD14[:2]
    assert sa["exports"] == 1 and sb["imports"] == 1


def test_pop_push_roundtrip_preserves_nodes():
    model = PfspModel(14, 1)
    eng = model.make_engine("gpu", 0, EngineOptions(max_parents=1024, ring_bytes=1 << 20))
    nodes, _, _, best = model.warmup(model.initial_best(1), 400_000)
    eng.begin(nodes, int(best))  # more than half the ring: the rest goes to the pinned spill
    st = eng.stats()
    assert st["host_nodes"] > 0
    out = eng.pop(len(nodes))
    assert len(out) == len(nodes)
    assert sorted(map(bytes, np.asarray(out))) == sorted(map(bytes, np.asarray(nodes)))
