"""Native RCCL transport (csrc/hip/rccl_transport.hpp) on one MI355X.

Two ranks cannot share one GPU under RCCL, so the multi-rank path runs only on a
multi-GPU node (bench.py, driver's scaling run); here the same code moves nodes over
a world-1 communicator: pool -> staging -> ncclSend to self / ncclRecv from self on
the engine's transfer stream -> staging -> pool, and the golden tree must survive."""
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel

pytestmark = pytest.mark.gpu


def test_rccl_library_is_torch_copy():
    import torch  # noqa: F401  (as in every entry point: torch first)

    H = ops.require_gpu(0)
    maps = open("/proc/self/maps").read()
    libs = {line.split()[-1] for line in maps.splitlines() if "librccl" in line}
    assert len(libs) == 1, libs  # one RCCL per process
    assert H.RcclTransport is not None


def test_rccl_self_loop_keeps_golden_tree():
    import torch  # noqa: F401

    H = ops.require_gpu(0)
    t = H.RcclTransport(H.RcclTransport.new_id(), 0, 1, 0)
    assert t.preflight(1 << 20)["peers"] == 0
    model = PfspModel(14, 1)
    eng = model.make_engine("gpu", 0, EngineOptions(max_parents=1 << 12, ring_bytes=1 << 30))
    nodes, t1, s1, best = model.warmup(1377, 25)
    eng.begin(nodes, best)
    moved = 0
    for _ in range(20):
        eng.run(max_launches=1)
        if eng.size() == 0:
            break
        moved += t.self_loop(eng, 5000)
    eng.run()
    st = eng.stats()
    assert moved > 0
    assert (st["tree"] + t1, st["sol"] + s1, st["best"]) == (2573652, 2648, 1377)
    assert t.rank == 0 and t.world == 1


def test_rccl_round_control_world1():
    # the control plane off the shm board: the round loop's status all-gather and final
    # reductions as ncclAllGather on the engine's transfer stream (world-1 communicator)
    import torch  # noqa: F401

    H = ops.require_gpu(0)
    t = H.RcclTransport(H.RcclTransport.new_id(), 0, 1, 0)
    model = PfspModel(14, 1)
    eng = model.make_engine("gpu", 0, EngineOptions(max_parents=1 << 14, ring_bytes=1 << 30))
    assert t.allgather_i64([7, -3, 1 << 40], eng).tolist() == [[7, -3, 1 << 40]]
    nodes, t1, s1, best = model.warmup(1377, 25)
    eng.begin(nodes, best)
    before = t.collectives
    out = H.dist_rounds(eng, 0, t, 0, 1, {}, t)
    assert t.collectives > before + 1  # status rounds + the final reductions
    assert (int(out["counts"][:, 0].sum()) + t1, int(out["counts"][:, 1].sum()) + s1, out["best"]) == \
        (2573652, 2648, 1377)
