"""Shared-memory control plane (csrc/core/shm_control.hpp) used by single-node
multi-process runs for the per-round status all-gather, barriers and final
reductions. Checked with real processes: ordering over many rounds (the two-slot
reuse rule), the incumbent MIN, failure detection when a rank never arrives, and
the distributed golden tree with the plane on and off."""
import os
import time

import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.parallel.launch import spawn_local
from dist_gpu_accelerated_tree_search_amd.parallel.workers import solve_rank

GOLD = (2573652, 2648, 1377)


def _rounds_rank(n_rounds: int):
    from dist_gpu_accelerated_tree_search_amd.parallel.comm import Comm

    comm = Comm(use_gpu=False)
    try:
        assert comm.ctl is not None
        rank, world = comm.rank, comm.world
        rng = np.random.default_rng(rank)
        for r in range(n_rounds):
            if rng.random() < 0.05:
                time.sleep(rng.random() * 1e-3)  # stragglers: a fast rank must not overwrite a slot being read
            n = 1 + (r % 15)
            g = comm.allgather_i64([rank * 1000003 + r * 7 + i for i in range(n)])
            want = np.array([[q * 1000003 + r * 7 + i for i in range(n)] for q in range(world)])
            assert g.shape == (world, n) and (g == want).all(), (r, g, want)
        f = comm.allgather_f64([rank + 0.5, -1.25])
        assert f.shape == (world, 2) and (f[:, 0] == np.arange(world) + 0.5).all() and (f[:, 1] == -1.25).all()
        s = comm.allreduce_i64([rank, 2 * rank], "sum")
        assert list(s) == [world * (world - 1) // 2, world * (world - 1)]
        assert comm.allreduce_i64([rank + 3], "min")[0] == 3
        comm.ctl.offer_best(1000 - rank)
        comm.barrier()
        best = comm.ctl.best
        return {"rank": rank, "rounds": int(comm.ctl.rounds), "best": int(best)}
    finally:
        comm.close()


@pytest.mark.parametrize("world", [2, 4])
def test_shm_allgather_many_rounds(world):
    res = spawn_local(world, _rounds_rank, (3000,), timeout=300)
    assert len({r["rounds"] for r in res}) == 1
    assert all(r["best"] == 1000 - (world - 1) for r in res)


def test_shm_segment_unlinked_after_setup():
    before = set(os.listdir("/dev/shm"))
    spawn_local(2, _rounds_rank, (10,), timeout=120)
    leaked = [f for f in set(os.listdir("/dev/shm")) - before if f.startswith("tts_ctl")]
    assert not leaked


def test_shm_missing_rank_times_out():
    C = ops.cpu()
    name = f"/tts_test_{os.getpid()}"
    a = C.ShmControl(name, 0, 2, True)
    try:
        b = C.ShmControl(name, 1, 2, False)
        t0 = time.perf_counter()
        with pytest.raises(RuntimeError, match="rank 1 did not reach round 1"):
            a.allgather(np.array([1], dtype=np.int64), 0.2)
        assert time.perf_counter() - t0 < 5
        del b
    finally:
        a.unlink()


def test_shm_world_mismatch_rejected():
    C = ops.cpu()
    name = f"/tts_test_w_{os.getpid()}"
    a = C.ShmControl(name, 0, 2, True)
    try:
        with pytest.raises(RuntimeError):
            C.ShmControl(name, 1, 4, False)
        with pytest.raises(ValueError):
            a.allgather(np.arange(16, dtype=np.int64), 1.0)
    finally:
        a.unlink()


@pytest.mark.parametrize("shm", ["1", "0"])
def test_distributed_golden_with_and_without_shm(shm):
    spec = {"problem": "pfsp", "inst": 14, "lb": 0, "backend": "cpu", "dist": {"slice_min_s": 0.0002}}
    res = spawn_local(3, solve_rank, (spec,), timeout=300, env={"TTS_SHM_CONTROL": shm})
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == GOLD
