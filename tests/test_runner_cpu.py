"""Native single-process multi-worker runner (csrc/core/runner.hpp) with CPU engines.

Parity: ref pfsp_multigpu_cuda.c (one thread per device + optional CPU worker,
steal-half sharing, incumbent sharing, termination). Lost or duplicated nodes in
the round protocol show up as a wrong golden tree."""
import subprocess

import pytest

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, QueensModel, ops
from dist_gpu_accelerated_tree_search_amd.search import solve_workers

OPTS = EngineOptions(cpu_batch=512)


def _cpu_engines(model, n, threads=1):
    C = ops.cpu()
    if model.kind == "pfsp":
        return [C.make_pfsp_cpu_engine(model.native, model.host_lb, 512, threads) for _ in range(n)]
    return [C.make_queens_cpu_engine(model.N, model.G, 512, threads) for _ in range(n)]


@pytest.mark.parametrize("W", [1, 2, 3, 4])
def test_runner_pfsp_golden(W):
    model = PfspModel(14, 1)
    r = solve_workers(model, devices=(), engines=_cpu_engines(model, W))
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
    assert len(r.workers) == W
    if W > 1:  # work actually moved between workers
        assert sum(r.extra["sent_nodes"]) > 0


def test_runner_lb2_and_no_sharing():
    model = PfspModel(14, 2)
    r = solve_workers(model, devices=(), engines=_cpu_engines(model, 3))
    assert (r.tree, r.sol, r.best) == (144639, 0, 1377)
    model = PfspModel(14, 0)
    r = solve_workers(model, devices=(), engines=_cpu_engines(model, 2), ws=False)
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
    assert sum(r.extra["sent_nodes"]) == 0


def test_runner_unknown_optimum_shares_incumbent():
    model = PfspModel.synthetic(8, 5, seed=3, lb=1)
    import itertools

    import numpy as np

    p = np.asarray(model.native.p).reshape(5, 8)

    def cmax(perm):
        c = [0] * 5
        for j in perm:
            for k in range(5):
                c[k] = max(c[k], c[k - 1] if k else 0) + int(p[k, j])
        return c[-1]

    opt = min(cmax(q) for q in itertools.permutations(range(8)))
    r = solve_workers(model, devices=(), engines=_cpu_engines(model, 3), ub=0, m=4)
    assert r.best == opt


def test_runner_queens_and_engine_reuse():
    model = QueensModel(11)
    engines = _cpu_engines(model, 3)
    for _ in range(2):
        r = solve_workers(model, devices=(), engines=engines)
        assert (r.tree, r.sol) == (166925, 2680)


def test_runner_cpu_worker_helper():
    # devices=() + cpu_threads builds one multithreaded CPU engine (-D 0 -C 1)
    r = solve_workers(PfspModel(14, 1), devices=(), cpu_threads=2, opts=OPTS)
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)


def test_runner_rejects_mixed_layouts():
    a = PfspModel(14, 1)  # 20 jobs -> 32-B nodes
    C = ops.cpu()
    engines = [C.make_pfsp_cpu_engine(a.native, 0, 512, 1), C.make_queens_cpu_engine(8, 1, 512, 1)]
    with pytest.raises(Exception):
        C.run_workers(engines, [a.root(), a.root()[:0].reshape(0, 16)], 1377)


def test_native_gpu_cli_fails_cleanly_without_device():
    from dist_gpu_accelerated_tree_search_amd.ops.build import BIN

    exe = BIN / "pfsp_gpu"
    if not exe.exists() or ops.gpu_count() > 0:
        pytest.skip("needs the built CLI on a host without GPUs")
    out = subprocess.run([str(exe), "-i", "14", "-l", "1", "-D", "1"], capture_output=True, text=True, timeout=60)
    assert out.returncode != 0
    assert "More GPU devices requested" in out.stdout


def test_runner_fault_injection_keeps_the_tree():
    # random per-round delays and 50 % of planned steals dropped: same tree, and
    # termination still happens (SURVEY §5.3 fault injection)
    model = PfspModel(14, 0)
    r = solve_workers(model, devices=(), engines=_cpu_engines(model, 4), m=10,
                      faults={"delay_us": 300, "steal_fail_pct": 50, "seed": 7})
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
    assert r.extra["dropped_transfers"] > 0


def test_runner_watchdog_reports_a_stalled_worker(capfd):
    model = QueensModel(11)
    r = solve_workers(model, devices=(), engines=_cpu_engines(model, 2), watchdog_s=0.05,
                      faults={"stall_worker": 1, "stall_s": 0.3})
    assert (r.tree, r.sol) == (166925, 2680)
    assert r.extra["watchdog_events"] >= 1
    assert "stuck in phase 'report'" in capfd.readouterr().err


def test_runner_env_faults(monkeypatch):
    monkeypatch.setenv("TTS_FAULT_STEAL_FAIL_PCT", "100")  # no transfer ever happens
    model = PfspModel(14, 1)
    r = solve_workers(model, devices=(), engines=_cpu_engines(model, 3))
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
    assert sum(r.extra["sent_nodes"]) == 0


def test_cpulist_parser():
    C = ops.cpu()
    assert C.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert C.parse_cpulist("") == []
    assert len(C.allowed_cpus()) >= 1


def test_knuth_estimate_brackets_known_trees():
    # unbiased random-probe estimate of the explored tree (csrc/core/estimate.hpp)
    from dist_gpu_accelerated_tree_search_amd import PfspModel, QueensModel, ops

    C = ops.cpu()
    m = PfspModel(14, 0)
    e = C.tree_estimate(m, m.best_known, 200000, 7, 6)  # deterministic for (probes, seed, threads)
    assert 0.5 * 2573652 < e["tree"] < 2.0 * 2573652, e["tree"]
    assert e["per_level"][0] == float(len(m.warmup(m.best_known, 2)[0]))  # level 1 is exact: the root's pushed children
    q = C.tree_estimate(QueensModel(10), 0, 20000, 5, 2)
    assert 0.7 * 35538 < q["tree"] < 1.3 * 35538, q["tree"]


def test_pool_weight_progress_on_cpu_engine():
    from dist_gpu_accelerated_tree_search_amd import PfspModel, ops
    from dist_gpu_accelerated_tree_search_amd.search import progress_weights

    m = PfspModel(14, 0)
    w = progress_weights(m)
    assert w[0] == 1.0 and abs(w[1] - 1 / 20) < 1e-15
    e = ops.cpu().make_pfsp_cpu_engine(m.native, 0, 64, 1)
    e.begin(m.root(), m.best_known)
    assert e.pool_weight(w) == 1.0
    e.run(max_launches=3)
    mid = e.pool_weight(w)
    assert 0.0 <= mid < 1.0
    e.run()
    assert e.pool_weight(w) == 0.0
