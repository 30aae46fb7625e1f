"""Native multi-worker runner with device engines (ref pfsp_multigpu_cuda.c -D/-C)
and the native GPU CLIs. On a one-GPU box several engines share device 0."""
import subprocess

import pytest

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, QueensModel, ops
from dist_gpu_accelerated_tree_search_amd.search import solve_workers

pytestmark = pytest.mark.gpu
SMALL = EngineOptions(ring_bytes=1 << 30, cpu_batch=1024)


@pytest.mark.parametrize("devices,cpu", [((0,), 0), ((0, 0), 0), ((0,), 2), ((0, 0, 0), 2)])
def test_runner_gpu_workers_golden(devices, cpu):
    r = solve_workers(PfspModel(14, 1), devices=devices, cpu_threads=cpu, opts=SMALL)
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
    assert len(r.workers) == len(devices) + (1 if cpu else 0)


def test_runner_gpu_lb2_and_queens():
    r = solve_workers(PfspModel(10, 2), devices=(0, 0), cpu_threads=2, opts=SMALL)
    assert (r.tree, r.sol, r.best) == (8122579, 0, 1108)
    r = solve_workers(QueensModel(14), devices=(0, 0), opts=EngineOptions(max_parents=1 << 20, ring_bytes=1 << 30))
    assert (r.tree, r.sol) == (27358552, 365596)


def test_runner_gpu_unknown_optimum():
    r = solve_workers(PfspModel(14, 0), devices=(0, 0), cpu_threads=2, ub=0, opts=SMALL)
    assert r.best == 1377


def _cli(name, *args, cwd=None):
    from dist_gpu_accelerated_tree_search_amd.ops.build import BIN

    exe = BIN / name
    if not exe.exists():
        pytest.fail(f"{exe} not built")
    return subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300, cwd=cwd)


def test_native_pfsp_gpu_cli(tmp_path):
    ops.require_gpu(0)
    out = _cli("pfsp_gpu", "-i", "14", "-l", "1", "-D", "1", "-C", "1", cwd=tmp_path)
    assert (tmp_path / "multigpu.csv").exists()
    assert out.returncode == 0, out.stdout + out.stderr
    assert "2573652" in out.stdout and "1377" in out.stdout


def test_native_nqueens_gpu_cli():
    ops.require_gpu(0)
    out = _cli("nqueens_gpu", "-N", "13", "-D", "1")
    assert out.returncode == 0, out.stdout + out.stderr
    assert "4674889" in out.stdout and "73712" in out.stdout


def test_runner_device_to_device_steals_and_pinning():
    # all initial work on engine 0: engine 1 must be fed by steals
    model = PfspModel(8, 0)
    H = ops.hip()
    nodes, t1, s1, best = model.warmup(model.initial_best(1), 50)
    for dev_steals in (True, False):
        engines = [model.make_engine("gpu", 0, SMALL) for _ in range(2)]
        out = H.run_workers(engines, [nodes, nodes[:0]], int(best), m=1000, pin=True, device_steals=dev_steals)
        ws = out["workers"]
        assert (t1 + sum(w["tree"] for w in ws), s1 + sum(w["sol"] for w in ws), out["best"]) == \
            (113458723, 808498, 1206)
        assert ws[1]["received"] > 0
        assert (ws[0]["device_transfers"] > 0) == dev_steals
    cpus = H.device_cpus(0)
    assert isinstance(cpus, list)
    assert ws[0]["pinned"] == bool(cpus and set(cpus) & set(H.allowed_cpus()))


def test_runner_faults_with_gpu_engines():
    r = solve_workers(PfspModel(14, 1), devices=(0, 0, 0), m=100, opts=SMALL,
                      faults={"delay_us": 200, "steal_fail_pct": 30})
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)


def test_python_cli_cpu_worker_and_single_process(tmp_path):
    import sys

    base = [sys.executable, "-m", "dist_gpu_accelerated_tree_search_amd", "pfsp", "-i", "14", "-l", "1",
            "--csv-dir", str(tmp_path), "--ring-gb", "1"]
    for extra in (["-D", "1", "-C", "1"], ["-D", "2", "--single-process", "--gpus-list", "0,0"]):
        out = subprocess.run(base + extra, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "2573652" in out.stdout and "1377" in out.stdout
    assert (tmp_path / "multigpu.csv").exists()
