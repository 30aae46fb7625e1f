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
    model = PfspModel(8, 0)  # 113M nodes: long enough for steals between the engines
    r = solve_workers(model, devices=(0, 0), m=1000, pin=True, opts=SMALL)
    assert (r.tree, r.sol, r.best) == (113458723, 808498, 1206)
    assert r.extra["device_transfers"] > 0
    H = ops.hip()
    cpus = H.device_cpus(0)
    assert isinstance(cpus, list)
    assert r.extra["pinned"][0] == bool(cpus and set(cpus) & set(H.allowed_cpus()))
    # host staging path (device_steals off) gives the same tree
    r = solve_workers(model, devices=(0, 0), m=1000, device_steals=False, opts=SMALL)
    assert (r.tree, r.sol, r.best) == (113458723, 808498, 1206)
    assert r.extra["device_transfers"] == 0


def test_runner_faults_with_gpu_engines():
    r = solve_workers(PfspModel(14, 1), devices=(0, 0, 0), m=100, opts=SMALL,
                      faults={"delay_us": 200, "steal_fail_pct": 30})
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
