"""Distributed runtime with GPU engines on one MI355X (ranks share the device; the
status/steal protocol runs over gloo). Nodes leave and enter the device pools
through the device-staged branch of Comm.execute_transfers (engine.export_to into
a device buffer on the transfer stream, a host hop around the gloo send/recv,
engine.import_from), so only the RCCL call itself is not exercised here."""
import pytest

from dist_gpu_accelerated_tree_search_amd.parallel.launch import spawn_local
from dist_gpu_accelerated_tree_search_amd.parallel.workers import solve_rank

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4])
def test_gpu_ranks_golden(world):
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "gpu", "comm": "gloo", "device": 0,
            "engine": {"ring_bytes": 1 << 28, "max_parents": 1 << 14},
            "dist": {"slice_min_s": 0.0001, "init_per_rank": 8}}
    res = spawn_local(world, solve_rank, (spec,), timeout=600)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == (2573652, 2648, 1377)


def test_gpu_native_session():
    # bench.py's N > 1 path: runtime.DistSolver (one native call per solve) with GPU engines
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "gpu", "comm": "gloo", "device": 0, "session": True,
            "repeat": 3, "engine": {"ring_bytes": 1 << 28, "max_parents": 1 << 16}}
    res = spawn_local(2, solve_rank, (spec,), timeout=600)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == (2573652, 2648, 1377)


def test_gpu_ranks_queens():
    spec = {"problem": "nqueens", "N": 13, "backend": "gpu", "comm": "gloo", "device": 0,
            "engine": {"ring_bytes": 1 << 28, "max_parents": 1 << 12}, "dist": {"slice_min_s": 0.0001}}
    res = spawn_local(2, solve_rank, (spec,), timeout=600)
    assert (res[0]["tree"], res[0]["sol"]) == (4674889, 73712)


def test_gpu_skewed_start_is_balanced_through_device_staging():
    # every Step-1 node starts on rank 0; GPU-scale thresholds (window 2^14: needy
    # below 4096 nodes, donors from 16384) must spread ta008 LB1_d over 4 ranks
    spec = {"problem": "pfsp", "inst": 8, "lb": 0, "backend": "gpu", "comm": "gloo", "device": 0,
            "engine": {"ring_bytes": 1 << 28, "max_parents": 1 << 14},
            "dist": {"start_on": 0, "split": False, "init_per_rank": 25}}
    res = spawn_local(4, solve_rank, (spec,), timeout=600)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == (113458723, 808498, 1206)
    per = [w["tree"] for w in res[0]["workers"]]
    mean = sum(per) / len(per)
    print("per-rank tree", per, "rounds", res[0]["extra"]["rounds"])
    assert max(per) <= 1.5 * mean, per
    assert res[0]["extra"]["needy_below"] == 4096 and res[0]["extra"]["donor_min"] == 16384
    assert sum(r["comm"]["device_transfers"] for r in res) > 0
    assert sum(r["comm"]["host_transfers"] for r in res) == 0
    assert sum(res[0]["extra"]["sent_nodes"]) == sum(res[0]["extra"]["received_nodes"]) > 0


@pytest.mark.parametrize("world", [1, 2])
def test_gpu_time_box(world):
    # bench.py's ta056 extra: a time-boxed LB2 solve stops on every rank together
    spec = {"problem": "pfsp", "inst": 56, "lb": 2, "backend": "gpu", "comm": "gloo", "device": 0, "session": True,
            "engine": {"ring_bytes": 1 << 30}, "dist": {"time_limit_s": 0.5}}
    res = spawn_local(world, solve_rank, (spec,), timeout=600)
    for r in res:
        assert r["extra"]["complete"] is False and r["tree"] > 0 and r["best"] == 3679
        assert r["t_search"] < 5.0


def test_gpu_session_round_robin_step1():
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "gpu", "comm": "gloo", "device": 0, "session": True,
            "repeat": 2, "engine": {"ring_bytes": 1 << 28, "max_parents": 1 << 16},
            "dist": {"split": False, "init_per_rank": 64}}
    res = spawn_local(2, solve_rank, (spec,), timeout=600)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == (2573652, 2648, 1377)


@pytest.mark.parametrize("live", [False, True])
def test_gpu_unknown_optimum_multi_rank(live):
    # -u 0 on 2 ranks: the optimum is found with and without the live incumbent exchange
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "gpu", "comm": "gloo", "device": 0, "session": True,
            "ub": 0, "engine": {"ring_bytes": 1 << 30, "max_parents": 1 << 16}, "dist": {"live_best": live}}
    res = spawn_local(2, solve_rank, (spec,), timeout=600, env={"TTS_DIVE": "0"})  # from +inf (no dive)
    assert all(r["best"] == 1377 for r in res)


@pytest.mark.parametrize("key,streams", [((14, 1), 2), ((14, 1), 3), ((8, 0), 3)])
def test_gpu_multi_engine_golden(key, streams):
    # sub-engines on one GPU (own stream and host thread each) as one engine
    from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.search import solve_engine

    gold = {(14, 1): (2573652, 2648, 1377), (8, 0): (113458723, 808498, 1206)}[key]
    model = PfspModel(*key)
    eng = model.make_engine("gpu", 0, EngineOptions(streams=streams, ring_bytes=3 << 30, max_parents=1 << 16))
    for _ in range(2):
        r = solve_engine(model, eng)
        assert (r.tree, r.sol, r.best) == gold


@pytest.mark.parametrize("key,streams", [((14, 1), 2), ((8, 0), 3)])
def test_gpu_multi_engine_split_golden(key, streams):
    # stream_split: the solve is split in the graph between the sub-engines (same begin
    # nodes, disjoint shares after the replicated prefix, two-level iterations included)
    from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.search import solve_engine

    gold = {(14, 1): (2573652, 2648, 1377), (8, 0): (113458723, 808498, 1206)}[key]
    model = PfspModel(*key)
    eng = model.make_engine("gpu", 0, EngineOptions(streams=streams, stream_split=512, ring_bytes=3 << 30))
    for _ in range(2):
        r = solve_engine(model, eng)
        assert (r.tree, r.sol, r.best) == gold


@pytest.mark.parametrize("split", [0, 512])
def test_gpu_multi_engine_queens(split):
    # (split 512: the default N-Queens configuration of the CLI and bench.py)
    from dist_gpu_accelerated_tree_search_amd import EngineOptions, QueensModel
    from dist_gpu_accelerated_tree_search_amd.search import solve_engine

    model = QueensModel(13, 1)
    eng = model.make_engine("gpu", 0, EngineOptions(streams=2, stream_split=split, ring_bytes=1 << 29,
                                                    max_parents=1 << 14))
    for _ in range(2):
        r = solve_engine(model, eng)
        assert (r.tree, r.sol) == (4674889, 73712)


def test_gpu_multi_engine_ranks():
    # 2 ranks, each rank engine = 2 sub-engines (4 engines on one GPU), native session
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "gpu", "comm": "gloo", "device": 0, "session": True,
            "repeat": 2, "engine": {"ring_bytes": 1 << 29, "max_parents": 1 << 15, "streams": 2}}
    res = spawn_local(2, solve_rank, (spec,), timeout=600)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == (2573652, 2648, 1377)


def test_gpu_cpu_worker_per_rank():
    # -C 1 under the process-per-GPU runtime: GPU engine + CPU worker per rank
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "gpu", "comm": "gloo", "device": 0, "session": True,
            "repeat": 2, "engine": {"ring_bytes": 1 << 29, "max_parents": 1 << 14},
            "dist": {"cpu_workers": 2, "cpu_batch": 256}}
    res = spawn_local(2, solve_rank, (spec,), timeout=600)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == (2573652, 2648, 1377)
    assert len(res[0]["workers"]) == 4


def test_gpu_cli_spawn_two_ranks_one_device(tmp_path):
    # the CLI's own -D 2 -C 0 path: forkserver first (cli.main), then two spawned rank
    # processes, both on device 0, node transfers over gloo
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "-m", "dist_gpu_accelerated_tree_search_amd", "pfsp", "-i", "14", "-l", "1",
                        "-D", "2", "-C", "0", "--comm", "gloo", "--device", "0", "--ring-gb", "0.25",
                        "--csv-dir", str(tmp_path)],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "Size of the explored tree: 2573652" in p.stdout, p.stdout
    assert "Optimal makespan: 1377" in p.stdout
    assert (tmp_path / "dist_multigpu.csv").exists()
