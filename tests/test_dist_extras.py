"""Round-3 runtime features on CPU ranks (gloo): the point-to-point preflight, time
boxes, the live incumbent exchange, the round-robin Step 1 of the native session,
checkpoint consistency, and bench.py's extras path (the other BASELINE configs run
in the same job as the headline)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd.parallel.launch import free_port, spawn_local
from dist_gpu_accelerated_tree_search_amd.parallel.workers import preflight_rank, solve_rank

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = (2573652, 2648, 1377)


@pytest.mark.parametrize("world", [2, 3])
def test_p2p_preflight_passes(world):
    res = spawn_local(world, preflight_rank, ({"nbytes": 1 << 15},), timeout=120)
    for r in res:
        assert r["ok"], r
        assert r["info"]["peers"] == world - 1 and r["info"]["bytes_per_peer"] == 1 << 15


def test_p2p_preflight_detects_corruption():
    res = spawn_local(3, preflight_rank, ({"nbytes": 1 << 12, "corrupt_rank": 1},), timeout=120)
    assert res[0]["ok"] and res[2]["ok"]
    assert not res[1]["ok"] and "does not match" in res[1]["error"] and "[0]" in res[1]["error"]


@pytest.mark.parametrize("world", [1, 2])
def test_time_box_stops_every_rank(world):
    # ta056 LB2 cannot finish: the session stops at the first round after the box on
    # every rank, reports complete=False and the nodes explored so far
    spec = {"problem": "pfsp", "inst": 56, "lb": 2, "backend": "cpu", "session": True,
            "dist": {"time_limit_s": 0.3}}
    res = spawn_local(world, solve_rank, (spec,), timeout=300)
    for r in res:
        assert r["extra"]["complete"] is False
        assert r["tree"] > 0 and r["best"] == 3679
        assert r["t_search"] < 30
    assert len({r["tree"] for r in res}) == 1


@pytest.mark.parametrize("world", [2, 3])
def test_session_round_robin_step1(world):
    # split=False: host BFS to world * init_per_rank nodes, rank-strided share
    # (ref roundRobin_distribution), then the rounds; golden tree
    spec = {"problem": "pfsp", "inst": 14, "lb": 0, "backend": "cpu", "session": True, "repeat": 2,
            "dist": {"split": False, "init_per_rank": 16}}
    res = spawn_local(world, solve_rank, (spec,), timeout=300)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == GOLD
    assert all(w["tree"] > 0 for w in res[0]["workers"])


@pytest.mark.parametrize("world", [2, 4])
def test_live_incumbent_with_unknown_optimum(world):
    # -u 0: the optimum must be found whatever the exchange; with the live exchange a
    # rank's better solution prunes the other ranks' pools between rounds too
    trees = {}
    for live in (False, True):
        spec = {"problem": "pfsp", "inst": 2, "lb": 0, "backend": "cpu", "ub": 0, "session": True,
                "dist": {"live_best": live}}
        # no dive: every rank starts from +inf, so incumbents really have to travel
        res = spawn_local(world, solve_rank, (spec,), timeout=300, env={"TTS_DIVE": "0"})
        assert all(r["best"] == 1359 for r in res)
        trees[live] = res[0]["tree"]
    assert trees[True] > 0 and trees[False] > 0


def test_checkpoint_rejects_mixed_rounds(tmp_path):
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel
    from dist_gpu_accelerated_tree_search_amd.parallel import checkpoint as ckpt

    model = PfspModel(14, 0)
    eng = model.make_engine("cpu")
    eng.begin(model.root(), 1377)
    eng.run(3)
    ckpt.save(str(tmp_path), 0, 2, model, eng, 10, 0, 1377, 5)
    ckpt.save(str(tmp_path), 1, 2, model, eng, 10, 0, 1377, 4)  # crashed before rewriting round 5
    with pytest.raises(ValueError, match="different rounds"):
        ckpt.load_all(str(tmp_path), model)
    ckpt.save(str(tmp_path), 1, 2, model, eng, 10, 0, 1377, 5)
    nodes, tree, sol, best, rounds = ckpt.load_all(str(tmp_path), model)
    assert rounds == 5 and tree == 20 and len(nodes) == 2 * eng.size()
    assert isinstance(nodes, np.ndarray)


def test_bench_extras_cpu_gloo():
    # the driver's launch line with 2 ranks (CPU engines, gloo): one JSON line with the
    # headline and the extras; small stand-ins keep it short (ta014 for the complete
    # LB1_d solve, a 0.5-s ta056 LB2 box, N-Queens N=11 for N=17)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2",
           "--steps", "1", "--warmup", "0", "--backend", "cpu", "--comm", "gloo", "--extra-inst-lb1d", "14",
           "--box-s", "0.5", "--extra-queens-n", "11"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and (rec["config"]["tree"], rec["config"]["sol"], rec["config"]["makespan"]) == GOLD
    ex = rec["extras"]
    assert (ex["ta021"]["tree"], ex["ta021"]["sol"], ex["ta021"]["makespan"]) == GOLD
    assert ex["ta021"]["complete"] is True
    assert ex["ta056"]["complete"] is False and ex["ta056"]["nodes_per_s"] > 0
    assert ex["ta056"]["time_box_s"] == 0.5
    assert (ex["nq17"]["tree"], ex["nq17"]["sol"]) == (166925, 2680) and ex["nq17"]["golden_ok"] is True


def test_bench_four_ranks_cpu_gloo():
    # the driver's N=4 launch line shape (4 ranks, one JSON line from rank 0, golden tree,
    # per-rank work shares), CPU engines
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "4",
           "--steps", "2", "--warmup", "1", "--backend", "cpu", "--comm", "gloo", "--no-extras"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["steps"] == 2 and rec["config"]["parallelism"] == "dp4+ws"
    assert (rec["config"]["tree"], rec["config"]["sol"], rec["config"]["makespan"]) == GOLD


def test_bench_runs_without_transfers_after_failed_preflight():
    # a rank whose point-to-point check fails (fault injection): bench.py reports it in
    # the JSON line and measures the headline without work sharing (static split), golden
    env = dict(os.environ, TTS_FAULT_P2P_RANK="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--backend", "cpu", "--no-extras"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["config"]["p2p_ok"] is False and rec["config"]["parallelism"] == "dp2"
    assert (rec["config"]["tree"], rec["config"]["sol"], rec["config"]["makespan"]) == GOLD
    assert "FAILED the preflight" in p.stderr


def test_bench_extras_failure_still_prints_headline():
    # an extra that fails is reported in the line; the headline is printed regardless
    cmd = [sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--backend", "cpu", "--extras", "nosuch"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][0])
    assert rec["value"] > 0 and rec["extras"]["nosuch"] == {"error": "unknown extra"}


@pytest.mark.parametrize("world,problem", [(1, "pfsp"), (2, "pfsp"), (2, "nqueens")])
def test_cpu_worker_per_rank(world, problem, tmp_path):
    # -C 1 in the process-per-rank runtime: every rank's engine is a hybrid of its main
    # engine and a CPU worker thread (csrc/core/hybrid_engine.hpp); golden tree, and the
    # CPU workers explore part of it (two workers per rank in the statistics)
    # N=12: a tree large enough that each rank's CPU worker is handed work even on a loaded host
    spec = {"problem": problem, "inst": 14, "lb": 1, "N": 12, "backend": "cpu", "session": True, "repeat": 2,
            "engine": {"cpu_batch": 64},
            "dist": {"cpu_workers": 2, "cpu_batch": 64, "m": 8, "init_per_rank": 16}}
    res = spawn_local(world, solve_rank, (spec,), timeout=300)
    gold = GOLD if problem == "pfsp" else (856188, 14200, None)
    for r in res:
        assert (r["tree"], r["sol"]) == gold[:2]
    ws = res[0]["workers"]
    assert len(ws) == 2 * world
    assert sum(w["tree"] for w in ws) + 0 <= gold[0]
    # the CPU workers took part (a loaded host may leave one rank's worker without a
    # hand-over on this small tree, so the check is on their sum)
    assert sum(ws[2 * k + 1]["tree"] for k in range(world)) > 0, ws
    from dist_gpu_accelerated_tree_search_amd.utils import report

    workers = [report.WorkerStats(**w) for w in ws]
    path = tmp_path / "dist_multigpu.csv"
    report.write_dist_multi_gpu_csv(str(path), 14, 1, 1, 1, 1, world, res[0]["best"] or 0, 8, 50000, 64,
                                    res[0]["elapsed"], res[0]["tree"], res[0]["sol"], workers,
                                    [w.dist_load_bal for w in workers], [w.t_load_bal for w in workers])
    row = path.read_text().splitlines()[1]
    assert row.count("[") >= 10 and row.endswith(",")


@pytest.mark.parametrize("streams", [2, 3])
def test_multi_engine_cpu_golden(streams):
    # several sub-engines as one engine (csrc/core/multi_engine.hpp): concurrent slices,
    # steal-half between them; repeated solves and time slices keep the golden tree
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.search import solve_engine

    model = PfspModel(14, 1)
    eng = model.make_engine("cpu", 0, EngineOptions(streams=streams, cpu_batch=64))
    for _ in range(2):
        r = solve_engine(model, eng)
        assert (r.tree, r.sol, r.best) == GOLD
    nodes, t1, s1, best = model.warmup(1377, 25)
    eng.begin(nodes, best)
    while eng.size() > 0:
        eng.run(max_seconds=0.003)
    st = eng.stats()
    assert (st["tree"] + t1, st["sol"] + s1) == GOLD[:2]


@pytest.mark.parametrize("streams", [2, 3])
def test_multi_engine_split_golden(streams):
    # stream_split: every solve is split in the graph between the sub-engines (same
    # begin nodes, disjoint shares after the replicated prefix); golden trees, and a
    # tree that dies out before the split point is counted once
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.search import solve_engine

    model = PfspModel(14, 1)
    eng = model.make_engine("cpu", 0, EngineOptions(streams=streams, stream_split=8, cpu_batch=64))
    for _ in range(2):
        r = solve_engine(model, eng)
        assert (r.tree, r.sol, r.best) == GOLD
    big = model.make_engine("cpu", 0, EngineOptions(streams=streams, stream_split=1 << 20, cpu_batch=64))
    r = solve_engine(model, big)  # the split point is never reached
    assert (r.tree, r.sol, r.best) == GOLD


def test_multi_engine_split_in_session():
    # rank split x sub-engine split (share rank * K + k of world * K), 2 ranks x 2 streams
    spec = {"problem": "pfsp", "inst": 14, "lb": 1, "backend": "cpu", "session": True, "repeat": 2,
            "engine": {"streams": 2, "stream_split": 8, "cpu_batch": 64}}
    res = spawn_local(2, solve_rank, (spec,), timeout=300)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == GOLD


def test_multi_engine_in_session():
    # a rank engine made of sub-engines inside the distributed session (2 ranks)
    spec = {"problem": "pfsp", "inst": 14, "lb": 0, "backend": "cpu", "session": True, "repeat": 2,
            "engine": {"streams": 2, "cpu_batch": 128}}
    res = spawn_local(2, solve_rank, (spec,), timeout=300)
    for r in res:
        assert (r["tree"], r["sol"], r["best"]) == GOLD


def _agreed_setup_rank(fail_rank: int) -> str:
    import importlib.util

    from dist_gpu_accelerated_tree_search_amd.parallel.comm import Comm

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    comm = Comm(use_gpu=False)
    try:
        def build():
            if comm.rank == fail_rank:
                raise MemoryError("no device memory (injected)")
            return "engine", "solver"

        try:
            bench._agreed_setup(comm, "ta021", build)
            return "ok"
        except RuntimeError as e:
            return str(e)
    finally:
        comm.close()


def test_extra_setup_failure_on_one_rank_stops_every_rank():
    # an extra whose engine cannot be built on one rank (device memory) must not leave the
    # other ranks waiting in a collective solve: every rank learns it and raises
    res = spawn_local(3, _agreed_setup_rank, (1,), timeout=120)
    assert all("setup failed on some rank" in r for r in res), res
    assert "injected" in res[1] and "injected" not in res[0]
    assert spawn_local(2, _agreed_setup_rank, (-1,), timeout=120) == ["ok", "ok"]
