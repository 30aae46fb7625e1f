#!/usr/bin/env python3
"""Headline benchmark: explored tree nodes per second, PFSP Taillard ta014, LB1, -u 1.

BASELINE.json metric: "tree-nodes/sec (whole node), PFSP ta014 LB1 at 1/2/4/8 MI355X".
One step = one complete cooperative B&B solve of ta014 with LB1 by all N GPUs
(Step-1 host warm-up + device search + work sharing + termination + reductions),
i.e. STRONG scaling: the tree (2,573,652 nodes, sol 2,648, makespan 1377) is the
same at every N. Each step's tree/sol/makespan is checked against the golden
values, so a skipped or truncated search fails instead of reporting a number.

After the timed headline loop the other BASELINE multi-GPU configs run in the same
job (all ranks cooperating, same runtime), unless --no-extras:
  * ta021 (20x20) LB1_d, one complete solve: makespan 2297 and the -u 1 tree
    (260,069,628,524 nodes, sol 14,963,858 — deterministic at every N) are checked;
  * ta056 (50x20) LB2, a fixed time box (--box-s, default 10 s): explored nodes/s
    (the tree is ~4.6e19 nodes, profiles/r2/ta056_projection.md: no complete solve);
  * N-Queens N=17 (g=1), best of 3 complete solves: tree 8,017,021,931 and 95,815,104
    solutions checked (the BASELINE single-GPU N-Queens config; all ranks cooperate).
They become fields of the same single JSON line ("extras"). An extra that fails is
reported there (and on stderr) and the headline line is still printed; a watchdog
(--extras-timeout) prints the line and ends every rank if an extra hangs.

Launch: python bench.py [--gpus 1 --steps K --warmup W]
        python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
               --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints exactly one JSON line on stdout; everything else goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

# ta014 LB1 (-u 1) golden values and the reference throughput on the same tree.
GOLDEN = {(14, 1): (2573652, 2648, 1377), (14, 0): (2573652, 2648, 1377), (14, 2): (144639, 0, 1377)}
# fastest reference implementation of this tree = pfsp_omp_c.out -C 8
# -l 0 (LB1_d, identical tree to LB1) at 23 M nodes/s; no published GPU number exists.
BASELINE_NODES_PER_S = 23.0e6
# ta021 LB1_d -u 1: tree / sol / makespan measured on one MI355X (profiles/r2/suite/);
# the makespan is Taillard's optimum. Reference single-GPU wall times (bound not
# recorded, pfsp/data/single-GPU.py:23,42): V100 CUDA 1308.79 s, MI50 HIP 2538.23 s.
TA021_GOLDEN = (260069628524, 14963858, 2297)
TA021_REF_S = 1308.79


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Emitter:
    """Prints the single JSON line exactly once (main thread or watchdog).

    Everything else a process writes to its standard output — including native
    libraries writing to file descriptor 1 directly (gloo's connection banner, HIP or
    RCCL messages) — goes to stderr: fd 1 is pointed at stderr for the whole run and
    the line is written through a private duplicate of the original stdout."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.lock = threading.Lock()
        self.done = False
        sys.stdout.flush()
        self.fd = os.dup(1)
        os.dup2(2, 1)

    def emit(self, rec: dict) -> None:
        with self.lock:
            if self.done:
                return
            self.done = True
            if self.rank == 0:
                os.write(self.fd, (json.dumps(rec) + "\n").encode())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--inst", type=int, default=14)
    ap.add_argument("--lb", type=int, default=1)
    ap.add_argument("--ub", type=int, default=1)
    ap.add_argument("--max-parents", type=int, default=1 << 19)
    ap.add_argument("--ring-gb", type=float, default=32.0)
    ap.add_argument("--init-per-rank", type=int, default=25)
    ap.add_argument("--streams", type=int, default=1,
                    help="headline engines per GPU (csrc/core/multi_engine.hpp), the solve split between them")
    ap.add_argument("--stream-split", type=int, default=512,
                    help="with --streams > 1: parents per engine at the in-graph split")
    ap.add_argument("--no-ws", action="store_true", help="static partition (ref -w 0 / -L 0)")
    ap.add_argument("--backend", choices=["gpu", "cpu"], default="gpu")
    ap.add_argument("--comm", choices=["nccl", "gloo"], default="nccl",
                    help="process group for node transfers (gloo: ranks may share one GPU, for tests)")
    ap.add_argument("--device", type=int, default=None, help="GPU of this rank (default LOCAL_RANK)")
    ap.add_argument("--no-extras", action="store_true", help="headline only (no ta021 / ta056 runs)")
    ap.add_argument("--extras", default="ta021,ta056,nq17", help="comma list of extras to run")
    ap.add_argument("--box-s", type=float, default=10.0, help="ta056 LB2 time box (seconds)")
    ap.add_argument("--extras-timeout", type=float, default=300.0,
                    help="watchdog: print the line and end every rank after this many seconds of extras")
    ap.add_argument("--extra-inst-lb1d", type=int, default=21, help=argparse.SUPPRESS)
    ap.add_argument("--extra-inst-lb2", type=int, default=56, help=argparse.SUPPRESS)
    ap.add_argument("--extra-queens-n", type=int, default=17, help=argparse.SUPPRESS)
    ap.add_argument("--extra-ring-gb", type=float, default=64.0)
    ap.add_argument("--extra-streams", type=int, default=3,
                    help="engines per GPU for the extras (csrc/core/multi_engine.hpp; 1 = one engine)")
    ap.add_argument("--extra-streams-lb2", type=int, default=4,
                    help="engines per GPU for the LB2 extra (ta056 0.177 -> 0.179 G nodes/s with 4; "
                         "ta021 keeps 3: profiles/r6/extras_streams_3_vs_4.txt)")
    ap.add_argument("--extra-max-parents", type=int, default=1 << 19)
    a = ap.parse_args()
    out = Emitter()  # before anything can write to stdout

    import torch  # noqa: F401  (before the HIP extension: one HIP runtime per process)

    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.parallel.comm import Comm
    from dist_gpu_accelerated_tree_search_amd.parallel.runtime import DistConfig, DistSolver

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # a failed RCCL point-to-point preflight is reported (stderr and the JSON line) and the
    # run continues WITHOUT node transfers (static in-search split, ref -w 0 -L 0), so the
    # numbers that need no transfer are still measured
    comm = Comm(use_gpu=(a.backend == "gpu" and a.comm == "nccl"), device=a.device, preflight_raise=False)
    if comm.preflight is not None:
        log(f"rank {comm.rank}: RCCL point-to-point preflight: {comm.preflight}")
    if not comm.p2p_ok:
        log(f"rank {comm.rank}: point-to-point transfers FAILED the preflight on some rank: "
            "running without work sharing (static partition)")
        a.no_ws = True
    model = PfspModel(a.inst, a.lb)
    opts = EngineOptions(max_parents=a.max_parents, ring_bytes=int(a.ring_gb * (1 << 30)), streams=max(1, a.streams),
                         stream_split=a.stream_split if a.streams > 1 else 0)
    device = (comm.topo.local_rank if a.device is None else a.device) if a.backend == "gpu" else 0
    engine = model.make_engine(a.backend, device, opts)
    cfg = DistConfig(init_per_rank=a.init_per_rank, ws=not a.no_ws, L=not a.no_ws)
    golden = GOLDEN.get((a.inst, a.lb)) if a.ub == 1 else None

    # one native call per solve (runtime.DistSolver): warm-up, split, rounds and reductions
    # at N > 1; at N = 1 the warm-up and the engine's fused solve, no interpreter between
    solver = DistSolver(model, engine, comm, cfg, window=a.max_parents)

    def step():
        raw = solver.solve_raw(a.ub)
        got = (raw[1], raw[2], raw[0])
        if golden and got != golden:
            raise SystemExit(f"wrong result {got} != golden {golden}")
        return raw, got[0]

    for _ in range(a.warmup):
        step()
    comm.barrier()
    t0 = time.perf_counter()
    tree = 0
    raw = None
    for _ in range(a.steps):
        raw, t = step()
        tree += t
    comm.barrier()
    dt_local = time.perf_counter() - t0
    last = solver.result(*raw)
    dt = float(comm.allgather_f64([dt_local]).max())
    value = tree / dt
    if comm.rank == 0:
        log(f"last step: elapsed {last.elapsed * 1e3:.3f} ms, init {last.t_init * 1e3:.3f} ms, "
            f"search {last.t_search * 1e3:.3f} ms, rounds {last.extra.get('rounds')}, "
            f"per-rank tree {[w.tree for w in last.workers]}, control plane "
            f"{'shm' if getattr(comm, 'ctl', None) is not None else comm.backend}")
    rec = {
        "metric": "tree-nodes/sec (whole node), PFSP ta014 LB1 at 1/2/4/8 MI355X",
        "value": value,
        "unit": "nodes/s",
        "n_gpus": comm.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": value / BASELINE_NODES_PER_S,
        "dtype": "int32",
        "data": "Taillard ta%03d regenerated from its seed (exact benchmark instance, no download)" % a.inst,
        "config": {
            "model": f"PFSP ta{a.inst:03d} ({model.jobs}x{model.machines}) {['LB1_d', 'LB1', 'LB2'][a.lb]} -u {a.ub}",
            "global_batch": a.max_parents,
            "seq_len": model.jobs,
            "parallelism": f"dp{comm.world}" + ("" if a.no_ws else "+ws"),
            "tree": last.tree,
            "sol": last.sol,
            "makespan": last.best,
            "rounds_last_step": last.extra.get("rounds"),
            "baseline": "reference pfsp_omp_c.out -C 8 -l 0, 23 M nodes/s (BASELINE.md, same tree)",
            "p2p_preflight": comm.preflight,
            "p2p_ok": comm.p2p_ok,
        },
    }
    del solver, engine

    if not a.no_extras:
        extras: dict = {}
        rec["extras"] = extras

        def fire():
            extras["error"] = f"watchdog: extras exceeded {a.extras_timeout:.0f} s; every rank exits"
            log(f"rank {comm.rank}: {extras['error']}")
            out.emit(rec)
            os._exit(3)  # the line is printed, but a hung extra is a failure

        dog = threading.Timer(a.extras_timeout, fire)
        dog.daemon = True
        dog.start()
        which = [x for x in a.extras.split(",") if x]
        ok = True
        for name in which:
            if not ok:
                extras[name] = {"skipped": "an earlier extra failed"}
                continue
            try:
                if name == "ta021":
                    extras[name] = run_solve_extra(a, comm, device, a.extra_inst_lb1d, 0, time_limit=0.0)
                elif name == "ta056":
                    extras[name] = run_solve_extra(a, comm, device, a.extra_inst_lb2, 2, time_limit=a.box_s)
                elif name == "nq17":
                    extras[name] = run_queens_extra(a, comm, device, a.extra_queens_n)
                else:
                    extras[name] = {"error": "unknown extra"}
                mine_ok = 1
            except Exception as e:  # noqa: BLE001 - reported in the line, headline still printed
                log(f"rank {comm.rank}: extra {name} failed: {e!r}")
                extras[name] = {"error": repr(e)[:300]}
                mine_ok = 0
            # every rank learns whether all ranks succeeded before the next collective solve
            ok = bool(comm.allreduce_i64([mine_ok], "min")[0])
        dog.cancel()
    out.emit(rec)
    comm.close()
    return 0


def _make_solver(model, a, device: int, opts, comm, cfg):
    from dist_gpu_accelerated_tree_search_amd.parallel.runtime import DistSolver

    engine = model.make_engine(a.backend, device, opts)
    return engine, DistSolver(model, engine, comm, cfg, window=opts.max_parents)


def _agreed_setup(comm, name: str, build):
    """Engine + solver of an extra on every rank, then one agreement: if any rank failed
    to set up (e.g. device memory), every rank raises before the collective solve, so no
    rank waits in a solve that another rank never enters."""
    made, err = None, None
    try:
        made = build()
    except Exception as e:  # noqa: BLE001 - agreed on below, re-raised on every rank
        err = e
        log(f"rank {comm.rank}: extra {name} setup failed: {e!r}")
    if not bool(comm.allreduce_i64([0 if err else 1], "min")[0]):
        made = None
        raise RuntimeError(f"{name}: setup failed on some rank" + (f" (here: {err!r})" if err else ""))
    return made


QUEENS_GOLDEN = {17: (8017021931, 95815104), 16: (1141190302, 14772512), 12: (856188, 14200), 11: (166925, 2680)}
QUEENS_REF_S = {17: 807.0}  # reference nqueens_c.out -N 17, sequential


def run_queens_extra(a, comm, device: int, N: int) -> dict:
    """N-Queens N (g=1): best of 3 cooperative solves with the headline's runtime."""
    from dist_gpu_accelerated_tree_search_amd.models.nqueens import QueensModel
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions
    from dist_gpu_accelerated_tree_search_amd.parallel.runtime import DistConfig

    model = QueensModel(N, 1)
    # engines per GPU with the solve split between them in the graph: N=17 74 -> 48 ms with
    # two (profiles/r3/queens/streams_probe.txt); with the wave-stack finishing and transfer
    # streams created on first use (each engine's compute stream on its own hardware queue)
    # three: 20.4 -> 18.2 ms (profiles/r6/queens/lazy_xfer_ab.txt)
    opts = EngineOptions(max_parents=1 << 19, ring_bytes=8 << 30, streams=3, stream_split=512) \
        if a.backend == "gpu" else EngineOptions(streams=2, stream_split=8)
    t_setup = time.perf_counter()
    engine, solver = _agreed_setup(comm, f"N-Queens N={N}", lambda: _make_solver(
        model, a, device, opts, comm, DistConfig(init_per_rank=a.init_per_rank, ws=not a.no_ws, L=not a.no_ws)))
    t_setup = time.perf_counter() - t_setup
    best_dt, r = None, None
    for _ in range(3):
        comm.barrier()
        t0 = time.perf_counter()
        raw = solver.solve_raw(1)
        comm.barrier()
        dt = float(comm.allgather_f64([time.perf_counter() - t0]).max())
        r = solver.result(*raw)
        best_dt = dt if best_dt is None else min(best_dt, dt)
    gold = QUEENS_GOLDEN.get(N)
    d = {"config": f"N-Queens N={N} g=1", "n_gpus": comm.world, "seconds": best_dt, "tree": r.tree, "sol": r.sol,
         "nodes_per_s": r.tree / best_dt, "engine_setup_s": t_setup, "engines_per_gpu": opts.streams,
         "golden_ok": gold is None or (r.tree, r.sol) == gold}
    if N in QUEENS_REF_S:
        d["ref_seconds_seq"] = QUEENS_REF_S[N]
        d["speedup_vs_ref"] = QUEENS_REF_S[N] / best_dt
    if not d["golden_ok"]:
        raise RuntimeError(f"N-Queens N={N}: (tree, sol) {(r.tree, r.sol)} != golden {gold}")
    del solver, engine
    return d


def run_solve_extra(a, comm, device: int, inst: int, lb: int, time_limit: float) -> dict:
    """One cooperative solve (or a time box) of another BASELINE config on all ranks,
    with the headline's runtime (DistSolver: same Step 1, split and rounds)."""
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.parallel.runtime import DistConfig

    model = PfspModel(inst, lb)
    # big trees: several engines per GPU fill it better than one (profiles/r3/streams*.txt)
    streams = max(1, a.extra_streams_lb2 if lb == 2 else a.extra_streams)
    opts = EngineOptions(ring_bytes=int(a.extra_ring_gb * (1 << 30)), streams=streams,
                         max_parents=a.extra_max_parents)
    t_setup = time.perf_counter()
    cfg = DistConfig(init_per_rank=a.init_per_rank, ws=not a.no_ws, L=not a.no_ws, time_limit_s=time_limit)
    engine, solver = _agreed_setup(comm, f"ta{inst:03d}", lambda: _make_solver(model, a, device, opts, comm, cfg))
    t_setup = time.perf_counter() - t_setup
    comm.barrier()
    t0 = time.perf_counter()
    raw = solver.solve_raw(1)
    comm.barrier()
    dt = float(comm.allgather_f64([time.perf_counter() - t0]).max())
    r = solver.result(*raw)
    name = f"ta{inst:03d} ({model.jobs}x{model.machines}) {['LB1_d', 'LB1', 'LB2'][lb]} -u 1"
    d = {"config": name, "n_gpus": comm.world, "seconds": dt, "tree": r.tree, "sol": r.sol, "makespan": r.best,
         "nodes_per_s": r.tree / dt, "complete": bool(r.extra.get("complete", True)),
         "rounds": r.extra.get("rounds"), "per_rank_tree": [w.tree for w in r.workers],
         "engine_setup_s": t_setup, "engines_per_gpu": streams, "max_parents": opts.max_parents,
         # where the ranks' time went (the round loop's clocks): idle without work, load
         # balancing (plan + transfers), termination checks; rounds that overlapped replays
         "per_rank_t_idle": [round(w.t_idle, 4) for w in r.workers],
         "per_rank_t_load_bal": [round(w.t_load_bal, 4) for w in r.workers],
         "per_rank_t_termination": [round(w.t_termination, 4) for w in r.workers],
         "overlapped_rounds": r.extra.get("overlapped_rounds")}
    if time_limit > 0:
        d["time_box_s"] = time_limit
    else:
        gold = TA021_GOLDEN if (inst, lb) == (21, 0) else None
        if gold is not None:
            d["golden_ok"] = (r.tree, r.sol, r.best) == gold
            d["ref_seconds_v100"] = TA021_REF_S
            d["speedup_vs_ref"] = TA021_REF_S / dt
            if not d["golden_ok"]:
                raise RuntimeError(f"{name}: (tree, sol, makespan) {(r.tree, r.sol, r.best)} != golden {gold}")
        elif r.best != model.best_known:
            raise RuntimeError(f"{name}: makespan {r.best} != best known {model.best_known}")
    del solver, engine
    return d


if __name__ == "__main__":
    raise SystemExit(main())
