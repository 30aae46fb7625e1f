"""Single-process search drivers (CPU sequential, CPU multi-core, one GPU).

The three-step structure of every reference driver is kept
(ref pfsp_multigpu_cuda.c:55-511, nqueens_gpu_cuda.cu:198-264):
  Step 1  host breadth-first warm-up until the pool holds `m` (x workers) nodes,
  Step 2  the parallel / device search,
  Step 3  host depth-first drain of whatever Step 2 leaves (nothing, on the GPU
          path: the device engine drains its pool completely).
Counting (tree / sol) and the -u incumbent rule are the reference's.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from . import ops
from .models.pfsp import EngineOptions
from .utils.report import WorkerStats


@dataclass
class SolveResult:
    best: int
    tree: int
    sol: int
    elapsed: float
    t_init: float = 0.0
    t_search: float = 0.0
    t_tail: float = 0.0
    workers: list = field(default_factory=list)
    extra: dict = field(default_factory=dict)

    @property
    def nodes_per_sec(self) -> float:
        return self.tree / self.elapsed if self.elapsed > 0 else float("inf")


def progress_weights(model) -> list[float]:
    """w[d] = share of the search space below a node of depth d: 1 / (N (N-1) ... (N-d+1))
    for PFSP permutations (the root stands for all N! of them); for N-Queens the same
    with N rows. 1 - engine.pool_weight(w) is the explored fraction of the space —
    pruned subtrees count as explored — used to project a time to solution."""
    n = model.jobs if model.kind == "pfsp" else model.N
    w, x = [], 1.0
    for d in range(n + 1):
        w.append(x)
        x /= max(1, n - d)
    return w


def solve_cpu(model, ub: int = 1, threads: int = 0, m: int = 25, batch: int = 20000, steal_cap: int = 250000,
              ws: bool = True, verbose: bool = False) -> SolveResult:
    """threads == 0: sequential (ref pfsp_c.c / nqueens_c.c); >0: multi-core WS
    (ref pfsp_omp_c.c)."""
    C = ops.cpu()
    if model.kind == "pfsp":
        r = C.run_pfsp(model.native, model.lb, model.initial_best(ub), threads=threads, m=m, batch=batch,
                       steal_cap=steal_cap, ws=ws, verbose=verbose)
    else:
        r = C.run_queens(model.N, model.G, threads=threads, m=m, batch=batch, steal_cap=steal_cap, ws=ws,
                         verbose=verbose)
    return SolveResult(best=r["best"], tree=r["tree"], sol=r["sol"], elapsed=r["elapsed"], t_init=r["t_init"],
                       t_search=r["t_search"], t_tail=r["t_tail"],
                       workers=[WorkerStats.from_dict(w) for w in r["workers"]])


def solve_engine(model, engine, ub: int = 1, m: int = 25, best: int | None = None,
                 verbose: bool = False) -> SolveResult:
    """One complete solve on an existing engine (GPU or CPU backend).

    The engine is reused across solves (allocation and graph capture are setup,
    like model initialisation); its counters are reset here."""
    t0 = time.perf_counter()
    best = model.search_best(ub) if best is None else best
    nodes, tree1, sol1, best = model.warmup(best, m)
    t1 = time.perf_counter()
    if verbose:
        from .utils.report import phase
        print(phase("Initial search on CPU completed", tree1, sol1, t1 - t0))
    st = engine.solve(nodes, int(best))  # reset + load + run to exhaustion, one native call
    launches = st["launches"]
    best = min(best, st["best"])
    t2 = time.perf_counter()
    tree, sol = tree1 + st["tree"], sol1 + st["sol"]
    if verbose:
        print(phase("Search on GPU completed", tree, sol, t2 - t1))
    # Step 3: the engine drains completely; anything left (none) goes to the host
    left = engine.size()
    if left:
        rest = engine.pop(left)
        tr, so, best = model.drain(best, rest)
        tree += tr
        sol += so
    t3 = time.perf_counter()
    if verbose:
        print(phase("Final on CPU completed", tree, sol, t3 - t2))
        print("\nExploration terminated.")
    w = WorkerStats(tree=st["tree"], sol=st["sol"], gen_child=st["tree"], t_memcpy=st["t_memcpy"],
                    t_malloc=st["t_malloc"], t_kernel=st["t_run"])
    return SolveResult(best=best, tree=tree, sol=sol, elapsed=t3 - t0, t_init=t1 - t0, t_search=t2 - t1,
                       t_tail=t3 - t2, workers=[w], extra={"launches": launches, "iters": st["iters"],
                                                           "parents": st["parents"], "syncs": st["syncs"]})


def solve_gpu(model, ub: int = 1, device: int = 0, m: int = 25, opts: EngineOptions | None = None,
              verbose: bool = False) -> SolveResult:
    """Single-GPU solve (ref pfsp_multigpu_cuda.c with -D 1 -C 0)."""
    eng = model.make_engine("gpu", device, opts)
    try:
        return solve_engine(model, eng, ub=ub, m=m, verbose=verbose)
    finally:
        del eng


def solve_workers(model, devices=(0,), cpu_threads: int = 0, ub: int = 1, m: int = 25, steal_cap: int = 250000,
                  ws: bool = True, opts: EngineOptions | None = None, engines=None, slice_min: float = 0.0005,
                  slice_max: float = 0.05, pin: bool = False, device_steals: bool = True, watchdog_s: float = 0.0,
                  faults: dict | None = None) -> SolveResult:
    """Several engines in ONE process — GPUs (`devices`, repeats allowed) plus an
    optional CPU worker with `cpu_threads` threads (-C 1) — driven by the native
    runner (csrc/core/runner.hpp), the analogue of ref pfsp_multigpu_cuda.c.
    Pass `engines` to reuse engines across solves.

    pin: pin each GPU's host thread to the CPUs of the GPU's NUMA node.
    device_steals: GPU -> GPU transfers through device staging (xGMI peer copies).
    watchdog_s / faults: stuck-phase reporting and fault injection
    ({"delay_us", "steal_fail_pct", "stall_worker", "stall_s", "seed"}; env
    TTS_FAULT_* / TTS_WATCHDOG_* also apply), see csrc/core/runner.hpp."""
    gpu = len(devices) > 0
    mod = ops.require_gpu(max(devices)) if gpu else ops.cpu()
    if engines is None:
        engines = [model.make_engine("gpu", d, opts) for d in devices]
        if cpu_threads > 0:
            engines.append(_cpu_worker(model, mod, cpu_threads, opts))
    W = len(engines)
    if W == 0:
        raise ValueError("no worker")
    t0 = time.perf_counter()
    best = model.search_best(ub)
    nodes, tree1, sol1, best = model.warmup(best, W * m)
    from .parallel.runtime import round_robin_share

    init = [np.ascontiguousarray(nodes[round_robin_share(len(nodes), w, W)]) for w in range(W)]
    # per-worker sharing thresholds: a GPU is needy below a quarter of its parent
    # window and donates from one window; a CPU worker keeps the reference's m / 2m
    # and receives at most 4*T nodes per steal (ref pfsp_multigpu_cuda.c:369-372)
    o = opts or EngineOptions()
    needy, donor, rcap = [], [], []
    for e in engines:
        if e.device >= 0:
            nb = max(m, int(o.max_parents) // 4)
            needy.append(nb)
            donor.append(max(2 * nb, int(o.max_parents)))
            rcap.append(steal_cap)
        else:
            needy.append(m)
            donor.append(2 * m)
            rcap.append(min(steal_cap, 4 * int(o.cpu_batch)))
    t1 = time.perf_counter()
    out = mod.run_workers(engines, init, int(best), m=m, steal_cap=steal_cap, slice_min=slice_min,
                          slice_max=slice_max, ws=ws, pin=pin, device_steals=device_steals,
                          watchdog_s=watchdog_s, faults=dict(faults or {}), needy_below=needy, donor_min=donor,
                          recv_cap=rcap)
    t2 = time.perf_counter()
    ws_ = out["workers"]
    tree = tree1 + sum(int(w["tree"]) for w in ws_)
    sol = sol1 + sum(int(w["sol"]) for w in ws_)
    workers = [WorkerStats(tree=int(w["tree"]), sol=int(w["sol"]), gen_child=int(w["tree"]),
                           steals=int(w["steals"]), success_steals=int(w["success_steals"]),
                           terminations=int(w["idle_rounds"]), t_memcpy=float(w["t_memcpy"]),
                           t_malloc=float(w["t_malloc"]), t_kernel=float(w["t_run_w"]),
                           t_pool_ops=float(w["t_comm"]), t_idle=float(w["t_idle"]),
                           t_termination=float(w["t_termination"])) for w in ws_]
    return SolveResult(best=min(int(best), int(out["best"])), tree=tree, sol=sol, elapsed=t2 - t0,
                       t_init=t1 - t0, t_search=t2 - t1, workers=workers,
                       extra={"rounds": max(int(w["rounds"]) for w in ws_), "engines": engines,
                              "sent_nodes": [int(w["sent"]) for w in ws_],
                              "device_transfers": sum(int(w["device_transfers"]) for w in ws_),
                              "dropped_transfers": sum(int(w["dropped_transfers"]) for w in ws_),
                              "watchdog_events": int(ws_[0]["watchdog_events"]),
                              "pinned": [bool(w["pinned"]) for w in ws_]})


def _cpu_worker(model, mod, threads: int, opts: EngineOptions | None):
    batch = (opts or EngineOptions()).cpu_batch
    if model.kind == "pfsp":
        return mod.make_pfsp_cpu_engine(model.jobs, model.machines, list(model.native.p), model.lb, batch, threads) \
            if hasattr(mod, "make_pfsp_engine") else mod.make_pfsp_cpu_engine(model.native, model.host_lb, batch,
                                                                              threads)
    return mod.make_queens_cpu_engine(model.N, model.G, batch, threads)
