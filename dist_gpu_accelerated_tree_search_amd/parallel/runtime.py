"""Distributed B&B runtime: one process (= one engine) per GPU, lock-step rounds.

Parity with the reference's two parallel engines:
  * intra-node multi-GPU (ref pfsp_multigpu_cuda.c): Step 1 BFS to workers*m nodes,
    round-robin split (roundRobin_distribution), per-GPU pools, random steal-half
    work stealing, BUSY/IDLE termination, incumbent sharing (checkBest);
  * distributed multi-node (ref pfsp_dist_multigpu_cuda.c): redundant Step 1 on
    every rank + rank-strided share, a comm thread doing Allreduce(best) /
    Allgather(termination, needs_work) / Allgatherv(nodes) rounds (DWS, -L 1) or a
    static partition (-L 0), final reductions.

Here every rank runs the same loop, natively (csrc/core/dist_rounds.hpp, no GIL):
    run its device pool for a time slice (fused kernels, no host round trips)
    -> one status all-gather {pool size, incumbent, split pending}
    -> incumbent = MIN over ranks          (replaces checkBest + Allreduce MIN)
    -> all pools empty => terminate        (exact: no node is in flight between rounds)
    -> steal-half plan, identical on all ranks, executed as targeted
       device-to-device transfers (replaces spin-lock steals and Allgatherv).
The slice adapts: it doubles while no rank is starving and resets when one is; a
rank that runs dry while a peer can donate calls the next round early through the
shared-memory board, so it waits one graph replay for work, not a whole slice.
Work-sharing thresholds are in units of the device parent window for GPU engines
(needy below window/4, donors from one window), the reference's m / 2m for CPU ones.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np

from .. import ops
from ..search import SolveResult
from ..utils.report import WorkerStats
from . import checkpoint as ckpt
from .comm import Comm
from .faults import Faults


@dataclass
class DistConfig:
    m: int = 25                  # CPU engines: needy below m nodes, donors need >= 2m (ref -m)
    init_per_rank: int = 25      # Step-1 nodes per rank (ref: workers * m)
    steal_cap: int = 250_000     # max nodes per transfer (ref 5*M)
    # GPU engines: needy below needy_below, donors hold >= donor_min (None: window/4
    # and one window, where window = the engine's parents per iteration)
    needy_below: int | None = None
    donor_min: int | None = None
    slice_min_s: float = 0.0005  # local work between rounds (adaptive)
    slice_max_s: float = 0.050
    early_rounds: bool = True    # a dry rank calls the next round early (shm board)
    ws: bool = True              # share within a node (ref -w)
    L: bool = True               # share across nodes (ref -L)
    # Step 1 on the engines instead of the host: every rank expands the root with
    # the same deterministic warm-up (warm_passes x 6 steps, warm_window parents
    # per step) and keeps the i % world == rank share of the resulting frontier.
    # Off by default: the host BFS to world * init_per_rank nodes costs ~30 us for
    # 8 ranks on ta014, the device warm-up ~6 dependent iterations plus a sync
    # and a gather (~80 us), and both give a strided sample of the frontier.
    engine_warmup: bool = False
    warm_window: int = 2048
    warm_passes: int = 1
    # Default Step 1 for world > 1: the in-search rank split (engine.set_split).
    # Every rank begins from the same small host warm-up (the N=1 Step 1) and
    # searches identically until its pool holds split_per_rank * world nodes;
    # that expansion is dealt out between ranks on the device, inside the same
    # graph replay — no host round trip, no collective, no replicated BFS on the
    # host. False: host BFS to world * init_per_rank nodes + round-robin share.
    # Load-balance tests: every Step-1 node starts on this rank (the others start empty)
    start_on: int | None = None
    split: bool = True
    split_per_rank: int = 512    # replicated iterations are narrow and run in parallel on
                                 # every rank: splitting late costs no latency and deals out
                                 # ~10^5 subtrees (balance), capped at window / children
    # checkpoint / resume (parallel/checkpoint.py): snapshot every
    # `checkpoint_every` rounds and when `max_rounds` (total, resume included) stops the solve
    checkpoint_dir: str | None = None
    checkpoint_every: int = 0
    max_rounds: int = 0
    resume: bool = False
    # throughput time box: every rank stops at the first round after time_limit_s
    # seconds on any rank (result.extra["complete"] is then False); 0: solve to the end
    time_limit_s: float = 0.0
    # exchange the incumbent through the node-wide board after every graph replay
    # (ref checkBest around every batch); False: only at round boundaries
    live_best: bool = True
    # overlapped rounds: a rank's slice may end with one graph replay still running,
    # and the round (all-gather, plan, transfers) runs while it does (ref: the comm
    # thread next to the GPU threads, pfsp_dist_multigpu_cuda.c:283,364-469)
    overlap: bool = True
    # record every rank's incumbent timeline (extra["incumbent_events"], diagnostics)
    trace_incumbent: bool = False
    # CPU worker next to each rank's GPU (ref -C 1 in pfsp_dist_multigpu_cuda.c:161-162,
    # 471-575): threads of the rank's CPU engine (0: none) and its batch (ref -T; a CPU
    # thief takes at most 4*T nodes). parallel/workers.py wraps the engines into one
    # hybrid engine (csrc/core/hybrid_engine.hpp)
    cpu_workers: int = 0
    cpu_batch: int = 5000
    # failure detection / fault injection (parallel/faults.py; env TTS_FAULT_*)
    watchdog_s: float = 0.0
    watchdog_abort: bool = False
    fault_delay_us: int | None = None
    fault_steal_fail_pct: int | None = None
    verbose: bool = False


def round_robin_share(n: int, rank: int, world: int) -> np.ndarray:
    """Indices rank, rank+world, ... ; the last rank also takes the tail
    (ref Pool_atom.c:14-36 roundRobin_distribution)."""
    c = n // world
    idx = rank + world * np.arange(c)
    if rank == world - 1:
        idx = np.concatenate([idx, np.arange(world * c, n)])
    return idx.astype(np.int64)


def distributed_solve(model, engine, comm: Comm, ub: int = 1, cfg: DistConfig | None = None,
                      window: int | None = None) -> SolveResult:
    """Cooperative solve of `model` by all ranks of `comm`; returns the global result
    (identical on every rank) with per-rank WorkerStats in `workers`. `window` is the
    engine's parents per iteration (GPU work-sharing thresholds)."""
    cfg = cfg or DistConfig()
    world, rank = comm.world, comm.rank
    t_start = time.perf_counter()

    # ---- Step 1: redundant, deterministic warm-up on every rank ----
    best = model.search_best(ub)
    if cfg.resume:
        if not cfg.checkpoint_dir:
            raise ValueError("resume needs checkpoint_dir")
        nodes, tree0, sol0, best0, rounds0 = ckpt.load_all(cfg.checkpoint_dir, model)
        best = min(int(best), best0)
        engine.begin(np.ascontiguousarray(nodes[rank::world]), int(best))
        t_init = time.perf_counter() - t_start
        return _rounds(model, engine, comm, cfg, t_start, t_init, best, tree0, sol0, window, rounds0)
    if world > 1 and cfg.engine_warmup:
        # on the engine: wide frontier in a few device iterations, strided share
        engine.begin(model.root(), int(best))
        engine.warm_split(rank, world, cfg.warm_window, cfg.warm_passes)
        return _rounds(model, engine, comm, cfg, t_start, time.perf_counter() - t_start, best, 0, 0, window)
    if world > 1 and cfg.split and cfg.start_on is None:
        nodes, tree1, sol1, best = model.warmup(best, cfg.m)
        engine.set_split(rank, world, cfg.split_per_rank * world)
        engine.begin(nodes, int(best))
        return _rounds(model, engine, comm, cfg, t_start, time.perf_counter() - t_start, best, tree1, sol1, window)
    nodes, tree1, sol1, best = model.warmup(best, world * cfg.init_per_rank)
    if cfg.start_on is not None:
        mine = np.ascontiguousarray(nodes if rank == cfg.start_on else nodes[:0])
    else:
        mine = np.ascontiguousarray(nodes[round_robin_share(len(nodes), rank, world)])
    t_init = time.perf_counter() - t_start
    if world == 1 and not cfg.max_rounds and not cfg.checkpoint_dir and not cfg.time_limit_s:  # one fused solve
        st = engine.solve(mine, int(best))
        elapsed = time.perf_counter() - t_start
        w = WorkerStats(tree=int(st["tree"]), sol=int(st["sol"]), gen_child=int(st["tree"]),
                        t_memcpy=float(st["t_memcpy"]), t_malloc=float(st["t_malloc"]), t_kernel=float(st["t_run"]))
        return SolveResult(best=min(int(best), int(st["best"])), tree=tree1 + int(st["tree"]),
                           sol=sol1 + int(st["sol"]), elapsed=elapsed, t_init=t_init,
                           t_search=elapsed - t_init, workers=[w],
                           extra={"rounds": 0, "sent_nodes": [0], "received_nodes": [0], "world": 1})
    engine.begin(mine, int(best))
    return _rounds(model, engine, comm, cfg, t_start, t_init, best, tree1, sol1, window)


def sharing_thresholds(cfg: DistConfig, engine, window: int | None) -> tuple[int, int]:
    """(needy_below, donor_min): GPU engines in units of the parent window, CPU
    engines the reference's m / 2m (ref popBackBulk ratio 2, pfsp_multigpu_cuda.c:343-404)."""
    gpu = bool(getattr(engine, "transfer_stream", 0))
    if gpu and window:
        needy = cfg.needy_below if cfg.needy_below is not None else max(cfg.m, int(window) // 4)
        donor = cfg.donor_min if cfg.donor_min is not None else max(2 * needy, int(window))
    else:
        needy = cfg.needy_below if cfg.needy_below is not None else cfg.m
        donor = cfg.donor_min if cfg.donor_min is not None else 2 * needy
    return int(needy), int(donor)


_OPTS_CACHE: dict = {}
_ENV_KEYS = ("TTS_WATCHDOG_S", "TTS_WATCHDOG_ABORT", "TTS_FAULT_DELAY_US", "TTS_FAULT_STEAL_FAIL_PCT", "TTS_FAULT_SEED")
_env_seen: tuple | None = None


def _env_snapshot() -> tuple:
    """The runtime's environment knobs, read once per process (os.environ lookups
    cost ~2.5 us each); refresh_env() re-reads them."""
    global _env_seen
    if _env_seen is None:
        _env_seen = tuple(os.environ.get(k) for k in _ENV_KEYS)
    return _env_seen


def refresh_env() -> None:
    global _env_seen
    _env_seen = None
    _OPTS_CACHE.clear()


def _native_options(cfg: DistConfig, engine, comm: Comm, window: int | None):
    """(needy_below, donor_min, options of the native loop), cached per configuration
    (a solve of a small tree must not pay ~20 us of Python setup each time)."""
    key = (tuple(vars(cfg).values()), bool(getattr(engine, "transfer_stream", 0)), window, comm.world,
           comm.topo.local_world, _env_snapshot())
    hit = _OPTS_CACHE.get(key)
    if hit is not None:
        return hit
    env = os.environ
    faults = Faults(comm.rank, cfg.fault_delay_us, cfg.fault_steal_fail_pct)
    needy, donor = sharing_thresholds(cfg, engine, window)
    share = comm.world > 1 and (cfg.ws or cfg.L)
    opts = dict(needy_below=needy, donor_min=donor, steal_cap=cfg.steal_cap, slice_min=cfg.slice_min_s,
                slice_max=cfg.slice_max_s, intra=bool(cfg.ws and share), inter=bool(cfg.L and share),
                local_world=comm.topo.local_world, early_rounds=cfg.early_rounds, max_rounds=cfg.max_rounds,
                time_limit=float(cfg.time_limit_s), live_best=bool(cfg.live_best),
                overlap=bool(cfg.overlap) and env.get("TTS_OVERLAP", "1") != "0",
                trace_incumbent=bool(cfg.trace_incumbent),
                checkpoint_every=cfg.checkpoint_every if cfg.checkpoint_dir else 0,
                watchdog_s=float(cfg.watchdog_s or float(env.get("TTS_WATCHDOG_S", "0") or 0)),
                watchdog_abort=bool(cfg.watchdog_abort or env.get("TTS_WATCHDOG_ABORT", "0") not in ("", "0")),
                fault_delay_us=faults.delay_us, fault_steal_fail_pct=faults.steal_fail_pct, fault_seed=faults.seed)
    if len(_OPTS_CACHE) > 64:
        _OPTS_CACHE.clear()
    _OPTS_CACHE[key] = (needy, donor, opts)
    return _OPTS_CACHE[key]


def _rounds(model, engine, comm: Comm, cfg: DistConfig, t_start: float, t_init: float, best: int, tree1: int,
            sol1: int, window: int | None, rounds0: int = 0) -> SolveResult:
    """Step 2 (native lock-step rounds until every pool is empty) and the final reductions."""
    world, rank = comm.world, comm.rank
    needy, donor, opts = _native_options(cfg, engine, comm, window)

    def transfer(plan):
        return comm.execute_transfers(plan, engine, model.node_bytes)

    def hook(rounds, gbest, replicated):
        est = engine.stats()
        if replicated:  # identical pools everywhere: rank 0 saves the one pool as a world-1 checkpoint
            if rank == 0:
                ckpt.save(cfg.checkpoint_dir, 0, 1, model, engine, int(est["tree"]) + tree1,
                          int(est["sol"]) + sol1, min(int(est["best"]), int(gbest)), int(rounds))
            keep = 1
        else:
            ckpt.save(cfg.checkpoint_dir, rank, world, model, engine,
                      int(est["tree"]) + (tree1 if rank == 0 else 0), int(est["sol"]) + (sol1 if rank == 0 else 0),
                      min(int(est["best"]), int(gbest)), int(rounds))
            keep = world
        comm.barrier()  # every file is complete before anyone may resume from it
        if rank == 0:
            ckpt.prune(cfg.checkpoint_dir, keep)
        comm.barrier()

    native = type(engine).__module__.rsplit(".", 1)[-1]
    mod = ops.hip() if native == "_tts_hip" else ops.cpu()
    t_loop = time.perf_counter()
    shm = comm.control_address(mod)
    # GPU ranks over RCCL: the native transport, no Python in the loop
    xfer = comm.transport(engine, model.node_bytes) if comm.rccl is not None else transfer
    out = mod.dist_rounds(engine, shm, None if shm else comm.round_allgather(engine), rank, world, opts, xfer,
                          hook if cfg.checkpoint_dir else None, int(rounds0), float(comm.timeout_s))
    t_search = time.perf_counter() - t_loop
    cnt, tms = out["counts"], out["times"]
    tree = int(cnt[:, 0].sum()) + tree1
    sol = int(cnt[:, 1].sum()) + sol1
    gbest = min(int(out["best"]), int(best))
    elapsed = time.perf_counter() - t_start
    return SolveResult(best=gbest, tree=tree, sol=sol, elapsed=elapsed, t_init=t_init,
                       t_search=t_search, t_tail=0.0, workers=RankTable(cnt, tms, bool(cfg.cpu_workers)),
                       extra={"rounds": int(out["rounds"]), "sent_nodes": cnt[:, 2].tolist(),
                              "received_nodes": cnt[:, 3].tolist(), "world": world,
                              "complete": bool(out["complete"]), "dropped_transfers": int(cnt[:, 10].sum()),
                              "watchdog_events": int(out["watchdog_events"]),
                              "early_rounds": cnt[:, 9].tolist(), "needy_below": needy, "donor_min": donor,
                              "overlapped_rounds": list(out.get("overlapped_rounds", [])),
                              "incumbent_events": list(out.get("incumbent_events", []))})


class RankTable(list):
    """Per-worker WorkerStats, built from the native round loop's count/time arrays on
    first use (the bench never needs them inside its timed loop). Fields keep the
    reference's meaning (ref PFSP_statistic.c:82-84, 133-135): gen_child = children the
    rank pushed (indexChildren), steals = rounds it asked for work, success_steals =
    rounds it received some, terminations = rounds it stayed idle. A rank with a CPU
    worker (hybrid engine, -C 1) gives two entries: its GPU, then its CPU worker (ref
    arrays of commSize * NB_THREADS entries, PFSP_statistic.c:115-167)."""

    def __init__(self, counts, times, hybrid: bool = False):
        super().__init__()
        self._src = (counts, times, hybrid)

    def _fill(self):
        if self._src is not None:
            c, t, hybrid = self._src
            self._src = None
            for r in range(len(c)):
                ct, cs = (int(c[r, 11]), int(c[r, 12])) if c.shape[1] > 12 else (0, 0)
                super().append(WorkerStats(
                    tree=int(c[r, 0]) - ct, sol=int(c[r, 1]) - cs, gen_child=int(c[r, 0]) - ct, steals=int(c[r, 6]),
                    success_steals=int(c[r, 7]), terminations=int(c[r, 8]), t_memcpy=float(t[r, 5]),
                    t_malloc=float(t[r, 6]), t_kernel=float(t[r, 0]), t_pool_ops=float(t[r, 1]),
                    t_idle=float(t[r, 2]), t_termination=float(t[r, 3]), t_load_bal=float(t[r, 4]),
                    dist_load_bal=int(c[r, 4])))
                if hybrid:
                    super().append(WorkerStats(tree=ct, sol=cs, gen_child=ct))

    def __len__(self):
        self._fill()
        return super().__len__()

    def __iter__(self):
        self._fill()
        return super().__iter__()

    def __getitem__(self, i):
        self._fill()
        return super().__getitem__(i)

    def __repr__(self):
        self._fill()
        return super().__repr__()


class DistSolver:
    """Reusable native session for repeated cooperative solves with the default Step 1
    (same host warm-up on every rank + in-search split; csrc/core/dist_session.hpp):
    one native call per solve — warm-up, split, rounds and final reductions run without
    the interpreter, which is what a 0.3-ms tree needs at N > 1 (bench.py). Per-rank
    statistics of the last solve: `last_outcome()` / `result(...).workers`."""

    def __init__(self, model, engine, comm: Comm, cfg: DistConfig | None = None, window: int | None = None):
        cfg = cfg or DistConfig()
        if cfg.checkpoint_dir or cfg.max_rounds or cfg.resume or cfg.engine_warmup or cfg.start_on is not None:
            raise ValueError("DistSolver runs the default Step 1 only; use distributed_solve for the other modes")
        self.model, self.engine, self.comm, self.cfg = model, engine, comm, cfg
        self.needy, self.donor, opts = _native_options(cfg, engine, comm, window)
        native = type(engine).__module__.rsplit(".", 1)[-1]
        mod = ops.hip() if native == "_tts_hip" else ops.cpu()
        shm = comm.control_address(mod)
        world = comm.world
        split = cfg.split and world > 1
        # Step 1: with the in-search split every rank starts from the 1-rank warm-up
        # (init_per_rank nodes); without it, a host BFS to world * init_per_rank nodes
        # and the round-robin share (ref roundRobin_distribution)
        warm = cfg.init_per_rank if split else world * cfg.init_per_rank
        self._xfer = comm.transport(engine, model.node_bytes)  # kept alive with the session
        self._s = mod.DistSession(engine, model, shm, None if shm else comm.round_allgather(engine), comm.rank, world, opts,
                                  self._xfer, None,
                                  int(warm), int(cfg.split_per_rank * world), float(comm.timeout_s), bool(split))

    def solve_raw(self, ub: int = 1) -> tuple:
        """(best, tree, sol, rounds, complete, t_init, t_search, elapsed), global values."""
        return self._s.solve(int(self.model.search_best(ub)))

    def solve(self, ub: int = 1) -> SolveResult:
        best, tree, sol, rounds, complete, t_init, t_search, elapsed = self.solve_raw(ub)
        return self.result(best, tree, sol, rounds, complete, t_init, t_search, elapsed)

    def last_outcome(self) -> dict:
        return self._s.outcome()

    def result(self, best, tree, sol, rounds, complete, t_init, t_search, elapsed) -> SolveResult:
        out = self._s.outcome()
        cnt, tms = out["counts"], out["times"]
        return SolveResult(best=int(best), tree=int(tree), sol=int(sol), elapsed=elapsed, t_init=t_init,
                           t_search=t_search, t_tail=0.0, workers=RankTable(cnt, tms, bool(self.cfg.cpu_workers)),
                           extra={"rounds": int(rounds), "sent_nodes": cnt[:, 2].tolist(),
                                  "received_nodes": cnt[:, 3].tolist(), "world": self.comm.world,
                                  "complete": bool(complete), "dropped_transfers": int(cnt[:, 10].sum()),
                                  "watchdog_events": int(out["watchdog_events"]),
                                  "early_rounds": cnt[:, 9].tolist(), "needy_below": self.needy,
                                  "donor_min": self.donor,
                                  "overlapped_rounds": list(out.get("overlapped_rounds", [])),
                                  "incumbent_events": list(out.get("incumbent_events", []))})
