"""Distributed B&B runtime: one process (= one engine) per GPU, lock-step rounds.

Parity with the reference's two parallel engines:
  * intra-node multi-GPU (ref pfsp_multigpu_cuda.c): Step 1 BFS to workers*m nodes,
    round-robin split (roundRobin_distribution), per-GPU pools, random steal-half
    work stealing, BUSY/IDLE termination, incumbent sharing (checkBest);
  * distributed multi-node (ref pfsp_dist_multigpu_cuda.c): redundant Step 1 on
    every rank + rank-strided share, a comm thread doing Allreduce(best) /
    Allgather(termination, needs_work) / Allgatherv(nodes) rounds (DWS, -L 1) or a
    static partition (-L 0), final reductions.

Here every rank runs the same loop:
    run its device pool for a time slice (fused kernels, no host round trips)
    -> one status all_gather {pool size, incumbent}
    -> incumbent = MIN over ranks          (replaces checkBest + Allreduce MIN)
    -> all pools empty => terminate        (exact: no node is in flight between rounds)
    -> steal-half plan, identical on all ranks, executed as targeted
       device-to-device transfers (replaces spin-lock steals and Allgatherv).
The slice adapts: it doubles while no rank is starving and resets when one is.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from ..search import SolveResult
from ..utils.report import WorkerStats
from . import checkpoint as ckpt
from .comm import Comm, plan_sharing
from .faults import Faults, Watchdog


@dataclass
class DistConfig:
    m: int = 25                  # needy below m nodes; donors need >= 2m (ref -m)
    init_per_rank: int = 25      # Step-1 nodes per rank (ref: workers * m)
    steal_cap: int = 250_000     # max nodes per transfer (ref 5*M)
    slice_min_s: float = 0.0005  # local work between rounds (adaptive)
    slice_max_s: float = 0.050
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
    split: bool = True
    split_per_rank: int = 512    # replicated iterations are narrow and run in parallel on
                                 # every rank: splitting late costs no latency and deals out
                                 # ~10^5 subtrees (balance), capped at window / children
    # checkpoint / resume (parallel/checkpoint.py): snapshot every
    # `checkpoint_every` rounds and when `max_rounds` stops the solve early
    checkpoint_dir: str | None = None
    checkpoint_every: int = 0
    max_rounds: int = 0
    resume: bool = False
    # failure detection / fault injection (parallel/faults.py; env TTS_FAULT_*)
    watchdog_s: float = 0.0
    watchdog_abort: bool = False
    fault_delay_us: int | None = None
    fault_steal_fail_pct: int | None = None
    verbose: bool = False


@dataclass
class RankStats:
    tree: int = 0
    sol: int = 0
    rounds: int = 0
    sent: int = 0
    received: int = 0
    transfers_in: int = 0
    transfers_out: int = 0
    t_run: float = 0.0
    t_comm: float = 0.0
    t_idle: float = 0.0
    t_init: float = 0.0


def round_robin_share(n: int, rank: int, world: int) -> np.ndarray:
    """Indices rank, rank+world, ... ; the last rank also takes the tail
    (ref Pool_atom.c:14-36 roundRobin_distribution)."""
    c = n // world
    idx = rank + world * np.arange(c)
    if rank == world - 1:
        idx = np.concatenate([idx, np.arange(world * c, n)])
    return idx.astype(np.int64)


def distributed_solve(model, engine, comm: Comm, ub: int = 1, cfg: DistConfig | None = None) -> SolveResult:
    """Cooperative solve of `model` by all ranks of `comm`; returns the global result
    (identical on every rank) with per-rank WorkerStats in `workers`."""
    cfg = cfg or DistConfig()
    rs = RankStats()
    world, rank = comm.world, comm.rank
    t_start = time.perf_counter()

    # ---- Step 1: redundant, deterministic warm-up on every rank ----
    best = model.initial_best(ub)
    if cfg.resume:
        if not cfg.checkpoint_dir:
            raise ValueError("resume needs checkpoint_dir")
        nodes, tree0, sol0, best0, rounds0 = ckpt.load_all(cfg.checkpoint_dir, model)
        best = min(int(best), best0)
        engine.begin(np.ascontiguousarray(nodes[rank::world]), int(best))
        rs.t_init = time.perf_counter() - t_start
        return _rounds(model, engine, comm, cfg, rs, t_start, best, tree0, sol0)
    if world > 1 and cfg.engine_warmup:
        # on the engine: wide frontier in a few device iterations, strided share
        tree1 = sol1 = 0
        engine.begin(model.root(), int(best))
        engine.warm_split(rank, world, cfg.warm_window, cfg.warm_passes)
        rs.t_init = time.perf_counter() - t_start
        return _rounds(model, engine, comm, cfg, rs, t_start, best, tree1, sol1)
    if world > 1 and cfg.split:
        nodes, tree1, sol1, best = model.warmup(best, cfg.m)
        engine.set_split(rank, world, cfg.split_per_rank * world)
        engine.begin(nodes, int(best))
        rs.t_init = time.perf_counter() - t_start
        return _rounds(model, engine, comm, cfg, rs, t_start, best, tree1, sol1)
    nodes, tree1, sol1, best = model.warmup(best, world * cfg.init_per_rank)
    mine = np.ascontiguousarray(nodes[round_robin_share(len(nodes), rank, world)])
    rs.t_init = time.perf_counter() - t_start
    if world == 1 and not cfg.max_rounds and not cfg.checkpoint_dir:  # one fused native solve, no rounds
        st = engine.solve(mine, int(best))
        elapsed = time.perf_counter() - t_start
        w = WorkerStats(tree=int(st["tree"]), sol=int(st["sol"]), gen_child=int(st["tree"]),
                        t_memcpy=float(st["t_memcpy"]), t_malloc=float(st["t_malloc"]), t_kernel=float(st["t_run"]))
        return SolveResult(best=min(int(best), int(st["best"])), tree=tree1 + int(st["tree"]),
                           sol=sol1 + int(st["sol"]), elapsed=elapsed, t_init=rs.t_init,
                           t_search=elapsed - rs.t_init, workers=[w],
                           extra={"rounds": 0, "sent_nodes": [0], "received_nodes": [0], "world": 1})
    engine.begin(mine, int(best))
    return _rounds(model, engine, comm, cfg, rs, t_start, best, tree1, sol1)


def _rounds(model, engine, comm: Comm, cfg: DistConfig, rs: RankStats, t_start: float, best: int, tree1: int,
            sol1: int) -> SolveResult:
    """Step 2 (lock-step rounds until every pool is empty) and the final reductions."""
    world, rank = comm.world, comm.rank

    # ---- Step 2: rounds ----
    share = cfg.ws or cfg.L
    node_of = lambda r: r // max(1, comm.topo.local_world)  # noqa: E731
    slice_s = cfg.slice_min_s
    faults = Faults(rank, cfg.fault_delay_us, cfg.fault_steal_fail_pct)
    dog = Watchdog(cfg.watchdog_s, cfg.watchdog_abort)
    complete = True
    t_loop = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        engine.run(max_seconds=slice_s, stop_below=1)
        t1 = time.perf_counter()
        rs.t_run += t1 - t0
        size = engine.size()
        mybest = engine.best
        faults.before_round()
        if dog.enabled:
            dog.arm(f"rank {rank}/{world} round {rs.rounds + 1} pool {size} best {mybest}")
        st = comm.allgather_i64([size, mybest, int(engine.split_pending())])
        dog.disarm()
        rs.rounds += 1
        # while any pool is still replicated (armed split not reached) nodes must not move
        replicated = bool(st[:, 2].any())
        gbest = int(st[:, 1].min())
        if gbest < mybest:
            engine.best = gbest
        sizes = st[:, 0]
        if int(sizes.sum()) == 0:
            rs.t_comm += time.perf_counter() - t1
            break
        starving = bool((sizes < cfg.m).any())
        if share and world > 1 and starving and not replicated:
            plan = plan_sharing(sizes, cfg.m, cfg.steal_cap, node_of, intra=cfg.ws, inter=cfg.L)
            plan = faults.filter_plan(plan, rs.rounds)
            if plan:
                sent, got = comm.execute_transfers(plan, engine, model.node_bytes)
                rs.sent += sent
                rs.received += got
                rs.transfers_out += sum(1 for d, _, _ in plan if d == rank)
                rs.transfers_in += sum(1 for _, r, _ in plan if r == rank)
            slice_s = cfg.slice_min_s
        else:
            slice_s = min(cfg.slice_max_s, slice_s * 2)
        if size == 0:
            rs.t_idle += time.perf_counter() - t0
        rs.t_comm += time.perf_counter() - t1
        stop = cfg.max_rounds > 0 and rs.rounds >= cfg.max_rounds
        if cfg.checkpoint_dir and not replicated and (stop or (cfg.checkpoint_every > 0 and
                                                              rs.rounds % cfg.checkpoint_every == 0)):
            est = engine.stats()
            ckpt.save(cfg.checkpoint_dir, rank, world, model, engine,
                      int(est["tree"]) + (tree1 if rank == 0 else 0), int(est["sol"]) + (sol1 if rank == 0 else 0),
                      min(int(est["best"]), int(gbest)), rs.rounds)
            comm.barrier()  # every file is complete before anyone may resume from it
        if stop:
            complete = False
            break
    t_search = time.perf_counter() - t_loop

    # ---- Step 3 (nothing left by construction) + reductions ----
    st = engine.stats()
    rs.tree, rs.sol = int(st["tree"]), int(st["sol"])
    best_local = min(int(st["best"]), int(best))
    # one collective for every final reduction (counts < 2^53 are exact in f64)
    per = comm.allgather_f64([rs.tree, rs.sol, rs.sent, rs.received, rs.transfers_in, rs.transfers_out,
                              rs.rounds, rs.t_run, rs.t_comm, rs.t_idle, rs.t_init,
                              float(st.get("t_memcpy", 0.0)), float(st.get("t_malloc", 0.0)), best_local])
    tot = (int(round(sum(float(r[0]) for r in per))) + tree1, int(round(sum(float(r[1]) for r in per))) + sol1)
    gbest = int(min(float(r[13]) for r in per))
    elapsed = time.perf_counter() - t_start
    workers = [WorkerStats(tree=int(r[0]), sol=int(r[1]), gen_child=int(r[0]), steals=int(r[4]),
                           success_steals=int(r[4]), terminations=int(r[6]), t_memcpy=float(r[11]),
                           t_malloc=float(r[12]), t_kernel=float(r[7]), t_pool_ops=float(r[8]),
                           t_idle=float(r[9]), t_termination=0.0) for r in per]
    return SolveResult(best=gbest, tree=int(tot[0]), sol=int(tot[1]), elapsed=elapsed, t_init=rs.t_init,
                       t_search=t_search, t_tail=0.0, workers=workers,
                       extra={"rounds": rs.rounds, "sent_nodes": [int(r[2]) for r in per],
                              "received_nodes": [int(r[3]) for r in per], "world": world, "complete": complete,
                              "dropped_transfers": faults.dropped, "watchdog_events": dog.events})
