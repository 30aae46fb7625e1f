"""Permutation Flow-shop Scheduling (PFSP) problem model.

Parity map (reference -> here):
  c_taillard.c                      -> utils/taillard.py + csrc/core/taillard.hpp
  c_bound_simple.c / c_bound_johnson.c (LB1, LB1_d, LB2)
                                    -> csrc/core/pfsp_bounds_cpu.hpp (host oracle)
                                       csrc/hip/pfsp_kernels.hpp     (gfx950 kernels)
  PFSP_lib.c decompose_* / generate_children
                                    -> csrc/core/problems.hpp (host) and the fused
                                       expand kernel (device)
  lb1_alloc_gpu / lb2_alloc_gpu     -> csrc/hip/pfsp_engine.hpp (tables owned by engine)

A model instance is what a driver needs: the native instance, the bound kind,
node layout, Step-1 warm-up / Step-3 drain on the host, and engine factories for
the CPU and the GPU backends (same engine contract, csrc/core/engine_api.hpp).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from .. import ops
from ..utils import nodes as nodes_mod
from ..utils import taillard as tl

INT_MAX = 2**31 - 1


@dataclass
class EngineOptions:
    max_parents: int = 1 << 18      # parents per device iteration (reference -M, sized for HBM)
    ring_bytes: int = 16 << 30      # device pool capacity
    iters_small: int = 6
    iters_large: int = 48
    iters_first: int = 18           # first graph replay after begin(): covers a 20-job tree (profiles/r1/r1ac)
    use_graphs: bool = True
    cpu_batch: int = 4096           # CPU engine batch
    cpu_threads: int = 1
    # sub-engines per device, one stream and host thread each, run as one engine
    # (csrc/core/multi_engine.hpp): large trees fill the GPU better (ta021 LB1_d 15.5 s
    # with 1, 9.9 s with 2, 9.1 s with 3 engines, profiles/r3/concurrency_probe.txt);
    # the ring is shared out between them. 1: a plain engine (latency-bound small trees)
    streams: int = 1
    # sub-engine sharing thresholds in units of the parent window: a sub-engine below
    # window * stream_needy nodes takes half of a pool of at least window * stream_donor
    # (same-device copies are cheap: far below the cross-GPU thresholds)
    stream_needy: float = 1 / 16
    stream_donor: float = 1 / 4
    # > 0: each solve is split in the graph between the sub-engines from the start
    # (every one begins from the same nodes and keeps a disjoint share once the pool
    # holds stream_split * streams parents). Measured on the ta014 headline: 0.224 ms
    # with one engine, 0.30 / 0.39 ms split over 2 / 3 streams (a latency-bound tree
    # gains nothing from concurrent streams; profiles/r3/probes/headline_streams_split_ab.txt)
    stream_split: int = 0
    # dynamic local DFS iterations of the LB1 / LB1_d front kernel (csrc/hip/pfsp_front_kernels.hpp
    # front_dyn): time budget of one iteration in us, work shared between the workgroups of
    # an XCD; 0 = fixed-step local iterations
    dyn_us: int = 0
    # -u 0 dive (csrc/hip/pool_device.hpp Slot::cap): a device solve begun without an
    # incumbent expands at most dive_window parents (the top of the stack) per iteration
    # until its first leaf, then the cap grows 2^dive_shift-fold per iteration back to
    # max_parents; every node is counted (reference -u 0 semantics: a search from +inf).
    # TTS_DIVE_WINDOW / TTS_DIVE_SHIFT override; 0 = off. 4096 / 2 on one MI355X (trees from
    # +inf, no dive -> dive): ta014 LB1 99-162 M -> 102 M nodes (9.3 -> 6.2 ms), ta008 LB1_d 273 ->
    # 230 M, ta003 LB1 232 -> 196 M (profiles/r6/dive_probe.txt; narrower windows and the
    # hold-while-improving growth were better on one instance and worse on another)
    dive_window: int = 4096
    dive_shift: int = 2


def make_multi(model, backend: str, device: int, opts: EngineOptions):
    """opts.streams engines of `model` on one device as one engine (ring shared out;
    sub-engines below a quarter of a parent window take half of the largest pool)."""
    from dataclasses import replace

    k = int(opts.streams)
    sub = replace(opts, streams=1, ring_bytes=max(1 << 26, opts.ring_bytes // k))
    engines = [model.make_engine(backend, device, sub) for _ in range(k)]
    mod = ops.hip() if backend == "gpu" else ops.cpu()
    window = opts.max_parents if backend == "gpu" else opts.cpu_batch
    return mod.make_multi_engine(engines, max(1, int(window * opts.stream_needy)), max(2, int(window * opts.stream_donor)),
                                 split_min=max(0, int(opts.stream_split)))


class PfspModel:
    kind = "pfsp"

    def __init__(self, inst: int | None = 14, lb: int = 1, *, jobs: int | None = None, machines: int | None = None,
                 p: np.ndarray | None = None, best_known: int | None = None):
        if lb not in (0, 1, 2):
            raise ValueError("lb must be 0 (LB1_d), 1 (LB1) or 2 (LB2)")
        C = ops.cpu()
        self.lb = lb
        if p is None:
            if inst is None:
                raise ValueError("give a Taillard id or a processing-time matrix")
            self.inst_id = int(inst)
            self.native = C.PfspInstance.taillard(self.inst_id)
        else:
            p = np.asarray(p, dtype=np.int64)
            if p.ndim != 2:
                raise ValueError("p must be a (machines, jobs) matrix")
            mm, n = p.shape
            if (jobs is not None and jobs != n) or (machines is not None and machines != mm):
                raise ValueError("jobs/machines do not match p")
            self.inst_id = 0
            self.native = C.PfspInstance.from_matrix(n, mm, p.reshape(-1).tolist(),
                                                     INT_MAX if best_known is None else int(best_known))
        self.jobs = self.native.jobs
        self.machines = self.native.machines
        self.best_known = self.native.best_known
        self._dive = None  # search_best(0): the beam dive's makespan, computed once
        # engines' node layout: front nodes (depth, unscheduled set, per-machine
        # completion times; csrc/core/pfsp_front.hpp) for LB1 / LB1_d on instances of
        # up to 20 jobs, the permutation node of the job-count bucket otherwise
        self.front_layout = bool(C.pfsp_front_layout(self.native, lb))
        self.node_bytes = int(C.pfsp_engine_node_bytes(self.native, lb))

    @classmethod
    def synthetic(cls, jobs: int, machines: int, seed: int, lb: int = 1) -> "PfspModel":
        return cls(None, lb, p=tl.synthetic(jobs, machines, seed))

    # ---- incumbent ----
    def initial_best(self, ub: int = 1) -> int:
        """-u 1: best-known makespan (deterministic tree); -u 0: +inf."""
        return self.best_known if ub == 1 else INT_MAX

    def search_best(self, ub: int = 1) -> int:
        """Initial incumbent of a device / distributed search. -u 1: as initial_best. -u 0:
        +inf, the reference's semantics (ref pfsp_c.c:55-63); the device engines then dive
        depth-first to their first leaves through a narrow parent window
        (EngineOptions.dive_window) and every node of that dive is counted.
        Opt-in (TTS_DIVE=<beam>, CLI --heuristic-ub): start from the best complete schedule of
        two host heuristics (csrc/core/pfsp_bounds_cpu.hpp) — a beam dive of LB1 and NEH +
        iterated greedy (TTS_NEH_BUDGET cell updates, ~5 ms). That tree is then NOT the
        reference's -u 0 quantity: the initial incumbent is recorded with the results
        (initial_ub)."""
        if ub == 1:
            return self.best_known
        beam = int(os.environ.get("TTS_DIVE", "0"))
        if beam <= 0:
            return INT_MAX
        if self._dive is None:
            C = ops.cpu()
            budget = int(os.environ.get("TTS_NEH_BUDGET", str(5_000_000)))
            self._dive = min(int(C.pfsp_dive(self.native, beam)), int(C.pfsp_neh(self.native, budget)))
        return self._dive

    # ---- host steps ----
    def root(self) -> np.ndarray:
        """Root node in the engines' layout, shape (1, node_bytes)."""
        return ops.cpu().pfsp_root(self.native, self.lb)

    def to_engine_layout(self, perm_nodes: np.ndarray) -> np.ndarray:
        """Permutation-layout nodes (utils.nodes.pfsp_pack) in the engines' layout."""
        return ops.cpu().pfsp_to_engine_layout(self.native, self.lb, np.ascontiguousarray(perm_nodes, dtype=np.uint8))

    @property
    def host_lb(self) -> int:
        """Bound used by host-side steps: LB1 is evaluated with the incremental LB1_d
        (identical values), as the reference's CPU workers do
        (ref pfsp_multigpu_cuda.c:152-154: `if (lb == 1) cpulb = 0`)."""
        return 0 if self.lb == 1 else self.lb

    def warmup(self, best: int, target: int):
        """Step 1 (ref pfsp_multigpu_cuda.c:111-118): breadth-first on the host until
        `target` nodes. Returns (nodes, tree, sol, best)."""
        return ops.cpu().pfsp_bfs(self.native, self.host_lb, int(best), int(target))

    def drain(self, best: int, nodes: np.ndarray):
        """Step 3 (ref :488-495): depth-first over leftovers. Returns (tree, sol, best)."""
        return ops.cpu().pfsp_drain(self.native, self.host_lb, int(best),
                                    np.ascontiguousarray(nodes, dtype=np.uint8))

    # ---- engines ----
    def make_engine(self, backend: str = "gpu", device: int = 0, opts: EngineOptions | None = None):
        opts = opts or EngineOptions()
        if opts.streams > 1:
            return make_multi(self, backend, device, opts)
        if backend == "cpu":
            return ops.cpu().make_pfsp_cpu_engine(self.native, self.lb, opts.cpu_batch, opts.cpu_threads)
        if backend != "gpu":
            raise ValueError(f"unknown backend {backend!r}")
        H = ops.require_gpu(device)
        return H.make_pfsp_engine(self.jobs, self.machines, list(self.native.p), self.lb, device=device,
                                  max_parents=opts.max_parents, ring_bytes=opts.ring_bytes,
                                  iters_small=opts.iters_small, iters_large=opts.iters_large,
                                  use_graphs=opts.use_graphs, taillard_id=self.inst_id,
                                  iters_first=opts.iters_first, dyn_us=opts.dyn_us,
                                  dive_window=int(os.environ.get("TTS_DIVE_WINDOW", opts.dive_window)),
                                  dive_shift=int(os.environ.get("TTS_DIVE_SHIFT", opts.dive_shift)))

    def make_hybrid(self, engine, backend: str, threads: int, m: int = 25, cap: int = 20000, batch: int = 5000):
        """`engine` plus a CPU worker of `threads` threads as one rank engine
        (csrc/core/hybrid_engine.hpp; ref -C 1 of the distributed driver). The CPU
        worker evaluates LB1 as LB1_d (same values, ref pfsp_multigpu_cuda.c:152-154)."""
        if backend == "gpu":
            H = ops.hip()
            cpu = H.make_pfsp_cpu_engine(self.jobs, self.machines, list(self.native.p), self.lb, batch, threads)
            return H.make_hybrid_engine(engine, cpu, m, cap)
        C = ops.cpu()
        cpu = C.make_pfsp_cpu_engine(self.native, self.host_lb, batch, threads)
        return C.make_hybrid_engine(engine, cpu, m, cap)

    # ---- bounds (reference evaluate_gpu semantics; used by tests/tools) ----
    def child_bounds_cpu(self, nodes: np.ndarray, best: int = INT_MAX) -> np.ndarray:
        C = ops.cpu()
        depths, perms = nodes_mod.pfsp_unpack(nodes, self.jobs)
        out = []
        for d, q in zip(depths, perms):
            d = int(d)
            if self.lb == 0:
                by_job = C.lb1_children(self.native, q.tolist(), d)
                out.extend(by_job[int(q[k])] for k in range(d, self.jobs))
                continue
            for k in range(d, self.jobs):
                c = q.copy()
                c[d], c[k] = c[k], c[d]
                out.append(C.lb1(self.native, c.tolist(), d + 1) if self.lb == 1 else
                           C.lb2(self.native, c.tolist(), d + 1, int(best)))
        return np.asarray(out, dtype=np.int64)

    def child_bounds_gpu(self, nodes: np.ndarray, best: int = INT_MAX, device: int = 0) -> np.ndarray:
        H = ops.require_gpu(device)
        return H.pfsp_bounds(self.jobs, self.machines, list(self.native.p), self.lb,
                             np.ascontiguousarray(nodes, dtype=np.uint8), int(best), device)

    def describe(self) -> dict:
        # the node layout is part of the identity: a 20-job front node (<= 10 machines) and a
        # 20-job permutation node are both 32 B, so node_bytes alone cannot tell them apart
        return {"problem": "pfsp", "inst": self.inst_id, "jobs": self.jobs, "machines": self.machines, "lb": self.lb,
                "best_known": self.best_known, "layout": "front" if self.front_layout else "perm"}
