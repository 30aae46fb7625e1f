#!/usr/bin/env python3
"""Headline benchmark: explored tree nodes per second, PFSP Taillard ta014, LB1, -u 1.

BASELINE.json metric: "tree-nodes/sec (whole node), PFSP ta014 LB1 at 1/2/4/8 MI355X".
One step = one complete cooperative B&B solve of ta014 with LB1 by all N GPUs
(Step-1 host warm-up + device search + work sharing + termination + reductions),
i.e. STRONG scaling: the tree (2,573,652 nodes, sol 2,648, makespan 1377) is the
same at every N. Each step's tree/sol/makespan is checked against the golden
values, so a skipped or truncated search fails instead of reporting a number.

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
import time

# ta014 LB1 (-u 1) golden values and the reference throughput on the same tree.
GOLDEN = {(14, 1): (2573652, 2648, 1377), (14, 0): (2573652, 2648, 1377), (14, 2): (144639, 0, 1377)}
# fastest reference implementation of this tree = pfsp_omp_c.out -C 8
# -l 0 (LB1_d, identical tree to LB1) at 23 M nodes/s; no published GPU number exists.
BASELINE_NODES_PER_S = 23.0e6


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
    ap.add_argument("--no-ws", action="store_true", help="static partition (ref -w 0 / -L 0)")
    ap.add_argument("--backend", choices=["gpu", "cpu"], default="gpu")
    ap.add_argument("--comm", choices=["nccl", "gloo"], default="nccl",
                    help="process group for node transfers (gloo: ranks may share one GPU, for tests)")
    ap.add_argument("--device", type=int, default=None, help="GPU of this rank (default LOCAL_RANK)")
    a = ap.parse_args()

    import torch  # noqa: F401  (before the HIP extension: one HIP runtime per process)

    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.parallel.comm import Comm
    from dist_gpu_accelerated_tree_search_amd.parallel.runtime import DistConfig, DistSolver

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    comm = Comm(use_gpu=(a.backend == "gpu" and a.comm == "nccl"), device=a.device)
    model = PfspModel(a.inst, a.lb)
    opts = EngineOptions(max_parents=a.max_parents, ring_bytes=int(a.ring_gb * (1 << 30)))
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
        ex = last.extra
        log(f"last step: elapsed {last.elapsed * 1e3:.3f} ms, init {last.t_init * 1e3:.3f} ms, "
            f"search {last.t_search * 1e3:.3f} ms, rounds {ex.get('rounds')}, "
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
            },
        }
        print(json.dumps(rec), flush=True)
    del engine
    comm.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
