"""Per-solve cost breakdown of the multi-rank runtime (one process per rank).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        scripts/round_cost.py [--backend cpu|gpu] [--comm gloo|nccl] [--inst 2] [--lb 1] [--solves 2000]

Times every phase of `distributed_solve` on a small tree, averaged over many solves:
  step1      host warm-up + set_split + begin (the engine upload is asynchronous)
  native     parallel/runtime -> dist_rounds (csrc/core/dist_rounds.hpp), split into
             run      the engine's time slices (device search)
             round    status all-gathers and transfers (waiting included)
             final    the two final all-gathers and the engine stats
  python     option lookup before the call + SolveResult after it
and prints one line per component for rank 0 (max over ranks for the total).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="cpu")
    ap.add_argument("--comm", default="gloo")
    ap.add_argument("--inst", type=int, default=2)
    ap.add_argument("--lb", type=int, default=1)
    ap.add_argument("--solves", type=int, default=2000)
    ap.add_argument("--device", type=int, default=None)
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401

    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.parallel import runtime as rt
    from dist_gpu_accelerated_tree_search_amd.parallel.comm import Comm

    comm = Comm(use_gpu=(a.backend == "gpu" and a.comm == "nccl"))
    model = PfspModel(a.inst, a.lb)
    dev = (comm.topo.local_rank if a.device is None else a.device) if a.backend == "gpu" else 0
    opts = EngineOptions(max_parents=1 << 19, ring_bytes=1 << 30)
    eng = model.make_engine(a.backend, dev, opts)
    cfg = rt.DistConfig()
    window = opts.max_parents if a.backend == "gpu" else None
    acc = np.zeros(7)
    for i in range(a.solves + 100):
        t0 = time.perf_counter()
        best = model.initial_best(1)
        nodes, t1, s1, best = model.warmup(best, cfg.m)
        if comm.world > 1:
            eng.set_split(comm.rank, comm.world, cfg.split_per_rank * comm.world)
        eng.begin(nodes, int(best))
        t1_ = time.perf_counter()
        r = rt._rounds(model, eng, comm, cfg, t0, t1_ - t0, best, t1, s1, window)
        t2 = time.perf_counter()
        if i >= 100:
            w0 = r.workers[comm.rank]
            acc += [t1_ - t0, r.t_search, w0.t_kernel, w0.t_pool_ops, 0.0, t2 - t0, 0.0]
    acc /= a.solves
    step1, native, run, rnd, _, total, _ = acc
    final = native - run - rnd
    python = total - step1 - native
    tot = comm.allgather_f64([total])
    if comm.rank == 0:
        print(f"world {comm.world} backend {a.backend}/{a.comm} ta{a.inst:03d} lb{a.lb} tree {r.tree}: "
              f"per solve (rank 0, mean of {a.solves})")
        for k, v in (("step1 (warm-up + begin)", step1), ("native: run slices", run), ("native: rounds", rnd),
                     ("native: final reductions", final), ("python (options + result)", python),
                     ("total", total), ("total, max over ranks", float(tot.max()))):
            print(f"  {k:28s} {v * 1e6:9.1f} us")
    comm.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
