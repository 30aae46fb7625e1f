#!/usr/bin/env python3
"""Single-GPU estimate of the multi-GPU critical path of the default multi-rank solve
(parallel/runtime.py: host warm-up, then engine.set_split -> identical device
iterations on every rank until the pool holds split_per_rank * W parents, then each
rank keeps its hashed share). For W ranks, each rank's whole solve (begin + run to
empty) is timed on one device; max over ranks ~ the W-GPU step time without the
status round (a few us on the shared-memory control plane)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: F401

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, QueensModel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inst", type=int, default=14)
    ap.add_argument("--lb", type=int, default=1)
    ap.add_argument("--queens", type=int, default=0)
    ap.add_argument("--per-rank", default="64,512,4096")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    model = QueensModel(a.queens) if a.queens else PfspModel(a.inst, a.lb)
    eng = model.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
    best = model.initial_best(1)
    nodes, t1, s1, b1 = model.warmup(best, 25)
    for _ in range(5):
        eng.solve(nodes, int(b1))
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        st = eng.solve(nodes, int(b1))
        ts.append(time.perf_counter() - t0)
    t_one = sorted(ts)[len(ts) // 2]
    print(f"fused solve W=1: {t_one*1e3:.3f} ms tree={t1 + st['tree']}", flush=True)
    for per in map(int, a.per_rank.split(",")):
        for W in (2, 4, 8):
            times, trees, iters = [], [], []
            for r in range(W):
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    eng.set_split(r, W, per * W)
                    eng.begin(nodes, int(b1))
                    eng.run()
                    eng.size()
                    ts.append(time.perf_counter() - t0)
                times.append(sorted(ts)[len(ts) // 2])
                st = eng.stats()
                trees.append(st["tree"])
                iters.append(st["iters"])
            print(f"split_per_rank={per} W={W}: max {max(times)*1e3:.3f} ms mean {sum(times)/W*1e3:.3f} ms "
                  f"tree={sum(trees) + t1} per-rank {min(trees)}..{max(trees)} iters {max(iters)} "
                  f"-> est speedup {t_one/max(times):.2f}x", flush=True)


if __name__ == "__main__":
    main()
