#!/usr/bin/env python3
"""Single-GPU estimate of the multi-GPU critical path: for W ranks, time each rank's
share (begin(root) + warm_split(r, W) + run to empty) on one device and report
max/mean over ranks. Excludes rounds and collectives (measured separately)."""
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
    ap.add_argument("--windows", default="512,2048,8192")
    ap.add_argument("--passes", default="1")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    model = QueensModel(a.queens) if a.queens else PfspModel(a.inst, a.lb)
    eng = model.make_engine("gpu", 0, EngineOptions(ring_bytes=4 << 30))
    best = model.initial_best(1)
    # reference single-rank fused solve
    nodes, t1, s1, b1 = model.warmup(best, 25)
    for _ in range(5):
        eng.solve(nodes, int(b1))
    t0 = time.perf_counter()
    for _ in range(a.reps):
        st = eng.solve(nodes, int(b1))
    t_one = (time.perf_counter() - t0) / a.reps
    print(f"fused solve W=1: {t_one*1e3:.3f} ms tree={t1 + st['tree']}")
    for passes in map(int, a.passes.split(",")):
        for win in map(int, a.windows.split(",")):
            for W in (1, 2, 4, 8):
                times, trees, warm = [], [], []
                for r in range(W):
                    best_t = 1e9
                    for _ in range(a.reps):
                        t0 = time.perf_counter()
                        eng.begin(model.root(), int(best))
                        n = eng.warm_split(r, W, win, passes)
                        t1_ = time.perf_counter()
                        eng.run()
                        eng.size()
                        t2 = time.perf_counter()
                        if t2 - t0 < best_t:
                            best_t, bw = t2 - t0, t1_ - t0
                    times.append(best_t)
                    warm.append(bw)
                    trees.append(eng.stats()["tree"])
                print(f"passes={passes} window={win} W={W}: max {max(times)*1e3:.3f} ms mean "
                      f"{sum(times)/W*1e3:.3f} ms warm {max(warm)*1e3:.3f} ms  tree={sum(trees)} "
                      f"-> est speedup {t_one/max(times):.2f}x")


if __name__ == "__main__":
    main()
