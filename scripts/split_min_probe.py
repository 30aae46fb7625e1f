"""In-search split point vs the per-rank critical path: ta014 LB1 emulated at `world` ranks
on one GPU (each rank's share solved alone, min of 10), for several split_min values.
Prints every rank's share time and tree; the job's time is the max over ranks."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel

m = PfspModel(14, 1)
eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=8 << 30))
nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
for world in (2, 4, 8):
    for smin in (1, 256 * world, 512 * world, 2048 * world):
        ts, trees = [], []
        for r in range(world):
            best_t = 1e9
            for _ in range(10):
                t0 = time.perf_counter()
                eng.set_split(r, world, smin)
                eng.begin(nodes, int(best))
                eng.run()
                st = eng.stats()
                best_t = min(best_t, time.perf_counter() - t0)
            ts.append(best_t * 1e3)
            trees.append(st["tree"])
        assert sum(trees) + tree1 == 2573652, (world, smin, sum(trees) + tree1)
        print(f"world {world} split_min {smin:6d}: max {max(ts):.3f} ms mean {sum(ts) / world:.3f} ms | "
              f"trees max/mean {max(trees) / (sum(trees) / world):.2f}", flush=True)
