"""Every rank's share of a W-way ta014 LB1 split, timed alone on one GPU (as
share_solve_probe.py for rank 0): the N=W headline step is bounded by the slowest share.

    python scripts/share_all_ranks.py [reps] [split_per_rank]
"""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
spr = int(sys.argv[2]) if len(sys.argv) > 2 else 512
m = PfspModel(14, 1)
eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
for world in (2, 4, 8):
    med, trees = [], []
    for rank in range(world):
        ts = []
        for rep in range(reps + 3):
            nodes, t1, s1, best = m.warmup(m.initial_best(1), 25)
            eng.set_split(rank, world, spr * world)
            t0 = time.perf_counter()
            eng.begin(nodes, int(best))
            eng.run()
            dt = time.perf_counter() - t0
            if rep >= 3:
                ts.append(dt)
        med.append(float(np.median(ts)) * 1e3)
        trees.append(eng.stats()["tree"])
    med = np.array(med)
    print(f"world {world} split_per_rank {spr}: share ms {np.round(med, 4).tolist()} max/mean {med.max() / med.mean():.2f}; "
          f"trees {trees} max/mean {max(trees) / np.mean(trees):.2f}", flush=True)
