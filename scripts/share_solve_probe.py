"""Rank r's share of a W-rank ta014 LB1 solve on one GPU, timed end to end as that
rank's engine runs it (warm-up, in-graph split at split_per_rank * W, search to empty):
the per-GPU critical path of the N=W headline without the other ranks.

    python scripts/share_solve_probe.py [reps]
Env knobs of the engine (TTS_FUSED_BPF, TTS_BLOCKS_PER_CU, ...) apply.
"""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
per_rank = int(sys.argv[2]) if len(sys.argv) > 2 else 512  # split_min = per_rank * world (DistConfig.split_per_rank)
m = PfspModel(14, 1)
eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
for world in (1, 2, 4, 8):
    ts, trees = [], []
    for rep in range(reps + 5):
        nodes, t1, s1, best = m.warmup(m.initial_best(1), 25)
        if world > 1:
            eng.set_split(0, world, per_rank * world)
        t0 = time.perf_counter()
        eng.begin(nodes, int(best))
        eng.run()
        dt = time.perf_counter() - t0
        st = eng.stats()
        if rep >= 5:
            ts.append(dt)
            trees.append(st["tree"])
    print(f"world {world}: rank 0 share median {np.median(ts) * 1e3:.4f} ms min {min(ts) * 1e3:.4f} ms, "
          f"tree {trees[-1]:,} iters {st['iters']}", flush=True)
