"""Cost of the replicated prefix of a multi-rank solve (default Step 1 = in-search split).

Every rank runs the same search from the same small host warm-up until its pool holds
split_per_rank * world nodes; that prefix is replicated work. This measures it on one
GPU as rank 0 of `world` ranks sees it: time and device iterations until the split.

    python scripts/split_probe.py
"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel

for inst, lb in ((14, 1), (21, 0), (56, 2)):
    m = PfspModel(inst, lb)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19 if lb != 2 else 1 << 18, ring_bytes=8 << 30))
    for world in (2, 4, 8):
        best_t, iters = 1e9, 0
        for rep in range(5):
            nodes, t1, s1, best = m.warmup(m.initial_best(1), 25)
            eng.set_split(0, world, 512 * world)
            t0 = time.perf_counter()
            eng.begin(nodes, int(best))
            while eng.split_pending() and eng.size() > 0:
                eng.run(max_launches=1)
            dt = time.perf_counter() - t0
            st = eng.stats()
            best_t = min(best_t, dt)
            iters = st["iters"]
            eng.run(max_seconds=0.05 if lb == 2 else 0)  # drain (LB2: just stop)
            if eng.size():
                eng.pop(eng.size())
        print(f"ta{inst:03d} lb{lb} world {world}: replicated prefix {best_t * 1e3:.3f} ms "
              f"({iters} device iterations incl. the first replay)", flush=True)
    del eng
