"""Dump the next expand windows of a time-boxed ta056 LB2 run (GPU engine) for the
host-side work model of the LB2 kernel (scripts/lb2_sched_sim.py).

    python scripts/lb2_pool_dump.py [out_dir] [seconds...]

For every time stamp: run the engine until then, copy the pool (oldest first), save the
top 16,384 nodes (the next window of the 50-job LB2 kernel: 2,048 chunks of 8 parents)
as ta056_top_<t>s.npy, and push the pool back.
"""
import os
import sys
import time

sys.path.insert(0, ".")
import numpy as np
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lb2_pool"
stamps = [float(x) for x in sys.argv[2:]] or [1.0, 4.0]
os.makedirs(out, exist_ok=True)
m = PfspModel(56, 2)
eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=16 << 30))
nodes, _, _, best = m.warmup(m.initial_best(1), 25)
eng.begin(nodes, int(best))
t0 = time.perf_counter()
for ts in stamps:
    left = ts - (time.perf_counter() - t0)
    if left > 0:
        eng.run(max_seconds=left)
    n = eng.size()
    pool = eng.pop(n)
    top = pool[-16384:]
    np.save(os.path.join(out, f"ta056_top_{ts:g}s.npy"), top)
    eng.push(pool)
    print(f"t={ts:g}s pool={n} saved {len(top)} nodes best={eng.best} tree={eng.stats()['tree']}", flush=True)
