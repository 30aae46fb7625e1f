"""Two-level (fused) iterations: ta014 LB1 solve time and iteration count at 1 rank and
for rank 0 of an 8-rank in-search split, with TTS_FUSE_MAX set to each argument
(0 = off; unset = the kernel's limit)."""
import os
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel

for fm in sys.argv[1:] or ["default", "0"]:
    os.environ.pop("TTS_FUSE_MAX", None)
    if fm != "default":
        os.environ["TTS_FUSE_MAX"] = fm
    m = PfspModel(14, 1)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=8 << 30))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    for world in (1, 8):
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            if world > 1:
                eng.set_split(0, world, 4096)
            eng.begin(nodes, int(best))
            eng.run()
            st = eng.stats()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print(f"fuse_max {fm:>8} world {world}: tree {st['tree']} iters {st['iters']} min {ts[0] * 1e3:.3f} ms "
              f"median {ts[15] * 1e3:.3f} ms", flush=True)
    del eng
