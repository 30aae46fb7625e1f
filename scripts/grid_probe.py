"""ta014 LB1 solve time and empty-replay cost vs workgroups per CU (TTS_BLOCKS_PER_CU)."""
import os
import sys
import time
sys.path.insert(0, ".")
import torch  # noqa
from dist_gpu_accelerated_tree_search_amd import PfspModel, EngineOptions, solve_engine

m = PfspModel(14, 1)
for per in ("1", "2", "3", "4", "0"):
    if per == "0":
        os.environ.pop("TTS_BLOCKS_PER_CU", None)
    else:
        os.environ["TTS_BLOCKS_PER_CU"] = per
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=8 << 30))
    ts = []
    for i in range(60):
        r = solve_engine(m, eng)
        assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
        ts.append(r.elapsed)
    ts.sort()
    # empty replays: a 24-iteration graph on an empty pool
    eng.begin(m.root()[:0], 1377)
    t0 = time.perf_counter()
    for i in range(50):
        eng.begin(m.root()[:0], 1377)
        eng.run(max_launches=1)
    te = (time.perf_counter() - t0) / 50
    print(f"blocks/CU={per}: median {ts[len(ts)//2]*1e3:.3f} ms min {ts[0]*1e3:.3f} ms; empty run {te*1e6:.1f} us", flush=True)
    del eng
