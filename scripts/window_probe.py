"""ta014 LB1 solve time against the parent window (max_parents) and the grid.

The widest ta014 iterations hold a whole window; with 2048 chunks of 256 parents and
fewer resident workgroups than chunks, part of the window runs as a second pass of
chunks. Usage: python scripts/window_probe.py [max_parents ...]
"""
import os
import sys

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, solve_engine

GOLD = (2573652, 2648, 1377)
sizes = [int(x) for x in sys.argv[1:]] or [1 << 19, 7 * 256 * 256, 6 * 256 * 256, 3 << 17, 1 << 18]
m = PfspModel(14, 1)
for mp in sizes:
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=mp, ring_bytes=8 << 30))
    ts, its = [], 0
    for _ in range(80):
        r = solve_engine(m, eng)
        assert (r.tree, r.sol, r.best) == GOLD, (mp, r.tree, r.sol, r.best)
        ts.append(r.elapsed)
    st = eng.stats()
    ts.sort()
    print(f"max_parents {mp:8d} blocks/CU {os.environ.get('TTS_BLOCKS_PER_CU', 'occ')}: median "
          f"{ts[len(ts) // 2] * 1e3:.4f} ms min {ts[0] * 1e3:.4f} ms, iterations/solve {st['iters'] / 80:.1f}",
          flush=True)
    del eng
