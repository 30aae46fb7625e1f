"""Iteration log of whole solves (TTS_ILOG, pool_device.hpp ilog_record): for every
device iteration its start time, window, shape and the explored tree so far.

    python scripts/ilog_probe.py [inst] [lb] [solves] [max_parents_log2] [world]

world > 1: rank 0's share of a world-way in-graph split (as scripts/share_solve_probe.py).

Prints, per iteration of the last solve: the gap to the next iteration's start (its
duration plus launch), the pool (S stack + C buffered children), the window B, the shape
(one / fused L levels / local with steps, strided), and the tree explored by it.
"""
import os
import sys
import tempfile

import numpy as np

path = os.path.join(tempfile.mkdtemp(), "ilog.bin")
os.environ["TTS_ILOG"] = path
sys.path.insert(0, ".")
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.search import solve_engine  # noqa: E402

inst = int(sys.argv[1]) if len(sys.argv) > 1 else 14
lb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
solves = int(sys.argv[3]) if len(sys.argv) > 3 else 3
mp = int(sys.argv[4]) if len(sys.argv) > 4 else 19
m = PfspModel(inst, lb)
eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << mp, ring_bytes=4 << 30))
world = int(sys.argv[5]) if len(sys.argv) > 5 else 1
if world > 1:
    for _ in range(solves):
        nodes, t1, s1, best = m.warmup(m.initial_best(1), 25)
        eng.set_split(0, world, 512 * world)
        eng.begin(nodes, int(best))
        eng.run()
    print(f"ta{inst:03d} lb {lb}: rank 0 of {world}: tree {eng.stats()['tree']}", flush=True)
else:
    for _ in range(solves):
        r = solve_engine(m, eng, ub=1)
    print(f"ta{inst:03d} lb {lb}: tree {r.tree} sol {r.sol} best {r.best} elapsed {r.elapsed * 1e3:.3f} ms", flush=True)
del eng
import gc  # noqa: E402

gc.collect()
from dist_gpu_accelerated_tree_search_amd import ops  # noqa: E402

ops.release_all() if hasattr(ops, "release_all") else None
if not os.path.exists(path):
    sys.exit("no iteration log written (engine not released?)")
rec = np.fromfile(path, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
# split into solves: the tree counter restarts
starts = [0] + [i for i in range(1, len(rec)) if rec[i, 5] < rec[i - 1, 5]]
last = rec[starts[-1]:]
clk_mhz = 100.0
print(f"{len(rec)} records, {len(starts)} solves; last solve {len(last)} iterations")
print("   dt_us        S        C        B  chunks  bp st  shape          tree_delta")
tree = last[:, 5]
for i, x in enumerate(last):
    dt = (last[i + 1, 0] - x[0]) / clk_mhz if i + 1 < len(last) else float("nan")
    sh = int(x[4])
    nch, bp, steps, fl, lev = sh & 0xFFFFF, (sh >> 20) & 0xFFFF, (sh >> 36) & 0xFF, (sh >> 44) & 0xF, (sh >> 48) & 0xF
    flags = (sh >> 44) & 0xFF
    kind = "empty" if x[3] == 0 else ("local" + ("/str" if flags & 2 else "") if flags & 1 else
                                        (f"fused L{lev}" if flags & 4 else "one"))
    if flags & 8:
        kind += " split"
    nxt = tree[i + 1] - tree[i] if i + 1 < len(last) else 0
    print(f"{dt:8.2f} {x[1]:8d} {x[2]:8d} {x[3]:8d} {nch:7d} {bp:3d} {steps:2d}  {kind:14s} {nxt:10d}")
