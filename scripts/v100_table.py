"""The reference's published single-GPU table (pfsp/data/single-GPU.py, 20x20
Taillard instances, -l 1 -u 1) measured on one MI355X: one complete solve per instance
with the bench's large-tree setup (3 engines on the GPU), the tree checked for the
best-known makespan, and the speed-up over the V100 CUDA and MI50 HIP wall times.

    python scripts/v100_table.py [inst,...]
"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.search import solve_engine  # noqa: E402

# pfsp/data/single-GPU.py:6,21,23 (V100 CUDA) and :40,42 (MI50 HIP), seconds
V100 = {29: 4.18, 30: 4.91, 22: 5.63, 27: 19.82, 23: 41.04, 28: 73.75, 25: 81.97, 26: 176.40, 24: 738.93, 21: 1308.79}
MI50 = {29: 7.56, 30: 9.14, 22: 10.52, 27: 38.08, 23: 79.44, 28: 140.81, 25: 159.35, 26: 379.45, 24: 1445.49,
        21: 2538.23}
insts = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [29, 30, 22, 27, 23, 28, 25, 26, 24, 21]
print(f"{'inst':>5} {'tree':>15} {'sol':>10} {'mksp':>5} {'seconds':>8} {'Gnodes/s':>9} {'V100 s':>8} {'x V100':>7} "
      f"{'x MI50':>7}", flush=True)
for inst in insts:
    m = PfspModel(inst, 1)
    eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=64 << 30, streams=3, max_parents=1 << 19))
    t0 = time.perf_counter()
    r = solve_engine(m, eng, ub=1)
    dt = time.perf_counter() - t0
    ok = r.best == m.best_known
    print(f"ta{inst:03d} {r.tree:>15} {r.sol:>10} {r.best:>5} {dt:>8.3f} {r.tree / dt / 1e9:>9.2f} {V100[inst]:>8.2f} "
          f"{V100[inst] / dt:>7.0f} {MI50[inst] / dt:>7.0f}{'' if ok else '  MAKESPAN != best known'}", flush=True)
    del eng
