"""Where the headline's non-kernel time goes (ta014 LB1, one GPU).

Times, over many solves: the host warm-up alone, the engine's fused solve from the
warm-up nodes (begin + one learned graph replay + the wait), and the bench's whole
step (DistSolver.solve_raw: warm-up + fused solve in one native call). Kernel time
per solve comes from the kernel trace (scripts/gpu_run.sh ktrace:ta014).
"""
import statistics
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel
from dist_gpu_accelerated_tree_search_amd.parallel.comm import Comm
from dist_gpu_accelerated_tree_search_amd.parallel.runtime import DistConfig, DistSolver

m = PfspModel(14, 1)
eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
best0 = m.initial_best(1)
R = 300


def med(f):
    ts = []
    for _ in range(R):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6, min(ts) * 1e6


nodes, t1, s1, best = m.warmup(best0, 25)
for _ in range(20):
    eng.solve(nodes, int(best))
print("warm-up (host BFS to 25 nodes): median %.1f us, min %.1f us" % med(lambda: m.warmup(best0, 25)), flush=True)
print("engine.solve (begin + replay + wait): median %.1f us, min %.1f us" % med(lambda: eng.solve(nodes, int(best))),
      flush=True)
comm = Comm(use_gpu=True)
solver = DistSolver(m, eng, comm, DistConfig(), window=1 << 19)
for _ in range(20):
    solver.solve_raw(1)
print("DistSolver.solve_raw (bench step): median %.1f us, min %.1f us" % med(lambda: solver.solve_raw(1)), flush=True)
st = eng.stats()
print("engine stats: syncs %d iters %d t_run %.3f s" % (st.get("syncs", -1), st["iters"], st["t_run"]), flush=True)
