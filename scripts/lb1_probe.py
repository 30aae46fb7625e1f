"""LB1/LB1_d timings on one GPU: ta014 headline solve, ta008 LB1_d, ta021 LB1_d steady rate."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, solve_engine

GOLD = {(14, 1): (2573652, 2648, 1377), (8, 0): (113458723, 808498, 1206)}
for key, reps in (((14, 1), 60), ((8, 0), 3)):
    m = PfspModel(*key)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
    ts = []
    for _ in range(reps):
        r = solve_engine(m, eng)
        assert (r.tree, r.sol, r.best) == GOLD[key], (key, r.tree, r.sol, r.best)
        ts.append(r.elapsed)
    ts.sort()
    print(f"ta{key[0]:03d} lb{key[1]}: median {ts[len(ts)//2]*1e3:.3f} ms min {ts[0]*1e3:.3f} ms "
          f"-> {r.tree/ts[0]/1e9:.2f} G nodes/s", flush=True)
    del eng
m = PfspModel(21, 0)
eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=16 << 30))
nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
eng.begin(nodes, int(best))
eng.run(max_seconds=0.3)
st0 = eng.stats()
t0 = time.perf_counter()
eng.run(max_seconds=2.0)
dt = time.perf_counter() - t0
st = eng.stats()
print(f"ta021 lb0 steady: {(st['tree'] - st0['tree'])/dt/1e9:.2f} G nodes/s", flush=True)
