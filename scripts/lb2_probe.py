"""LB2 timings on one GPU: golden trees (ta014/ta010/ta020) and a time-boxed ta056 run.

    python scripts/lb2_probe.py [ta056_seconds]
"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, solve_engine

GOLD = {14: (144639, 0, 1377), 10: (8122579, 0, 1108), 20: (4870386, 0, 1591), 3: (80062, 0, 1081)}
for inst in (14, 3, 10, 20):
    m = PfspModel(inst, 2)
    eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=8 << 30))
    ts = []
    for _ in range(3):
        r = solve_engine(m, eng)
        assert (r.tree, r.sol, r.best) == GOLD[inst], (inst, r.tree, r.sol, r.best)
        ts.append(r.elapsed)
    st = eng.stats()
    print(f"ta{inst:03d} lb2: tree={r.tree} t={min(ts)*1e3:.2f} ms iters={st['iters']} "
          f"-> {r.tree/min(ts)/1e9:.3f} G nodes/s", flush=True)
    del eng

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
m = PfspModel(56, 2)
eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=32 << 30))
nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
eng.begin(nodes, int(best))
t0 = time.perf_counter()
done = False
while time.perf_counter() - t0 < secs:
    eng.run(max_seconds=2.0)
    st = eng.stats()
    el = time.perf_counter() - t0
    print(f"ta056 lb2 {el:6.1f} s: tree={st['tree']} pool={eng.size()} iters={st['iters']} "
          f"-> {st['tree']/el/1e9:.3f} G nodes/s", flush=True)
    if eng.size() == 0:
        done = True
        break
print("ta056 lb2", "solved" if done else "time-boxed", f"best={eng.best}")
