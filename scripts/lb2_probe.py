"""LB2 on one GPU: golden trees (ta014/ta003/ta010/ta020, best of 3) and a time-boxed
ta056 (50x20) run with a progress projection.

    python scripts/lb2_probe.py [ta056_seconds] [report_every_s]

Progress: W = pool_weight, the share of the permutation space still held by the pool
(a node of depth d stands for 1/(N(N-1)...(N-d+1)) of it; pruned subtrees count as
explored). The projection W / (-dW/dt) uses the rate at which W fell over the last
report interval; it is a rough indicator (B&B progress is not linear), not a bound.
"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, solve_engine
from dist_gpu_accelerated_tree_search_amd.search import progress_weights

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
every = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
m = PfspModel(56, 2)
w = progress_weights(m)
eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=32 << 30))
nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
eng.begin(nodes, int(best))
t0 = time.perf_counter()
done = False
W0, tw = eng.pool_weight(w), 0.0
while time.perf_counter() - t0 < secs:
    eng.run(max_seconds=every)
    st = eng.stats()
    el = time.perf_counter() - t0
    W = eng.pool_weight(w)
    rate = (W0 - W) / max(el - tw, 1e-9)
    proj = W / rate if rate > 0 else float("inf")
    W0, tw = W, el
    print(f"ta056 lb2 {el:7.1f} s: tree={st['tree']} pool={eng.size()} iters={st['iters']} "
          f"-> {st['tree']/el/1e9:.3f} G nodes/s, space left {W:.6e} (-{rate:.3e}/s), "
          f"projection {proj/3600:.3g} h on 1 GPU ({proj/3600/8:.3g} h on 8 at linear scaling)", flush=True)
    if eng.size() == 0:
        done = True
        break
print("ta056 lb2", "solved" if done else "time-boxed", f"best={eng.best}", flush=True)
