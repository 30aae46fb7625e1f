"""Per-config timings on one GPU (solve time, iterations, launches) for tuning."""
import sys, time, json
sys.path.insert(0, ".")
import torch  # noqa
from dist_gpu_accelerated_tree_search_amd import PfspModel, QueensModel, EngineOptions, solve_engine

def run(model, opts, reps=5, ub=1):
    eng = model.make_engine("gpu", 0, opts)
    out = []
    for i in range(reps):
        r = solve_engine(model, eng, ub=ub)
        out.append(r)
    best = min(out, key=lambda r: r.elapsed)
    st = eng.stats()
    del eng
    return best, st

cases = [("ta014 lb1", PfspModel(14, 1)), ("ta014 lb0", PfspModel(14, 0)), ("ta014 lb2", PfspModel(14, 2)),
         ("ta008 lb0", PfspModel(8, 0)), ("ta010 lb2", PfspModel(10, 2)), ("ta020 lb2", PfspModel(20, 2))]
for mp in (1 << 16, 1 << 18, 1 << 20):
    for name, m in cases[:2]:
        r, st = run(m, EngineOptions(max_parents=mp, ring_bytes=8 << 30))
        print(f"{name} mp={mp}: tree={r.tree} t={r.elapsed*1e3:.3f} ms init={r.t_init*1e3:.3f} search={r.t_search*1e3:.3f} "
              f"iters={r.extra['iters']} launches={r.extra['launches']} -> {r.tree/r.elapsed/1e9:.2f} G/s", flush=True)
for name, m in cases[2:]:
    r, st = run(m, EngineOptions(max_parents=1 << 18, ring_bytes=8 << 30), reps=2)
    print(f"{name}: tree={r.tree} sol={r.sol} best={r.best} t={r.elapsed*1e3:.2f} ms iters={r.extra['iters']} -> {r.tree/r.elapsed/1e9:.3f} G/s", flush=True)
for N in (15, 16, 17):
    r, st = run(QueensModel(N), EngineOptions(max_parents=1 << 20, ring_bytes=32 << 30), reps=1 if N == 17 else 2)
    print(f"queens N={N}: tree={r.tree} sol={r.sol} t={r.elapsed*1e3:.2f} ms iters={r.extra['iters']} -> {r.tree/r.elapsed/1e9:.2f} G/s", flush=True)
