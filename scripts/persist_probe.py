"""Persistent iterations (lb1_small_persist) on one GPU: goldens and solve times, on vs off.

    python scripts/persist_probe.py
Each configuration is a fresh engine (the TTS_PERSIST_* knobs are read at construction)."""
import os
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, solve_engine

G = {(14, 1): (2573652, 2648, 1377), (8, 0): (113458723, 808498, 1206)}


def run(inst, lb, env, reps, ub=1):
    for k in [k for k in os.environ if k.startswith("TTS_PERSIST")]:
        del os.environ[k]
    os.environ.update(env)
    m = PfspModel(inst, lb)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=8 << 30))
    ts = []
    r = None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = solve_engine(m, eng, ub=ub)
        ts.append(time.perf_counter() - t0)
        if ub == 1 and (r.tree, r.sol, r.best) != G[(inst, lb)]:
            print(f"ta{inst:03d} lb{lb} {env}: WRONG {(r.tree, r.sol, r.best)} != {G[(inst, lb)]}", flush=True)
            return False
    ts.sort()
    st = eng.stats()
    print(f"ta{inst:03d} lb{lb} ub{ub} {env or 'default'}: tree {r.tree} sol {r.sol} best {r.best} | "
          f"min {ts[0] * 1e3:.3f} ms median {ts[len(ts) // 2] * 1e3:.3f} ms | launches {st['launches']} iters {st['iters']} | "
          f"per solve: steps {st['p_steps'] / reps:.0f} donations {st['p_donations'] / reps:.0f} waits {st['p_waits'] / reps:.0f} "
          f"wait {st['p_wait_us'] / reps:.0f} us (summed over workgroups)", flush=True)
    del eng
    return True


def run_split(world, env, reps=30, split_min=4096):
    """Rank 0's share of a `world`-rank in-search split solve of ta014 LB1 (the per-GPU
    critical path of the multi-GPU headline), timed on one GPU."""
    for k in [k for k in os.environ if k.startswith("TTS_PERSIST")]:
        del os.environ[k]
    os.environ.update(env)
    m = PfspModel(14, 1)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=8 << 30))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.set_split(0, world, split_min)
        eng.begin(nodes, int(best))
        eng.run()
        st = eng.stats()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"ta014 split rank 0 of {world} {env or 'default'}: tree {st['tree']} | min {ts[0] * 1e3:.3f} ms "
          f"median {ts[len(ts) // 2] * 1e3:.3f} ms | iters {st['iters']}", flush=True)
    del eng
    return True


ok = True
if len(sys.argv) > 1 and sys.argv[1] == "split":
    for w in (1, 2, 4, 8):
        for env in ({"TTS_PERSIST_MIN": "0"}, {"TTS_PERSIST_MIN": "256"}, {"TTS_PERSIST_MIN": "20000"}):
            run_split(w, env)
    sys.exit(0)
cfgs = [a.split(",") for a in sys.argv[1:]] if len(sys.argv) > 1 else None
if cfgs:
    for c in cfgs:  # inst,lb,reps[,K=V...]
        ok &= run(int(c[0]), int(c[1]), dict(x.split("=") for x in c[3:]), int(c[2]))
else:
    ok &= run(14, 1, {}, 30)
    ok &= run(14, 1, {"TTS_PERSIST_WT": "0"}, 30)
    ok &= run(14, 1, {"TTS_PERSIST_MIN": "0"}, 30)
    ok &= run(14, 1, {"TTS_PERSIST_MIN": "4096"}, 30)
    ok &= run(14, 1, {"TTS_PERSIST_US": "10"}, 10)
    ok &= run(14, 1, {"TTS_PERSIST_DMIN": "512"}, 10)
    ok &= run(14, 1, {"TTS_PERSIST_DMIN": "512", "TTS_PERSIST_WT": "0"}, 10)
    ok &= run(14, 1, {}, 5, ub=0)
    ok &= run(8, 0, {}, 2)
    ok &= run(8, 0, {"TTS_PERSIST_MIN": "0"}, 2)
    ok &= run(8, 0, {"TTS_PERSIST_US": "200"}, 2)
print("persist probe", "OK" if ok else "FAILED")
sys.exit(0 if ok else 1)
