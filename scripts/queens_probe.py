"""N-Queens on one GPU: golden counts and solve times for subtree-finishing depths.

    python scripts/queens_probe.py [N ...]
TTS_QUEENS_FINISH = columns left at which a parent's thread explores its subtree to the
end (0 = level-by-level through the device pool). Engine construction is outside the
timed solves (min / median of 5)."""
import os
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, QueensModel, solve_engine

GOLD = {12: (856188, 14200), 14: (27358552, 365596), 15: (171129071, 2279184), 17: (8017021931, 95815104)}
ok = True
for N in [int(x) for x in sys.argv[1:]] or [16, 17]:
    for k in [int(x) for x in os.environ.get("KS", "0,6,7,8,9").split(",")]:
        os.environ["TTS_QUEENS_FINISH"] = str(k)
        m = QueensModel(N)
        eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 20, ring_bytes=16 << 30))
        ts = []
        for _ in range(5 if N < 17 else 3):
            t0 = time.perf_counter()
            r = solve_engine(m, eng)
            ts.append(time.perf_counter() - t0)
        if N not in GOLD:  # no golden tree: the level-by-level run (finish 0) is the reference
            GOLD[N] = (r.tree, r.sol)
        good = (r.tree, r.sol) == GOLD[N]
        ok &= good
        ts.sort()
        print(f"N={N} finish={k:2d}: tree {r.tree} sol {r.sol} {'ok' if good else 'WRONG'} | min {ts[0] * 1e3:.2f} ms "
              f"median {ts[len(ts) // 2] * 1e3:.2f} ms -> {r.tree / ts[0] / 1e9:.1f} G nodes/s | iters {eng.stats()['iters']}",
              flush=True)
        del eng
print("queens probe", "OK" if ok else "FAILED")
sys.exit(0 if ok else 1)
