"""Per-instance regression table for the device engine's defaults: every change of a
production heuristic (local-DFS steps, stride, fusion, dynamic iterations) is checked on
trees of different shapes, at one engine and at three engines per GPU.

    python scripts/regress.py [rows] [--env K=V ...]

rows: comma list of inst:lb (default 3:1,8:0,14:1,21:0). Each row prints seconds (best
of `reps` solves after one untimed solve; ta021 one solve), tree, nodes/s and whether
(tree, sol, makespan) equals the golden. The engine is built outside the timed solves.
"""
import os
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.search import solve_engine  # noqa: E402

GOLDEN = {(3, 1): (2573133, 5689, 1081), (8, 0): (113458723, 808498, 1206), (14, 1): (2573652, 2648, 1377),
          (21, 0): (260069628524, 14963858, 2297)}
REPS = {(21, 0): 1, (8, 0): 3}

rows = [tuple(int(x) for x in r.split(":")) for r in (sys.argv[1] if len(sys.argv) > 1 and ":" in sys.argv[1]
                                                       else "3:1,8:0,14:1,21:0").split(",")]
engines = [int(x) for x in os.environ.get("TTS_REGRESS_ENGINES", "1,3").split(",")]
print(f"{'inst':>5} {'lb':>5} {'eng':>3} {'seconds':>10} {'tree':>14} {'Gnodes/s':>9}  golden", flush=True)
for inst, lb in rows:
    model = PfspModel(inst, lb)
    for k in engines:
        opts = EngineOptions(ring_bytes=(64 << 30) if (inst, lb) == (21, 0) else (8 << 30), streams=k,
                             max_parents=1 << 19 if k > 1 else 1 << 18)
        eng = model.make_engine("gpu", 0, opts)
        reps = REPS.get((inst, lb), 10)
        if reps > 1:
            solve_engine(model, eng, ub=1)  # graphs, first-graph learning
        best = float("inf")
        r = None
        for _ in range(reps):
            t0 = time.perf_counter()
            r = solve_engine(model, eng, ub=1)
            best = min(best, time.perf_counter() - t0)
        ok = (r.tree, r.sol, r.best) == GOLDEN.get((inst, lb), (r.tree, r.sol, model.best_known))
        print(f"ta{inst:03d} {['LB1_d', 'LB1', 'LB2'][lb]:>5} {k:>3} {best:>10.4f} {r.tree:>14} "
              f"{r.tree / best / 1e9:>9.3f}  {'ok' if ok else 'MISMATCH'}", flush=True)
        del eng
