#!/usr/bin/env python3
"""-u 0 device dive (pool_device.hpp Slot::cap): explored trees and times of searches
from +inf for several dive windows / growth shifts, against no dive (window 0) and the
opt-in heuristic start (TTS_DIVE beam dive + NEH). One GPU; --worlds adds multi-rank
runs (gloo, every rank on device 0) of the chosen settings.

    python scripts/dive_probe.py [--cases 14:1,8:0] [--windows 0,64,256,1024,4096] [--shifts 1,2,3]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dist_gpu_accelerated_tree_search_amd.parallel.launch import spawn_local, warm_forkserver  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="14:1,8:0,3:1")
    ap.add_argument("--windows", default="0,64,256,1024,4096")
    ap.add_argument("--shifts", default="1,2,3", help="growth shift per iteration (+256: hold while improving)")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--worlds", default="")
    ap.add_argument("--world-window", type=int, default=1024)
    ap.add_argument("--world-shift", type=int, default=2)
    ap.add_argument("--max-parents", type=int, default=1 << 18)
    a = ap.parse_args()
    warm_forkserver()
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions, PfspModel
    from dist_gpu_accelerated_tree_search_amd.parallel.workers import solve_rank
    from dist_gpu_accelerated_tree_search_amd.search import solve_engine

    print(f"{'case':>10} {'window':>6} {'shift':>5} {'tree min':>12} {'tree max':>12} {'best':>5} {'ms (per repeat)':>30}", flush=True)
    for case in a.cases.split(","):
        inst, lb = (int(x) for x in case.split(":"))
        model = PfspModel(inst, lb)
        name = f"ta{inst:03d}/{['LB1_d', 'LB1', 'LB2'][lb]}"
        runs = [(w, s) for w in (int(x) for x in a.windows.split(",")) for s in
                ((0,) if w == 0 else (int(x) for x in a.shifts.split(",")))]
        runs.append(("heur", 0))
        for w, s in runs:
            heur = w == "heur"
            os.environ["TTS_DIVE"] = "32" if heur else "0"
            eng = model.make_engine("gpu", 0, EngineOptions(ring_bytes=8 << 30, dive_window=0 if heur else w,
                                                            dive_shift=s, max_parents=a.max_parents))
            ts, r, trees = [], None, []
            for _ in range(a.repeat):
                t0 = time.perf_counter()
                r = solve_engine(model, eng, ub=0)
                ts.append((time.perf_counter() - t0) * 1e3)
                trees.append(r.tree)
                assert r.best == model.best_known, (name, r.best, model.best_known)
            del eng
            print(f"{name:>10} {str(w):>6} {s:>5} {min(trees):>12} {max(trees):>12} {r.best:>5} "
                  f"{' '.join(f'{t:.2f}' for t in ts):>30}", flush=True)
        os.environ["TTS_DIVE"] = "0"
        for world in (int(x) for x in a.worlds.split(",") if x):
            spec = {"problem": "pfsp", "inst": inst, "lb": lb, "backend": "gpu", "comm": "gloo", "device": 0,
                    "session": True, "ub": 0, "repeat": 1,
                    "engine": {"ring_bytes": 4 << 30, "dive_window": a.world_window, "dive_shift": a.world_shift,
                               "max_parents": a.max_parents}}
            trees, ts = [], []
            for _ in range(a.repeat):
                res = spawn_local(world, solve_rank, (spec,), timeout=600, env={"TTS_DIVE": "0"})
                assert res[0]["best"] == model.best_known
                trees.append(res[0]["tree"])
                ts.append(res[0]["t_search"] * 1e3)
            print(f"{name:>10} world {world} window {a.world_window} shift {a.world_shift}: trees {trees} "
                  f"t_search ms {' '.join(f'{t:.1f}' for t in ts)}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
