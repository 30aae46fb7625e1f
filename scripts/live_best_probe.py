#!/usr/bin/env python3
"""-u 0 trees with and without the live incumbent exchange (round 3).

With -u 0 the explored tree depends on how fast a good incumbent reaches every
rank. Ranks exchange the incumbent at every round (status all-gather) and, with
DistConfig.live_best (default), after every graph replay through the node-wide
board (ShmControl::exchange_best; ref checkBest around every batch,
pfsp_multigpu_cuda.c:30-50,307-312). This runs ta014 LB1 and ta008 LB1_d at
1, 2 and 4 ranks sharing one GPU (gloo for the node payloads) and prints the trees.

    python scripts/live_best_probe.py [--worlds 1,2,4] [--repeat 2]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dist_gpu_accelerated_tree_search_amd.parallel.launch import spawn_local, warm_forkserver  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.parallel.workers import solve_rank  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4")
    ap.add_argument("--cases", default="14:1,8:0")
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    warm_forkserver()
    opt = {14: 1377, 8: 1206}
    print(f"{'case':>10} {'world':>5} {'live':>5} {'tree (per repeat)':>40} {'best':>5} {'t_search ms':>12}")
    for case in a.cases.split(","):
        inst, lb = (int(x) for x in case.split(":"))
        for world in (int(x) for x in a.worlds.split(",")):
            for live in ((True,) if world == 1 else (False, True)):
                spec = {"problem": "pfsp", "inst": inst, "lb": lb, "backend": "gpu", "comm": "gloo", "device": 0,
                        "session": True, "ub": 0, "repeat": 1,
                        "engine": {"ring_bytes": 8 << 30}, "dist": {"live_best": live}}
                trees, ts, best = [], [], None
                for _ in range(a.repeat):
                    res = spawn_local(world, solve_rank, (spec,), timeout=900)
                    trees.append(res[0]["tree"])
                    ts.append(res[0]["t_search"] * 1e3)
                    best = res[0]["best"]
                    assert best == opt[inst], (inst, best)
                name = f"ta{inst:03d}/{['LB1_d', 'LB1', 'LB2'][lb]}"
                print(f"{name:>10} {world:>5} {str(live):>5} {str(trees):>40} {best:>5} "
                      f"{' '.join(f'{t:.1f}' for t in ts):>12}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
