#!/usr/bin/env python3
"""Where does the -u 0 multi-rank tree inflation come from? (round-4 verdict item 8)

Runs ta008 LB1_d (and ta014 LB1) with -u 0 at 1, 2 and 4 ranks sharing one GPU (gloo
for node payloads, shared-memory board for the incumbent) with the incumbent timeline
on (DistConfig.trace_incumbent): per rank, every change of its incumbent with the time
since the rounds began, the tree the rank had explored, and whether the rank's own
leaves or a peer's exchange brought it. Prints, per rank, when the optimum became
known and how much it had explored by then, and the whole trees.

    python scripts/incumbent_probe.py [--worlds 1,2,4] [--cases 8:0,14:1] [--window N]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dist_gpu_accelerated_tree_search_amd.parallel.launch import spawn_local, warm_forkserver  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.parallel.workers import solve_rank  # noqa: E402

OPT = {14: 1377, 8: 1206, 10: 1108}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4")
    ap.add_argument("--cases", default="8:0,14:1")
    ap.add_argument("--window", type=int, default=0, help="max_parents (0: engine default)")
    ap.add_argument("--extra", default="", help="extra dist options k=v,k=v (ints)")
    a = ap.parse_args()
    warm_forkserver()
    for case in a.cases.split(","):
        inst, lb = (int(x) for x in case.split(":"))
        for world in (int(x) for x in a.worlds.split(",")):
            eng = {"ring_bytes": 8 << 30}
            if a.window:
                eng["max_parents"] = a.window
            dist = {"trace_incumbent": True}
            for kv in filter(None, a.extra.split(",")):
                k, v = kv.split("=")
                dist[k] = int(v)
            spec = {"problem": "pfsp", "inst": inst, "lb": lb, "backend": "gpu", "comm": "gloo", "device": 0,
                    "session": True, "ub": 0, "repeat": 1, "engine": eng, "dist": dist}
            res = spawn_local(world, solve_rank, (spec,), timeout=900)
            print(f"ta{inst:03d} lb{lb} world {world}: tree {res[0]['tree']:,} best {res[0]['best']} "
                  f"t_search {res[0]['t_search'] * 1e3:.1f} ms, per-rank tree "
                  f"{[w['tree'] for w in res[0]['workers']]}", flush=True)
            for r in sorted(res, key=lambda x: x["rank"]):
                ev = r["extra"].get("incumbent_events", [])
                first = ev[0] if ev else None
                opt = next((e for e in ev if e[3] <= OPT.get(inst, 0)), None)
                src = lambda e: "own" if e[2] <= e[3] else "peer"  # noqa: E731
                line = f"   rank {r['rank']}: {len(ev)} incumbent changes"
                if first:
                    line += f"; first {int(first[3])} at {first[0] * 1e3:.2f} ms after {int(first[1]):,} nodes ({src(first)})"
                if opt:
                    line += f"; optimum {int(opt[3])} at {opt[0] * 1e3:.2f} ms after {int(opt[1]):,} nodes ({src(opt)})"
                print(line, flush=True)
                for e in ev[:12]:
                    print(f"      {e[0] * 1e3:8.2f} ms  tree {int(e[1]):>12,}  own {int(e[2]):>10}  now {int(e[3]):>6} "
                          f"({src(e)})", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
