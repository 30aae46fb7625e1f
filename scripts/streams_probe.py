#!/usr/bin/env python3
"""Sub-engines per GPU (EngineOptions.streams, csrc/core/multi_engine.hpp) on the big
BASELINE trees: ta021 LB1_d complete solve, ta056 LB2 time box, ta008 LB1_d, and the
ta014 headline (where one engine should stay best: latency-bound).

    python scripts/streams_probe.py [--streams 1,2,3,4] [--box 5]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.search import solve_engine  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--box", type=float, default=5.0)
    ap.add_argument("--mp", type=int, default=1 << 19)
    ap.add_argument("--needy", type=float, default=1 / 16)
    ap.add_argument("--donor", type=float, default=1 / 4)
    ap.add_argument("--only", default="ta014,ta008,ta021,ta056")
    a = ap.parse_args()
    only = a.only.split(",")
    for k in (int(x) for x in a.streams.split(",")):
        opts = EngineOptions(streams=k, max_parents=a.mp, ring_bytes=48 << 30, stream_needy=a.needy,
                             stream_donor=a.donor)
        if "ta014" in only:
            m = PfspModel(14, 1)
            eng = m.make_engine("gpu", 0, opts)
            ts = []
            for _ in range(30):
                r = solve_engine(m, eng)
                assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
                ts.append(r.elapsed)
            ts.sort()
            print(f"streams {k} ta014 LB1: median {ts[15] * 1e3:.3f} ms min {ts[0] * 1e3:.3f} ms", flush=True)
            del eng
        if "ta008" in only:
            m = PfspModel(8, 0)
            eng = m.make_engine("gpu", 0, opts)
            ts = []
            for _ in range(5):
                r = solve_engine(m, eng)
                assert (r.tree, r.sol, r.best) == (113458723, 808498, 1206)
                ts.append(r.elapsed)
            ts.sort()
            print(f"streams {k} ta008 LB1_d: median {ts[2] * 1e3:.2f} ms -> {r.tree / ts[2] / 1e9:.2f} G nodes/s",
                  flush=True)
            del eng
        if "ta021" in only:
            m = PfspModel(21, 0)
            eng = m.make_engine("gpu", 0, opts)
            t0 = time.perf_counter()
            r = solve_engine(m, eng)
            dt = time.perf_counter() - t0
            assert (r.tree, r.sol, r.best) == (260069628524, 14963858, 2297), (r.tree, r.sol, r.best)
            print(f"streams {k} window {a.mp} needy {a.needy:.4f} donor {a.donor:.4f} ta021 LB1_d: {dt:.2f} s -> {r.tree / dt / 1e9:.2f} G nodes/s", flush=True)
            del eng
        if "ta056" in only:
            m = PfspModel(56, 2)
            eng = m.make_engine("gpu", 0, opts)
            nodes, _, _, best = m.warmup(m.initial_best(1), 25)
            eng.begin(nodes, int(best))
            eng.run(max_seconds=0.5)
            s0 = eng.stats()
            t0 = time.perf_counter()
            eng.run(max_seconds=a.box)
            dt = time.perf_counter() - t0
            s1 = eng.stats()
            print(f"streams {k} ta056 LB2: {(s1['tree'] - s0['tree']) / dt / 1e9:.4f} G nodes/s over {dt:.1f} s",
                  flush=True)
            del eng
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
