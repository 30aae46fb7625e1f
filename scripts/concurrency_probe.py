#!/usr/bin/env python3
"""Does one engine fill the GPU? Rates of big trees with one engine (parent window,
grid) vs several engines on the same device (separate streams, native runner).

Round 3 finding: two ranks sharing one MI355X solved ta021 LB1_d in 9.8 s against
15.4 s for one rank, and ran ta056 LB2 at 0.169 vs 0.116 G nodes/s. This separates
the causes: window size (chunks per iteration vs the resident grid) and concurrency.

    python scripts/concurrency_probe.py [--box 2.0]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.search import solve_workers  # noqa: E402


def steady_rate(model, opts, box, env=None):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        eng = model.make_engine("gpu", 0, opts)
        nodes, _, _, best = model.warmup(model.initial_best(1), 25)
        eng.begin(nodes, int(best))
        eng.run(max_seconds=0.3)
        s0 = eng.stats()
        t0 = time.perf_counter()
        eng.run(max_seconds=box)
        dt = time.perf_counter() - t0
        s1 = eng.stats()
        del eng
        return (s1["tree"] - s0["tree"]) / dt, (s1["iters"] - s0["iters"]) / dt
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--box", type=float, default=2.0)
    a = ap.parse_args()
    for inst, lb in ((21, 0), (56, 2)):
        m = PfspModel(inst, lb)
        for mp in (1 << 16, 1 << 18, 1 << 19, 1 << 20):
            for bpc in (None, "8", "16"):
                env = {"TTS_BLOCKS_PER_CU": bpc} if bpc else {}
                r, it = steady_rate(m, EngineOptions(max_parents=mp, ring_bytes=16 << 30), a.box, env)
                print(f"ta{inst:03d} lb{lb} max_parents {mp:>8} blocks/CU {bpc or 'occ':>3}: "
                      f"{r / 1e9:7.3f} G nodes/s, {it:8.0f} iterations/s", flush=True)
    # several engines on one device, native runner (complete ta021 solve)
    m = PfspModel(21, 0)
    for k in (1, 2, 3):
        t0 = time.perf_counter()
        r = solve_workers(m, devices=(0,) * k, opts=EngineOptions(ring_bytes=16 << 30))
        dt = time.perf_counter() - t0
        print(f"ta021 lb0 runner with {k} engine(s) on GPU 0: {dt:.2f} s, tree {r.tree}, "
              f"{r.tree / dt / 1e9:.2f} G nodes/s", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
