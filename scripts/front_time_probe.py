"""Time single front-kernel iterations over ta014 BFS windows under each iteration
shape (one level, 2/3/4-level chunks), with per-workgroup phase stamps.

    python scripts/front_time_probe.py [inst] [lb]
Stamps (pfsp_front_kernels.hpp front_stamp): 0 entry, 1 pool_begin done, 2 tables in
LDS, multi-level: 3 parents staged, 4..7 after level 0..3, 8 chunk done; one level:
4 bounds done, 5 scan done, 6 children stored; local DFS (LOC): 4..7 after step 0..3;
15 workgroup exit.
"""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd import ops  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel  # noqa: E402

inst = int(sys.argv[1]) if len(sys.argv) > 1 else 14
lb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
m = PfspModel(inst, lb)
H = ops.require_gpu(0)
best = m.best_known
depths = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else list(range(2, 20))
# rank share of an S-rank split: every S-th node of the level (TTS_PROBE_SHARE=S)
share = int(os.environ.get("TTS_PROBE_SHARE", "1"))
shapes = [("one", dict(fuse_max=0)), ("L2", dict(deep_levels=2, wide_levels=1)),
          ("L3", dict(deep_levels=3, deep_per3=1 << 20, wide_levels=1)),
          ("L4", dict(deep_levels=4, deep_per3=1 << 20, deep_per4=1 << 20, wide_levels=1)),
          ("W2", dict(deep_levels=2, wide_levels=2)), ("W3", dict(deep_levels=2, wide_levels=3)),
          ("LOC", dict(local_min=1, local_steps=4)), ("LOC2", dict(local_min=1, local_steps=2))]
if len(sys.argv) > 4:
    shapes = [x for x in shapes if x[0] in sys.argv[4].split(",")]
for dep in depths:
    nodes = ops.cpu().pfsp_bfs_level(m.native, m.host_lb, best, dep)[::share]
    if len(nodes) == 0:
        continue
    depth = np.bincount(nodes[:, 0])
    print(f"window {len(nodes)} nodes, depths {dict((i, int(c)) for i, c in enumerate(depth) if c)}", flush=True)
    for name, kw in shapes:
        d = H.pfsp_front_time(m.jobs, m.machines, list(m.native.p), m.lb, nodes, best, reps=20, **kw)
        st = d["stamps_us"]
        used = st[:, 0] > 0 if False else np.ones(len(st), bool)
        ent = st[:, 0]
        ex = st[:, 15]
        live = ex > 0
        parts = []
        prev = 0
        for k in (1, 2, 3, 4, 5, 6, 7, 8):
            col = st[live, k]
            ok = col > 0
            if ok.sum() == 0:
                continue
            base = st[live, prev][ok] if prev else ent[live][ok]
            dt = col[ok] - base
            parts.append(f"s{k} {dt.mean():.2f}/{dt.max():.2f}")
            prev = k
        if os.environ.get("TTS_PROBE_DETAIL"):  # exit time by XCD (workgroup i runs on XCD i % 8) and spread
            xcd = np.arange(len(st)) % 8
            by = [f"{ex[live & (xcd == x)].mean():.1f}/{ex[live & (xcd == x)].max():.1f}" for x in range(8)]
            q = np.percentile(ex[live], [10, 50, 90, 99])
            print(f"    exit by XCD (mean/max): {' '.join(by)} | p10/50/90/99 {q.round(1).tolist()}", flush=True)
            if st[live, 4].any():
                s0 = st[live, 4] - st[live, 2]
                print(f"    step0 p10/50/90/99 {np.percentile(s0, [10, 50, 90, 99]).round(1).tolist()}; "
                      f"corr(exit, step0) {np.corrcoef(ex[live], s0)[0, 1]:.2f}", flush=True)
        print(f"  {name:4s} {d['ms_min'] * 1e3:7.2f} us (median {d['ms_median'] * 1e3:.2f}) grid {d['grid']} "
              f"out chunks {d['nch_out']} | entry max {ent[live].max():.2f} exit mean {ex[live].mean():.2f} "
              f"max {ex[live].max():.2f} | " + " ".join(parts), flush=True)
