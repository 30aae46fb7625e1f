"""Where does a local-DFS front kernel's tail come from? Per-workgroup stamps plus the
hardware placement (HW_ID / XCC_ID read at entry) of one timed iteration per window.

    python scripts/lb_probe.py [inst] [depths] [steps] [dyn_us]

For each ta014 BFS window (depth d): the exit-time spread over workgroups, the same
grouped by CU (max exit per CU: is the kernel bound by one slow workgroup or by whole
CUs?), the correlation of a workgroup's exit with its own work (nodes expanded), with
its CU's total work, and with its dispatch rank inside the CU (age priority).
"""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd import ops  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel  # noqa: E402

inst = int(sys.argv[1]) if len(sys.argv) > 1 else 14
depths = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [9, 11, 13, 15]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
dyn_us = int(sys.argv[4]) if len(sys.argv) > 4 else 0
m = PfspModel(inst, 1)
H = ops.require_gpu(0)
best = m.best_known


def corr(x, y):
    if np.std(x) == 0 or np.std(y) == 0:
        return float("nan")
    return float(np.corrcoef(x, y)[0, 1])


for dep in depths:
    nodes = ops.cpu().pfsp_bfs_level(m.native, m.host_lb, best, dep)
    if len(nodes) == 0:
        continue
    d = H.pfsp_front_time(m.jobs, m.machines, list(m.native.p), m.lb, nodes, best, reps=10, local_min=1,
                          local_steps=steps, dyn_us=dyn_us)
    st = d["stamps_us"]
    ent, ex = st[:, 0], st[:, 15]
    live = ex > 0
    hw = st[:, 12].astype(np.int64)
    xcc = st[:, 13].astype(np.int64) & 0xF
    simd = (hw >> 4) & 3
    cu_key = xcc * 256 + ((hw >> 8) & 0xFF)
    cnt = st[:, 14].astype(np.int64)
    inner = cnt & 0xFFFFFFFF
    left = cnt >> 32
    print(f"window depth {dep}: {len(nodes)} nodes, kernel {d['ms_min'] * 1e3:.2f} us, grid {d['grid']}", flush=True)
    q = np.percentile(ex[live], [10, 50, 90, 100])
    print(f"  exit p10/50/90/max {q.round(1).tolist()} mean {ex[live].mean():.1f}; entry max {ent[live].max():.2f}")
    print(f"  work (inner nodes) p10/50/90/max {np.percentile(inner[live], [10, 50, 90, 100]).astype(int).tolist()} "
          f"left on stack mean {left[live].mean():.0f}")
    keys, inv = np.unique(cu_key[live], return_inverse=True)
    exl, inl, entl, simdl = ex[live], inner[live], ent[live], simd[live]
    ncu = len(keys)
    cu_max = np.zeros(ncu)
    cu_work = np.zeros(ncu)
    cu_n = np.zeros(ncu, int)
    rank = np.zeros(len(exl), int)
    for c in range(ncu):
        idx = np.where(inv == c)[0]
        cu_max[c] = exl[idx].max()
        cu_work[c] = inl[idx].sum()
        cu_n[c] = len(idx)
        order = idx[np.argsort(entl[idx], kind="stable")]
        rank[order] = np.arange(len(idx))
    print(f"  CUs {ncu}, workgroups per CU {np.bincount(cu_n).tolist()} (index = count)")
    print(f"  per-CU max exit p10/50/90/max {np.percentile(cu_max, [10, 50, 90, 100]).round(1).tolist()}; "
          f"per-CU work p10/50/90/max {np.percentile(cu_work, [10, 50, 90, 100]).astype(int).tolist()}")
    print(f"  corr(exit, own work) {corr(exl, inl):.2f}; corr(CU max exit, CU work) {corr(cu_max, cu_work):.2f}; "
          f"corr(exit, rank in CU) {corr(exl, rank):.2f}")
    by_rank = [f"{exl[rank == r].mean():.1f}" for r in range(rank.max() + 1)]
    print(f"  mean exit by dispatch rank in CU: {' '.join(by_rank)}")
    print(f"  wave-0 SIMD histogram {np.bincount(simdl, minlength=4).tolist()}")
    steps_t = []
    prev = st[live, 2]
    for k in (4, 5, 6, 7):
        col = st[live, k]
        ok = col > 0
        if ok.sum() == 0:
            break
        dt = col[ok] - prev[ok]
        steps_t.append(f"step{k - 4} n={ok.sum()} {dt.mean():.1f}/{np.percentile(dt, 90):.1f}/{dt.max():.1f}")
        prev = np.where(ok, col, prev)
    print("  " + " | ".join(steps_t), flush=True)
    if dyn_us:
        cw = st[live, 9].astype(np.int64)
        nstep, ndon, ncl = cw & 0x3FF, (cw >> 10) & 0x3FF, (cw >> 20) & 0x3FF
        idle = st[live, 10] / 100.0  # 100 MHz ticks -> us
        print(f"  dyn: steps p10/50/90/max {np.percentile(nstep, [10, 50, 90, 100]).astype(int).tolist()} "
              f"donations total {int(ndon.sum())} (wgs {int((ndon > 0).sum())}) claims total {int(ncl.sum())} "
              f"idle us mean {idle.mean():.1f} max {idle.max():.1f}; left on stacks {int(left[live].sum())}",
              flush=True)
    if os.environ.get("TTS_PROBE_DUMP"):
        np.save(f"gpurun_out/lb_probe_d{dep}.npy", st)
