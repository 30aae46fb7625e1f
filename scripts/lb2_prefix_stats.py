"""How many LB2 walk steps a chunk-shared record list would save (ta056 windows).

Each Johnson walk of the LB2 kernel steps over all 50 records of a machine pair; the
jobs its child's parent has scheduled are no-op steps. Records of jobs scheduled in
EVERY parent of a chunk could be dropped from a per-chunk list that all the chunk's
walks share. For windows dumped by scripts/lb2_pool_dump.py this prints, per chunk
layout (strided as the kernel deals them, or blocked), the mean number of records a
walk needs with such a list (50 - |common scheduled set|) against the 50 it walks now
and the per-parent minimum (50 - depth).

    python scripts/lb2_prefix_stats.py gpurun_out/<dir>/lb2_pool/*.npy
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from dist_gpu_accelerated_tree_search_amd.utils import nodes as nd  # noqa: E402

N, BP = 50, 8
for path in sys.argv[1:]:
    raw = np.load(path)
    depths, perms = nd.pfsp_unpack(raw, N)
    n = len(depths)
    sched = np.zeros((n, N), dtype=bool)
    for i in range(n):
        sched[i, perms[i, :depths[i]]] = True
    nch = (n + BP - 1) // BP
    out = [f"{path.split('/')[-1]}: {n} parents, depth mean {depths.mean():.1f} (min {depths.min()}, max {depths.max()}), "
           f"per-parent unscheduled mean {N - depths.mean():.1f}"]
    for name, groups in (("strided", [np.arange(c, n, nch) for c in range(nch)]),
                         ("blocked", [np.arange(c * BP, min(n, (c + 1) * BP)) for c in range(nch)])):
        common = np.array([sched[g].all(axis=0).sum() for g in groups if len(g)])
        out.append(f"  {name} chunks of {BP}: common scheduled jobs mean {common.mean():.1f} -> "
                   f"{N - common.mean():.1f} records per walk (now {N})")
    out.append(f"  whole window: common scheduled jobs {sched.all(axis=0).sum()}")
    print("\n".join(out), flush=True)
