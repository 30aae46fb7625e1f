"""ta014 LB1 solve time vs replay schedule (first-graph length, parent window,
polled vs event completion). Env TTS_POLL is read at engine construction."""
import os
import sys
sys.path.insert(0, ".")
import torch  # noqa
from dist_gpu_accelerated_tree_search_amd import PfspModel, EngineOptions, solve_engine

m = PfspModel(14, 1)
for poll in ("1", "0"):
    os.environ["TTS_POLL"] = poll
    for first in (0, 12, 24):
        for mp in (1 << 18, 1 << 19):
            eng = m.make_engine("gpu", 0, EngineOptions(max_parents=mp, ring_bytes=8 << 30, iters_first=first))
            ts = []
            for i in range(60):
                r = solve_engine(m, eng)
                assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377)
                ts.append(r.elapsed)
            ts.sort()
            print(f"poll={poll} iters_first={first:2d} mp={mp:7d}: median {ts[len(ts)//2]*1e3:.3f} ms "
                  f"min {ts[0]*1e3:.3f} ms iters={r.extra['iters']} launches={r.extra['launches']}", flush=True)
            del eng
