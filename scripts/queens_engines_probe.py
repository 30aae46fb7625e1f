"""N-Queens N=17 (g=1) on one GPU: engines per GPU x in-graph split point, best of 3 solves
each (engine built outside the timed solves), checked against the golden counts.

    python scripts/queens_engines_probe.py [N]
"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd import EngineOptions, QueensModel  # noqa: E402
from dist_gpu_accelerated_tree_search_amd.search import solve_engine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 17
GOLD = {17: (8017021931, 95815104), 16: (1141190302, 14772512)}
m = QueensModel(N, 1)
CONFIGS = ((2, 512, 1 << 19), (3, 512, 1 << 19), (4, 512, 1 << 19), (4, 512, 1 << 18), (8, 512, 1 << 17))
if len(sys.argv) > 2:
    CONFIGS = tuple(tuple(int(x) for x in c.split(":")) for c in sys.argv[2].split(","))
for streams, split, mp in CONFIGS:
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=mp, ring_bytes=8 << 30, streams=streams,
                                                stream_split=split))
    solve_engine(m, eng)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = solve_engine(m, eng)
        ts.append(time.perf_counter() - t0)
        assert (r.tree, r.sol) == GOLD[N], (r.tree, r.sol)
    print(f"N={N} engines {streams} split {split} window {mp}: best {min(ts) * 1e3:.2f} ms "
          f"({r.tree / min(ts) / 1e9:.1f} G nodes/s)", flush=True)
    del eng
