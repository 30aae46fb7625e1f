"""N-Queens N=17 on one GPU with 1-3 engines (own stream each): plain sharing between
slices, or the solve split in the graph between the engines (stream_split).

    python scripts/queens_streams_probe.py [N]
"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401

from dist_gpu_accelerated_tree_search_amd import EngineOptions, QueensModel
from dist_gpu_accelerated_tree_search_amd.search import solve_engine

N = int(sys.argv[1]) if len(sys.argv) > 1 else 17
GOLD = {17: (8017021931, 95815104), 16: (1141190302, 14772512)}.get(N)
m = QueensModel(N, 1)
for streams, split in ((1, 0), (2, 0), (2, 512), (3, 512), (4, 512)):
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 20, ring_bytes=8 << 30, streams=streams,
                                                 stream_split=split))
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        r = solve_engine(m, eng)
        ts.append(time.perf_counter() - t0)
        assert GOLD is None or (r.tree, r.sol) == GOLD, (streams, split, r.tree, r.sol)
    print(f"N={N} streams {streams} split {split}: best {min(ts) * 1e3:.1f} ms, median {sorted(ts)[2] * 1e3:.1f} ms "
          f"-> {r.tree / min(ts) / 1e9:.1f} G nodes/s", flush=True)
    del eng
