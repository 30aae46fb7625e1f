"""Median solve time of the 20-job Taillard instances (ta001-ta030, LB1, -u 1) on one GPU:
how the first graph replay's length (TTS_ITERS_FIRST) fits trees of different depths."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, solve_engine

insts = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else range(1, 21))]
tot = 0.0
for i in insts:
    m = PfspModel(i, 1)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
    r = solve_engine(m, eng)
    if r.elapsed > 0.5:
        continue  # big trees: the first replay does not matter
    ts = []
    for _ in range(7):
        r = solve_engine(m, eng)
        ts.append(r.elapsed)
    st = eng.stats()
    t = sorted(ts)[3]
    tot += t
    print(f"ta{i:03d} lb1 tree={r.tree} iters={st['iters']} launches={st['launches']} median {t*1e3:.3f} ms", flush=True)
    del eng
print(f"sum of medians {tot*1e3:.3f} ms", flush=True)
