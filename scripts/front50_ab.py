"""50-job LB1_d node rate, front-carrying nodes vs permutation nodes (TTS_FRONT=0):

    python scripts/front50_ab.py [seconds] [inst,...]

Each instance runs -u 1 from a host warm-up for a time box (or to the end of its tree)
on one engine; prints nodes, seconds, G nodes/s and whether the tree finished."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401,E402

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel  # noqa: E402

box = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
insts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [31, 41, 51]
for inst in insts:
    m = PfspModel(inst, 0)
    eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=16 << 30))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    t0 = time.perf_counter()
    eng.begin(nodes, int(best))
    eng.run(max_seconds=box)
    eng.synchronize()
    dt = time.perf_counter() - t0
    st = eng.stats()
    done = eng.size() == 0
    print(f"ta{inst:03d} LB1_d layout {m.describe()['layout']}: {st['tree']} nodes in {dt:.3f} s, "
          f"{st['tree'] / dt / 1e9:.4f} G nodes/s, {'tree done' if done else 'time box'}", flush=True)
    del eng
