"""LB2 throughput of one instance in a time box on one GPU (several engines optional).

    python scripts/lb2_box_probe.py INST [seconds] [streams]
"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel

inst = int(sys.argv[1])
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
streams = int(sys.argv[3]) if len(sys.argv) > 3 else 1
m = PfspModel(inst, 2)
eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=16 << 30, streams=streams))
nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
eng.begin(nodes, int(best))
eng.run(max_seconds=0.5)
st0 = eng.stats()
t0 = time.perf_counter()
eng.run(max_seconds=secs)
dt = time.perf_counter() - t0
st = eng.stats()
print(f"ta{inst:03d} ({m.jobs}x{m.machines}) LB2, {streams} engine(s): {(st['tree'] - st0['tree']) / dt / 1e9:.4f} "
      f"G nodes/s over {dt:.1f} s (best {st['best']}, pool {eng.size()})", flush=True)
