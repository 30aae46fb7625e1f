"""Drive the RCCL node-transfer branch of Comm.execute_transfers on ONE GPU.

RCCL refuses two ranks on one GPU, so the multi-rank tests use gloo; this probe runs
the real RCCL path with a one-rank process group and a self-loop plan (rank 0 sends k
nodes to itself): pool -> device staging (export_to on the engine's transfer stream)
-> RCCL batch_isend_irecv (send and receive to/from rank 0, ExternalStream) -> peer
staging -> pool (import_from), then the solve must still find the golden tree.
It also runs the P2P preflight (pattern check) over the same one-rank group.

    python scripts/rccl_selfloop_probe.py
"""
import os
import sys
import time

sys.path.insert(0, ".")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
os.environ["RANK"] = "0"
os.environ["WORLD_SIZE"] = "1"
import torch
import torch.distributed as dist

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel
from dist_gpu_accelerated_tree_search_amd.parallel.comm import Comm

torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
comm = Comm(use_gpu=True)
print("process group:", dist.get_backend(), "world", dist.get_world_size(), flush=True)
try:
    pf = comm.preflight_p2p(1 << 20)
    print("preflight over RCCL (self-loop):", pf, flush=True)
except Exception as e:  # noqa: BLE001
    print("preflight over RCCL (self-loop) raised:", repr(e)[:400], flush=True)

m = PfspModel(14, 1)
eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=4 << 30))
nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 2000)
for k in (1, 500, len(nodes) // 2):
    eng.begin(nodes, int(best))
    before = eng.size()
    t0 = time.perf_counter()
    sent, got = comm.execute_transfers([(0, 0, k)], eng, m.node_bytes)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    after = eng.size()
    eng.run()
    st = eng.stats()
    tree, sol = st["tree"] + tree1, st["sol"] + sol1
    ok = (tree, sol, st["best"]) == (2573652, 2648, 1377)
    print(f"self-loop transfer of {k} nodes over RCCL: sent {sent} received {got} in {dt * 1e3:.2f} ms, "
          f"pool {before} -> {after}; solve after it: tree {tree} sol {sol} best {st['best']} golden {ok}, "
          f"device transfers {comm.device_transfers}", flush=True)
    assert ok and sent == k and got == k and before == after
dist.destroy_process_group()
print("rccl self-loop probe ok", flush=True)
