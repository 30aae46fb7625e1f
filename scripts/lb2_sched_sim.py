"""Work model of the LB2 expand kernel's B2 phase on real ta056 windows.

    python scripts/lb2_sched_sim.py [dump_dir]

Input: windows dumped by scripts/lb2_pool_dump.py (GPU run). For each child the host
oracle (`lb2_child_profile`) gives LB1, the number of machine pairs in the learned order
until the partial LB2 reaches best (P if it never does) and the full LB2. The walks a
child needs are its `until` first pairs (children with LB1 >= best need none: B1 filter).

Two schedulers of a chunk (8 parents, one 256-lane workgroup) are replayed:
  rounds  the production B2: rounds of 8, 16, 32, ... pairs; a round's (pair, child)
          tasks are dealt to the 256 lanes, pair-major; children decided in a round
          leave the task list at the next round (barriers between rounds)
  wave    persistent waves: each wave keeps up to 64 live children, pulled from the
          chunk's active list, and deals its 64 lanes over them every batch (child i
          gets floor/ceil(64/n) consecutive pairs of its own order); decided children
          leave after each batch and are replaced from the chunk list
Reported per scheduler: lane slots (64 x wave-steps, each one Johnson walk), useful
walks, lane utilisation, and the chunk critical path in walk steps (max over waves).
"""
import glob
import os
import sys

sys.path.insert(0, ".")
import numpy as np
from dist_gpu_accelerated_tree_search_amd import PfspModel
from dist_gpu_accelerated_tree_search_amd.ops import cpu

BLOCK, WAVE, BP = 256, 64, 8


def rounds_chunk(need, P):
    """need: pairs each active child needs (<= P). Returns (slots, walks, path)."""
    alive = list(range(len(need)))
    q0, R, slots, walks, path = 0, 8, 0, 0, 0
    while q0 < P and alive:
        nq = min(P - q0, R)
        na = len(alive)
        ntask = nq * na
        # wave w holds lanes 64w..64w+63; lane tid runs tasks tid, tid+256, ...
        iters = [max(0, -(-(ntask - WAVE * w) // BLOCK)) if ntask > WAVE * w else 0 for w in range(BLOCK // WAVE)]
        slots += sum(iters) * WAVE
        path += max(iters)
        for q in range(q0, q0 + nq):
            for c in alive:
                if q < need[c]:
                    walks += 1
        q0 += nq
        R *= 2
        alive = [c for c in alive if need[c] > q0]
    return slots, walks, path


def wave_chunk(need, P, nwaves=BLOCK // WAVE):
    queue = list(range(len(need)))
    qi = 0
    live = [[] for _ in range(nwaves)]  # per wave: [child, next pair]
    steps = [0] * nwaves
    slots = walks = 0
    while True:
        progressed = False
        for w in range(nwaves):
            L = live[w]
            while len(L) < WAVE and qi < len(queue):
                L.append([queue[qi], 0])
                qi += 1
            if not L:
                continue
            progressed = True
            n = len(L)
            base, extra = divmod(WAVE, n)
            for i, e in enumerate(L):
                k = base + (1 if i < extra else 0)
                c, q = e
                take = min(k, P - q)
                walks += min(take, max(0, need[c] - q))
                e[1] = q + take
            slots += WAVE
            steps[w] += 1
            live[w] = [e for e in L if e[1] < need[e[0]]]
        if not progressed:
            break
    return slots, walks, max(steps) if steps else 0


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lb2_pool"
    files = sorted(glob.glob(os.path.join(d, "*.npy")))
    m = PfspModel(56, 2)
    best = m.initial_best(1)
    P = m.native.npairs
    C = cpu()
    for f in files:
        nodes = np.load(f)
        nodes = nodes[: (len(nodes) // BP) * BP][:4096]
        prof = C.lb2_child_profile(m.native, nodes, best)
        depth = nodes[:, 0].astype(int) if nodes.dtype == np.uint8 else None
        # children per parent: N - depth (same order as the oracle's loops)
        N = m.jobs
        counts = [N - int(x) for x in depth]
        tot = {"rounds": [0, 0, 0], "wave": [0, 0, 0]}
        pos = 0
        nact_all = []
        for ch in range(0, len(nodes), BP):
            need = []
            for p in range(ch, ch + BP):
                for k in range(counts[p]):
                    lb1, until, lb = prof[pos]
                    pos += 1
                    if counts[p] == 1:  # leaf children: decided in B1
                        continue
                    if lb1 < best:
                        need.append(int(until))
            nact_all.append(len(need))
            for name, fn in (("rounds", rounds_chunk), ("wave", wave_chunk)):
                s, wk, pth = fn(need, P)
                t = tot[name]
                t[0] += s
                t[1] += wk
                t[2] += pth
        nch = len(nact_all)
        print(f"{os.path.basename(f)}: {len(nodes)} parents, mean depth {np.mean(depth):.1f}, "
              f"active children per chunk {np.mean(nact_all):.1f} (max {max(nact_all)})")
        for name, (s, wk, pth) in tot.items():
            print(f"  {name:6s}: lane slots {s / nch:9.1f}/chunk  useful walks {wk / nch:8.1f}/chunk  "
                  f"utilisation {wk / max(s, 1):.3f}  critical path {pth / nch:6.1f} walks/chunk")


if __name__ == "__main__":
    main()
