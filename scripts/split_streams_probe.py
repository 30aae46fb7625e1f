"""ta014 LB1 split between K engines on ONE GPU (own stream + host thread each).

Each engine begins from the same host warm-up with an in-graph rank split
(set_split(k, K, 512 K): identical replicated iterations, then a disjoint 1/K share)
and the K solves run concurrently; per solve: wall time from the first begin to the
last engine's end, tree summed and checked against the golden value. Question: do
concurrent streams hide each other's per-kernel fixed cost on a latency-bound tree?

    python scripts/split_streams_probe.py [K ...]
"""
import statistics
import sys
import threading
import time

sys.path.insert(0, ".")
import torch  # noqa: F401

from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel

GOLD = (2573652, 2648)
m = PfspModel(14, 1)
nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
for K in [int(x) for x in sys.argv[1:]] or [1, 2, 3]:
    engs = [m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=4 << 30)) for _ in range(K)]
    go = [threading.Event() for _ in range(K)]
    done = [threading.Event() for _ in range(K)]
    stop = False

    def worker(k):
        while True:
            go[k].wait()
            go[k].clear()
            if stop:
                return
            engs[k].run()
            done[k].set()

    th = [threading.Thread(target=worker, args=(k,), daemon=True) for k in range(1, K)]
    for t in th:
        t.start()
    ts = []
    for rep in range(80):
        t0 = time.perf_counter()
        for k, e in enumerate(engs):
            if K > 1:
                e.set_split(k, K, 512 * K)
            e.begin(nodes, int(best))
        for k in range(1, K):
            go[k].set()
        engs[0].run()
        for k in range(1, K):
            done[k].wait()
            done[k].clear()
        dt = time.perf_counter() - t0
        tree = sum(e.stats()["tree"] for e in engs) + tree1
        sol = sum(e.stats()["sol"] for e in engs) + sol1
        assert (tree, sol) == GOLD, (K, tree, sol)
        if rep >= 10:
            ts.append(dt)
    stop = True
    for k in range(1, K):
        go[k].set()
    print(f"K={K} engines on one GPU: median {statistics.median(ts) * 1e3:.4f} ms, min {min(ts) * 1e3:.4f} ms "
          f"per ta014 solve", flush=True)
    del engs
