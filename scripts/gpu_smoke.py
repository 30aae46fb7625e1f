"""First-contact GPU check: kernel bounds vs CPU oracle, golden trees, timings."""
import sys, time
import numpy as np
sys.path.insert(0, ".")
from dist_gpu_accelerated_tree_search_amd import _tts_cpu as C
from dist_gpu_accelerated_tree_search_amd import _tts_hip as H

print("devices", H.device_count(), H.device_info(0), flush=True)
rng = np.random.default_rng(0)

def rand_nodes(inst, n):
    N = inst.jobs; nb = C.pfsp_node_bytes(N)
    arr = np.zeros((n, nb), np.uint8)
    perms = []
    for i in range(n):
        d = int(rng.integers(0, N))
        p = rng.permutation(N)
        arr[i, 0] = d; arr[i, 1:1 + N] = p
        perms.append((d, p))
    return arr, perms

for tid in (14, 21, 3):
    inst = C.PfspInstance.taillard(tid)
    arr, perms = rand_nodes(inst, 3000)
    for lb in (1, 2):
        for best in (2**31 - 1, inst.best_known):
            g = H.pfsp_bounds(inst.jobs, inst.machines, list(inst.p), lb, arr, best, 0)
            ref = []
            for d, p in perms:
                for k in range(d, inst.jobs):
                    q = p.copy(); q[d], q[k] = q[k], q[d]
                    ref.append(C.lb1(inst, list(q), d + 1) if lb == 1 else C.lb2(inst, list(q), d + 1, best))
            ref = np.array(ref)
            print(f"ta{tid:03d} lb{lb} best={best}: n={len(ref)} mismatches={(g != ref).sum()}", flush=True)

for lb in (1, 0, 2):
    inst = C.PfspInstance.taillard(14)
    eng = H.make_pfsp_engine(inst.jobs, inst.machines, list(inst.p), lb, 0, max_parents=1 << 18, ring_bytes=4 << 30)
    for rep in range(3):
        t0 = time.perf_counter()
        nodes, t1, s1, b = C.pfsp_bfs(inst, lb, inst.best_known, 25)
        eng.reset_counters(); eng.best = b; eng.push(nodes)
        launches = eng.run()
        st = eng.stats()
        dt = time.perf_counter() - t0
        print(f"ta014 lb{lb} rep{rep}: tree={t1 + st['tree']} sol={s1 + st['sol']} best={st['best']} "
              f"t={dt*1e3:.2f} ms launches={launches} iters={st['iters']} syncs={st['syncs']} "
              f"Mnodes/s={(t1 + st['tree'])/dt/1e6:.1f}", flush=True)
    del eng

for N in (10, 12, 14):
    eng = H.make_queens_engine(N, 1, 0, max_parents=1 << 20, ring_bytes=4 << 30)
    t0 = time.perf_counter()
    nodes, t1, s1 = C.queens_bfs(N, 1, 25)
    eng.reset_counters(); eng.push(nodes); eng.run()
    st = eng.stats(); dt = time.perf_counter() - t0
    print(f"queens N={N}: tree={t1 + st['tree']} sol={s1 + st['sol']} t={dt*1e3:.2f} ms iters={st['iters']}", flush=True)
