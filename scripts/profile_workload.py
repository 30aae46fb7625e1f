"""Fixed workloads for rocprofv3 runs (kernel trace / PMC counters)."""
import sys
sys.path.insert(0, ".")
import torch  # noqa: F401
import os
if os.environ.get("TTS_DUMP_MAPS"):  # the process mappings at exit (resolve a crash PC from a finalizer)
    import atexit
    atexit.register(lambda: open(os.environ["TTS_DUMP_MAPS"], "w").write(open("/proc/self/maps").read()))
from dist_gpu_accelerated_tree_search_amd import EngineOptions, PfspModel, QueensModel, solve_engine

which = sys.argv[1] if len(sys.argv) > 1 else "ta014"
if which == "ta014":
    m = PfspModel(14, 1); eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
    for _ in range(20):
        r = solve_engine(m, eng)
elif which == "ta014_w8":  # rank 0 of an 8-rank split solve (the per-GPU critical path at N=8)
    m = PfspModel(14, 1); eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 19, ring_bytes=32 << 30))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    for _ in range(20):
        eng.set_split(0, 8, 4096)
        eng.begin(nodes, int(best))
        eng.run()
    st = eng.stats()
    print(which, st["tree"], st["iters"])
    raise SystemExit(0)
elif which == "ta008":
    m = PfspModel(8, 0); eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=32 << 30))
    r = solve_engine(m, eng)
elif which == "lb2":
    m = PfspModel(20, 2); eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=32 << 30))
    r = solve_engine(m, eng)
elif which == "ta056":  # LB2 50x20, time-boxed (the full tree takes far longer)
    m = PfspModel(56, 2); eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=32 << 30))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    eng.begin(nodes, int(best))
    eng.run(max_seconds=1.5)
    st = eng.stats()
    print(which, st["tree"], st["iters"], "pool", eng.size())
    raise SystemExit(0)
elif which == "ta081":  # LB2 100x20 (two-word job sets), time-boxed
    m = PfspModel(81, 2); eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=32 << 30))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    eng.begin(nodes, int(best))
    eng.run(max_seconds=1.5)
    st = eng.stats()
    print(which, st["tree"], st["iters"], "pool", eng.size())
    raise SystemExit(0)
elif which == "ta021":  # LB1_d 20x20 (BASELINE 8-GPU config), time-boxed
    m = PfspModel(21, 0); eng = m.make_engine("gpu", 0, EngineOptions(ring_bytes=32 << 30))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    eng.begin(nodes, int(best))
    eng.run(max_seconds=2.0)
    st = eng.stats()
    print(which, st["tree"], st["iters"], "pool", eng.size())
    raise SystemExit(0)
elif which == "spill":  # pinned spill/refill: a ring smaller than the pool (copies overlapping replays)
    m = PfspModel(14, 1); eng = m.make_engine("gpu", 0, EngineOptions(max_parents=256, ring_bytes=1 << 20))
    for _ in range(2):
        r = solve_engine(m, eng, m=200_000)
    st = eng.stats()
    assert (r.tree, r.sol, r.best) == (2573652, 2648, 1377), (r.tree, r.sol, r.best)
    print(which, "ta014 spilled", st["spilled"], "refilled", st["refilled"], "pinned MB", st["pinned_bytes"] >> 20,
          "capacity", st["capacity"], f"{r.elapsed * 1e3:.1f} ms")
elif which.startswith("spill021"):  # spill021[:ring_MB[:seconds]]: ta021 LB1_d, 2^14-parent window, small ring
    parts = which.split(":")
    ring_mb = int(parts[1]) if len(parts) > 1 else 256
    box = float(parts[2]) if len(parts) > 2 else 3.0
    import time
    m = PfspModel(21, 0)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 14, ring_bytes=ring_mb << 20))
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 25)
    eng.begin(nodes, int(best))
    t0 = time.perf_counter()
    eng.run(max_seconds=box)
    dt = time.perf_counter() - t0
    st = eng.stats()
    print(which, f"ring {ring_mb} MB capacity {st['capacity']} nodes: {st['tree'] / dt / 1e9:.3f} G nodes/s over "
          f"{dt:.2f} s, spilled {st['spilled']} refilled {st['refilled']} pinned MB {st['pinned_bytes'] >> 20} "
          f"pool device {st['device_nodes']} host {st['host_nodes']}")
    raise SystemExit(0)
elif which.startswith("spillbig"):  # spillbig[:seconds]: ta021 LB1_d begun from a 2M-node host frontier on a
    # 1024-parent window and the smallest ring it allows (~10 MB): the frontier spills to pinned host
    # blocks at begin() and comes back through refills while graph replays run
    import time
    parts = which.split(":")
    box = float(parts[1]) if len(parts) > 1 else 3.0
    ring = int(parts[2]) << 20 if len(parts) > 2 else 1 << 20
    m = PfspModel(21, 0)
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 2_000_000)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 10, ring_bytes=ring))
    t0 = time.perf_counter()
    eng.begin(nodes, int(best))
    eng.run(max_seconds=box)
    dt = time.perf_counter() - t0
    st = eng.stats()
    print(which, f"{len(nodes)} begin nodes, capacity {st['capacity']} nodes: {st['tree'] / dt / 1e9:.3f} G nodes/s "
          f"over {dt:.2f} s, spilled {st['spilled']} refilled {st['refilled']} pinned MB {st['pinned_bytes'] >> 20} "
          f"pool device {st['device_nodes']} host {st['host_nodes']}")
    del eng
    raise SystemExit(0)
elif which.startswith("spill014"):  # spill014[:ring_MB]: ta014 LB1 solved to the end from a 400K-node host
    # frontier on a 1024-parent window: with the smallest ring (1 MB -> its floor) most of the frontier
    # waits in pinned host blocks and comes back through refills while replays run; golden tree checked
    import time
    parts = which.split(":")
    ring = int(parts[1]) << 20 if len(parts) > 1 else 1 << 20
    m = PfspModel(14, 1)
    nodes, tree1, sol1, best = m.warmup(m.initial_best(1), 400_000)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 10, ring_bytes=ring))
    ts = []
    for rep in range(4):
        # the last solve records the replay / copy timeline (TTS_EXIT_MODE=notrace: none)
        eng.set_trace(rep == 3 and os.environ.get("TTS_EXIT_MODE") != "notrace")
        t0 = time.perf_counter()
        eng.begin(nodes, int(best))
        eng.run()
        eng.synchronize()
        ts.append(time.perf_counter() - t0)
        st = eng.stats()
        assert (st["tree"] + tree1, st["sol"] + sol1) == (2573652, 2648), (st["tree"] + tree1, st["sol"] + sol1)
    print(which, f"{len(nodes)} begin nodes, capacity {st['capacity']} nodes: {min(ts[:3]) * 1e3:.2f} ms per solve "
          f"(best of 3 untraced), spilled {st['spilled']} refilled {st['refilled']} (last solve), "
          f"pinned MB {st['pinned_bytes'] >> 20}")
    if os.environ.get("TTS_EXIT_MODE") == "notrace":
        del eng
        raise SystemExit(0)
    tr = eng.trace()
    import numpy as np
    g = tr[tr[:, 0] == 0][:, 1:]
    for kind, name in ((1, "spill D2H"), (2, "refill H2D")):
        c = tr[tr[:, 0] == kind][:, 1:]
        tot = float((c[:, 1] - c[:, 0]).sum()) if len(c) else 0.0
        ov = 0.0
        for a, b in c:  # overlap with the union of replay intervals (replays are serial on one stream)
            ov += float(np.clip(np.minimum(g[:, 1], b) - np.maximum(g[:, 0], a), 0, None).sum())
        print(f"  {name}: {len(c)} copies (enqueue-to-complete spans), {tot:.3f} ms, {ov:.3f} ms "
              f"({100 * ov / tot if tot else 0:.0f} %) while a graph replay ran")
    print(f"  replays: {len(g)}, {float((g[:, 1] - g[:, 0]).sum()):.3f} ms; traced solve {ts[3] * 1e3:.2f} ms")
    # exit-crash diagnosis under rocprofv3 --memory-copy-trace (profiles/r4/spill/README.md):
    # TTS_EXIT_MODE=sleep waits before the engine is released, =keep never releases it
    mode = os.environ.get("TTS_EXIT_MODE", "")
    if mode == "sleep":
        time.sleep(1.0)
    if mode == "keep":
        import builtins
        builtins._tts_keep = eng
        raise SystemExit(0)
    del eng
    raise SystemExit(0)
elif which == "queens17":  # the bench's N-Queens extra: N=17, two split engines on the GPU
    m = QueensModel(17)
    eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 20, ring_bytes=8 << 30, streams=2, stream_split=512))
    for _ in range(2):
        r = solve_engine(m, eng)
elif which == "queens":
    m = QueensModel(16); eng = m.make_engine("gpu", 0, EngineOptions(max_parents=1 << 20, ring_bytes=32 << 30))
    r = solve_engine(m, eng)
print(which, r.tree, r.sol, r.best, f"{r.elapsed*1e3:.2f} ms")
