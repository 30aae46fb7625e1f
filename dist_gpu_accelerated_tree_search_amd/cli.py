"""Command line (parity with the reference executables' flags, defaults and output).

    python -m dist_gpu_accelerated_tree_search_amd pfsp  [-i 14 -l 1 -u 1 -m 25 -M 50000 -T 5000 -D 1 -C 1 -w 1 -L 1 -p 50]
    python -m dist_gpu_accelerated_tree_search_amd nqueens [-N 14 -g 1 -m 25 -M 50000 -D 1]

pfsp:  -D 0            CPU only: -C threads (0/1 = sequential, ref pfsp_c / pfsp_omp_c)
       -D 1            one GPU (ref pfsp_multigpu_cuda.out -D 1)
       -D N            N GPUs. Routing:
                         -C 1 (the default, ref -C 1), no torchrun: ONE process drives
                           every GPU plus a CPU worker (native runner, one host thread
                           per GPU, xGMI peer steals: ref pfsp_multigpu_cuda), as does
                           --single-process;
                         -C 0, no torchrun: one process per GPU, spawned here
                           (RCCL between them: ref pfsp_dist_multigpu_cuda layout);
                         under torchrun: one process per GPU, with -C 1 each rank also
                           runs a CPU worker thread (hybrid rank engine, ref -C 1 of
                           the distributed driver).
                       -w / -L enable work sharing inside a node / across nodes.
       --streams K     K engines per GPU, run concurrently (large trees).
nqueens: -D 0 CPU sequential (ref nqueens_c), -D >= 1 GPU(s).
Results: the reference's stdout blocks, plus a CSV row (singlegpu.csv,
multigpu.csv or dist_multigpu.csv) and optionally a JSON record (--json).
-M is the reference's per-offload batch cap; the device engine's per-iteration
parent window is --max-parents (default 262144, sized for 288 GB HBM).
"""
from __future__ import annotations

import argparse
import os
import sys

from .utils import report

INT_MAX = 2**31 - 1


def _pfsp_parser(cls=argparse.ArgumentParser) -> argparse.ArgumentParser:
    ap = cls(prog="pfsp", description="PFSP Branch-and-Bound (Taillard instances)")
    ap.add_argument("-i", "--inst", type=int, default=14)
    ap.add_argument("-l", "--lb", type=int, default=1)
    ap.add_argument("-u", "--ub", type=int, default=1)
    ap.add_argument("-m", "--m", type=int, default=25)
    ap.add_argument("-M", "--M", type=int, default=50000)
    ap.add_argument("-T", "--T", type=int, default=5000)
    ap.add_argument("-D", "--D", type=int, default=1)
    ap.add_argument("-C", "--C", type=int, default=1)  # ref PFSP_lib.c:182 (*C = 1)
    ap.add_argument("-w", "--ws", type=int, default=1)
    ap.add_argument("-L", "--L", type=int, default=1)
    ap.add_argument("-p", "--perc", type=int, default=50)
    ap.add_argument("--max-parents", type=int, default=1 << 18)
    ap.add_argument("--single-process", action="store_true",
                    help="all GPUs driven by one process (native runner) instead of one process per GPU")
    ap.add_argument("--gpus-list", default=None, help="comma-separated device ids (single-process mode)")
    ap.add_argument("--steal-cap", type=int, default=None, help="max nodes per transfer (default 5*M)")
    ap.add_argument("--comm-period", type=float, default=0.5,
                    help="minimum local search between coordination rounds, ms (adaptive up to 50 ms)")
    ap.add_argument("--pin", type=int, default=1, help="pin GPU host threads to the GPU's NUMA node")
    ap.add_argument("--ring-gb", type=float, default=16.0)
    ap.add_argument("--streams", type=int, default=1,
                    help="engines per GPU, one stream and host thread each, run as one (large trees: 3)")
    ap.add_argument("--comm", choices=["nccl", "gloo"], default="nccl",
                    help="one process per GPU: node transfers over RCCL (default) or gloo (ranks may share a GPU)")
    ap.add_argument("--device", type=int, default=None,
                    help="one process per GPU: put every rank on this device (tests; use with --comm gloo)")
    ap.add_argument("--heuristic-ub", action="store_true",
                    help="-u 0: start from a heuristic incumbent (LB1 beam dive + NEH) instead of +inf; the "
                         "explored tree is then not the reference's -u 0 quantity (recorded as initial_ub)")
    ap.add_argument("--json", default=None, help="append a JSON run record to this file")
    ap.add_argument("--csv-dir", default=".", help="directory of the CSV statistics files")
    ap.add_argument("--no-csv", action="store_true")
    return ap


def _validate_pfsp(a) -> None:
    def fail(msg):
        sys.stderr.write(msg + "\n")
        raise SystemExit(1)

    if not 1 <= a.inst <= 120:
        fail("Error: unsupported Taillard's instance")
    if a.lb not in (0, 1, 2):
        fail("Error: unsupported lower bound function")
    if a.ub not in (0, 1):
        fail("Error: unsupported upper bound initialization")
    if a.m < 1:
        fail("Error: unsupported minimal pool for GPU initialization")
    if a.M < a.m:
        fail("Error: unsupported maximal pool for GPU initialization")
    if a.T < a.m:
        fail("Error: unsupported maximal pool for CPU multi-core")
    if a.D < 0:
        fail("Error: unsupported number of GPU(s)")
    if a.C < 0:
        fail("Error: unsupported number of CPU Core(s)")
    if a.D >= 1 and a.C > 1:
        fail("C is set to %d. Invalid option for this version.\nChoose 0 to unable and 1 to enable multi-core. "
             "Mapping automatically done." % a.C)
    if a.ws not in (0, 1):
        fail("Error: unsupported Intra-node Work Stealing option")
    if a.L not in (0, 1):
        fail("Error: unsupported distributed dynamic load balancing option")
    if not 0 < a.perc <= 100:
        fail("Error: unsupported WS percentage for popFrontBulkFree")
    if a.device is not None and a.comm != "gloo":
        # RCCL builds one communicator per rank on that rank's own GPU (LOCAL_RANK) and
        # refuses two ranks on one device: ranks pinned to one GPU need the gloo transport
        fail("Error: --device puts every rank on one GPU; use it with --comm gloo")


def _steal_cap(a) -> int:
    return a.steal_cap if a.steal_cap else 5 * a.M


def _rank_spec(a, world: int = 1) -> dict:
    # -C 1 under torchrun: a CPU worker thread per rank (ref NB_THREADS_GPU - 1 threads).
    # The host's cores are shared by the ranks of THIS node (LOCAL_WORLD_SIZE), not by
    # the whole job: on several nodes the global WORLD_SIZE would under-provision them.
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    cpu = max(1, _cpu_worker_threads(local, a.streams) // max(1, local)) if a.C == 1 else 0
    return {"problem": "pfsp", "inst": a.inst, "lb": a.lb, "ub": a.ub, "backend": "gpu",
            "engine": {"max_parents": a.max_parents, "ring_bytes": int(a.ring_gb * (1 << 30)),
                       "streams": max(1, a.streams)},
            "dist": {"m": a.m, "init_per_rank": a.m, "steal_cap": _steal_cap(a), "ws": bool(a.ws), "L": bool(a.L),
                     "slice_min_s": a.comm_period * 1e-3, "cpu_workers": max(0, cpu), "cpu_batch": a.T},
            "pin": bool(a.pin), "comm": a.comm, **({} if a.device is None else {"device": a.device})}


def _cpu_worker_threads(n_gpus: int, engines_per_gpu: int = 1) -> int:
    """ref pfsp_multigpu_cuda.c:61-69: nprocs/deviceCount threads per GPU, one of which
    drives the GPU; here the CPU threads of all GPUs form one multithreaded worker.
    Every engine has a host thread of its own (--streams engines per GPU), so the CPU
    worker gets the cores left after those: no oversubscribed host."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, n - n_gpus * max(1, engines_per_gpu))


def _pfsp_single_process(a, model) -> int:
    from .models.pfsp import EngineOptions
    from .ops import gpu_count
    from .search import solve_workers

    devices = [int(x) for x in a.gpus_list.split(",")] if a.gpus_list else list(range(a.D))
    if len(devices) != a.D and a.gpus_list:
        a.D = len(devices)
    if devices and max(devices) >= gpu_count():
        print("Execution Terminated. More GPU devices requested than the ones available")
        return 1
    threads = _cpu_worker_threads(len(devices), a.streams) if a.C == 1 else 0
    print(report.pfsp_settings(a.inst, model.machines, model.jobs, a.ub, a.lb, a.D, a.C, a.ws, 1, a.L, 2,
                               _init_ub(a, model)))
    opts = EngineOptions(max_parents=a.max_parents, ring_bytes=int(a.ring_gb * 2**30), cpu_batch=a.T,
                         cpu_threads=max(1, threads), streams=max(1, a.streams))
    r = solve_workers(model, devices=tuple(devices), cpu_threads=threads, ub=a.ub, m=a.m, steal_cap=_steal_cap(a),
                      ws=bool(a.ws), opts=opts, slice_min=a.comm_period * 1e-3, pin=bool(a.pin))
    print(report.phase("Initial search on CPU completed", 0, 0, r.t_init))
    print(report.phase("Search on Parallel GPU completed", r.tree, r.sol, r.t_search))
    print("\nExploration terminated.")
    print(report.pfsp_results(r.best, r.tree, r.sol, r.elapsed))
    if not a.no_csv:
        report.write_multi_gpu_csv(os.path.join(a.csv_dir, "multigpu.csv"), a.inst, a.lb, len(devices),
                                   1 if threads else 0, a.ws, r.best, a.m, a.M, a.T, r.elapsed, r.tree, r.sol,
                                   r.workers)
    _json(a, model, r, len(devices))
    return 0


def pfsp_main(argv: list[str]) -> int:
    a = _pfsp_parser().parse_args(argv)
    _validate_pfsp(a)
    if a.heuristic_ub:
        os.environ.setdefault("TTS_DIVE", "32")  # models.pfsp.PfspModel.search_best
    from .models.pfsp import EngineOptions, PfspModel
    from .search import solve_cpu, solve_engine

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    model = PfspModel(a.inst, a.lb)
    if a.D == 0:
        version = 0 if a.C <= 1 else 2
        print(report.pfsp_settings(a.inst, model.machines, model.jobs, a.ub, a.lb, 0, a.C, a.ws, 1, a.L, version))
        r = solve_cpu(model, ub=a.ub, threads=a.C if a.C > 1 else 0, m=a.m, batch=20000, steal_cap=5 * a.M,
                      ws=bool(a.ws), verbose=a.C > 1)
        if a.C <= 1:
            print("\nExploration terminated.")
        print(report.pfsp_results(r.best, r.tree, r.sol, r.elapsed))
        if not a.no_csv and a.C > 1:
            report.write_multi_gpu_csv(os.path.join(a.csv_dir, "multigpu.csv"), a.inst, a.lb, 0, a.C, a.ws, r.best,
                                       a.m, a.M, a.T, r.elapsed, r.tree, r.sol, r.workers)
        _json(a, model, r, 0)
        return 0

    if world_env == 1 and (a.C == 1 or a.single_process or a.gpus_list):
        return _pfsp_single_process(a, model)

    if a.D == 1 and world_env == 1:
        print(report.pfsp_settings(a.inst, model.machines, model.jobs, a.ub, a.lb, 1, a.C, a.ws, 1, a.L, 2,
                                   _init_ub(a, model)))
        eng = model.make_engine("gpu", 0, EngineOptions(max_parents=a.max_parents, ring_bytes=int(a.ring_gb * 2**30),
                                                        streams=max(1, a.streams)))
        r = solve_engine(model, eng, ub=a.ub, m=a.m, verbose=True)
        print(report.pfsp_results(r.best, r.tree, r.sol, r.elapsed))
        if not a.no_csv:
            w = r.workers[0]
            report.write_single_gpu_csv(os.path.join(a.csv_dir, "singlegpu.csv"), a.inst, a.lb, r.best, a.m, a.M,
                                        r.elapsed, w.t_memcpy, w.t_malloc, w.t_kernel, w.t_gen_child, r.tree, r.sol)
            report.write_multi_gpu_csv(os.path.join(a.csv_dir, "multigpu.csv"), a.inst, a.lb, 1, 0, a.ws, r.best,
                                       a.m, a.M, a.T, r.elapsed, r.tree, r.sol, r.workers)
        _json(a, model, r, 1)
        return 0

    # ---- several GPUs: one process per GPU ----
    from .parallel.workers import solve_rank

    spec = _rank_spec(a, world_env if world_env > 1 else a.D)
    if a.heuristic_ub:
        spec["heuristic_ub"] = True
    if world_env == 1:
        spec["dist"]["cpu_workers"] = 0  # spawned ranks: -C 0 (with -C 1 this was the native runner)
    if world_env > 1:  # already under torchrun
        res = solve_rank(spec)
        if res["rank"] != 0:
            return 0
    else:
        from .ops import gpu_count
        from .parallel.launch import spawn_local, warm_forkserver

        warm_forkserver()  # before gpu_count: the ranks never come from a GPU-initialised process
        if (a.D > gpu_count()) if a.device is None else (a.device >= gpu_count()):
            print("Execution Terminated. More GPU devices requested than the ones available")
            return 1
        res = spawn_local(a.D, solve_rank, (spec,))[0]
    D = res["world"]
    print(report.pfsp_settings(a.inst, model.machines, model.jobs, a.ub, a.lb, D, a.C, a.ws, 1, a.L, 2,
                               _init_ub(a, model)))
    print(report.phase("Search on Parallel GPU completed", res["tree"], res["sol"], res["t_search"]))
    print("\nExploration terminated.")
    print(report.pfsp_results(res["best"], res["tree"], res["sol"], res["elapsed"]))
    workers = [report.WorkerStats(**w) for w in res["workers"]]
    # C column: 1 when every rank ran a CPU worker next to its GPU (hybrid rank engine)
    C = 1 if spec["dist"]["cpu_workers"] > 0 else 0
    if not a.no_csv:
        report.write_multi_gpu_csv(os.path.join(a.csv_dir, "multigpu.csv"), a.inst, a.lb, D, C, a.ws, res["best"],
                                   a.m, a.M, a.T, res["elapsed"], res["tree"], res["sol"], workers)
        # one process per GPU = the reference's distributed driver layout (one GPU per rank)
        report.write_dist_multi_gpu_csv(os.path.join(a.csv_dir, "dist_multigpu.csv"), a.inst, a.lb, 1, C, a.L, D,
                                        res["best"], a.m, a.M, a.T, res["elapsed"], res["tree"], res["sol"], workers,
                                        [w.dist_load_bal for w in workers], [w.t_load_bal for w in workers])
    if a.json:
        report.write_json_record(a.json, {**model.describe(), "n_gpus": D, "tree": res["tree"], "sol": res["sol"],
                                           "best": res["best"], "elapsed": res["elapsed"],
                                           "nodes_per_sec": res["tree"] / max(res["elapsed"], 1e-12),
                                           "rounds": res["extra"]["rounds"], "workers": res["workers"],
                                           "initial_ub": _init_ub(a, model)})
    return 0


def _json(a, model, r, n_gpus) -> None:
    if a.json:
        from dataclasses import asdict

        report.write_json_record(a.json, {**model.describe(), "n_gpus": n_gpus, "tree": r.tree, "sol": r.sol,
                                          "best": r.best, "elapsed": r.elapsed, "nodes_per_sec": r.nodes_per_sec,
                                          "workers": [asdict(w) for w in r.workers], "initial_ub": _init_ub(a, model)})


def _init_ub(a, model) -> int | None:
    """The incumbent the device search starts from: the best-known makespan with -u 1,
    None (+inf) with -u 0, the heuristic schedule's makespan with --heuristic-ub."""
    if a.ub == 1:
        return int(model.best_known)
    if getattr(a, "heuristic_ub", False) and a.D >= 1:
        return int(model.search_best(0))
    return None


def _nqueens_parser(cls=argparse.ArgumentParser) -> argparse.ArgumentParser:
    ap = cls(prog="nqueens", description="N-Queens backtracking")
    ap.add_argument("-N", type=int, default=14)
    ap.add_argument("-g", type=int, default=1)
    ap.add_argument("-m", type=int, default=25)
    ap.add_argument("-M", type=int, default=50000)
    ap.add_argument("-D", type=int, default=1)
    ap.add_argument("--max-parents", type=int, default=1 << 19)
    # engines per GPU, the solve split in the graph between them: N=17 74 -> 48 ms on one
    # MI355X with 2 (profiles/r3/queens/streams_probe.txt); with the wave-stack finishing
    # and each engine's compute stream on its own hardware queue, 3: 20.4 -> 18.2 ms
    # (profiles/r6/queens/lazy_xfer_ab.txt; the kernel's window is at most 2^19 parents)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--stream-split", type=int, default=512)
    return ap


def nqueens_main(argv: list[str]) -> int:
    a = _nqueens_parser().parse_args(argv)
    for name, v in (("N", a.N), ("g", a.g), ("m", a.m)):
        if v < 1:
            sys.stderr.write(f"Error: {name} must be a positive integer.\n")
            return 1
    if a.M < a.m:
        sys.stderr.write("Error: M must be a positive integer, greater or equal to m.\n")
        return 1
    from .models.nqueens import QueensModel
    from .models.pfsp import EngineOptions
    from .search import solve_cpu, solve_engine

    model = QueensModel(a.N, a.g)
    if a.D == 0:
        print(report.queens_settings(a.N, a.g, "Sequential C++"))
        r = solve_cpu(model)
        print("\nExploration terminated.")
        print(report.queens_results(r.tree, r.sol, r.elapsed))
        return 0
    if a.D == 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        print(report.queens_settings(a.N, a.g, "Single-GPU C++/HIP (MI355X)"))
        eng = model.make_engine("gpu", 0, EngineOptions(max_parents=a.max_parents, streams=max(1, a.streams),
                                                        stream_split=a.stream_split if a.streams > 1 else 0))
        r = solve_engine(model, eng, m=a.m, verbose=True)
        print(report.queens_results(r.tree, r.sol, r.elapsed))
        return 0
    from .parallel.workers import solve_rank

    spec = {"problem": "nqueens", "N": a.N, "G": a.g, "backend": "gpu",
            "engine": {"max_parents": a.max_parents, "streams": max(1, a.streams),
                       "stream_split": a.stream_split if a.streams > 1 else 0},
            "dist": {"m": a.m, "init_per_rank": a.m}}
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        res = solve_rank(spec)
        if res["rank"] != 0:
            return 0
    else:
        from .parallel.launch import spawn_local, warm_forkserver

        warm_forkserver()
        res = spawn_local(a.D, solve_rank, (spec,))[0]
    print(report.queens_settings(a.N, a.g, f"Multi-GPU C++/HIP+RCCL ({res['world']} GPUs)"))
    print(report.phase("Search on GPU completed", res["tree"], res["sol"], res["t_search"]))
    print("\nExploration terminated.")
    print(report.queens_results(res["tree"], res["sol"], res["elapsed"]))
    return 0


class _QuietParser(argparse.ArgumentParser):
    def error(self, message):  # parse errors are reported by the real parse in *_main
        raise ValueError(message)


def _spawn_planned(argv: list[str]) -> bool:
    """Will this command start one process per GPU itself (spawn_local)? Decided with the
    same parsers and the same routing tests as pfsp_main / nqueens_main (so `-D2`,
    `--D=3` and abbreviated long options count), before anything touches HIP."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or not argv:
        return False
    try:
        if argv[0] == "nqueens":
            a = _nqueens_parser(_QuietParser).parse_args(argv[1:])
            return a.D > 1
        a = _pfsp_parser(_QuietParser).parse_args(argv[1:])
    except (ValueError, SystemExit):
        return False
    # pfsp_main: D == 0 is CPU only; C == 1 / --single-process / --gpus-list is the native
    # runner; D == 1 is the single-GPU path; every other D goes through spawn_local
    return a.D > 1 and not (a.C == 1 or a.single_process or a.gpus_list)


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("pfsp", "nqueens"):
        sys.stderr.write(__doc__ or "")
        return 2
    if _spawn_planned(argv):
        # the rank processes come from a forkserver that must exist before this process
        # makes any HIP call (gpu_count, engines): a GPU-initialised process never forks
        # and execs a rank (ref launch: pfsp_dist_multigpu_cuda.c:907-919, one MPI rank per GPU)
        from .parallel.launch import warm_forkserver

        warm_forkserver()
    return pfsp_main(argv[1:]) if argv[0] == "pfsp" else nqueens_main(argv[1:])
