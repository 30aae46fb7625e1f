"""Stdout blocks and CSV statistics (byte-compatible with the reference).

Parity: ref pfsp/lib/PFSP_lib.c:133-170 (print_settings / print_results),
pfsp/lib/PFSP_statistic.c:7-167 (singlegpu.csv, multigpu.csv, dist_multigpu.csv:
quoted "[a,b]" arrays, "%.4f" times, trailing comma on multi/dist rows) and
nqueens/*: print_settings / print_results. The native CLIs (csrc/core/report.hpp)
emit the same blocks.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field
from typing import Sequence

LB_NAMES = {0: "lb1_d", 1: "lb1", 2: "lb2"}

BANNER = "================================================="


def pfsp_settings(inst: int, machines: int, jobs: int, ub: int, lb: int, D: int, C: int, ws: int, comm_size: int,
                  L: int, version: int, init_ub: int | None = None) -> str:
    """init_ub: with -u 0, the opt-in heuristic starting incumbent (--heuristic-ub), printed
    instead of "inf" so the explored tree is not mistaken for the reference's -u 0 tree."""
    if version == 0:
        head = "Sequential C++"
    elif version == 1:
        head = "Single-GPU C++/HIP (MI355X)"
    elif version == 2:
        head = f"Multi-core Multi-GPU C++/HIP (%d GPU(s) - [%d] Multi-core - [%d] Work Stealing)" % (D, C, ws)
    else:
        head = f"Distributed Multi-GPU C++/HIP+RCCL (%d processes x ( %d GPU(s) - [%d] Multi-core ) - [%d] LB)" % (
            comm_size, D, C, L)
    lines = [
        "",
        BANNER,
        head,
        "",
        f"Resolution of PFSP Taillard's instance: ta{inst} (m = {machines}, n = {jobs})",
        ("Initial upper bound: opt" if ub != 0 else
         "Initial upper bound: inf" if init_ub is None or init_ub >= 2**31 - 1 else
         f"Initial upper bound: heuristic ({init_ub})"),
        f"Lower bound function: {LB_NAMES.get(lb, 'lb2')}",
        "Branching rule: fwd",
        BANNER,
    ]
    return "\n".join(lines)


def pfsp_results(optimum: int, tree: int, sol: int, elapsed: float) -> str:
    return "\n".join([
        "",
        BANNER,
        f"Size of the explored tree: {tree}",
        f"Number of explored solutions: {sol}",
        f"Optimal makespan: {optimum}",
        f"Elapsed time: {elapsed:.4f} [s]",
        BANNER,
    ])


def phase(title: str, tree: int, sol: int, t: float) -> str:
    return "\n".join(["", title, f"Size of the explored tree: {tree}", f"Number of explored solutions: {sol}",
                      f"Elapsed time: {t:f} [s]"])


def queens_settings(N: int, G: int, backend: str) -> str:
    return "\n".join(["", BANNER, backend, "", f"Resolution of the {N}-Queens instance",
                      f"  with {G} safety check(s) per evaluation", BANNER])


def queens_results(tree: int, sol: int, elapsed: float) -> str:
    return "\n".join(["", BANNER, f"Size of the explored tree: {tree}", f"Number of explored solutions: {sol}",
                      f"Elapsed time: {elapsed:.4f} [s]", BANNER])


@dataclass
class WorkerStats:
    """Per-worker counters/timers; the reference's CSV array columns."""

    tree: int = 0
    sol: int = 0
    gen_child: int = 0
    steals: int = 0
    success_steals: int = 0
    terminations: int = 0
    t_memcpy: float = 0.0
    t_malloc: float = 0.0
    t_kernel: float = 0.0
    t_gen_child: float = 0.0
    t_pool_ops: float = 0.0
    t_idle: float = 0.0
    t_termination: float = 0.0
    # distributed runs: transfers received (DWS, ref nbSDistLoadBal) and time spent moving nodes (timeLoadBal)
    dist_load_bal: int = 0
    t_load_bal: float = 0.0

    @classmethod
    def from_dict(cls, d: dict) -> "WorkerStats":
        return cls(**{k: d[k] for k in asdict(cls()) if k in d})


def _ull(v: Sequence[int]) -> str:
    return '"[' + ",".join(str(int(x)) for x in v) + ']",'


def _dbl(v: Sequence[float]) -> str:
    return '"[' + ",".join(f"{float(x):.4f}" for x in v) + ']",'


def _open_with_header(path: str, header: str):
    fresh = not os.path.exists(path) or os.path.getsize(path) == 0
    f = open(path, "a")
    if fresh:
        f.write(header)
    return f


SINGLE_HEADER = ("instance_id,lower_bound,optimum,m,M,total_time,gpu_memcpy_time,gpu_malloc_time,gpu_kernel_time,"
                 "gen_child_time,explored_tree,explored_sol\n")
MULTI_HEADER = ("instance_id,D,C,lower_bound,work_stealing,optimum,m,M,T,total_time,total_tree,total_sol,"
                "exp_tree_gpu,exp_sol_gpu,gen_child_gpu,steals_gpu,success_steals_gpu,termination_gpu,"
                "gpu_memcpy_time,gpu_malloc_time,gpu_kernel_time,gpu_gen_child_time,pool_ops_time,gpu_idle_time,"
                "termination_time\n")
DIST_HEADER = ("instance_id,D,C,comm_size,lower_bound,load_balancing,optimum,m,M,T,total_time,total_tree,total_sol,"
               "all_exp_tree_gpu,all_exp_sol_gpu,all_gen_child_gpu,all_steals_gpu,all_success_steals_gpu,"
               "all_termination_gpu,all_dist_load_bal,all_gpu_memcpy_time,all_gpu_malloc_time,all_gpu_kernel_time,"
               "all_gpu_gen_child_time,all_pool_ops_time,all_gpu_idle_time,all_termination_time,all_time_load_bal\n")


def _worker_cols(ws: Sequence[WorkerStats]) -> str:
    return "".join([
        _ull([w.tree for w in ws]), _ull([w.sol for w in ws]), _ull([w.gen_child for w in ws]),
        _ull([w.steals for w in ws]), _ull([w.success_steals for w in ws]), _ull([w.terminations for w in ws]),
    ])


def _worker_times(ws: Sequence[WorkerStats]) -> str:
    return "".join([
        _dbl([w.t_memcpy for w in ws]), _dbl([w.t_malloc for w in ws]), _dbl([w.t_kernel for w in ws]),
        _dbl([w.t_gen_child for w in ws]), _dbl([w.t_pool_ops for w in ws]), _dbl([w.t_idle for w in ws]),
        _dbl([w.t_termination for w in ws]),
    ])


def write_single_gpu_csv(path: str, inst: int, lb: int, optimum: int, m: int, M: int, total_time: float,
                         t_memcpy: float, t_malloc: float, t_kernel: float, t_gen_child: float, tree: int,
                         sol: int) -> None:
    with _open_with_header(path, SINGLE_HEADER) as f:
        f.write(f"{inst},{lb},{optimum},{m},{M},{total_time:.4f},{t_memcpy:.4f},{t_malloc:.4f},{t_kernel:.4f},"
                f"{t_gen_child:.4f},{tree},{sol}\n")


def write_multi_gpu_csv(path: str, inst: int, lb: int, D: int, C: int, ws: int, optimum: int, m: int, M: int, T: int,
                        total_time: float, tree: int, sol: int, workers: Sequence[WorkerStats]) -> None:
    with _open_with_header(path, MULTI_HEADER) as f:
        f.write(f"{inst},{D},{C},{lb},{ws},{optimum},{m},{M},{T},{total_time:.4f},{tree},{sol},")
        f.write(_worker_cols(workers) + _worker_times(workers) + "\n")


def write_dist_multi_gpu_csv(path: str, inst: int, lb: int, D: int, C: int, L: int, comm_size: int, optimum: int,
                             m: int, M: int, T: int, total_time: float, tree: int, sol: int,
                             workers: Sequence[WorkerStats], dist_load_bal: Sequence[int],
                             time_load_bal: Sequence[float]) -> None:
    with _open_with_header(path, DIST_HEADER) as f:
        f.write(f"{inst},{D},{C},{comm_size},{lb},{L},{optimum},{m},{M},{T},{total_time:.4f},{tree},{sol},")
        f.write(_worker_cols(workers) + _ull(dist_load_bal) + _worker_times(workers) + _dbl(time_load_bal) + "\n")


def write_json_record(path: str, record: dict) -> None:
    """One JSON line per run (nodes/sec + per-worker breakdown); new in this framework."""
    with open(path, "a") as f:
        f.write(json.dumps(record) + "\n")
