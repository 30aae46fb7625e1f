#!/usr/bin/env python3
"""Analysis of run statistics (ref pfsp/data/*.py: speedup, workload balance, DWS
counts plots), reading this framework's byte-compatible CSVs and JSON records.

    python bench/analyze.py multigpu.csv [--plot out.png]
    python bench/analyze.py dist_multigpu.csv
    python bench/analyze.py bench/results/headline.jsonl     (bench.py lines)

Prints a markdown table: per (instance, lb, D, C): mean time, speedup vs the
smallest D of the same instance, per-worker tree balance (max/mean), steals.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dist_gpu_accelerated_tree_search_amd.utils import stats  # noqa: E402


def _arr(s: str) -> list[float]:
    s = s.strip().strip('"').strip()
    if not s.startswith("["):
        return []
    body = s[1:-1].strip()
    return [float(x) for x in body.split(",") if x.strip()] if body else []


def read_csv(path: str) -> list[dict]:
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            r = {k: v for k, v in r.items() if k}  # trailing comma -> empty column
            rows.append(r)
    return rows


def analyze_csv(path: str) -> list[dict]:
    rows = read_csv(path)
    dist = "comm_size" in (rows[0] if rows else {})
    groups = defaultdict(list)
    for r in rows:
        D = int(r["D"]) * (int(r["comm_size"]) if dist else 1)
        key = (int(r["instance_id"]), int(r["lower_bound"]), D, int(r["C"]))
        tree_col = "all_exp_tree_gpu" if dist else "exp_tree_gpu"
        steal_col = "all_success_steals_gpu" if dist else "success_steals_gpu"
        groups[key].append({"time": float(r["total_time"]), "tree": int(r["total_tree"]),
                            "per": _arr(r.get(tree_col, "")), "steals": sum(_arr(r.get(steal_col, "")))})
    base = {}
    for (inst, lb, D, C), g in sorted(groups.items()):
        t = stats.median([x["time"] for x in g])
        base.setdefault((inst, lb), (D, t))
    out = []
    for (inst, lb, D, C), g in sorted(groups.items()):
        t = stats.median([x["time"] for x in g])
        d0, t0 = base[(inst, lb)]
        per = g[-1]["per"]
        out.append({"instance": inst, "lb": lb, "D": D, "C": C, "runs": len(g), "time_s": t,
                    "tree": g[-1]["tree"], "nodes_per_s": g[-1]["tree"] / t if t > 0 else 0.0,
                    "speedup": t0 / t if t > 0 else 0.0, "base_D": d0,
                    "balance": stats.imbalance(per) if per and sum(per) > 0 else 1.0,
                    "steals": stats.median([x["steals"] for x in g])})
    return out


def analyze_jsonl(path: str) -> list[dict]:
    recs = [json.loads(line) for line in open(path) if line.strip().startswith("{")]
    by_n = {}
    for r in recs:
        by_n.setdefault(int(r.get("n_gpus", 1)), r)
    v1 = by_n.get(1, {}).get("value")
    out = []
    for n, r in sorted(by_n.items()):
        eff = (r["value"] / (n * v1)) if v1 else None
        out.append({"n_gpus": n, "value": r["value"], "unit": r.get("unit"), "ms_per_step": r.get("ms_per_step"),
                    "speedup": (r["value"] / v1) if v1 else None, "efficiency": eff})
    return out


def table(rows: list[dict]) -> str:
    if not rows:
        return "(no rows)"
    keys = list(rows[0])
    fmt = lambda v: f"{v:.4g}" if isinstance(v, float) else str(v)  # noqa: E731
    lines = ["| " + " | ".join(keys) + " |", "|" + "---|" * len(keys)]
    lines += ["| " + " | ".join(fmt(r[k]) for k in keys) + " |" for r in rows]
    return "\n".join(lines)


def plot(rows: list[dict], out: str) -> None:
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots(1, 2, figsize=(10, 4))
    if rows and "n_gpus" in rows[0]:
        n = [r["n_gpus"] for r in rows]
        ax[0].plot(n, [r["speedup"] for r in rows], "o-", label="measured")
        ax[0].plot(n, n, "k--", label="ideal")
        ax[1].bar([str(x) for x in n], [r["value"] for r in rows])
        ax[1].set_ylabel(rows[0].get("unit") or "value")
    else:
        for (inst, lb) in sorted({(r["instance"], r["lb"]) for r in rows}):
            rr = [r for r in rows if (r["instance"], r["lb"]) == (inst, lb)]
            ax[0].plot([r["D"] for r in rr], [r["speedup"] for r in rr], "o-", label=f"ta{inst:03d} lb{lb}")
            ax[1].plot([r["D"] for r in rr], [r["balance"] for r in rr], "o-", label=f"ta{inst:03d}")
        ax[1].set_ylabel("tree max/mean per worker")
    ax[0].set_xlabel("GPUs")
    ax[0].set_ylabel("speedup")
    ax[0].legend()
    fig.tight_layout()
    fig.savefig(out, dpi=120)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--plot", default=None)
    a = ap.parse_args(argv)
    rows = analyze_jsonl(a.path) if a.path.endswith(".jsonl") or a.path.endswith(".json") else analyze_csv(a.path)
    print(table(rows))
    if a.plot:
        plot(rows, a.plot)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
