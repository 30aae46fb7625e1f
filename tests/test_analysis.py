"""Run-statistics helpers (ref common/util.c stats, pfsp/data/*.py analysis)."""
import json
import os
import sys

import pytest

from dist_gpu_accelerated_tree_search_amd.utils import report, stats

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "bench"))
import analyze  # noqa: E402


def test_stats_helpers():
    v = [1, 2, 3, 4, 100]
    assert stats.find_min(v) == 1 and stats.find_max(v) == 100
    assert stats.median(v) == 3
    assert stats.quartiles([1, 2, 3, 4]) == (1.75, 2.5, 3.25)
    assert stats.percentile([5], 90) == 5
    assert stats.stddev([2, 4, 4, 4, 5, 5, 7, 9]) == pytest.approx(2.0)
    b = stats.boxplot(v)
    assert b.outliers == [100] and b.upper_whisker == 4
    assert stats.imbalance([1, 1, 2]) == pytest.approx(1.5)


def test_analyze_multi_and_dist_csv(tmp_path):
    W = report.WorkerStats
    p = tmp_path / "multigpu.csv"
    for D, t in ((1, 2.0), (2, 1.0), (4, 0.6)):
        ws = [W(tree=100 // D, sol=1, steals=D) for _ in range(D)]
        report.write_multi_gpu_csv(str(p), 14, 1, D, 0, 1, 1377, 25, 50000, 5000, t, 100, 2, ws)
    rows = analyze.analyze_csv(str(p))
    assert [r["D"] for r in rows] == [1, 2, 4]
    assert rows[1]["speedup"] == pytest.approx(2.0)
    assert rows[2]["balance"] == pytest.approx(1.0)
    q = tmp_path / "dist_multigpu.csv"
    ws = [W(tree=30), W(tree=10)]
    report.write_dist_multi_gpu_csv(str(q), 14, 1, 1, 0, 1, 2, 1377, 25, 50000, 5000, 1.0, 40, 1, ws, [1, 0],
                                    [0.1, 0.0])
    rows = analyze.analyze_csv(str(q))
    assert rows[0]["D"] == 2 and rows[0]["balance"] == pytest.approx(1.5)
    assert "| instance |" in analyze.table(rows)


def test_analyze_bench_jsonl(tmp_path):
    p = tmp_path / "h.jsonl"
    with open(p, "w") as f:
        for n, v in ((1, 10.0), (2, 15.0), (8, 40.0)):
            f.write(json.dumps({"metric": "m", "value": v, "unit": "nodes/s", "n_gpus": n, "ms_per_step": 1.0}) + "\n")
    rows = analyze.analyze_jsonl(str(p))
    assert rows[1]["speedup"] == pytest.approx(1.5) and rows[2]["efficiency"] == pytest.approx(0.5)
    analyze.plot(rows, str(tmp_path / "x.png"))
    assert (tmp_path / "x.png").stat().st_size > 0
