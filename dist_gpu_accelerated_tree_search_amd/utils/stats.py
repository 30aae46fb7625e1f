"""Descriptive statistics for run analysis (ref common/util.c:40-201: findMin,
findMaxInt, get_min/max/median/quartile/percentile/stddev, compute_boxplot_stats;
none of which the reference's drivers call). Percentiles use linear interpolation
between closest ranks, as the reference's get_percentile does."""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Sequence


def find_min(v: Sequence[float]) -> float:
    return min(v)


def find_max(v: Sequence[float]) -> float:
    return max(v)


def percentile(v: Sequence[float], p: float) -> float:
    """p in [0, 100]."""
    if not v:
        raise ValueError("empty sample")
    s = sorted(v)
    if len(s) == 1:
        return float(s[0])
    x = (len(s) - 1) * p / 100.0
    lo = math.floor(x)
    hi = min(lo + 1, len(s) - 1)
    return float(s[lo] + (s[hi] - s[lo]) * (x - lo))


def median(v: Sequence[float]) -> float:
    return percentile(v, 50)


def quartiles(v: Sequence[float]) -> tuple[float, float, float]:
    return percentile(v, 25), percentile(v, 50), percentile(v, 75)


def stddev(v: Sequence[float], sample: bool = False) -> float:
    n = len(v)
    if n < 2:
        return 0.0
    mu = sum(v) / n
    return math.sqrt(sum((x - mu) ** 2 for x in v) / (n - 1 if sample else n))


@dataclass
class Boxplot:
    min: float
    q1: float
    median: float
    q3: float
    max: float
    iqr: float
    lower_whisker: float
    upper_whisker: float
    outliers: list


def boxplot(v: Sequence[float]) -> Boxplot:
    q1, q2, q3 = quartiles(v)
    iqr = q3 - q1
    lo_f, hi_f = q1 - 1.5 * iqr, q3 + 1.5 * iqr
    inside = [x for x in v if lo_f <= x <= hi_f]
    return Boxplot(min=float(min(v)), q1=q1, median=q2, q3=q3, max=float(max(v)), iqr=iqr,
                   lower_whisker=float(min(inside)) if inside else q1,
                   upper_whisker=float(max(inside)) if inside else q3,
                   outliers=[x for x in v if x < lo_f or x > hi_f])


def imbalance(work: Sequence[float]) -> float:
    """max / mean of per-worker work (1.0 = perfect balance)."""
    mu = sum(work) / len(work)
    return float(max(work) / mu) if mu > 0 else 1.0
