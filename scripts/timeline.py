"""Kernel timeline from a rocprofv3 --kernel-trace CSV: the last `n` dispatches with
their duration and the idle gap before each, plus per-solve totals.

    python scripts/timeline.py <dir-or-csv> [n] [--md]
"""
import csv
import glob
import os
import sys


def load(path):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not cands:
            raise SystemExit(f"no kernel_trace.csv under {path}")
        path = max(cands, key=os.path.getsize)
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    name = name.replace("tts::dev::", "").replace("tts::", "").replace("void ", "")
    return name.split("(")[0] if "(" in name else name


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    md = "--md" in sys.argv
    rows = load(args[0])
    n = int(args[1]) if len(args) > 1 else 80
    tail = rows[-n:]
    prev_end = None
    busy = 0
    if md:
        print("| kernel | duration us | gap before us |\n|---|---|---|")
    for s, e, k in tail:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        busy += e - s
        prev_end = e
        if md:
            print(f"| {short(k)} | {(e - s) / 1e3:.2f} | {gap:.2f} |")
        else:
            print(f"{(e - s) / 1e3:8.2f} us  gap {gap:8.2f} us  {short(k)}")
    span = (tail[-1][1] - tail[0][0]) / 1e3
    print(f"\nlast {len(tail)} dispatches: span {span:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / 1e3 / span:.0f}%)")


if __name__ == "__main__":
    main()
