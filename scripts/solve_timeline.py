"""Last-solve kernel timeline from a rocprofv3 kernel trace.

    python scripts/solve_timeline.py <rocprofv3 output dir> [dispatches]

Prints the last `dispatches` kernels (duration, gap to the previous one, name) and the
span / busy share of that stretch: where a short solve's time goes (kernel work, empty
iterations, host gaps between graph replays, copies)."""
import csv
import glob
import os
import sys

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")) for r in rows)[-n:]
prev = None
busy = 0
for s, e, name in ev:
    gap = 0 if prev is None else max(0, s - prev)
    busy += e - s
    print(f"{(e - s) / 1e3:9.2f} us  gap {gap / 1e3:8.2f} us  {name.split('(')[0].replace('void ', '')[:60]}")
    prev = e
span = ev[-1][1] - ev[0][0]
print(f"\nlast {len(ev)} dispatches: span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / span:.0f}%)")
