"""Sum rocprofv3 counter-collection CSVs per kernel and print derived ratios.

    python scripts/pmc_summary.py <rocprofv3 output dir> [kernel substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "")
            if want not in k:
                continue
            name = k.split("(")[0].replace("void ", "").replace("tts::dev::", "")
            tot[name][row["Counter_Name"]] += float(row["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", x[1].get("SQ_WAVES", 0))):
    print(k)
    for n in sorted(c):
        print(f"  {n:28s} {c[n]:.4e}")
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if n in c:
                print(f"  {n + ' / SQ_WAVE_CYCLES':44s} {c[n] / wc:.3f}")
    if c.get("SQ_INSTS_LDS") and c.get("SQ_LDS_BANK_CONFLICT"):
        print(f"  {'bank-conflict cycles per LDS instruction':44s} {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.3f}")
    if c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
        print(f"  {'VALU instructions per wave':44s} {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.1f}")
