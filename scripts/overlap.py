"""Copy / kernel overlap from a rocprofv3 trace (--kernel-trace --memory-copy-trace).

    python scripts/overlap.py <rocprofv3 output dir>

Prints the time spent in host<->device copies and how much of it ran while an
expand kernel was executing (engine.hpp: spills and refills on the transfer stream
are meant to overlap the graph replays on the compute stream)."""
import csv
import glob
import os
import sys


def load(pattern):
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", pattern), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


krows = load("*kernel_trace.csv")
mrows = load("*memory_copy_trace.csv")
if mrows:
    print("memory-copy trace fields:", ",".join(mrows[0].keys()))
allk = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")) for r in krows]
# HIP moves pinned-host <-> device async copies with blit kernels on the issuing stream
# (__amd_rocclr_copyBuffer...): count them as copies, the search kernels as compute
blit = lambda n: "rocclr" in n or "copyBuffer" in n  # noqa: E731
kern = sorted(k for k in allk if not blit(k[2]))
copies = [(s, e, "blit " + n.split("(")[0].split(" ")[-1], 0) for s, e, n in allk if blit(n)]
copies += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "")),
            int(r.get("Bytes", r.get("Size", r.get("Copy_Bytes", 0))) or 0)) for r in mrows]
# merge kernel intervals into busy spans
busy = []
for s, e, _ in kern:
    if busy and s <= busy[-1][1]:
        busy[-1][1] = max(busy[-1][1], e)
    else:
        busy.append([s, e])


def overlap(s, e):
    t = 0
    for bs, be in busy:
        if be <= s:
            continue
        if bs >= e:
            break
        t += min(e, be) - max(s, bs)
    return t


by = {}
for s, e, d, b in copies:
    x = by.setdefault(d, [0, 0, 0, 0])
    x[0] += 1
    x[1] += e - s
    x[2] += overlap(s, e)
    x[3] += b
print(f"kernels: {len(kern)} dispatches, busy {sum(e - s for s, e in busy) / 1e6:.3f} ms")
for d, (n, t, o, b) in sorted(by.items()):
    print(f"copies {d}: {n}, {b / 2**20:.1f} MiB, {t / 1e6:.3f} ms, {o / 1e6:.3f} ms ({100 * o / max(t, 1):.0f} %) "
          f"while a kernel ran")
big = sorted(copies, key=lambda c: c[1] - c[0], reverse=True)[:8]
for s, e, d, b in big:
    print(f"  {d} {b / 2**20:8.2f} MiB {(e - s) / 1e3:9.1f} us, overlapped {overlap(s, e) / 1e3:9.1f} us")

# timeline excerpt around the longest copies: every kernel/copy start-end (us, relative)
ev = sorted([(s, e, "K " + n.split("(")[0].split(" ")[-1][:40]) for s, e, n in allk if not blit(n)] +
            [(s, e, "C " + d) for s, e, d, _ in copies])
for s0, e0, d0, _ in big[:2]:
    i = next(k for k, x in enumerate(ev) if x[0] == s0)
    print(f"--- around a {(e0 - s0) / 1e3:.1f} us copy")
    for s, e, n in ev[max(0, i - 8): i + 8]:
        print(f"  {(s - s0) / 1e3:9.2f} .. {(e - s0) / 1e3:9.2f}  {n}")
