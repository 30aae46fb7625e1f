"""Per-kernel register / LDS / occupancy table from hipcc's resource-usage remarks.

    python scripts/kernel_resources.py [file.hip ...]   (default: every csrc/hip/*.hip)
"""
import glob
import re
import subprocess
import sys

FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch",
          "Occupancy [waves/SIMD]": "occ", "LDS Size [bytes/block]": "lds", "SGPRs Spill": "sspill",
          "VGPRs Spill": "vspill"}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), text=True,
                         capture_output=True).stdout.split("\n")
    return [re.sub(r"\(.*", "", o).replace("tts::dev::", "").replace("tts::", "") for o in out]


def resources(src):
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o",
                        "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m2 = re.search(r"remark: Function Name: (\S+)", line)
        if m2:
            cur = {"name": m2.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(.*?): (\S+) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2)
        if cur is not None and k in FIELDS:
            cur[FIELDS[k]] = v
    for row, d in zip(rows, demangle([x["name"] for x in rows])):
        row["name"] = d
    return rows


def main():
    srcs = sys.argv[1:] or sorted(glob.glob("dist_gpu_accelerated_tree_search_amd/csrc/hip/*.hip"))
    print(f"| kernel | VGPR | SGPR | LDS B | scratch B/lane | waves/SIMD | VGPR spill | SGPR spill |\n|---|---|---|---|---|---|---|---|")
    seen = set()
    for s in srcs:
        for r in resources(s):
            if r["name"] in seen:
                continue
            seen.add(r["name"])
            print(f"| {r['name']} | {r.get('vgpr')} | {r.get('sgpr')} | {r.get('lds')} | {r.get('scratch')} | "
                  f"{r.get('occ')} | {r.get('vspill')} | {r.get('sspill')} |")


if __name__ == "__main__":
    main()
