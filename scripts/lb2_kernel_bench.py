"""Time the LB2 expand kernel on real ta056 windows (one iteration each) and check
that every variant gives the same bounds as the default path.

    python scripts/lb2_kernel_bench.py [window_dir] [reps]

Windows: scripts/lb2_pool_dump.py output (16,384 pool-top parents = 2,048 chunks).
Per window and variant: min/median ms per launch on the engine's grid, the
per-chunk shader clocks of phases A / B1 / B2 / B3+C, and G parents/s.
Variants are (label, probe variant, environment).
"""
import glob
import os
import sys

sys.path.insert(0, ".")
import numpy as np
import torch  # noqa: F401
from dist_gpu_accelerated_tree_search_amd import PfspModel
from dist_gpu_accelerated_tree_search_amd.ops import hip

VARIANTS = [
    ("plain walk, blocked chunks", 1, {"TTS_LB2_PIPE": "0", "TTS_LB2_STRIDE": "0"}),
    ("packed 2-child, blocked", 4, {"TTS_LB2_PIPE": "1", "TTS_LB2_STRIDE": "0"}),
    ("packed 2-child, strided", 4, {"TTS_LB2_PIPE": "1", "TTS_LB2_STRIDE": "1"}),
]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "scratch/lb2_windows"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    H = hip()
    m = PfspModel(56, 2)
    best = m.initial_best(1)
    p = list(m.native.p)
    for f in sorted(glob.glob(os.path.join(d, "*.npy"))):
        nodes = np.ascontiguousarray(np.load(f))
        ref = None
        for label, var, env in VARIANTS:
            for k, v in env.items():
                os.environ[k] = v
            out = H.pfsp_expand_probe(m.jobs, m.machines, p, 2, nodes, best, 0, var)
            dec = out < best
            if ref is None:
                ref = dec
            assert np.array_equal(dec, ref), (label, int((dec != ref).sum()))
            t = H.pfsp_expand_time(m.jobs, m.machines, p, 2, nodes, best, 0, var, reps)
            print(f"{os.path.basename(f)} {label:28s}: {t['ms_min']:.3f} ms (median {t['ms_median']:.3f}) "
                  f"-> {len(nodes) / t['ms_min'] / 1e6:.3f} G parents/s; clocks/chunk A {t['clk_a']:.0f} "
                  f"B1 {t['clk_b1']:.0f} B2 {t['clk_b2']:.0f} C {t['clk_c']:.0f} ({t['chunks']:.0f} chunks); "
                  f"workgroup clocks max {t['clk_block_max']:.0f} mean {t['clk_block_mean']:.0f} (grid {t['grid']:.0f})",
                  flush=True)
            tl = t["timeline_us"]
            if len(tl):
                ends = np.sort(tl[:, 2])
                print(f"    workgroups (us from the first entry): entry max {tl[:, 0].max():.1f}, prologue "
                      f"mean {np.mean(tl[:, 1] - tl[:, 0]):.1f} max {np.max(tl[:, 1] - tl[:, 0]):.1f}, exit "
                      f"p10 {ends[len(ends) // 10]:.1f} p50 {ends[len(ends) // 2]:.1f} p90 {ends[9 * len(ends) // 10]:.1f} "
                      f"max {ends[-1]:.1f}; busy share {np.sum(tl[:, 2] - tl[:, 0]) / (len(tl) * ends[-1]):.2f}",
                      flush=True)
            for k in env:
                os.environ.pop(k, None)


if __name__ == "__main__":
    main()
