"""A/B an environment knob on one GPU: each command runs once per setting, settings
alternating, repeated; prints the JSON value / probe lines per run.

    python scripts/ab_env.py VAR v1,v2 REPEATS -- cmd args...
"""
import json
import os
import subprocess
import sys

var, vals, reps = sys.argv[1], sys.argv[2].split(","), int(sys.argv[3])
cmd = sys.argv[sys.argv.index("--") + 1:]
for r in range(reps):
    for v in vals:
        env = dict(os.environ, **{var: v})
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            print(f"{var}={v} run {r}: exit {p.returncode}\n{p.stderr[-2000:]}", flush=True)
            raise SystemExit(1)
        out = p.stdout.strip().splitlines()
        try:
            rec = json.loads(out[-1])
            print(f"{var}={v} run {r}: {rec['ms_per_step']:.4f} ms/step, {rec['value'] / 1e9:.3f} G nodes/s", flush=True)
        except (ValueError, IndexError, KeyError):
            for line in out:
                if "amdgpu.ids" not in line:
                    print(f"{var}={v} run {r}: {line}", flush=True)
