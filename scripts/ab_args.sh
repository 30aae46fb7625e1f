#!/bin/bash
# A/B bench.py argument sets on one GPU, alternating: scripts/ab_args.sh OUT REPEATS "args1" "args2" ...
out=$1; reps=$2; shift 2
for r in $(seq 1 "$reps"); do
  for args in "$@"; do
    timeout -k 10 300 python bench.py $args > "$out.tmp" 2>> "$out.err" || { echo "failed: $args"; exit 1; }
    python3 -c "import json,sys; r=json.loads(open('$out.tmp').read().strip().splitlines()[-1]); print('$args', 'run', $r, '%.4f ms/step %.3f G nodes/s' % (r['ms_per_step'], r['value']/1e9))" >> "$out"
  done
done
rm -f "$out.tmp"
