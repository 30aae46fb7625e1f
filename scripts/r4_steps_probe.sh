#!/bin/bash
# Local DFS steps (TTS_LOCAL_STEPS) on the rank shares and ta021 / ta056
set -o pipefail
for v in 3 4 2; do
  echo "== TTS_LOCAL_STEPS=$v"
  TTS_LOCAL_STEPS=$v timeout -k 10 300 python -u scripts/share_solve_probe.py 20 2>&1 | grep -v amdgpu || exit 1
  TTS_LOCAL_STEPS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --extras ta021 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['ms_per_step'], {k: (e.get('seconds'), e.get('nodes_per_s')) for k, e in d['extras'].items()})" || exit 1
done
