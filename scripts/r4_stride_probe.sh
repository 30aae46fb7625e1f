#!/bin/bash
# Strided local DFS windows (TTS_LOCAL_STRIDE): ta021 and the rank shares
set -o pipefail
for v in 1 0; do
  echo "== TTS_LOCAL_STRIDE=$v"
  TTS_LOCAL_STRIDE=$v timeout -k 10 300 python -u scripts/share_solve_probe.py 20 2>&1 | grep -v amdgpu || exit 1
  TTS_LOCAL_STRIDE=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --extras ta021,ta056 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print({k: (e.get('seconds'), e.get('nodes_per_s')) for k, e in d['extras'].items()})" || exit 1
done
