#!/bin/bash
# Local DFS from narrower windows (TTS_LOCAL_MIN) on the rank shares and on ta021
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
for v in 0 20000 8000 4000; do
  echo "== TTS_LOCAL_MIN=$v"
  TTS_LOCAL_MIN=$v timeout -k 10 300 python -u scripts/share_solve_probe.py 30 2>&1 | grep -v amdgpu || exit 1
done
for v in 0 16384; do
  echo "== ta021 TTS_LOCAL_MIN=$v"
  TTS_LOCAL_MIN=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --extras ta021 > "$out/ta021_$v.json" 2> "$out/ta021_$v.err" || { tail -5 "$out/ta021_$v.err"; exit 1; }
  python -c "import json,sys; r=json.load(open('$out/ta021_$v.json')); e=r['extras']['ta021']; print(r['ms_per_step'], e['seconds'], e['tree'], e['golden_ok'])"
done
