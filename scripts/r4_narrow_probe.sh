#!/bin/bash
# Steps of narrow strided local windows (TTS_LOCAL_NARROW_STEPS; 0 = the default)
set -o pipefail
bash scripts/r4_session.sh "$1" ab:TTS_LOCAL_NARROW_STEPS=6,0:3 || exit 1
for v in 6 0; do
  echo "== TTS_LOCAL_NARROW_STEPS=$v"
  TTS_LOCAL_NARROW_STEPS=$v timeout -k 10 300 python -u scripts/share_solve_probe.py 20 2>&1 | grep -v amdgpu || exit 1
done
