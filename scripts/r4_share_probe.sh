#!/bin/bash
# Kernel shapes on a rank's share of an S-rank split (TTS_PROBE_SHARE) and at N=1
set -o pipefail
for S in 8 1; do
  echo "== share 1/$S"
  TTS_PROBE_SHARE=$S timeout -k 10 300 python -u scripts/front_time_probe.py 14 1 ${1:-4,6,8,9,10,11,12,13,14,15,16,17,18} one,L2,L3 2>&1 | grep -v amdgpu || exit 1
done
