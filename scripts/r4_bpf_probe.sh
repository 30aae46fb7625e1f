#!/bin/bash
# Two-level chunk size cap (TTS_FUSED_BPF) on the rank shares and the N=1 headline
set -o pipefail
for b in 12 24 32; do
  echo "== TTS_FUSED_BPF=$b"
  TTS_FUSED_BPF=$b timeout -k 10 300 python -u scripts/share_solve_probe.py 30 2>&1 | grep -v amdgpu || exit 1
done
