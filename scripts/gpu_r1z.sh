#!/bin/bash
# local DFS gated on the pool backlog: A/B over TTS_LOCAL_STEPS / TTS_LOCAL_MIN
o=gpurun_out/r1z; mkdir -p $o
for cfg in "0 0" "4 0" "8 0" "4 1" "4 3145728"; do
  set -- $cfg
  TTS_LOCAL_STEPS=$1 TTS_LOCAL_MIN=$2 timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe_L$1_min$2.txt 2>&1 || exit $?
done
for f in $o/lb1_probe_*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
