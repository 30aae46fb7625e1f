#!/bin/bash
# first graph replay length: ta014 (W=1, W=8 estimate) and small 20-job trees
o=gpurun_out/r1ac; mkdir -p $o
for F in 18 24 12; do
  TTS_ITERS_FIRST=$F timeout -k 10 100 python -u scripts/lb1_probe.py > $o/lb1_F$F.txt 2>&1 || exit $?
  TTS_ITERS_FIRST=$F timeout -k 10 100 python -u scripts/scaling_probe.py --per-rank 512 --reps 10 > $o/scal_F$F.txt 2>&1 || exit $?
  TTS_ITERS_FIRST=$F timeout -k 10 100 python -u scripts/first_graph_probe.py 3,4,13,14,7,12,2 > $o/small_F$F.txt 2>&1 || exit $?
done
for F in 12 18 24; do echo "== F$F"; grep -v amdgpu $o/lb1_F$F.txt | head -1; grep "W=8" $o/scal_F$F.txt; grep -v amdgpu $o/small_F$F.txt; done
