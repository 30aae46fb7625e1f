#!/bin/bash
# narrow local DFS (small windows): A/B over TTS_NARROW_STEPS / TTS_NARROW_CAP / TTS_NARROW_BP
o=gpurun_out/r1ab; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread > $o/gpu_search_tests.log 2>&1 || { tail -30 $o/gpu_search_tests.log; exit 1; }
for cfg in "0 512 16" "16 512 16" "8 512 16" "32 512 16" "16 256 16" "16 1024 16" "16 512 4" "16 512 64"; do
  set -- $cfg
  n=S$1_C$2_B$3
  TTS_NARROW_STEPS=$1 TTS_NARROW_CAP=$2 TTS_NARROW_BP=$3 timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_$n.txt 2>&1 || exit $?
  TTS_NARROW_STEPS=$1 TTS_NARROW_CAP=$2 TTS_NARROW_BP=$3 timeout -k 10 200 python -u scripts/scaling_probe.py --per-rank 512 --reps 10 > $o/scal_$n.txt 2>&1 || exit $?
done
tail -2 $o/gpu_search_tests.log
for f in $o/lb1_*.txt; do n=${f#$o/lb1_}; echo "== $n $(grep -v amdgpu $f | tr '\n' ' ')"; grep "W=8" $o/scal_$n; done
