#!/bin/bash
# local DFS on full windows only: A/B over TTS_LOCAL_STEPS, then GPU tests
o=gpurun_out/r1y; mkdir -p $o
for L in 0 2 4 8; do
  TTS_LOCAL_STEPS=$L timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe_L$L.txt 2>&1 || exit $?
done
TTS_LOCAL_STEPS=4 TTS_LOCAL_MIN=65536 timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe_L4_min64k.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?
tail -2 $o/gpu_tests.log; for f in $o/lb1_probe_*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
exit $rc
