#!/bin/bash
# LB2 B2 in rounds of pairs with re-compaction: tests, then A/B (TTS_LB2_ROUNDS=0 = off)
o=gpurun_out/r1ak; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_rounds.txt 2>&1 &&
TTS_LB2_ROUNDS=0 timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_norounds.txt 2>&1
rc=$?
tail -3 $o/gpu_tests.log; grep -v amdgpu $o/lb2_rounds.txt; grep -v amdgpu $o/lb2_norounds.txt
exit $rc
