#!/bin/bash
# LB2 packed LDS records for the leading pairs: tests, then A/B (TTS_LB2_LDS_PAIRS=0 = off)
o=gpurun_out/r1ag; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_lds.txt 2>&1 &&
TTS_LB2_LDS_PAIRS=0 timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_nolds.txt 2>&1
rc=$?
tail -3 $o/gpu_tests.log; grep -v amdgpu $o/lb2_lds.txt; grep -v amdgpu $o/lb2_nolds.txt
exit $rc
