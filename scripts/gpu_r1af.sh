#!/bin/bash
# LB2 wave-uniform pair walks: GPU kernel/search tests, then A/B on ta014/3/10/20 + ta056 time box
o=gpurun_out/r1af; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
TTS_LB2_WAVE=1 timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_wave1.txt 2>&1 &&
TTS_LB2_WAVE=0 timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_wave0.txt 2>&1
rc=$?
tail -3 $o/gpu_tests.log; grep -v amdgpu $o/lb2_wave1.txt; grep -v amdgpu $o/lb2_wave0.txt
exit $rc
