#!/bin/bash
# 8-parent LB2 chunks for 50-job instances: tests, then ta014/3/10/20 + ta056 time box
o=gpurun_out/r1aj; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_bp8.txt 2>&1
rc=$?
tail -3 $o/gpu_tests.log; grep -v amdgpu $o/lb2_bp8.txt
exit $rc
