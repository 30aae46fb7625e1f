#!/bin/bash
# LB2 task-parallel kernel: numerics + golden trees, then timings
o=gpurun_out/r1m; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/lb2_probe.py 30 > $o/lb2_probe.txt 2>&1
rc=$?
tail -3 $o/gpu_tests.log; cat $o/lb2_probe.txt
exit $rc
