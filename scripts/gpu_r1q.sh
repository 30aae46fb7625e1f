#!/bin/bash
o=gpurun_out/r1q; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe.txt 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err
rc=$?
tail -2 $o/gpu_tests.log; cat $o/lb1_probe.txt $o/n1.json
exit $rc
