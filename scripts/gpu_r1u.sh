#!/bin/bash
o=gpurun_out/r1u; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe.txt 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err &&
timeout -k 10 200 python -u scripts/scaling_probe.py --per-rank 512 > $o/scaling_probe.txt 2>&1
rc=$?
tail -3 $o/gpu_tests.log; cat $o/lb1_probe.txt $o/n1.json $o/scaling_probe.txt
exit $rc
