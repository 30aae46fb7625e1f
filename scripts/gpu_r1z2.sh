#!/bin/bash
# defaults after the local-DFS / two-level iteration work: tests, bench, probes
o=gpurun_out/r1z2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err &&
timeout -k 10 200 python -u scripts/scaling_probe.py --per-rank 512 > $o/scaling_probe.txt 2>&1 &&
timeout -k 10 300 python -u bench/suite.py --gpus 1 --limit 90 > $o/suite_n1.jsonl 2> $o/suite.err
rc=$?
tail -2 $o/gpu_tests.log; cat $o/n1.json $o/scaling_probe.txt $o/suite_n1.jsonl
exit $rc
