#!/bin/bash
# local-DFS LB1 iterations: correctness (gpu tests), then A/B with TTS_LOCAL_STEPS=0
o=gpurun_out/r1w; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
TTS_LOCAL_STEPS=0 timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe_off.txt 2>&1 &&
timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe_on.txt 2>&1 &&
TTS_LOCAL_STEPS=4 timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe_4.txt 2>&1 &&
timeout -k 10 200 python -u scripts/scaling_probe.py --per-rank 512 > $o/scaling_probe_on.txt 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err
rc=$?
tail -3 $o/gpu_tests.log; cat $o/lb1_probe_*.txt $o/scaling_probe_*.txt $o/n1.json
exit $rc
