#!/bin/bash
o=gpurun_out/r1r; mkdir -p $o
timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe.txt 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err
rc=$?
cat $o/lb1_probe.txt $o/n1.json
exit $rc
