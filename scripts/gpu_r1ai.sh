#!/bin/bash
# bench repeatability after the PfspArgs layout change (3 runs of N=1)
o=gpurun_out/r1ai; mkdir -p $o
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $o/n1_a.json 2> $o/err_a &&
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $o/n1_b.json 2> $o/err_b &&
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $o/n1_c.json 2> $o/err_c
rc=$?
for f in a b c; do python -c "import json;d=json.load(open('$o/n1_$f.json'));print(d['ms_per_step'], d['value']/1e9)"; done
exit $rc
