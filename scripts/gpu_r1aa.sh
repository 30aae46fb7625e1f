#!/bin/bash
# grid size (workgroups per CU) vs ta014 / ta008 / ta021 and the 8-rank estimate
o=gpurun_out/r1aa; mkdir -p $o
for b in 2 3 4 6 8; do
  TTS_BLOCKS_PER_CU=$b timeout -k 10 200 python -u scripts/lb1_probe.py > $o/lb1_probe_b$b.txt 2>&1 || exit $?
  TTS_BLOCKS_PER_CU=$b timeout -k 10 200 python -u scripts/scaling_probe.py --per-rank 512 --reps 10 > $o/scaling_b$b.txt 2>&1 || exit $?
done
for f in $o/*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
