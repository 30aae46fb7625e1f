#!/bin/bash
# kernel timelines of ta014 (1 rank, rank 0 of 8) with local DFS steps 8 / 2 / 0
o=gpurun_out/r1x; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in 8 2 0; do
  TTS_LOCAL_STEPS=$L timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t1_$L -o run --output-format csv -- python scripts/profile_workload.py ta014 > $o/t1_$L.log 2>&1 || exit $?
  python scripts/timeline.py $o/t1_$L 45 > $o/timeline_w1_L$L.txt || exit $?
  TTS_LOCAL_STEPS=$L timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t8_$L -o run --output-format csv -- python scripts/profile_workload.py ta014_w8 > $o/t8_$L.log 2>&1 || exit $?
  python scripts/timeline.py $o/t8_$L 30 > $o/timeline_w8_L$L.txt || exit $?
done
rm -rf $o/t1_* $o/t8_*/
