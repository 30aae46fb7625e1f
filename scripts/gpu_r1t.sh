#!/bin/bash
# kernel timelines: ta014 N=1 solve and rank 0 of an 8-rank split solve
o=gpurun_out/r1t; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t1 -o run --output-format csv -- python scripts/profile_workload.py ta014 > $o/t1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/t8 -o run --output-format csv -- python scripts/profile_workload.py ta014_w8 > $o/t8.log 2>&1 &&
python scripts/timeline.py $o/t1 27 > $o/timeline_w1.txt && python scripts/timeline.py $o/t8 27 > $o/timeline_w8.txt
rc=$?
paste $o/timeline_w1.txt $o/timeline_w8.txt
exit $rc
