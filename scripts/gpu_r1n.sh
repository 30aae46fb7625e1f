#!/bin/bash
# kernel timeline of the headline solve + counters of the LB2 kernel on ta056
o=gpurun_out/r1n; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python scripts/profile_workload.py ta014 > $o/trace.log 2>&1 &&
python scripts/timeline.py $o/trace 30 > $o/timeline.txt &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES --kernel-trace --stats -d $o/pmc56 -o run --output-format csv -- python scripts/profile_workload.py ta056 > $o/pmc56.log 2>&1
rc=$?
cat $o/timeline.txt; tail -3 $o/pmc56.log
exit $rc
