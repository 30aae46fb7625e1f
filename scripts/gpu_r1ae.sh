#!/bin/bash
# ta056 LB2 (50x20): kernel time split + PMC passes on the LB2 expand kernel
o=gpurun_out/r1ae; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python scripts/profile_workload.py ta056 > $o/trace.log 2>&1 &&
timeout -s KILL 120 bash scripts/pmc_pass.sh $o/p1 ta056 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS > $o/p1.log 2>&1 &&
timeout -s KILL 120 bash scripts/pmc_pass.sh $o/p2 ta056 SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS FETCH_SIZE > $o/p2.log 2>&1
rc=$?
find $o -name "*stats.csv" | head; tail -3 $o/trace.log
exit $rc
