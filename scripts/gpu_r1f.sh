#!/bin/bash
# kernel timelines of ta014 LB1 solves with and without speculative replays
o=gpurun_out/r1f; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TTS_SPECULATE=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/spec0 -o run --output-format csv -- python scripts/profile_workload.py ta014 > $o/spec0.log 2>&1 &&
TTS_SPECULATE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/spec1 -o run --output-format csv -- python scripts/profile_workload.py ta014 > $o/spec1.log 2>&1 &&
python scripts/timeline.py $o/spec0 62 > $o/spec0_timeline.txt && python scripts/timeline.py $o/spec1 62 > $o/spec1_timeline.txt
