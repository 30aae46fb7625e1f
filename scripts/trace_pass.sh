#!/bin/bash
# usage: scripts/trace_pass.sh <outdir> <workload>   (kernel trace + stats, no counters)
out=$1; shift; wl=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv -- python scripts/profile_workload.py "$wl"
