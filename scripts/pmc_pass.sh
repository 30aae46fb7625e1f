#!/bin/bash
# usage: scripts/pmc_pass.sh <outdir> <workload> <counters...>
out=$1; shift; wl=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --stats -d "$out" -o run --output-format csv -- python scripts/profile_workload.py "$wl"
