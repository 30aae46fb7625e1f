#!/bin/bash
# PMC passes over fixed workloads: scripts/gpu_pmc.sh <out-dir> <workload>[@ENV=V,...] ...
# Two counter passes per workload (8 SQ counters each), each its own rocprofv3 run
# under a time limit; summaries via scripts/pmc_summary.py.
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"
for spec in "$@"; do
  wl="${spec%%@*}"; envs=""; [ "$spec" != "$wl" ] && envs="${spec#*@}"
  tag="$wl${envs:+_$(echo "$envs" | tr ',=' '__')}"
  mkdir -p "$out/$tag"
  for pass in 1 2; do
    ctrs=$([ $pass = 1 ] && echo "$P1" || echo "$P2")
    ( IFS=','; for e in $envs; do export "$e"; done
      timeout -s KILL 180 rocprofv3 --pmc $ctrs --kernel-trace --stats -d "$out/$tag/p$pass" -o run --output-format csv \
        -- python3 scripts/profile_workload.py "$wl" > "$out/$tag/p$pass.log" 2>&1 ) \
      || { echo "pass $pass of $tag failed"; tail -5 "$out/$tag/p$pass.log"; exit 1; }
  done
  python3 scripts/pmc_summary.py "$out/$tag" "${KFILTER:-pfsp_expand}" > "$out/$tag/summary.txt"
  for pass in 1 2; do  # keep the per-kernel stats, drop the raw traces (gpurun_out must stay small)
    find "$out/$tag/p$pass" -name "*kernel_stats.csv" -exec cp {} "$out/$tag/p${pass}_kernel_stats.csv" \; 2>/dev/null
    rm -rf "$out/$tag/p$pass"
  done
  echo "== $tag"; cat "$out/$tag/summary.txt"; grep -v "^W20\|amdgpu.ids" "$out/$tag/p1.log" | tail -2
done
