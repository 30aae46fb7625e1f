#!/bin/bash
# Scaling and instance-class launcher (ref pfsp/launch_scripts/mgpu_launch.sh,
# dmgpu_launch.sh: SLURM batches over Taillard classes with repetitions).
#
#   bench/run_scaling.sh headline [steps] [warmup]        bench.py at 1/2/4/8 GPUs (JSON lines)
#   bench/run_scaling.sh class -j 20 -g 20 -l 1 -D 8 -r 3 [-w 1] [-L 1] [-C 0]
#        every Taillard instance of that class through the CLI (multigpu.csv rows)
#
# One process per GPU over RCCL (torchrun, loopback rendezvous). Results go to
# ${OUT:-bench/results}/.
set -euo pipefail
cd "$(dirname "$0")/.."
. scripts/env-mi355x.sh >/dev/null
OUT=${OUT:-bench/results}
mkdir -p "$OUT"
NGPU_MAX=$(python -c "import torch; print(torch.cuda.device_count())")

run_n() {  # run_n <n> <args...>
  local n=$1; shift
  if [ "$n" -eq 1 ]; then
    python "$@"
  else
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $((29500 + RANDOM % 1000)) "$@"
  fi
}

instances_of_class() {  # Taillard ids for jobs x machines (ref mgpu_launch.sh ordering for 20x20)
  local j=$1 g=$2
  case "${j}x${g}" in
    20x5) seq 1 10 ;; 20x10) seq 11 20 ;; 20x20) echo 29 30 22 27 23 28 25 26 24 21 ;;
    50x5) seq 31 40 ;; 50x10) seq 41 50 ;; 50x20) echo 52 53 56 57 58 ;;  # 51 54 55 59 60 open
    100x5) seq 61 70 ;; 100x10) seq 71 80 ;; 100x20) echo 82 83 84 90 ;;  # 81 85-89 open
    200x10) seq 91 100 ;; 200x20) echo 101 103 104 105 106 107 108 109 110 ;;  # 102 open
    500x20) seq 111 120 ;;
    *) echo "unknown class ${j}x${g}" >&2; return 1 ;;
  esac
}

mode=${1:-headline}; shift || true
case "$mode" in
  headline)
    steps=${1:-100}; warmup=${2:-10}
    for n in 1 2 4 8; do
      [ "$n" -le "$NGPU_MAX" ] || continue
      run_n "$n" bench.py --gpus "$n" --steps "$steps" --warmup "$warmup" | tee -a "$OUT/headline.jsonl"
    done
    ;;
  class)
    J=20; G=20; LB=1; D=1; R=1; WS=1; L=1; C=0
    while getopts "j:g:l:D:r:w:L:C:" o; do
      case $o in j) J=$OPTARG ;; g) G=$OPTARG ;; l) LB=$OPTARG ;; D) D=$OPTARG ;; r) R=$OPTARG ;;
                 w) WS=$OPTARG ;; L) L=$OPTARG ;; C) C=$OPTARG ;; *) exit 2 ;; esac
    done
    for inst in $(instances_of_class "$J" "$G"); do
      for rep in $(seq 1 "$R"); do
        echo "== ta$(printf %03d "$inst") lb=$LB D=$D rep=$rep"
        if [ "$C" -eq 1 ] || [ "$D" -eq 1 ]; then
          python -m dist_gpu_accelerated_tree_search_amd pfsp -i "$inst" -l "$LB" -D "$D" -C "$C" -w "$WS" -L "$L" \
            --csv-dir "$OUT" --json "$OUT/runs.jsonl"
        else
          run_n "$D" -m dist_gpu_accelerated_tree_search_amd pfsp -i "$inst" -l "$LB" -D "$D" -w "$WS" -L "$L" \
            --csv-dir "$OUT" --json "$OUT/runs.jsonl"
        fi
      done
    done
    ;;
  *) echo "usage: $0 headline|class ..." >&2; exit 2 ;;
esac
