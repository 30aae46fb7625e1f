#!/bin/bash
# One GPU session of round 3: GPU tests, headline bench with extras, LB1 probes,
# 2 ranks on one GPU (gloo) with extras, -u 0 live-incumbent probe.
# Usage (on the GPU box): bash scripts/r3_gpu_session.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r3}
mkdir -p "$OUT"
step() { echo "== $(date +%T) $*" >> "$OUT/steps.txt"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gputests.log" 2>&1 || exit 11
step bench_n1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err" || exit 12
step lb1_probe
timeout -k 10 200 python scripts/lb1_probe.py > "$OUT/lb1_probe.txt" 2>&1 || exit 13
step bench_n2_shared
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --comm gloo --device 0 --steps 50 --warmup 5 \
  > "$OUT/bench_n2_shared.json" 2> "$OUT/bench_n2_shared.err" || exit 14
step live_best
timeout -k 10 300 python scripts/live_best_probe.py > "$OUT/live_best.txt" 2> "$OUT/live_best.err" || exit 15
step done
