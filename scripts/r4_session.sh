#!/bin/bash
# Round-4 GPU session helper: scripts/r4_session.sh <out> <step>...
#   probe            pytest -m gpu -k front_probe
#   tests            full pytest -m gpu
#   ab:VAR=v1,v2[:reps]   headline A/B (bench.py --no-extras) over an env knob
#   bench            bench.py default (with extras)
#   ktrace:<wl>      kernel timeline (scripts/gpu_run.sh ktrace)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
for step in "$@"; do
  case "$step" in
    probe)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_front_probe.py -m gpu -x -v --timeout 300 \
        --timeout-method thread > "$out/probe_tests.log" 2>&1 || { tail -40 "$out/probe_tests.log"; exit 1; }
      tail -3 "$out/probe_tests.log" ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
      tail -3 "$out/gpu_tests.log" ;;
    ab:*)
      arg="${step#ab:}"; reps=3; [[ "$arg" == *:* ]] && { reps="${arg##*:}"; arg="${arg%:*}"; }
      var="${arg%%=*}"; vals="${arg#*=}"
      timeout -k 10 600 python -u scripts/ab_env.py "$var" "$vals" "$reps" -- python bench.py --steps 50 --warmup 10 \
        --no-extras > "$out/ab_$var.txt" 2>&1 || { tail -20 "$out/ab_$var.txt"; exit 1; }
      cat "$out/ab_$var.txt" ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$out/bench_n1.json" 2> "$out/bench_n1.err" \
        || { tail -20 "$out/bench_n1.err"; exit 1; }
      cat "$out/bench_n1.json" ;;
    ktrace:*)
      bash scripts/gpu_run.sh "${out#gpurun_out/}" "$step" || exit 1 ;;
    rccl)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$out/rccl_tests.log" 2>&1 || { tail -30 "$out/rccl_tests.log"; exit 1; }
      tail -3 "$out/rccl_tests.log" ;;
    shared2:*)  # shared2:<extras>: 2 ranks on one GPU (gloo), headline + extras, overlap on
      ex="${step#shared2:}"
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --comm gloo --device 0 --extras "$ex" \
        > "$out/bench_n2_shared.json" 2> "$out/bench_n2_shared.err" || { tail -20 "$out/bench_n2_shared.err"; exit 1; }
      cat "$out/bench_n2_shared.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[r4_session] all steps ok"
