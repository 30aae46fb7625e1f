#!/bin/bash
# Parameterised GPU-box session: scripts/gpu_run.sh <out-dir> <step>...
# steps: tests[:<k1>,<k2>...] (pytest -k "k1 or k2") | bench1 | bench2shared | smoke | lb2:<ta056 seconds>[@ENV=V,...] | trace:<workload>
# Every step runs under its own timeout; the session stops at the first failure.
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
for step in "$@"; do
  case "$step" in
    tests*)
      k="${step#tests}"; k="${k#:}"; k="${k//,/ or }"   # tests:a,b -> -k "a or b"
      echo "[gpu_run] pytest -m gpu ${k:+-k $k}"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${k:+-k "$k"} \
        > "$out/gpu_tests.log" 2>&1 || { tail -30 "$out/gpu_tests.log"; exit 1; }
      tail -3 "$out/gpu_tests.log" ;;
    bench1)
      timeout -k 10 180 python bench.py --steps 20 --warmup 5 > "$out/bench_n1.json" 2> "$out/bench_n1.err" \
        || { tail -20 "$out/bench_n1.err"; exit 1; }
      cat "$out/bench_n1.json" ;;
    bench2shared)
      timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --comm gloo --device 0 \
        > "$out/bench_n2_shared.json" 2> "$out/bench_n2_shared.err" || { tail -20 "$out/bench_n2_shared.err"; exit 1; }
      cat "$out/bench_n2_shared.json"; grep "last step" "$out/bench_n2_shared.err" ;;
    lb2:*)  # lb2:<seconds>[@ENV=V,...]
      arg="${step#lb2:}"; secs="${arg%%@*}"; envs=""; [ "$arg" != "$secs" ] && envs="${arg#*@}"
      tag="lb2_probe${envs:+_$(echo "$envs" | tr ',=' '__')}"
      ( IFS=','; for e in $envs; do export "$e"; done
        timeout -k 10 $((secs + 240)) python -u scripts/lb2_probe.py "$secs" 10 > "$out/$tag.txt" 2>&1 ) \
        || { tail -20 "$out/$tag.txt"; exit 1; }
      cat "$out/$tag.txt" ;;
    trace:*)  # trace:<workload>: kernel + memory-copy trace, copy/kernel overlap summary
      wl="${step#trace:}"
      ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
        timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace -d "$out/trace_$wl" -o run --output-format csv \
          -- python3 scripts/profile_workload.py "$wl" > "$out/trace_$wl.log" 2>&1 ) || { tail -20 "$out/trace_$wl.log"; exit 1; }
      python3 scripts/overlap.py "$out/trace_$wl" > "$out/overlap_$wl.txt"; rm -rf "$out/trace_$wl"
      grep -v "^W20\|^E20\|amdgpu.ids" "$out/trace_$wl.log" | tail -2; cat "$out/overlap_$wl.txt" ;;
    ktrace:*)  # ktrace:<workload>: kernel trace only, timeline of the last solve
      wl="${step#ktrace:}"
      ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
        timeout -k 10 150 rocprofv3 --kernel-trace -d "$out/ktrace_$wl" -o run --output-format csv \
          -- python3 scripts/profile_workload.py "$wl" > "$out/ktrace_$wl.log" 2>&1 ) || { tail -20 "$out/ktrace_$wl.log"; exit 1; }
      python3 scripts/solve_timeline.py "$out/ktrace_$wl" 80 > "$out/timeline_$wl.txt"; rm -rf "$out/ktrace_$wl"
      tail -3 "$out/timeline_$wl.txt" ;;
    py:*)  # py:<script.py>: any probe script, output to <out>/<script>.txt
      sc="${step#py:}"; nm=$(basename "$sc" .py)
      timeout -k 10 300 python -u "$sc" > "$out/$nm.txt" 2>&1 || { tail -20 "$out/$nm.txt"; exit 1; }
      grep -v "amdgpu.ids" "$out/$nm.txt" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
        || { tail -20 "$out/smoke.log"; exit 1; }
      tail -1 "$out/smoke.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_run] all steps ok"
