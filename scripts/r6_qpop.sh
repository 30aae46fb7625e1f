# N-Queens finishing: one or two nodes per lane and pass (tests on both, then N=17 same box)
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
for v in pop2 pop1; do
  cp build/ab/$v/$(basename $mod) $mod || exit 1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_queens_finish.py tests/test_gpu_search.py -k "queens or finish" -x -q --timeout 120 --timeout-method thread > $out/tests_$v.txt 2>&1 || { tail -20 $out/tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 $out/tests_$v.txt)"
done
for v in pop1 pop2 pop1 pop2; do
  cp build/ab/$v/$(basename $mod) $mod || exit 1
  echo "== $v" | tee -a $out/qpop.txt
  timeout -k 10 200 python -u scripts/queens_engines_probe.py 17 2:512:524288,3:512:524288 2>/dev/null | grep "N=17" | tee -a $out/qpop.txt || exit 1
done
cp build/ab/pop1/$(basename $mod) $mod
