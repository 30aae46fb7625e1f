# Wave-cooperative N-Queens finishing: tests under each stack size (96 forces the register
# fallback often), then a same-box A/B of N=17 against the per-lane register walk.
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
for v in s96 s448 base; do
  cp build/ab/$v/$(basename $mod) $mod || exit 1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_queens_finish.py tests/test_gpu_search.py -k "queens or finish" -x -q --timeout 120 --timeout-method thread > $out/tests_$v.txt 2>&1 || { echo "tests $v failed"; tail -20 $out/tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 $out/tests_$v.txt)"
done
bash scripts/ab_so.sh 3 base,reg,s448 -- python bench.py --steps 5 --warmup 2 --extras nq17 | tee $out/ab.txt
