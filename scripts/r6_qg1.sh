# N-Queens finishing specialised for -g 1 (g1: 99 VGPRs, 4 waves per SIMD; g1w5: forced to
# 5 waves) against one loop for every -g (gany, the previous code): tests, then N=17
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
cp build/ab/g1w5/$(basename $mod) $mod || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_queens_finish.py tests/test_gpu_search.py -k "queens or finish" -x -q --timeout 120 --timeout-method thread > $out/tests_g1w5.txt 2>&1 || { tail -20 $out/tests_g1w5.txt; exit 1; }
tail -1 $out/tests_g1w5.txt
for v in gany g1 g1w5 gany g1 g1w5; do
  cp build/ab/$v/$(basename $mod) $mod || exit 1
  echo "== $v" | tee -a $out/qg1.txt
  timeout -k 10 200 python -u scripts/queens_engines_probe.py 17 3:512:524288 2>/dev/null | grep "N=17" | tee -a $out/qg1.txt || exit 1
done
cp build/ab/g1w5/$(basename $mod) $mod
