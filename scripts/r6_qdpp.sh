# N-Queens finishing prefix on a DPP wave scan (dpp) vs four ballots (ballot): the scan
# checked alone first, then the queens tests, then N=17 same box
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
timeout -k 10 30 ./build/bin/dpp_scan_check || exit 1
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
cp build/ab/dpp/$(basename $mod) $mod || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_queens_finish.py tests/test_gpu_search.py -k "queens or finish" -x -q --timeout 120 --timeout-method thread > $out/tests_dpp.txt 2>&1 || { tail -20 $out/tests_dpp.txt; exit 1; }
tail -1 $out/tests_dpp.txt
for v in ballot dpp ballot dpp; do
  cp build/ab/$v/$(basename $mod) $mod || exit 1
  echo "== $v" | tee -a $out/qdpp.txt
  timeout -k 10 200 python -u scripts/queens_engines_probe.py 17 3:512:524288,2:512:524288 2>/dev/null | grep "N=17" | tee -a $out/qdpp.txt || exit 1
done
cp build/ab/dpp/$(basename $mod) $mod
