# N-Queens: next-to-last column counted in the lane (pl*), and a 2048-chunk window
# (2^19 parents) that frees 8 KB of LDS per workgroup (c2k*): N=17, same box
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
for v in pl448 plc2k504; do
  cp build/ab/$v/$(basename $mod) $mod || exit 1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_queens_finish.py tests/test_gpu_search.py -k "queens or finish" -x -q --timeout 120 --timeout-method thread > $out/tests_$v.txt 2>&1 || { tail -20 $out/tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 $out/tests_$v.txt)"
done
for k in 9 10; do
  echo "== TTS_QUEENS_FINISH=$k" | tee -a $out/ab5.txt
  TTS_QUEENS_FINISH=$k bash scripts/ab_so.sh 2 new,pl448,c2k448,c2k504,plc2k504 -- python bench.py --steps 5 --warmup 2 --extras nq17 | tee -a $out/ab5.txt
done
