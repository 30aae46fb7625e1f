# N-Queens wave finishing: finishing depth (columns left) x stack size at N=17 (same box)
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
cp build/ab/q448/$(basename $mod) $mod || exit 1
TTS_QUEENS_FINISH=12 timeout -k 10 300 python -u -m pytest tests/test_gpu_queens_finish.py -x -q --timeout 120 --timeout-method thread > $out/tests_q448_k12.txt 2>&1 || { tail -20 $out/tests_q448_k12.txt; exit 1; }
tail -1 $out/tests_q448_k12.txt
for k in 9 10 11 12; do
  echo "== TTS_QUEENS_FINISH=$k" | tee -a $out/ab3.txt
  TTS_QUEENS_FINISH=$k bash scripts/ab_so.sh 2 q448,q640 -- python bench.py --steps 5 --warmup 2 --extras nq17 | tee -a $out/ab3.txt
done
