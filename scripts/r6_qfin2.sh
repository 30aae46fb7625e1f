# N-Queens wave finishing: stack size / occupancy sweep at N=17 (same box), then the
# finishing depth (columns left) at two stack sizes
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
bash scripts/ab_so.sh 3 s448,s320,s256,s192,s448b4,s256b4 -- python bench.py --steps 5 --warmup 2 --extras nq17 | tee $out/ab2.txt
for k in 6 8 9; do
  echo "== TTS_QUEENS_FINISH=$k" | tee -a $out/ab2.txt
  TTS_QUEENS_FINISH=$k bash scripts/ab_so.sh 2 s448,s256 -- python bench.py --steps 5 --warmup 2 --extras nq17 | tee -a $out/ab2.txt
done
