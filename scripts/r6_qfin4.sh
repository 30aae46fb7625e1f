# wave finishing defaults (448-node stacks, 9 columns): GPU suite and bench, then the
# same-box N=17 A/B against the previous default (register walk from 7 columns)
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
bash scripts/r6_check.sh || exit 1
for r in 1 2 3; do
  bash scripts/ab_so.sh 1 new -- python bench.py --steps 5 --warmup 2 --extras nq17 | tee -a $out/ab4.txt || exit 1
  TTS_QUEENS_FINISH=7 bash scripts/ab_so.sh 1 reg,new -- python bench.py --steps 5 --warmup 2 --extras nq17 | sed 's/^/k7 /' | tee -a $out/ab4.txt || exit 1
done
