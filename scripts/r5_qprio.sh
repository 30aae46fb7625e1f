set -o pipefail
out=gpurun_out/r5qprio; mkdir -p $out
bash scripts/ab_so.sh 3 base,qprio -- python bench.py --steps 1 --warmup 0 --extras nq17 | tee $out/nq17_ab.txt
