set -o pipefail
out=gpurun_out/r6ab3; mkdir -p $out
bash scripts/ab_so.sh 3 nopad,base -- python bench.py --steps 20 --warmup 5 | tee $out/ab.txt
