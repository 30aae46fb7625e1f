set -o pipefail
out=gpurun_out/r5learn; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
bash scripts/ab_so.sh 3 base,round -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/learn_ab.txt
