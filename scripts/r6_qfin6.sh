# N-Queens finishing: waves take 64-parent groups from a kernel-wide counter (dyn) against
# static chunk dealing (static): tests, then N=17 same box
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_queens_finish.py tests/test_gpu_search.py tests/test_gpu_distributed.py -k "queens or finish or Queens" -x -q --timeout 120 --timeout-method thread > $out/tests_dyn.txt 2>&1 || { tail -20 $out/tests_dyn.txt; exit 1; }
tail -1 $out/tests_dyn.txt
bash scripts/ab_so.sh 3 dyn,static -- python bench.py --steps 5 --warmup 2 --extras nq17 | tee $out/ab6.txt
