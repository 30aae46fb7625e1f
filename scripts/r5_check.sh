set -o pipefail
out=gpurun_out/r5check; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-extras > $out/bench_n1.json 2>/dev/null && python3 -c "import json;d=json.load(open('$out/bench_n1.json'));print('N=1', round(d['ms_per_step'],4), 'ms')"
bash scripts/r5_n2.sh
