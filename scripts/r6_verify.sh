set -o pipefail
out=gpurun_out/r6verify; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_queens_finish.py tests/test_gpu_kernels.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for r in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_$r.json 2>/dev/null && python3 -c "
import json;d=json.load(open('$out/bench_$r.json'));e=d['extras']
print('run $r headline', round(d['ms_per_step'],4), 'ms; ta021', round(e['ta021']['seconds'],2), 's; ta056', round(e['ta056']['nodes_per_s']/1e9,4), 'G/s; nq17', round(e['nq17']['seconds']*1e3,1), 'ms')"; done
