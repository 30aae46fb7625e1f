# Round-6 GPU check: the GPU test suite, then the driver's bench command (with extras).
set -o pipefail
out=gpurun_out/r6check; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_n1.json 2> $out/bench_n1.err && python3 -c "import json;d=json.load(open('$out/bench_n1.json'));e=d['extras'];print('N=1', round(d['ms_per_step'],4), 'ms; ta021', round(e['ta021']['seconds'],2), 's; ta056', round(e['ta056']['nodes_per_s']/1e9,4), 'G/s; nq17', round(e['nq17']['seconds']*1e3,1), 'ms')"
