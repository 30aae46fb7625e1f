set -o pipefail
# Round-6 record: smoke, every GPU test, the driver's bench command, kernel timelines and
# the rocprofv3 kernel stats of the headline solve (N=1 and rank 0 of an 8-way split)
out=${END_OUT:-gpurun_out/r6end}; mkdir -p $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_n1.json 2> $out/bench_n1.err || { tail -30 $out/bench_n1.err; exit 1; }
python3 -c "
import json;d=json.load(open('$out/bench_n1.json'))
print('headline', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G nodes/s')
for k,e in d.get('extras',{}).items(): print(k, {x: e.get(x) for x in ('seconds','nodes_per_s','golden_ok')})"
[ -n "$NO_TRACE" ] && exit 0
bash scripts/trace_pass.sh $out/trace ta014 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
python3 scripts/solve_timeline.py $out/trace 30 > $out/ta014_n1_timeline.txt && tail -12 $out/ta014_n1_timeline.txt
cp $(find $out/trace -name '*kernel_stats.csv' | head -1) $out/ta014_n1_kernel_stats.csv && rm -rf $out/trace
bash scripts/trace_pass.sh $out/trace8 ta014_w8 > $out/trace8.log 2>&1 || { tail -20 $out/trace8.log; exit 1; }
python3 scripts/solve_timeline.py $out/trace8 30 > $out/ta014_rank0_of_8_timeline.txt && tail -10 $out/ta014_rank0_of_8_timeline.txt
cp $(find $out/trace8 -name '*kernel_stats.csv' | head -1) $out/ta014_rank0_of_8_kernel_stats.csv && rm -rf $out/trace8
