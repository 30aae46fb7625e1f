set -o pipefail
out=gpurun_out/r5final; mkdir -p $out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_n1.json 2> $out/bench_n1.err || { tail -30 $out/bench_n1.err; exit 1; }
python3 -c "
import json;d=json.load(open('$out/bench_n1.json'))
print('headline', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G nodes/s')
for k,e in d.get('extras',{}).items(): print(k, {x: e.get(x) for x in ('seconds','nodes_per_s','golden_ok','tree')})"
bash scripts/trace_pass.sh $out/trace ta014 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
python3 scripts/solve_timeline.py $out/trace 40 > $out/ta014_n1_timeline.txt && rm -rf $out/trace && tail -14 $out/ta014_n1_timeline.txt
bash scripts/trace_pass.sh $out/trace8 ta014_w8 > $out/trace8.log 2>&1 || { tail -20 $out/trace8.log; exit 1; }
python3 scripts/solve_timeline.py $out/trace8 30 > $out/ta014_rank0_of_8_timeline.txt && rm -rf $out/trace8 && tail -10 $out/ta014_rank0_of_8_timeline.txt
