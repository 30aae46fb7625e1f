# The driver's bench command twice (ta056 extra at 4 engines), then the 2-rank one-GPU rehearsal
set -o pipefail
out=gpurun_out/r6fb; mkdir -p $out
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_$r.json 2> $out/bench_$r.err || { tail -20 $out/bench_$r.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/bench_$r.json'));e=d['extras']
print('run $r', round(d['ms_per_step'],4), 'ms; ta021', round(e['ta021']['seconds'],2), e['ta021']['golden_ok'], '; ta056', round(e['ta056']['nodes_per_s']/1e9,4), e['ta056']['engines_per_gpu'], 'engines; nq17', round(e['nq17']['seconds']*1e3,1), 'ms')"
done
N8OUT=$out WORLDS=2 bash scripts/r6_n8.sh
