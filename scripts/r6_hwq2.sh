# The driver's bench command under 4 / 8 / 16 HIP hardware queues per process (the extras
# run 2-3 engines per GPU, each with a compute and a transfer stream), same box
set -o pipefail
out=gpurun_out/r6qe; mkdir -p $out
run() {
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 $3 > $out/hwq_b.json 2>/dev/null || { echo "q=$1 failed"; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/hwq_b.json'));e=d['extras']
print('q=$1 $2', round(d['ms_per_step'],4), 'ms; ta021', round(e['ta021']['seconds'],2), 's', e['ta021']['golden_ok'], '; ta056', round(e['ta056']['nodes_per_s']/1e9,4), 'G/s; nq17', round(e['nq17']['seconds']*1e3,1), 'ms', e['nq17']['golden_ok'])" | tee -a $out/hwq2.txt
}
for r in 1 2; do
  for q in 4 8 16; do run $q "" "" || exit 1; done
done
run 16 "extra-streams 4" "--extra-streams 4" || exit 1
