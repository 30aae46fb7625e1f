# ta021 / ta056 extras at 3 vs 4 engines per GPU (transfer streams created on first use)
set -o pipefail
out=gpurun_out/r6qe; mkdir -p $out
for r in 1 2; do for s in 3 4; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --extra-streams $s --extras ta021,ta056 > $out/s34.json 2>/dev/null || { echo "s=$s failed"; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/s34.json'));e=d['extras']
print('streams $s: ta021', round(e['ta021']['seconds'],2), 's', e['ta021']['golden_ok'], '; ta056', round(e['ta056']['nodes_per_s']/1e9,4), 'G/s')" | tee -a $out/s34.txt
done; done
