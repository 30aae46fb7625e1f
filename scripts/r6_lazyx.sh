# Transfer streams created on first use (lazy) vs with the engine (eager): engines per GPU
# on N=17, then the driver's bench command, same box
set -o pipefail
out=gpurun_out/r6qe; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
for v in lazy eager; do
  cp build/ab/$v/$(basename $mod) $mod || exit 1
  echo "== $v" | tee -a $out/lazyx.txt
  timeout -k 10 200 python -u scripts/queens_engines_probe.py 17 2:512:524288,3:512:524288,4:512:524288 2>/dev/null | grep "N=17" | tee -a $out/lazyx.txt || exit 1
done
bash scripts/ab_so.sh 2 lazy,eager -- python bench.py --steps 20 --warmup 5 | tee -a $out/lazyx.txt
cp build/ab/lazy/$(basename $mod) $mod
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-streams 2 --extras ta021,ta056 > $out/lazy_s2.json 2>/dev/null && python3 -c "
import json;d=json.load(open('$out/lazy_s2.json'));e=d['extras']
print('lazy extra-streams 2: ta021', round(e['ta021']['seconds'],2), 's', e['ta021']['golden_ok'], '; ta056', round(e['ta056']['nodes_per_s']/1e9,4))" | tee -a $out/lazyx.txt
