set -o pipefail
out=gpurun_out/r5t; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
bash scripts/ab_so.sh 2 base,lb2prio -- python bench.py --steps 1 --warmup 1 --extras ta056 | tee $out/ta056_prio.txt
for k in 2 4; do
  timeout -k 10 120 python bench.py --steps 1 --warmup 1 --extras ta056 --extra-streams $k > $out/ta056_s$k.json 2>/dev/null || exit 1
  python3 -c "import json;e=json.load(open('$out/ta056_s$k.json'))['extras']['ta056'];print('ta056 engines $k', round(e['nodes_per_s']/1e9,4), 'G nodes/s')" | tee -a $out/ta056_prio.txt
done
bash scripts/trace_pass.sh $out/trace ta014 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
python3 scripts/solve_timeline.py $out/trace 40 > $out/ta014_n1_timeline.txt && rm -rf $out/trace && cat $out/ta014_n1_timeline.txt | tail -22
cp build/ab/ilog/$(basename $mod) $mod
timeout -k 10 120 python -u scripts/ilog_probe.py 14 1 3 19 > $out/ilog.txt 2>&1; rc=$?
cp build/ab/base/$(basename $mod) $mod
grep -v amdgpu.ids $out/ilog.txt; exit $rc
