set -o pipefail
out=gpurun_out/r5dyn4; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dyn.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
grep -cE "PASSED" $out/tests.log
for us in 60 200; do
  TTS_LOCAL_STRIDE=1 timeout -k 10 120 python -u scripts/lb_probe.py 14 8,9,11 4 $us > $out/lb_dyn_$us.txt 2>&1 || { tail -20 $out/lb_dyn_$us.txt; exit 1; }
  grep -v amdgpu.ids $out/lb_dyn_$us.txt | grep -E "window|exit p10|dyn:|per-CU max"
done
for us in 0 40 100 300 1000; do
  TTS_DYN_US=$us timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-extras > $out/bench_$us.json 2> $out/bench_$us.err || { tail -20 $out/bench_$us.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/bench_$us.json'));print('dyn_us $us', round(d['ms_per_step'],4), 'ms', d['config']['tree'])"
done
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so); cp $mod /tmp/base.so; cp build/ab/ilog/$(basename $mod) $mod
for us in 100 1000; do
  TTS_DYN_US=$us timeout -k 10 120 python -u scripts/ilog_probe.py 14 1 3 19 > $out/ilog_$us.txt 2>&1 || { tail -20 $out/ilog_$us.txt; cp /tmp/base.so $mod; exit 1; }
  grep -v amdgpu.ids $out/ilog_$us.txt
done
cp /tmp/base.so $mod
