set -o pipefail
out=gpurun_out/r5dyn2; mkdir -p $out
timeout -k 10 400 python -u -m pytest "tests/test_gpu_front_probe.py::test_front_probe_machine_buckets" "tests/test_gpu_front_probe.py::test_front_probe_fifty_jobs" tests/test_gpu_front_probe.py::test_front_probe_synthetic_machine_padding -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" $out/tests.log
for us in 0 30 100 300 2000; do
  TTS_DYN_US=$us timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-extras > $out/bench_$us.json 2> $out/bench_$us.err || { tail -20 $out/bench_$us.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/bench_$us.json'));print('dyn_us $us', round(d['ms_per_step'],4), 'ms', d['config']['tree'])"
done
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so); cp $mod /tmp/base.so; cp build/ab/ilog/$(basename $mod) $mod
for us in 0 300; do
  TTS_DYN_US=$us timeout -k 10 120 python -u scripts/ilog_probe.py 14 1 3 19 > $out/ilog_$us.txt 2>&1 || { tail -20 $out/ilog_$us.txt; cp /tmp/base.so $mod; exit 1; }
  grep -v amdgpu.ids $out/ilog_$us.txt
done
cp /tmp/base.so $mod
for dive in 0 32; do
  TTS_DIVE=$dive timeout -k 10 200 python -u scripts/live_best_probe.py --worlds 1,2 > $out/u0_dive$dive.txt 2>&1 || { tail -20 $out/u0_dive$dive.txt; exit 1; }
  grep -v amdgpu.ids $out/u0_dive$dive.txt | tail -12
done
