set -o pipefail
# local-DFS step counts re-tuned under the step priority; per-instance table; PMC
out=gpurun_out/r5steps; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_front_probe.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/probe_tests.txt 2>&1 || { tail -20 $out/probe_tests.txt; exit 1; }
tail -1 $out/probe_tests.txt
timeout -k 10 400 python scripts/ab_env.py TTS_LOCAL_WIDE_STEPS 3,4,5 3 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/wide_steps.txt
timeout -k 10 300 python scripts/ab_env.py TTS_LOCAL_STEPS 4,5,6 2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/local_steps.txt
timeout -k 10 300 python scripts/ab_env.py TTS_LOCAL_NARROW_STEPS 4,6,8 1 -- python scripts/share_solve_probe.py 20 | tee $out/narrow_steps_share.txt
timeout -k 10 240 python -u scripts/regress.py > $out/table.txt 2>&1 || { tail -20 $out/table.txt; exit 1; }
grep -v amdgpu.ids $out/table.txt
timeout -k 10 300 python scripts/ab_env.py TTS_LOCAL_STEPS 4,6 1 -- python scripts/regress.py 21:0 | tee $out/ta021_steps.txt
KFILTER=pfsp_front bash scripts/gpu_pmc.sh r5steps/pmc ta021 ta014 && KFILTER=pfsp_expand bash scripts/gpu_pmc.sh r5steps/pmc ta056
