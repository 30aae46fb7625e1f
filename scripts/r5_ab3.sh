set -o pipefail
out=gpurun_out/r5ab3; mkdir -p $out
timeout -k 10 400 python scripts/ab_env.py TTS_DEEP_P3 8,4,16 2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/deep_p3.txt
timeout -k 10 400 python scripts/ab_env.py TTS_WIDE_LEVELS 1,2 2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/wide_levels.txt
timeout -k 10 200 python scripts/share_solve_probe.py 30 2>&1 | grep -v amdgpu.ids | tee $out/share.txt
timeout -k 10 300 python -u scripts/regress.py 2>&1 | grep -v amdgpu.ids | tee $out/table.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_front_probe.py tests/test_gpu_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
