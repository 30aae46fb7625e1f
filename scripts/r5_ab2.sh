set -o pipefail
out=gpurun_out/r5ab2; mkdir -p $out
timeout -k 10 400 python scripts/ab_env.py TTS_DEEP_LEVELS 2,3,4 2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/deep_levels.txt
timeout -k 10 400 python scripts/ab_env.py TTS_LOCAL_MIN 16384,4096,1024 2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/local_min.txt
TTS_REGRESS_ENGINES=1,3 timeout -k 10 400 python scripts/ab_env.py TTS_LOCAL_BACKLOG_STEPS 0,8 1 -- python scripts/regress.py 21:0,8:0 | tee $out/backlog_steps.txt
