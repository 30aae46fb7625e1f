set -o pipefail
out=gpurun_out/r5steps2; mkdir -p $out
timeout -k 10 400 python scripts/ab_env.py TTS_LOCAL_STEPS 4,6,7,8 2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/local_steps.txt
timeout -k 10 300 python scripts/ab_env.py TTS_LOCAL_STEPS 6,8 1 -- python scripts/share_solve_probe.py 20 | tee $out/share.txt
timeout -k 10 300 python scripts/ab_env.py TTS_LOCAL_STEPS 6,8 1 -- python scripts/regress.py 21:0,8:0 | tee $out/ta021.txt
