set -o pipefail
out=gpurun_out/r5bpc10; mkdir -p $out
[ -n "$SKIP_HEAD" ] || timeout -k 10 400 python scripts/ab_env.py TTS_BLOCKS_PER_CU 6,5,4 2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/bpc.txt
TTS_REGRESS_ENGINES=1,3 timeout -k 10 300 python scripts/ab_env.py TTS_BLOCKS_PER_CU 6,5 2 -- python scripts/regress.py 3:1,8:0,14:1 | tee $out/bpc_table.txt
timeout -k 10 300 python scripts/ab_env.py TTS_BLOCKS_PER_CU 6,5 1 -- python scripts/share_solve_probe.py 30 | tee $out/bpc_share.txt
