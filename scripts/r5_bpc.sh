set -o pipefail
out=gpurun_out/r5bpc; mkdir -p $out
TTS_REGRESS_ENGINES=1,3 timeout -k 10 500 python scripts/ab_env.py TTS_BLOCKS_PER_CU 4,5 2 -- python scripts/regress.py 21:0 | tee $out/bpc_ta021.txt
