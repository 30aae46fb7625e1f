set -o pipefail
out=gpurun_out/r5dyn021; mkdir -p $out
TTS_REGRESS_ENGINES=1,3 timeout -k 10 700 python scripts/ab_env.py TTS_DYN_US 0,300,1000 1 -- python scripts/regress.py 21:0,8:0 | tee $out/dyn_ta021.txt
