set -o pipefail
out=gpurun_out/r5f50; mkdir -p $out
timeout -k 10 300 python scripts/ab_env.py TTS_FRONT 1,0 1 -- python scripts/front50_ab.py 3 31,41,51 | tee $out/front50_ab.txt
bash scripts/ab_so.sh 3 base,fuseprio -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/fuseprio_ab.txt
