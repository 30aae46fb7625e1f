set -o pipefail
# local-DFS finishing of small leftover stacks (TTS_LOCAL_FINISH): headline, rank shares, ta008 / ta021
out=gpurun_out/r6finish; mkdir -p $out
timeout -k 10 600 python scripts/ab_env.py TTS_LOCAL_FINISH 0,64,256,1024 3 -- python bench.py --steps 100 --warmup 10 --no-extras | tee $out/headline.txt
for v in 0 256; do echo "== TTS_LOCAL_FINISH=$v" | tee -a $out/share.txt; TTS_LOCAL_FINISH=$v timeout -k 10 150 python scripts/share_all_ranks.py 10 2>/dev/null | tee -a $out/share.txt; done
for v in 0 256; do echo "== TTS_LOCAL_FINISH=$v" | tee -a $out/regress.txt; TTS_LOCAL_FINISH=$v TTS_REGRESS_ENGINES=1,3 timeout -k 10 250 python -u scripts/regress.py 8:0,21:0,3:1 2>/dev/null | tee -a $out/regress.txt; done
