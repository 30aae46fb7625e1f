set -o pipefail
# ta008 LB1_d -u 0 at 1 / 2 / 4 ranks sharing one GPU: does a shorter first replay (earlier incumbent exchange) cut the multi-rank tree?
out=gpurun_out/r6u0; mkdir -p $out
for e in "TTS_X=0" "TTS_LEARN_FIRST=0 TTS_ITERS_FIRST=6" "TTS_LEARN_FIRST=0 TTS_ITERS_FIRST=12"; do
  echo "== $e" | tee -a $out/ranks.txt
  env $e timeout -k 10 400 python -u scripts/dive_probe.py --cases 8:0 --windows 4096 --shifts 2 --repeat 2 --worlds 2,4 2>/dev/null | grep -v Gloo | tee -a $out/ranks.txt
done
