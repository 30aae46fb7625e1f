# N=17 at three engines: finishing depth 8 / 9 / 10 columns (same box)
set -o pipefail
out=gpurun_out/r6qfin; mkdir -p $out
for r in 1 2; do for k in 8 9 10; do
  echo "== TTS_QUEENS_FINISH=$k" | tee -a $out/qk3.txt
  TTS_QUEENS_FINISH=$k timeout -k 10 200 python -u scripts/queens_engines_probe.py 17 3:512:524288 2>/dev/null | grep "N=17" | tee -a $out/qk3.txt || exit 1
done; done
