set -o pipefail
out=gpurun_out/r5bpcq; mkdir -p $out
for rep in 1 2; do for b in 6 5 4 8; do
  TTS_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 1 --warmup 0 --extras nq17 > $out/nq_$b.json 2>/dev/null || exit 1
  python3 -c "import json;e=json.load(open('$out/nq_$b.json'))['extras']['nq17'];print('nq17 blocks/CU $b', round(e['seconds']*1e3,2), 'ms')" | tee -a $out/nq.txt
done; done
