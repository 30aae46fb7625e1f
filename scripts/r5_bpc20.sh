set -o pipefail
out=gpurun_out/r5bpc20; mkdir -p $out
TTS_REGRESS_ENGINES=1,3 timeout -k 10 400 python scripts/ab_env.py TTS_BLOCKS_PER_CU 4,3 1 -- python scripts/regress.py 21:0 | tee $out/ta021.txt
for b in 4 3; do
  TTS_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 1 --warmup 0 --extras ta056 > $out/ta056_$b.json 2>/dev/null || exit 1
  python3 -c "import json;e=json.load(open('$out/ta056_$b.json'))['extras']['ta056'];print('ta056 blocks/CU $b', round(e['nodes_per_s']/1e9,4))" | tee -a $out/ta056.txt
done
