set -o pipefail
out=gpurun_out/r5mp021; mkdir -p $out
for rep in 1 2; do for mp in 262144 524288 1048576; do
  timeout -k 10 120 python bench.py --steps 1 --warmup 0 --extras ta021 --extra-max-parents $mp > $out/mp_$mp.json 2>/dev/null || exit 1
  python3 -c "import json;e=json.load(open('$out/mp_$mp.json'))['extras']['ta021'];print('max_parents $mp', round(e['seconds'],3), 's golden', e['golden_ok'])" | tee -a $out/mp.txt
done; done
