set -o pipefail
mkdir -p gpurun_out/r2j
for mp in 262144 393216 458752 524288 786432 1048576; do
  timeout -k 10 120 python bench.py --steps 40 --warmup 5 --max-parents $mp > gpurun_out/r2j/mp_$mp.json 2>/dev/null || exit 1
  echo "max_parents $mp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2j/mp_$mp.json)"
done
