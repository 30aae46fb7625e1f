# N=17 engines per process against the HIP hardware queues per process (GPU_MAX_HW_QUEUES)
set -o pipefail
out=gpurun_out/r6qe; mkdir -p $out
for q in 4 8 16; do
  echo "== GPU_MAX_HW_QUEUES=$q" | tee -a $out/hwq.txt
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u scripts/queens_engines_probe.py 17 2>/dev/null | grep "N=17" | tee -a $out/hwq.txt || exit 1
done
