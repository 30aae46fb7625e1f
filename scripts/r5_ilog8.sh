set -o pipefail
out=${ILOG_OUT:-gpurun_out/r5ilog8}; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
cp build/ab/ilog/$(basename $mod) $mod
for w in 1 8; do
  timeout -k 10 120 python -u scripts/ilog_probe.py 14 1 3 19 $w > $out/ilog_w$w.txt 2>&1 || { cp build/ab/base/$(basename $mod) $mod; tail -20 $out/ilog_w$w.txt; exit 1; }
  grep -v amdgpu.ids $out/ilog_w$w.txt
done
cp build/ab/base/$(basename $mod) $mod
