set -o pipefail
mkdir -p gpurun_out/r5ilog
timeout -k 10 120 python -u scripts/ilog_probe.py 14 1 3 19 > gpurun_out/r5ilog/ta014.txt 2>&1 || { tail -20 gpurun_out/r5ilog/ta014.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5ilog/ta014.txt
