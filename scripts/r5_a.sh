set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || { tail -20 gpurun_out/r5a/bench.err; exit 1; }
cat gpurun_out/r5a/bench.json
TTS_LOCAL_STRIDE=1 timeout -k 10 200 python -u scripts/lb_probe.py 14 9,11,13,15 4 > gpurun_out/r5a/lb_stride.txt 2>&1 || { tail -20 gpurun_out/r5a/lb_stride.txt; exit 1; }
TTS_LOCAL_STRIDE=0 timeout -k 10 200 python -u scripts/lb_probe.py 14 9,11,13,15 4 > gpurun_out/r5a/lb_contig.txt 2>&1 || { tail -20 gpurun_out/r5a/lb_contig.txt; exit 1; }
cat gpurun_out/r5a/lb_stride.txt gpurun_out/r5a/lb_contig.txt | grep -v amdgpu.ids
