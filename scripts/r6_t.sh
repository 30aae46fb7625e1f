# Round-6: GPU tests of the changed paths (dive, dyn, RCCL control, distributed, CLI spawn)
set -o pipefail
out=gpurun_out/r6t; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dive.py tests/test_gpu_dyn.py tests/test_gpu_rccl.py tests/test_gpu_distributed.py tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
