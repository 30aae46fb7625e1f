#!/bin/bash
# validation of the defaults: GPU tests, smoke, bench (N=1), 2-rank rehearsal on one GPU (gloo)
o=gpurun_out/r1al; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err &&
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 10 --comm gloo --device 0 > $o/n2_shared_gpu.json 2> $o/n2.err &&
timeout -k 10 150 python -u scripts/lb2_probe.py 12 > $o/lb2_default.txt 2>&1
rc=$?
tail -2 $o/gpu_tests.log; cat $o/smoke.log $o/n1.json $o/n2_shared_gpu.json; grep -v amdgpu $o/lb2_default.txt
exit $rc
