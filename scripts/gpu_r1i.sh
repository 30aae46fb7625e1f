#!/bin/bash
o=gpurun_out/r1i; mkdir -p $o
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 &&
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $o/n1.json 2> $o/n1.err &&
timeout -k 10 180 $T --nproc-per-node 2 --master-port 29531 bench.py --gpus 2 --comm gloo --device 0 --steps 100 --warmup 10 > $o/n2.json 2> $o/n2.err &&
timeout -k 10 180 $T --nproc-per-node 4 --master-port 29532 bench.py --gpus 4 --comm gloo --device 0 --steps 100 --warmup 10 > $o/n4.json 2> $o/n4.err
rc=$?
tail -3 $o/gpu_tests.log
for f in $o/n*.json; do echo "== $f"; grep metric $f | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['n_gpus'], r['ms_per_step'], r['value']/1e9)"; done
grep -h "last step" $o/*.err
exit $rc
