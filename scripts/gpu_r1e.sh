#!/bin/bash
# speculation A/B at N=1, then 2 and 4 ranks sharing one GPU (gloo transfers, shm control plane)
set -o pipefail
o=gpurun_out/r1e; mkdir -p $o
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
TTS_SPECULATE=0 timeout -k 10 120 python bench.py --steps 100 --warmup 10 > $o/n1_spec0.json 2> $o/n1_spec0.err &&
TTS_SPECULATE=1 timeout -k 10 120 python bench.py --steps 100 --warmup 10 > $o/n1_spec1.json 2> $o/n1_spec1.err &&
timeout -k 10 180 $T --nproc-per-node 2 --master-port 29517 bench.py --gpus 2 --comm gloo --device 0 --steps 50 --warmup 5 > $o/n2_shared.json 2> $o/n2_shared.err &&
TTS_SHM_CONTROL=0 timeout -k 10 180 $T --nproc-per-node 2 --master-port 29518 bench.py --gpus 2 --comm gloo --device 0 --steps 50 --warmup 5 > $o/n2_shared_noshm.json 2> $o/n2_shared_noshm.err &&
timeout -k 10 180 $T --nproc-per-node 4 --master-port 29519 bench.py --gpus 4 --comm gloo --device 0 --steps 50 --warmup 5 > $o/n4_shared.json 2> $o/n4_shared.err
rc=$?
for f in $o/*.json; do echo "== $f"; cat $f; done
grep -h "last step" $o/*.err
exit $rc
