set -o pipefail
# Rehearsal of the driver's multi-GPU bench on ONE GPU: N ranks (torchrun) sharing GPU 0,
# node transfers over gloo (RCCL refuses two ranks on one device), shm control plane,
# the headline plus every extra; small rings so N ranks fit one card.
out=${N8OUT:-gpurun_out/r6n8}; mkdir -p $out
for n in ${WORLDS:-4 8}; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 --comm gloo --device 0 --ring-gb 2 --extra-ring-gb 4 --extra-max-parents 131072 ${EXTRA_ARGS:-} > $out/bench_n$n.json 2> $out/bench_n$n.err || { tail -30 $out/bench_n$n.err; exit 1; }
python3 -c "
import json;d=json.load(open('$out/bench_n$n.json'))
print('N=$n headline', round(d['ms_per_step'],4), 'ms', d['config']['parallelism'], 'tree', d['config']['tree'])
for k,e in d['extras'].items(): print(' ', k, {x: e.get(x) for x in ('seconds','nodes_per_s','golden_ok','rounds','per_rank_tree','per_rank_t_idle','overlapped_rounds','error')})"
done
