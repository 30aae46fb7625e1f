set -o pipefail
# 2 ranks sharing GPU 0 (gloo transfers), headline + ta021 extra with per-rank idle / load-balance clocks
out=${N2OUT:-gpurun_out/r5n2}; mkdir -p $out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --comm gloo --device 0 --extras ta021 > $out/bench_n2.json 2> $out/bench_n2.err || { tail -30 $out/bench_n2.err; exit 1; }
python3 -c "
import json;d=json.load(open('$out/bench_n2.json'))
e=d['extras']['ta021']
print('headline', round(d['ms_per_step'],4), 'ms; ta021', round(e['seconds'],3), 's golden', e.get('golden_ok'), 'rounds', e['rounds'])
for k in ('per_rank_tree','per_rank_t_idle','per_rank_t_load_bal','per_rank_t_termination','overlapped_rounds'): print(k, e.get(k))"
