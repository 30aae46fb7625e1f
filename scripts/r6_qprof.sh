set -o pipefail
out=gpurun_out/r6q; mkdir -p $out
bash scripts/trace_pass.sh $out/trace queens17 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
tail -2 $out/trace.log
cp $(find $out/trace -name '*kernel_stats.csv' | head -1) $out/nq17_kernel_stats.csv
python3 - <<'PY'
import csv, glob
f = max(glob.glob('gpurun_out/r6q/trace/**/*kernel_trace.csv', recursive=True), key=lambda x: len(x))
rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in csv.DictReader(open(f)))
# last solve: from the last load kernel
import collections
d = [(e - s) / 1e3 for s, e, n in rows if 'queens_expand' in n]
print('expand kernels', len(d), 'total ms', round(sum(d) / 1e3, 2))
h = collections.Counter(int(x // 20) * 20 for x in d)
print('duration histogram (us bucket: count)', sorted(h.items())[:30])
top = sorted(d)[-20:]
print('longest', [round(x, 1) for x in top])
span = (rows[-1][1] - rows[0][0]) / 1e6
print('trace span ms', round(span, 1))
PY
rm -rf $out/trace
