#!/bin/bash
# Same-box A/B of module variants built by scripts/build_variant.py:
#   bash scripts/ab_so.sh <reps> <variant,variant,...> -- <command...>
# each run copies build/ab/<variant>/_tts_hip*.so over the package's module (a scratch
# tree on the GPU box), runs the command and prints its JSON ms_per_step or its output
set -o pipefail
reps=$1; vars=$2; shift 3
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
for r in $(seq 1 "$reps"); do
  for v in ${vars//,/ }; do
    cp "build/ab/$v/$(basename "$mod")" "$mod" || exit 1
    o=$(timeout -k 10 300 "$@" 2>/dev/null) || { echo "$v run $r: failed"; exit 1; }
    echo "$o" | python3 -c "import json,sys
lines=[l for l in sys.stdin.read().splitlines() if l.strip()]
try:
    d=json.loads(lines[-1])
    ex=' '.join(('%s %.3f s %.4f Gn/s' % (k, e['seconds'], e.get('nodes_per_s', 0) / 1e9)) for k, e in d.get('extras', {}).items() if 'seconds' in e)
    print('$v run $r: %.4f ms/step %s' % (d['ms_per_step'], ex))
except Exception:
    print('\n'.join('$v run $r: '+l for l in lines))"
  done
done
cp "build/ab/${vars%%,*}/$(basename "$mod")" "$mod"
