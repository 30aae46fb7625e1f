set -o pipefail
# wave priority by step (prio1) / by stack size (prio2) in the fixed-step local DFS: headline A/B,
# per-workgroup exits (lb_probe), ta021 at 1 and 3 engines
out=gpurun_out/r5prio; mkdir -p $out
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
bash scripts/ab_so.sh 3 base,prio1,prio2 -- python bench.py --steps 50 --warmup 10 --no-extras | tee $out/headline_ab.txt
for v in base prio1; do
  cp build/ab/$v/$(basename $mod) $mod
  timeout -k 10 120 python -u scripts/lb_probe.py 14 9,11,13 > $out/lb_$v.txt 2>&1 || { tail -20 $out/lb_$v.txt; cp build/ab/base/$(basename $mod) $mod; exit 1; }
  echo "== $v"; grep -E "window|exit p10|per-CU max|rank in CU" $out/lb_$v.txt
done
for v in base prio1 prio2; do
  cp build/ab/$v/$(basename $mod) $mod
  timeout -k 10 120 python -u scripts/regress.py 21:0 > $out/ta021_$v.txt 2>&1 || { tail -20 $out/ta021_$v.txt; cp build/ab/base/$(basename $mod) $mod; exit 1; }
  echo "== $v"; grep ta021 $out/ta021_$v.txt
done
cp build/ab/base/$(basename $mod) $mod
# LB2 active slots parity-split in LDS (lb2par = the package module): tests, then ta056 A/B
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_search.py -m gpu -k "lb2 or ta056" -x -q --timeout 120 --timeout-method thread > $out/lb2_tests.txt 2>&1 || { tail -20 $out/lb2_tests.txt; exit 1; }
tail -2 $out/lb2_tests.txt
bash scripts/ab_so.sh 2 base,lb2par -- python bench.py --steps 1 --warmup 1 --extras ta056 | tee $out/ta056_ab.txt
