set -o pipefail
# same-box A/B of module variants: headline + the N-Queens extra, then the element-wise front probe under the B side
out=gpurun_out/r6ab2; mkdir -p $out
V=${VARIANTS:-base,prepad}
bash scripts/ab_so.sh ${REPS:-3} $V -- python bench.py --steps 100 --warmup 10 --extras nq17 | tee $out/ab_${V//,/_}.txt
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
B=${V##*,}
cp build/ab/$B/$(basename $mod) $mod
timeout -k 10 400 python -u -m pytest tests/test_gpu_front_probe.py tests/test_gpu_search.py tests/test_gpu_queens_finish.py -x -q --timeout 120 --timeout-method thread > $out/tests_$B.txt 2>&1; tail -1 $out/tests_$B.txt
cp build/ab/base/$(basename $mod) $mod
