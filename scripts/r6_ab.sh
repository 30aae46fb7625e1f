set -o pipefail
# same-box A/B of module variants (scripts/build_variant.py): headline, then ta008 / ta021 at 3 engines
out=gpurun_out/r6ab; mkdir -p $out
V=${VARIANTS:-base,remain}
bash scripts/ab_so.sh ${REPS:-4} $V -- python bench.py --steps 100 --warmup 10 --no-extras | tee $out/headline_${V//,/_}.txt
mod=$(ls dist_gpu_accelerated_tree_search_amd/_tts_hip*.so)
for v in ${V//,/ }; do
  cp build/ab/$v/$(basename $mod) $mod
  echo "== $v" | tee -a $out/regress_${V//,/_}.txt
  TTS_REGRESS_ENGINES=3 timeout -k 10 200 python -u scripts/regress.py ${ROWS:-8:0,21:0} 2>/dev/null | tee -a $out/regress_${V//,/_}.txt
done
cp build/ab/base/$(basename $mod) $mod
