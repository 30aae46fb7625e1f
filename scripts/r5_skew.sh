set -o pipefail
out=gpurun_out/r5skew; mkdir -p $out
for v in ${SKEW_VARIANTS:-"X=0" "TTS_OVERLAP=0" "TTS_LOCAL_STEPS=4" "TTS_DEEP_LEVELS=2"}; do
  env $v timeout -k 10 200 python -u -m pytest "tests/test_gpu_distributed.py::test_gpu_skewed_start_is_balanced_through_device_staging" -m gpu -q -s --timeout 150 --timeout-method thread > $out/skew.log 2>&1; rc=$?
  echo "$v rc $rc $(grep 'per-rank tree' $out/skew.log)"
  [ $rc -le 1 ] || exit 1
done
