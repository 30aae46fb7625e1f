set -o pipefail
# three-level fused iterations while a rank split is pending (TTS_ARMED_DEEP): goldens, then rank shares
out=gpurun_out/r6armed; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_front_probe.py tests/test_gpu_distributed.py tests/test_gpu_dyn.py tests/test_gpu_learned.py -x -q --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for pr in 512 256 128; do
for d in 0 1; do echo "== TTS_ARMED_DEEP=$d split_per_rank $pr" | tee -a $out/share.txt; TTS_ARMED_DEEP=$d timeout -k 10 120 python scripts/share_solve_probe.py 20 $pr 2>/dev/null | tee -a $out/share.txt; done
done
