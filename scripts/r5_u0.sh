set -o pipefail
out=gpurun_out/r5u0; mkdir -p $out
for dive in 0 32; do
  TTS_DIVE=$dive timeout -k 10 200 python -u scripts/live_best_probe.py > $out/u0_dive$dive.txt 2>&1 || { tail -20 $out/u0_dive$dive.txt; exit 1; }
  grep -v amdgpu.ids $out/u0_dive$dive.txt | tail -20
done
