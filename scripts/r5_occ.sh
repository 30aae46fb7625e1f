set -o pipefail
mkdir -p gpurun_out/r5occ
for b in 1 2 3 4 5 6; do
  TTS_BLOCKS_PER_CU=$b TTS_LOCAL_STRIDE=1 timeout -k 10 120 python -u scripts/lb_probe.py 14 11,13 4 > gpurun_out/r5occ/bpc$b.txt 2>&1 || { tail -20 gpurun_out/r5occ/bpc$b.txt; exit 1; }
  echo "== bpc $b"; grep -v amdgpu.ids gpurun_out/r5occ/bpc$b.txt | grep -E "window|per-CU|step0"
done
