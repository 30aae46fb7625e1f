set -o pipefail
out=gpurun_out/r5sweep; mkdir -p $out
timeout -k 10 200 python scripts/share_solve_probe.py 30 2>&1 | grep -v amdgpu.ids | tee $out/share.txt
TTS_REGRESS_ENGINES=1,2,3,4 timeout -k 10 300 python -u scripts/regress.py 3:1,8:0,14:1,21:0 2>&1 | grep -v amdgpu.ids | tee $out/table.txt
