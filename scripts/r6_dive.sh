set -o pipefail
out=gpurun_out/r6dive; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dive.py -x -q --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
timeout -k 10 600 python -u scripts/dive_probe.py --cases 14:1,8:0,3:1 --windows 0,16,64,256,1024,4096 --shifts 2,257,258,259 --repeat 3 > $out/dive.txt 2> $out/dive.err || { tail -20 $out/dive.err; exit 1; }
cat $out/dive.txt
