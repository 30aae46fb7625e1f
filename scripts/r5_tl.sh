set -o pipefail
out=gpurun_out/r5tl; mkdir -p $out
bash scripts/trace_pass.sh $out/trace ta014 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
python3 scripts/solve_timeline.py $out/trace 30 > $out/ta014_n1_timeline.txt && rm -rf $out/trace && tail -12 $out/ta014_n1_timeline.txt
bash scripts/trace_pass.sh $out/trace8 ta014_w8 > $out/trace8.log 2>&1 || { tail -20 $out/trace8.log; exit 1; }
python3 scripts/solve_timeline.py $out/trace8 30 > $out/ta014_rank0_of_8_timeline.txt && rm -rf $out/trace8 && tail -10 $out/ta014_rank0_of_8_timeline.txt
