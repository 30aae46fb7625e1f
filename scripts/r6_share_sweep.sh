set -o pipefail
# rank-0 share of 1/2/4/8-way ta014 splits (scripts/share_solve_probe.py) under engine knobs
out=gpurun_out/r6share; mkdir -p $out
run() { echo "== $*" | tee -a $out/sweep.txt; env "$@" timeout -k 10 120 python scripts/share_solve_probe.py 20 2>/dev/null | tee -a $out/sweep.txt; }
run TTS_X=0
run TTS_LOCAL_MIN=4096
run TTS_LOCAL_MIN=2048
run TTS_LOCAL_STEPS=8
run TTS_LOCAL_MIN=4096 TTS_LOCAL_STEPS=8
run TTS_LOCAL_MIN=2048 TTS_LOCAL_STEPS=8 TTS_LOCAL_WIDE_STEPS=8
run TTS_DEEP_LEVELS=4
# -u 0 from +inf: no dive vs the default dive at the bench's 2^19 window; ta008 at 2 / 4 ranks
timeout -k 10 300 python -u scripts/dive_probe.py --cases 14:1,8:0 --windows 0,4096 --shifts 2 --repeat 3 --max-parents 524288 2>/dev/null | tee $out/dive_w19.txt
for w in 0 4096; do timeout -k 10 400 python -u scripts/dive_probe.py --cases 8:0 --windows $w --shifts 2 --repeat 2 --worlds 2,4 --world-window $w 2>/dev/null | tee -a $out/dive_worlds.txt; done
