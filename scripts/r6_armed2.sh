set -o pipefail
# every rank's share (the N=W step is bounded by the slowest): armed three-level iterations x split point
out=gpurun_out/r6armed; mkdir -p $out
for cfg in "0 512" "1 512" "1 256" "1 128" "1 64"; do
set -- $cfg
echo "== TTS_ARMED_DEEP=$1 split_per_rank $2" | tee -a $out/all_ranks.txt
TTS_ARMED_DEEP=$1 timeout -k 10 150 python scripts/share_all_ranks.py 10 $2 2>/dev/null | tee -a $out/all_ranks.txt
done
