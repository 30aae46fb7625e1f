set -o pipefail
# does a longer untimed warm-up change the headline (GPU clock ramp)?
out=gpurun_out/r6warm; mkdir -p $out
bash scripts/ab_args.sh $out/warm.txt 3 "--steps 20 --warmup 5 --no-extras" "--steps 20 --warmup 3000 --no-extras" "--steps 500 --warmup 5 --no-extras" || exit 1
cat $out/warm.txt
