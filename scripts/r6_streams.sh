set -o pipefail
# headline with 1 engine vs 2 / 3 engines on the GPU, the solve split in the graph between them
out=gpurun_out/r6streams; mkdir -p $out
bash scripts/ab_args.sh $out/headline.txt 3 "--steps 100 --warmup 10 --no-extras" "--steps 100 --warmup 10 --no-extras --streams 2 --stream-split 256" "--steps 100 --warmup 10 --no-extras --streams 2 --stream-split 512" "--steps 100 --warmup 10 --no-extras --streams 2 --stream-split 2048" "--steps 100 --warmup 10 --no-extras --streams 3 --stream-split 512" || exit 1
cat $out/headline.txt
