set -e
OUT=gpurun_out/r04ab; mkdir -p $OUT
for k in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m > $OUT/base$k.json 2> $OUT/base$k.err
BENCH_LOSS_SIDE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m > $OUT/side$k.json 2> $OUT/side$k.err
done
