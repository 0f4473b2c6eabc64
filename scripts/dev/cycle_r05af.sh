#!/bin/bash
# r05af: rehearsal of the multi-rank bench flow on one GPU (KAOLIN_BENCH_SHARED_GPU=1: the ranks
# share the device, gloo instead of RCCL): 2 ranks with the p2m leg, 4 ranks headline only
set -e
R=$(pwd); OUT=gpurun_out/r05af; mkdir -p $OUT
KAOLIN_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --no-extra > $OUT/n2.json 2> $OUT/n2.err
tail -c 600 $OUT/n2.json; echo
KAOLIN_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 4 --steps 8 --warmup 2 --no-cpu-baseline --no-extra --no-p2m > $OUT/n4.json 2> $OUT/n4.err
tail -c 600 $OUT/n4.json; echo
