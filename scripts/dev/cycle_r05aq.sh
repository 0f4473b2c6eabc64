#!/bin/bash
# r05aq: the bench step's loss on a side stream beside the backward (default) against in line
# (KAOLIN_BENCH_LOSS_STREAM=0): short cfg3 / cfg5 lines alternated (eager and graph modes)
set -e
R=$(pwd); OUT=gpurun_out/r05aq; mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_side_$k.json 2> $OUT/cfg3_side_$k.err
  KAOLIN_BENCH_LOSS_STREAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_inline_$k.json 2> $OUT/cfg3_inline_$k.err
done
for k in 1 2; do
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_side_$k.json 2> $OUT/cfg5_side_$k.err
  KAOLIN_BENCH_LOSS_STREAM=0 timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_inline_$k.json 2> $OUT/cfg5_inline_$k.err
done
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],'eager',d['eager']['ms_per_step'],'graph',d['hip_graph']['ms_per_step'],d['graph_replay_check'])"; done
