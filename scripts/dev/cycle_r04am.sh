#!/bin/bash
# one-launch loss (last-workgroup sum): loss + graph tests, headline bench twice, kernel stats
set -e
OUT=gpurun_out/r04am; mkdir -p $OUT
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "loss_dot2 or graph or fused" > $OUT/tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/bench1.json 2> $OUT/bench1.err
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/bench2.json 2> $OUT/bench2.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
