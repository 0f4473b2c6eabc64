#!/bin/bash
# gather batch 3: dibr tests + headline bench twice
set -e
OUT=gpurun_out/r04ax; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dibr or rasteriz or soft or gather or fused or tutorial" > $OUT/tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/bench1.json 2> $OUT/bench1.err
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/bench2.json 2> $OUT/bench2.err
