#!/bin/bash
# p2m with staged reciprocals (qdiv): division self-check, p2m tests (incl. cfg2 full size), p2m timing
set -e
OUT=gpurun_out/r04as; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "qdiv or reciprocal or p2m or point_to_mesh or triangle_distance or cfg2" > $OUT/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 10 > $OUT/bench.json 2> $OUT/bench.err
