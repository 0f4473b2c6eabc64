#!/bin/bash
# dibr_backward A/B under dev bits: 0 | raster hash off (1<<25) | the per-face gather path (1<<21)
# | old per-face gather path (1<<21); then a rocprof pass of the product path's kernels
set -e
R=$(pwd)
OUT=${OUT:-gpurun_out/db_ab}
mkdir -p $OUT
timeout -k 10 120 python scripts/dev/gather_ab.py 0 0x2000000 0x200000 > $OUT/ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/scripts/dev/gather_ab.py 0 > $R/$OUT/prof.log 2>&1
