#!/bin/bash
# r06s: the cost of the raster / soft launches' unused workgroups (grids cut by dev params 28 / 29)
set -e
R=$(pwd); OUT=gpurun_out/r06s; mkdir -p $OUT
timeout -k 10 300 python scripts/dev/grid_ab.py 28=2200 28=2600 28=3000 28=4096 29=2400 29=2800 29=3200 29=4000 28=3000,29=3200 > $OUT/grid_ab.txt 2>&1 || { tail $OUT/grid_ab.txt; exit 1; }
grep params $OUT/grid_ab.txt
