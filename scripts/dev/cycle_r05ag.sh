#!/bin/bash
# r05ag: sweeps of the split parameters on this build (param_ab combos, alternated with the default):
# rasterizer heavy-tile split (dev params 4 = split_from, 5 = split_log2) and the soft split
# (0 = b4, 1 = b8, 2 = cap4, 3 = cap8)
set -e
R=$(pwd); OUT=gpurun_out/r05ag; mkdir -p $OUT
timeout -k 10 300 python scripts/dev/param_ab.py combo 9=0 4=4 9=0 4=6 9=0 5=1 9=0 5=3 9=0 4=4,5=3 9=0 > $OUT/rast.txt 2>&1
grep dibr $OUT/rast.txt
timeout -k 10 300 python scripts/dev/param_ab.py combo 9=0 0=4 9=0 1=5 9=0 2=512 9=0 3=256 9=0 1=5,3=256 9=0 0=6,1=7 9=0 > $OUT/soft.txt 2>&1
grep dibr $OUT/soft.txt
