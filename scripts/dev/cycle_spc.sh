#!/bin/bash
# SPC / voxel tests + the cfg4 probe under rocprofv3 kernel stats (development aid)
set -e
OUT=${OUT:-gpurun_out/spc}
mkdir -p $OUT
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -k "spc or octree or cfg4 or raytrace or voxel or morton" > $OUT/tests.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 5 > $OUT/probe.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/c4 -o run -- python3 $R/scripts/dev/cfg4_probe.py 5 > $R/$OUT/probe_prof.txt 2>&1
