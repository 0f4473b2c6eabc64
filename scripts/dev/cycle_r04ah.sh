#!/bin/bash
# mesh_to_spc by node ranks: SPC tests, cfg4 timings against the sorted-pairs path (dev param 14=2),
# kernel stats of the new path
set -e
OUT=gpurun_out/r04ah; mkdir -p $OUT
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "mesh_to_spc or cfg4 or spc" > $OUT/tests.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 8 > $OUT/probe_new.txt 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 8 14=2 > $OUT/probe_old.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/scripts/dev/cfg4_probe.py 5 > $R/$OUT/probe_prof.txt 2>&1
