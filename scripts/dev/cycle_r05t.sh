#!/bin/bash
# r05t: sided and deftet A/B (the suite passed in r05s), deftet kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05t; mkdir -p $OUT
timeout -k 10 120 python scripts/dev/sided_ab.py > $OUT/sided_ab.log 2>&1
timeout -k 10 120 python scripts/dev/deftet_ab.py > $OUT/deftet_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_dt -o run -- python3 $R/scripts/dev/deftet_ab.py > $R/$OUT/deftet_prof.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_sd -o run -- python3 $R/scripts/dev/sided_ab.py > $R/$OUT/sided_prof.log 2>&1
