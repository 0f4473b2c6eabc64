#!/bin/bash
# r05r: sided_distance forward split over p2's tiles: GPU suite, sided A/B
set -e
R=$(pwd); OUT=gpurun_out/r05r; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/dev/sided_ab.py > $OUT/sided_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_sd -o run -- python3 $R/scripts/dev/sided_ab.py > $R/$OUT/sided_prof.log 2>&1
