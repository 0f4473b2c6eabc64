#!/bin/bash
# r05s: deftet tile walk in a Morton pixel order (+ the r05r sided split): GPU suite, A/B, deftet stats
set -e
R=$(pwd); OUT=gpurun_out/r05s; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/dev/sided_ab.py > $OUT/sided_ab.log 2>&1
timeout -k 10 120 python scripts/dev/deftet_ab.py > $OUT/deftet_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_dt -o run -- python3 $R/scripts/dev/deftet_ab.py > $R/$OUT/deftet_prof.log 2>&1
