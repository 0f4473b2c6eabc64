#!/bin/bash
# r05q: hit-list raytrace with the scans folded into its count / write passes (eager and fixed),
# dot2 back to r04: GPU suite, raytrace A/B + kernel stats, bench line (sub-lines included)
set -e
R=$(pwd); OUT=gpurun_out/r05q; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_rt -o run -- python3 $R/scripts/dev/rt_ab.py > $R/$OUT/rt_prof.log 2>&1
