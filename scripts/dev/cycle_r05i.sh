#!/bin/bash
# r05i: gather spans removed, gather soft re-zeroing A/B (dev param 17), depth-first raytrace march:
# full GPU suite, A/B timings, raytrace kernel stats, bench kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05i; mkdir -p $OUT
rc=0; timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python scripts/dev/param_ab.py 17 0 1 3 0 1 3 > $OUT/param_ab.log 2>&1
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_rt -o run -- python3 $R/scripts/dev/rt_ab.py > $R/$OUT/rt_prof.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
