#!/bin/bash
# r05l: chip order kernel race fix (barrier before the histogram reads; r05k faulted at cfg5) and
# register cap walk, DFS raytrace without scratch arrays: GPU suite (stop on any failure), A/B, stats
set -e
R=$(pwd); OUT=gpurun_out/r05l; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/order_stamps.py > $OUT/order_stamps.log 2>&1
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
timeout -k 10 200 python scripts/dev/param_ab.py combo 18=0 18=2 18=2,1=5,3=512 18=2,0=4,1=5,2=1024,3=512 18=0 18=2 18=2,1=5,3=512 18=2,0=4,1=5,2=1024,3=512 > $OUT/param_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_rt -o run -- python3 $R/scripts/dev/rt_ab.py > $R/$OUT/rt_prof.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
