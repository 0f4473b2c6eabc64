#!/bin/bash
# r05n: hit-list raytrace march (eager default), per-level fixed, soft walk appends four entries per
# step, order-kernel histogram stamp: GPU suite, fwd/bwd timing, stamps, raytrace A/B, bench stats
set -e
R=$(pwd); OUT=gpurun_out/r05n; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 160 python scripts/dev/param_ab.py combo 18=0 20=2 18=2 18=2,20=2 18=0 20=2 18=2 18=2,20=2 > $OUT/param_ab.log 2>&1
KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/order_stamps.py > $OUT/order_stamps.log 2>&1
STAMPS_FLAGS=0 KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so STAMPS_DUMP=$R/$OUT/stamps.npy timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps.log 2>&1
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
