#!/bin/bash
# r05k: r05j (never got a box) + unbanded item order A/B (dev 18), rotated soft slot lists (dev 19):
# placement, sibling-batched depth-first raytrace, p2m per-point pair queue: GPU suite, A/B, stats
set -e
R=$(pwd); OUT=gpurun_out/r05k; mkdir -p $OUT
rc=0; timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python scripts/dev/param_ab.py 18 0 2 3 0 2 3 > $OUT/param_ab18.log 2>&1
timeout -k 10 120 python scripts/dev/param_ab.py 19 0 1 0 1 > $OUT/param_ab19.log 2>&1
KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/order_stamps.py > $OUT/order_stamps.log 2>&1
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
timeout -k 10 300 python scripts/dev/p2m_ab.py 11=0 11=4 11=0 11=4 > $OUT/p2m_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_rt -o run -- python3 $R/scripts/dev/rt_ab.py > $R/$OUT/rt_prof.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
