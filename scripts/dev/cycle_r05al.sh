#!/bin/bash
# r05al: the order kernel's segmented scans by DPP: GPU suite, order-kernel time A/B against
# devlib/head (rocprofv3 kernel stats over param_ab for each build)
set -e
R=$(pwd); OUT=gpurun_out/r05al; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 0 > $OUT/ab_new.txt 2>&1
KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 0 > $OUT/ab_head.txt 2>&1
grep -H dibr $OUT/ab_*.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_new -o run -- python3 $R/scripts/dev/param_ab.py 20 0 > $R/$OUT/prof_new.log 2>&1
KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_head -o run -- python3 $R/scripts/dev/param_ab.py 20 0 > $R/$OUT/prof_head.log 2>&1
