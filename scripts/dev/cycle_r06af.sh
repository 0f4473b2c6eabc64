#!/bin/bash
# r06af: deftet backward gather at 5 waves per EU: deftet GPU tests, the A/B
set -e
R=$(pwd); OUT=gpurun_out/r06af; mkdir -p $OUT
rc=0; timeout -k 10 300 python -u -m pytest tests/test_deftet.py -m gpu -q -x -rs --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 200 python scripts/dev/deftet_gather_ab.py > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
