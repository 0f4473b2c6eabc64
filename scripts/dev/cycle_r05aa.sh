#!/bin/bash
# r05aa: soft backward with the next item's index and row data in flight (and 4-row soft items
# again): GPU suite, DIB-R fwd/bwd A/B against devlib/head (the previous commit, with dev param
# 20 = 1 for the same 4-row items), short cfg3 / cfg5 bench lines both ways
set -e
R=$(pwd); OUT=gpurun_out/r05aa; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 20 0 > $OUT/ab_new_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 1 > $OUT/ab_head_$k.txt 2>&1
done
grep -H dibr $OUT/ab_*.txt
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_new_$k.json 2> $OUT/cfg3_new_$k.err
  KAOLIN_DEV_PARAMS=20=1 KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_head_$k.json 2> $OUT/cfg3_head_$k.err
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_new_$k.json 2> $OUT/cfg5_new_$k.err
  KAOLIN_DEV_PARAMS=20=1 KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_head_$k.json 2> $OUT/cfg5_head_$k.err
done
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
