#!/bin/bash
# r05ad: soft backward hash with 2 / 4 copies per face slot (devlib/nc2: 256 slots x 2, devlib/nc4:
# 128 x 4) against 512 x 1: DIB-R fwd/bwd alternated, short cfg3 bench lines, soft tests per build
set -e
R=$(pwd); OUT=gpurun_out/r05ad; mkdir -p $OUT
for v in nc2 nc4; do
  KAOLIN_HIP_LIB=$R/devlib/$v/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "dibr or soft" --timeout 120 --timeout-method thread > $OUT/tests_$v.log 2>&1
  tail -1 $OUT/tests_$v.log
done
for k in 1 2 3; do
  timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_nc1_$k.txt 2>&1
  for v in nc2 nc4; do
    KAOLIN_HIP_LIB=$R/devlib/$v/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_${v}_$k.txt 2>&1
  done
done
grep -H dibr $OUT/ab_*.txt
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_nc1_$k.json 2> $OUT/cfg3_nc1_$k.err
  for v in nc2 nc4; do
    KAOLIN_HIP_LIB=$R/devlib/$v/libkaolin_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_${v}_$k.json 2> $OUT/cfg3_${v}_$k.err
  done
done
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
