#!/bin/bash
# r05ao: the soft evaluation's hits in flight per lane at 4-row items (LDS-bound occupancy): U = 2
# (this build) against devlib/u3, devlib/u4: DIB-R fwd alternated, short cfg3 / cfg5 lines
set -e
R=$(pwd); OUT=gpurun_out/r05ao; mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_u2_$k.txt 2>&1
  for v in u3 u4; do
    KAOLIN_HIP_LIB=$R/devlib/$v/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_${v}_$k.txt 2>&1
  done
done
grep -H dibr $OUT/ab_*.txt
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_u2_$k.json 2> $OUT/cfg3_u2_$k.err
  KAOLIN_HIP_LIB=$R/devlib/u4/libkaolin_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_u4_$k.json 2> $OUT/cfg3_u4_$k.err
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_u2_$k.json 2> $OUT/cfg5_u2_$k.err
  KAOLIN_HIP_LIB=$R/devlib/u4/libkaolin_hip.so timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_u4_$k.json 2> $OUT/cfg5_u4_$k.err
done
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
