#!/bin/bash
# r05ab: soft forward fill with 3 candidate chunks per wave and step (devlib/fc3) against 2 (this
# build): DIB-R fwd/bwd and short cfg3 / cfg5 bench lines, alternated
set -e
R=$(pwd); OUT=gpurun_out/r05ab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "dibr or soft" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
for k in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_fc2_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/devlib/fc3/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_fc3_$k.txt 2>&1
done
grep -H dibr $OUT/ab_*.txt
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_fc2_$k.json 2> $OUT/cfg3_fc2_$k.err
  KAOLIN_HIP_LIB=$R/devlib/fc3/libkaolin_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_fc3_$k.json 2> $OUT/cfg3_fc3_$k.err
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_fc2_$k.json 2> $OUT/cfg5_fc2_$k.err
  KAOLIN_HIP_LIB=$R/devlib/fc3/libkaolin_hip.so timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_fc3_$k.json 2> $OUT/cfg5_fc3_$k.err
done
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
