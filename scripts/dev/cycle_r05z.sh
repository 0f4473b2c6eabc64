#!/bin/bash
# r05z: cfg5 / cfg3 A/B of the soft forward defaults: this build, dev param 20 = 1 (4-row items),
# and the r05t build (devlib/oldtr: ST_EVAL_U = 4, 4-row items, the branchy transpose)
set -e
R=$(pwd); OUT=gpurun_out/r05z; mkdir -p $OUT
for k in 1 2; do
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_def_$k.json 2> $OUT/cfg5_def_$k.err
  KAOLIN_DEV_PARAMS=20=1 timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_p20_$k.json 2> $OUT/cfg5_p20_$k.err
  KAOLIN_HIP_LIB=$R/devlib/oldtr/libkaolin_hip.so timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_old_$k.json 2> $OUT/cfg5_old_$k.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_def_$k.json 2> $OUT/cfg3_def_$k.err
  KAOLIN_DEV_PARAMS=20=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_p20_$k.json 2> $OUT/cfg3_p20_$k.err
  KAOLIN_HIP_LIB=$R/devlib/oldtr/libkaolin_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_old_$k.json 2> $OUT/cfg3_old_$k.err
done
for f in $OUT/*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
