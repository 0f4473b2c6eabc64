#!/bin/bash
# r05aj: owner searches in two LDS round trips (common.h owner64) instead of six: GPU suite, then
# DIB-R fwd/bwd, raytrace and short cfg3 / cfg5 lines against devlib/head (the previous commit)
set -e
R=$(pwd); OUT=gpurun_out/r05aj; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_new_$k.txt 2>&1
  KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 20 0 0 > $OUT/ab_head_$k.txt 2>&1
done
grep -H dibr $OUT/ab_*.txt
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_new.log 2>&1
KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_head.log 2>&1
grep -H "mode 0:" $OUT/rt_*.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_new_$k.json 2> $OUT/cfg3_new_$k.err
  KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_head_$k.json 2> $OUT/cfg3_head_$k.err
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_new_$k.json 2> $OUT/cfg5_new_$k.err
  KAOLIN_HIP_LIB=$R/devlib/head/libkaolin_hip.so timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_head_$k.json 2> $OUT/cfg5_head_$k.err
done
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
