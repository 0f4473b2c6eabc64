#!/bin/bash
# r05ac: soft work items flagged live by the rasterizer: GPU suite, DIB-R fwd/bwd A/B (dev param
# 26 = 1: unflagged), short cfg3 / cfg5 bench lines both ways
set -e
R=$(pwd); OUT=gpurun_out/r05ac; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/dev/param_ab.py 26 0 1 0 1 0 1 > $OUT/ab.txt 2>&1
grep dibr $OUT/ab.txt
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_on_$k.json 2> $OUT/cfg3_on_$k.err
  KAOLIN_DEV_PARAMS=26=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3_off_$k.json 2> $OUT/cfg3_off_$k.err
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_on_$k.json 2> $OUT/cfg5_on_$k.err
  KAOLIN_DEV_PARAMS=26=1 timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 20 > $OUT/cfg5_off_$k.json 2> $OUT/cfg5_off_$k.err
done
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
