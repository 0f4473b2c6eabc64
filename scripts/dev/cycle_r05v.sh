#!/bin/bash
# r05v: soft forward defaults ST_EVAL_U = 2 and 2-row items at knum 30 (LDS for 5 workgroups per CU):
# GPU suite, DIB-R fwd/bwd (dev param 20 = 1: the 4-row items), short bench line + kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05v; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 160 python scripts/dev/param_ab.py 20 0 1 0 1 > $OUT/param_ab.txt 2>&1
grep dibr $OUT/param_ab.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
