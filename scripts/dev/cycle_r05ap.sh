#!/bin/bash
# r05ap: soft backward shard selection unrolled + persistent grid 3 (default) against 4 / 5
# workgroups per CU (dev param 27); the loss with every thread's loads in flight: GPU suite,
# param_ab combos alternated, short bench line + kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05ap; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/dev/param_ab.py combo 27=3 27=4 27=3 27=4 27=3 27=5 27=3 27=4 27=3 27=5 > $OUT/ab.txt 2>&1
grep dibr $OUT/ab.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/cfg3.json 2> $OUT/cfg3.err
python -c "import json;d=json.load(open('$OUT/cfg3.json'));print(d['value'],d['ms_per_step'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
