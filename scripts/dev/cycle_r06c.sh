#!/bin/bash
# r06c: product library without dev controls + dev library: full GPU suite (devlib tests in the
# wrapper's child process), smoke, bench
set -e
R=$(pwd); OUT=gpurun_out/r06c; mkdir -p $OUT
rc=0; timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -15 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'],d['mode'],d['p2m']['ms'],d['cfg4']['mesh_to_spc']['roofline']['frac'],d['raytrace']['roofline']['frac'])"
