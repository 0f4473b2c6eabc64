#!/bin/bash
# r05x: two-level grid tickets (common.h grid_last) in dot2 and the raytrace passes: GPU suite,
# smoke, raytrace A/B, gather lane-utilisation model, short bench line + kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05x; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 200 python scripts/dev/rt_ab.py > $OUT/rt_ab.log 2>&1
grep "mode [0-9]*:" $OUT/rt_ab.log
timeout -k 10 300 python scripts/dev/gather_sim.py > $OUT/gather_sim.log 2>&1
grep -v amdgpu.ids $OUT/gather_sim.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
