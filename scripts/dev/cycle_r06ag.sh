#!/bin/bash
# r06ag: final validation of round 6's last tree (deftet walk at 8 waves per EU, the underflow-edge test):
# the whole GPU suite (devlib + RCCL children), smoke, FETCH / WRITE passes over the sub-line legs
# (-> profiles/pmc_traffic_sub.json), the default bench line, kernel stats of the step and of the legs
set -e
R=$(pwd); OUT=gpurun_out/r06ag; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
cd /tmp; export TMPDIR=/tmp
n=0
for grp in FETCH_SIZE WRITE_SIZE; do
  n=$((n + 1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'deftet_|cs_|sided_|BboxSrc|bbox_bin|countorder' --output-format csv \
    -d $R/$OUT/pmc_sub_$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-p2m --steps 4 --warmup 1 > $R/$OUT/pmc_sub_$n.log 2>&1
done
cd $R
python scripts/pmc_traffic.py $OUT/pmc_traffic_sub.json $OUT/pmc_sub_1 $OUT/pmc_sub_2 "r06ag: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py's extra legs (deftet, check_sign, cfg1 sided, _C soft mask), scripts/dev/cycle_r06ag.sh"
cp $OUT/pmc_traffic_sub.json profiles/pmc_traffic_sub.json
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));t=d['deftet'];print('bench',d['value'],d['ms_per_step'],d['mode'],d['roofline']['frac'],'p2m',d['p2m']['ms'],'csm',d['soft_mask_C']['ms'],'vox',d['cfg4']['voxelgrid']['ms'],'m2s',d['cfg4']['mesh_to_spc']['ms'],'rt',d['raytrace']['ms'],'deftet',t['ms'],t['fwd_ms'],t['value'],t['roofline']['frac'],t['roofline']['traffic'])"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_sub -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 > $R/$OUT/bench_prof_sub.json 2> $R/$OUT/bench_prof_sub.err
echo done
