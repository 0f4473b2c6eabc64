#!/bin/bash
# r06aa: deftet forward through counted cell lists (no sort, no host sync): deftet GPU tests (+ the devlib
# child), the A/B on the bench workload, FETCH / WRITE passes over the sub-line legs, a bench line
set -e
R=$(pwd); OUT=gpurun_out/r06aa; mkdir -p $OUT
rc=0; timeout -k 10 300 python -u -m pytest tests/test_deftet.py -m gpu -q -x -rs --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
rc=0; timeout -k 10 400 python -u -m pytest tests/test_gpu_devlib.py -m gpu -q -x -rs --timeout 380 --timeout-method thread > $OUT/devlib.log 2>&1 || rc=$?
tail -4 $OUT/devlib.log; [ $rc -eq 0 ] || exit $rc
KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 200 python scripts/dev/deftet_cells_ab.py > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
cd /tmp; export TMPDIR=/tmp
n=0
for grp in FETCH_SIZE WRITE_SIZE; do
  n=$((n + 1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'deftet_|cs_|sided_|BboxSrc|bbox_bin|countorder' --output-format csv \
    -d $R/$OUT/pmc_sub_$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-p2m --steps 4 --warmup 1 > $R/$OUT/pmc_sub_$n.log 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_sub -o run -- python3 $R/bench.py --no-cpu-baseline --no-p2m --steps 8 > $R/$OUT/bench_prof_sub.json 2> $R/$OUT/bench_prof_sub.err
cd $R
python scripts/pmc_traffic.py $OUT/pmc_traffic_sub.json $OUT/pmc_sub_1 $OUT/pmc_sub_2 "r06aa: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py's extra legs (deftet, check_sign, cfg1 sided, _C soft mask), scripts/dev/cycle_r06aa.sh"
cp $OUT/pmc_traffic_sub.json profiles/pmc_traffic_sub.json
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));t=d['deftet'];print('bench',d['value'],d['ms_per_step'],'deftet',t['ms'],t['fwd_ms'],t['value'],t['roofline']['frac'],t['roofline']['traffic'])"
