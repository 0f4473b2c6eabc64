#!/bin/bash
# r05ar: validation + artifacts: GPU suite, smoke, FETCH / WRITE passes -> pmc_traffic.json (read by
# the bench line), full bench line, cfg5, bench kernel stats, SQ passes on the DIB-R kernels
set -e
R=$(pwd); OUT=gpurun_out/r05ar; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
cd /tmp; export TMPDIR=/tmp
n=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'kl::' --output-format csv \
    -d $R/$OUT/pmcf$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2 > $R/$OUT/pmcf$n.log 2>&1
done
cd $R
python scripts/pmc_traffic.py $OUT/pmc_traffic.json $OUT/pmcf1 $OUT/pmcf2 "r05ar: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py (cfg3, 5 steps + 2 warm-up), scripts/dev/cycle_r05ar.sh"
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m > $OUT/cfg5.json 2> $OUT/cfg5.err
python -c "import json;d=json.load(open('$OUT/cfg5.json'));print(d['value'],d['ms_per_step'])"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "bin_word|countorder|soft_tile|gather2|raster_tile|dot2" --output-format csv \
    -d $R/$OUT/pmcs$n -o run -- python3 $R/scripts/dev/param_ab.py 9 0 > $R/$OUT/pmcs$n.log 2>&1
done
