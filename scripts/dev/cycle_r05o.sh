#!/bin/bash
# r05o: validation + artifacts: GPU suite, smoke, full bench line, cfg5, kernel stats, FETCH / WRITE
# passes (profiles/pmc_traffic.json), SQ counter passes on the DIB-R kernels, A/B of the soft order
set -e
R=$(pwd); OUT=gpurun_out/r05o; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 160 python scripts/dev/param_ab.py combo 18=1 18=0 18=1 18=0 > $OUT/param_ab.log 2>&1
KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/order_stamps.py > $OUT/order_stamps.log 2>&1
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m > $OUT/cfg5.json 2> $OUT/cfg5.err
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
n=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'kl::' --output-format csv \
    -d $R/$OUT/pmcf$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2 > $R/$OUT/pmcf$n.log 2>&1
done
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "bin_word|countorder|soft_tile|gather2|raster_tile|dot2" --output-format csv \
    -d $R/$OUT/pmcs$n -o run -- python3 $R/scripts/dev/param_ab.py 9 0 > $R/$OUT/pmcs$n.log 2>&1
done
