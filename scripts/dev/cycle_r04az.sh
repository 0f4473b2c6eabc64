#!/bin/bash
# round-end validation (after the gather batch change): headline bench (full line), its kernel stats, FETCH / WRITE passes, cfg5
set -e
OUT0=gpurun_out/r04az; mkdir -p $OUT0
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT0/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT0/smoke.log 2>&1
OUT=gpurun_out/r04az; mkdir -p $OUT; R=$(pwd)
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m > $OUT/cfg5.json 2> $OUT/cfg5.err
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
n=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'kl::' --output-format csv \
    -d $R/$OUT/pmcf$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2 > $R/$OUT/pmcf$n.log 2>&1
done
