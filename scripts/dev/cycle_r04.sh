#!/bin/bash
# r04 development cycle on the GPU box: selected GPU tests, optional A/B probe, a short bench line,
# optional rocprofv3 kernel stats of it.  Every GPU step has its own time limit; the first failure
# ends the script.
# usage: OUT=gpurun_out/x TESTS='tests/a.py' TESTK='expr' AB='scripts/dev/gather_ab.py 0 p7=1' PROF=1 \
#        bash scripts/dev/cycle_r04.sh
set -e
OUT=${OUT:-gpurun_out/r04}
mkdir -p "$OUT"
ROOT=$(pwd)
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
    ${TESTK:+-k "$TESTK"} > "$OUT/tests.log" 2>&1
fi
if [ -n "$AB" ]; then
  timeout -k 10 240 python $AB > "$OUT/ab.log" 2>&1
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
if [ -n "$PROF" ]; then
  cd /tmp
  export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra --no-p2m --steps 10 > "$ROOT/$OUT/prof_bench.log" 2>&1
fi
