#!/bin/bash
# r03 development cycle: selected GPU tests, a short bench line, rocprofv3 kernel stats of it.
# usage: TESTS='tests/x.py' TESTK='expr' OUT=gpurun_out/x bash scripts/dev/cycle_r03.sh
set -e
OUT=${OUT:-gpurun_out/r03}
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > "$OUT/tests.log" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra --no-p2m --steps 10 > "$ROOT/$OUT/prof_bench.log" 2>&1
if [ -n "$HOSTPROF" ]; then
  cd "$ROOT"
  timeout -k 10 240 python scripts/dev/host_profile.py 200 > "$OUT/host_profile.txt" 2>&1
fi
