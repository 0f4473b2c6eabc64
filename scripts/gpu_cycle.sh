#!/bin/bash
# One GPU verification cycle (run on the MI355X box from the repo root):
# GPU parity tests -> bench line -> rocprofv3 kernel stats of a short bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${TESTS_ARGS:-} > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 480 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra --no-p2m --steps 10 > "$ROOT/$OUT/prof_bench.log" 2>&1
