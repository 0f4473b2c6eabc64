#!/bin/bash
# soft-mask iteration: GPU parity tests, stamps (STAMP_FLAGS), short bench with rocprof stats
set -e
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_full_size.py} -m gpu > gpurun_out/soft_tests.log 2>&1
if [ "${STAMP_FLAGS:-0}" != none ]; then STAMP_FLAGS="${STAMP_FLAGS:-0}" bash scripts/dev/cycle_stamps.sh; fi
cd /tmp; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 10 > $R/gpurun_out/prof_bench.log 2>&1
