#!/bin/bash
# quick GPU check: selected tests (TESTS), then optional stamps dump
set -e
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread ${TESTS:-tests -m gpu} > gpurun_out/quick_tests.log 2>&1
if [ -n "$STAMPS" ]; then
  KAOLIN_HIP_LIB=$R/scripts/dev/_bin/stamps/libkaolin_hip.so STAMPS_DUMP=$R/gpurun_out/stamps.npy timeout -k 10 120 python scripts/dev/stamps.py > gpurun_out/stamps.log 2>&1
fi
