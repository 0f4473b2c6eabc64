#!/bin/bash
# round-end validation part 1: the whole GPU suite and smoke
set -e
OUT=gpurun_out/r04ap; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
