#!/bin/bash
# fixed-capacity (capturable) mesh_to_spc: SPC tests + cfg4 timings
set -e
OUT=gpurun_out/r04al; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "mesh_to_spc or cfg4 or spc" > $OUT/tests.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 8 > $OUT/probe_new.txt 2>&1
