#!/bin/bash
# mesh_to_spc by node ranks (static scan tiles, wave look-back): SPC tests, cfg4 timings, kernel
# trace, one counter pass over the node kernels
set -e
OUT=gpurun_out/r04ak; mkdir -p $OUT
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "mesh_to_spc or cfg4 or spc" > $OUT/tests.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 8 > $OUT/probe_new.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/scripts/dev/cfg4_probe.py 3 > $R/$OUT/probe_prof.txt 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-include-regex 'm2s_' --output-format csv -d $R/$OUT/pmc1 -o run -- python3 $R/scripts/dev/cfg4_probe.py 1 > $R/$OUT/pmc1.log 2>&1
