#!/bin/bash
# r02b: full GPU cycle + soft_tile_fwd counters + per-wave stamps
set -e
R=$(pwd)
bash scripts/gpu_cycle.sh
bash scripts/dev/probe_pmc.sh
cd $R
KAOLIN_HIP_LIB=$R/scripts/dev/_bin/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/stamps.py > gpurun_out/stamps.log 2>&1
