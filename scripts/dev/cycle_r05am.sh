#!/bin/bash
# r05am: gather lane model with per-round balancing
set -e
OUT=gpurun_out/r05am; mkdir -p $OUT
timeout -k 10 300 python scripts/dev/gather_sim.py > $OUT/gather_sim.log 2>&1
grep -v amdgpu $OUT/gather_sim.log
