#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel trace only) over a probe command,
# restricted to the kernels matching $REGEX.  Run on the MI355X box from the repo root.
# usage: OUT=gpurun_out/x REGEX='gather2' PROBE='scripts/dev/gather_ab.py 0' bash scripts/dev/pmc_probe.sh
set -e
OUT=${OUT:-gpurun_out/pmc_probe}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS}; do
  n=$((n + 1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${REGEX:-kl::}" --output-format csv \
    -d "$ROOT/$OUT/pmc$n" -o run -- python3 "$ROOT/"$PROBE > "$ROOT/$OUT/pmc$n.log" 2>&1
done
