#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, kernel trace only) over a
# short bench run, restricted to the kaolin kernels.  Run on the MI355X box from the
# repo root; writes $OUT/pmc<N>/.  Summarise locally with scripts/pmc_summary.py.
set -e
OUT=${OUT:-gpurun_out}
ROOT=$(pwd)
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:---no-cpu-baseline --no-p2m --steps 5 --warmup 2}
cd /tmp
export TMPDIR=/tmp
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS}; do
  n=$((n + 1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'kl::' --output-format csv \
    -d "$ROOT/$OUT/pmc$n" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/pmc$n.log" 2>&1
done
