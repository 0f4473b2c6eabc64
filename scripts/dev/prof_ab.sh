#!/bin/bash
# rocprofv3 kernel stats of param_ab.py, one profiled run per parameter combo (development aid).
# usage: OUT=gpurun_out/x bash scripts/dev/prof_ab.sh 9=2 9=256 ...
set -e
OUT=${OUT:-gpurun_out/prof_ab}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/p_$c" -o run \
    -- python3 "$ROOT/scripts/dev/param_ab.py" combo "$c" > "$ROOT/$OUT/p_$c.log" 2>&1
done
