#!/bin/bash
# soft split A/B on the headline bench: default against all-non-empty-tiles-in-4-parts
set -e
export BENCH_PARAMS="- 0=1,2=4096 0=2,2=4096 - 0=1,2=4096 0=2,2=4096"
export OUT=gpurun_out/r04ag
bash scripts/dev/bench_params.sh
for f in $OUT/bench_*.json; do echo "$f $(cat $f)"; done | python -c "
import sys, json
for l in sys.stdin:
    f, j = l.split(' ', 1)
    d = json.loads(j)
    print(f, d['value'], d['ms_per_step'], d.get('mode'), d.get('hip_graph'))
"
