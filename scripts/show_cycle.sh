#!/bin/bash
# Summarise the outputs of scripts/gpu_cycle.sh (run locally after gpurun merges them).
OUT=${OUT:-gpurun_out}
tail -3 "$OUT/gpu_tests.log" 2>/dev/null
tail -1 "$OUT/bench.log" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['ops']))" 2>/dev/null
python3 - "$OUT/prof/run_kernel_stats.csv" <<'PY' 2>/dev/null
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(r['Name'][:64].ljust(66), r['Calls'].rjust(5), '%9.1f us' % (float(r['AverageNs']) / 1e3), r['Percentage'][:5])
PY
