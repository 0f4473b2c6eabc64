#!/bin/bash
# r06a: baseline of this round's boxes + the RCCL world-1 test + bench with the loss all_gather in the step
set -e
R=$(pwd); OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 200 --timeout-method thread > $OUT/rccl.log 2>&1 || { tail -40 $OUT/rccl.log; exit 1; }
tail -2 $OUT/rccl.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('plain',d['value'],d['ms_per_step'],d['mode'],d['p2m']['ms'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --collectives > $OUT/bench_coll.json 2> $OUT/bench_coll.err
python -c "import json;d=json.load(open('$OUT/bench_coll.json'));print('collectives',d['value'],d['ms_per_step'],d['mode'],d['process_group'],d['p2m']['ms'])"
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -3 $OUT/tests.log; exit $rc
