#!/bin/bash
# r05d: the double-backward test, soft-forward stamps, order kernel A/B, bench kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "double_backward" > $OUT/tests.log 2>&1
STAMPS_FLAGS=0 KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so STAMPS_DUMP=$R/$OUT/stamps_0.npy \
  timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps_0.log 2>&1
timeout -k 10 120 python scripts/dev/param_ab.py 15 0 1 0 1 > $OUT/param_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
