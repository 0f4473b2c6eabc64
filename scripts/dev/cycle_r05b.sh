#!/bin/bash
# r05: the new GPU tests (sharding emulation, double backward, m2s overflow, cfg3 full size), then
# the baseline soft-forward stamps, fwd/bwd A/B timing and the bench kernel stats
set -e
R=$(pwd); OUT=gpurun_out/r05b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sharding.py \
  "tests/test_gpu_parity.py::test_torch_reference_nodes_double_backward" \
  "tests/test_gpu_parity.py::test_compiled_nodes_refuse_double_backward" \
  "tests/test_gpu_parity.py::test_mesh_to_spc_pair_overflow_fallback" \
  "tests/test_gpu_parity.py::test_sided_vs_oracle_and_grad" \
  "tests/test_gpu_full_size.py::test_cfg3_full_size_vs_oracle" > $OUT/tests.log 2>&1
STAMPS_FLAGS=0 KAOLIN_HIP_LIB=$R/devlib/stamps/libkaolin_hip.so STAMPS_DUMP=$R/$OUT/stamps_0.npy \
  timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps_0.log 2>&1
timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/param_ab.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
