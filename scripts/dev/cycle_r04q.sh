set -e
OUT=gpurun_out/r04q; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_parity.py::test_dibr_fused_tile_kernel_equals_two_kernel_path > $OUT/tests.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 5 15=1 > $OUT/cfg4_k64.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 5 > $OUT/cfg4.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-p2m > $OUT/bench.json 2> $OUT/bench.err
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/m2s" -o run -- python3 "$ROOT/scripts/dev/cfg4_probe.py" 5 > "$ROOT/$OUT/m2s.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra --no-p2m --steps 10 > "$ROOT/$OUT/prof_bench.log" 2>&1
