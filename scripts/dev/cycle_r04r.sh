set -e
OUT=gpurun_out/r04r; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mesh_to_spc or cfg4 or octree or morton" > $OUT/tests.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 8 15=1 > $OUT/cfg4_k64.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 8 > $OUT/cfg4.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/m2s" -o run -- python3 "$ROOT/scripts/dev/cfg4_probe.py" 5 > "$ROOT/$OUT/m2s.log" 2>&1
