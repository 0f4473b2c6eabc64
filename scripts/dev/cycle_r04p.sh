set -e
OUT=gpurun_out/r04p; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mesh_to_spc or cfg4" > $OUT/tests.log 2>&1
timeout -k 10 180 python scripts/dev/p2m_ab.py 11=0 11=3 11=2 11=0 11=2 > $OUT/p2m_ab.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 5 14=1 > $OUT/cfg4_old.log 2>&1
KAOLIN_HIP_LIB=$ROOT/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/order_stamps.py > $OUT/stamps.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/m2s" -o run -- python3 "$ROOT/scripts/dev/cfg4_probe.py" 5 > "$ROOT/$OUT/m2s.log" 2>&1
