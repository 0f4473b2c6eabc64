set -e
OUT=gpurun_out/r04u; mkdir -p $OUT; ROOT=$(pwd)
KAOLIN_HIP_LIB=$ROOT/devlib/stamps/libkaolin_hip.so timeout -k 10 120 python scripts/dev/stamps.py > $OUT/stamps.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-p2m > $OUT/bench.json 2> $OUT/bench.err
