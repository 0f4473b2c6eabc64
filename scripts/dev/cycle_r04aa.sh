set -e
OUT=gpurun_out/r04aa; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "soft or dibr or rasterize or cfg5 or compiled" > $OUT/tests.log 2>&1
timeout -k 10 200 python scripts/dev/param_ab.py combo 9=0 9=0 9=0 > $OUT/ab.log 2>&1
OUT=$OUT/pab bash scripts/dev/prof_ab.sh 9=0
