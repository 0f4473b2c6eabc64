set -e
OUT=gpurun_out/r04z; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "soft or dibr or rasterize or cfg5" --deselect tests/test_gpu_parity.py::test_dibr_fused_tile_kernel_equals_two_kernel_path > $OUT/tests.log 2>&1
OUT=$OUT/pab bash scripts/dev/prof_ab.sh 9=0
