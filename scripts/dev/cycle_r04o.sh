set -e
OUT=gpurun_out/r04o; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mesh_to_spc or p2m or cfg4 or cfg2 or raytrace or dibr_fused or soft_mask_compact" > $OUT/tests.log 2>&1
timeout -k 10 180 python scripts/dev/p2m_ab.py 11=1 11=0 11=1 11=0 > $OUT/p2m_ab.log 2>&1
timeout -k 10 180 python scripts/dev/cfg4_probe.py 5 > $OUT/cfg4.log 2>&1
OUT=$OUT/pab bash scripts/dev/prof_ab.sh 10=1 12=0 12=1 12=2 12=3 13=2 13=3
