#!/bin/bash
# r06x: the one-wave soft rows' walk two hits per iteration (default) against one (dev param 29 = 1)
set -e
R=$(pwd); OUT=gpurun_out/r06x; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -q -x -k "dibr or soft_mask or cfg3 or cfg5 or rasterize" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "soft_walk_pairs or soft_mask_C or soft_live" --timeout 200 --timeout-method thread > $OUT/tests_dev.log 2>&1 || { tail -30 $OUT/tests_dev.log; exit 1; }
tail -2 $OUT/tests_dev.log
timeout -k 10 200 python scripts/dev/param_ab.py 29 0 1 0 1 0 1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
grep params $OUT/ab.txt
timeout -k 10 200 python scripts/dev/csm_ab.py 29=0 29=1 > $OUT/csm_ab.txt 2>&1 || { tail $OUT/csm_ab.txt; exit 1; }
grep params $OUT/csm_ab.txt
