#!/bin/bash
# r06o: _C contract soft mask -- word binning + chip order kernel (soft bitmap only), both padding the first
# rows of the slot tensors; tests (product + dev library) and the A/B
set -e
R=$(pwd); OUT=gpurun_out/r06o; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "soft_mask" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
KAOLIN_NO_EXT=1 KAOLIN_HIP_LIB=$R/kaolin-windows_amd/kaolin/_lib/dev/libkaolin_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "soft_mask_C" --timeout 200 --timeout-method thread > $OUT/tests_dev.log 2>&1 || { tail -30 $OUT/tests_dev.log; exit 1; }
tail -2 $OUT/tests_dev.log
timeout -k 10 300 python scripts/dev/csm_ab.py 28=0 31=1 28=1,29=1 28=4,29=4 28=5,29=3 > $OUT/csm_ab.txt 2>&1 || { tail $OUT/csm_ab.txt; exit 1; }
grep params $OUT/csm_ab.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/scripts/dev/csm_ab.py 28=0 > $R/$OUT/prof.log 2>&1
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06o/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'kl::' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
