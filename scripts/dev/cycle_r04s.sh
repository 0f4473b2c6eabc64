set -e
OUT=gpurun_out/r04s; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mesh_to_spc or cfg4 or octree or morton" > $OUT/tests.log 2>&1
timeout -k 10 120 python scripts/dev/cfg4_probe.py 8 > $OUT/cfg4.log 2>&1
cd /tmp; export TMPDIR=/tmp
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "bin_word|countorder|soft_tile|gather2|raster_tile" --output-format csv \
    -d "$ROOT/$OUT/pmc$n" -o run -- python3 "$ROOT/scripts/dev/param_ab.py" combo 9=0 > "$ROOT/$OUT/pmc$n.log" 2>&1
done
