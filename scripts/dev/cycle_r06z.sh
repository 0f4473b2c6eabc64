#!/bin/bash
# r06z: final validation + artifacts of round 6: the whole GPU suite (devlib + RCCL children), smoke,
# FETCH / WRITE passes for the cfg3 step, the sub-lines and cfg5 (-> profiles/pmc_traffic*.json, read by
# the bench lines), bench lines (default, cfg5), kernel stats, SQ passes on the DIB-R kernels
set -e
R=$(pwd); OUT=gpurun_out/r06z; mkdir -p $OUT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
for i in 1 2; do timeout -k 10 100 python scripts/dev/rt_trace.py >> $OUT/rt.txt 2>&1; done; grep raytrace $OUT/rt.txt
cd /tmp; export TMPDIR=/tmp
pmc() {  # name, kernel regex, bench args
  local n=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    n=$((n + 1))
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$2" --output-format csv \
      -d $R/$OUT/pmc_$1_$n -o run -- python3 $R/bench.py $3 > $R/$OUT/pmc_$1_$n.log 2>&1
  done
}
pmc step 'kl::' "--no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2"
pmc sub 'deftet_|cs_|sided_|BboxSrc|bbox_bin|countorder' "--no-cpu-baseline --no-p2m --steps 4 --warmup 1"
pmc cfg5 'kl::' "--config cfg5 --no-cpu-baseline --no-extra --no-p2m --steps 3 --warmup 1"
cd $R
python scripts/pmc_traffic.py $OUT/pmc_traffic.json $OUT/pmc_step_1 $OUT/pmc_step_2 "r06z: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py (cfg3 step, 5 steps + 2 warm-up), scripts/dev/cycle_r06z.sh"
python scripts/pmc_traffic.py $OUT/pmc_traffic_sub.json $OUT/pmc_sub_1 $OUT/pmc_sub_2 "r06z: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py's extra legs (deftet, check_sign, cfg1 sided, _C soft mask), scripts/dev/cycle_r06z.sh"
python scripts/pmc_traffic.py $OUT/pmc_traffic_cfg5.json $OUT/pmc_cfg5_1 $OUT/pmc_cfg5_2 "r06z: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --config cfg5 (3 steps + 1 warm-up), scripts/dev/cycle_r06z.sh"
cp $OUT/pmc_traffic.json $OUT/pmc_traffic_sub.json $OUT/pmc_traffic_cfg5.json profiles/
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'],d['mode'],d['roofline']['frac'],d['roofline']['traffic'],'p2m',d['p2m']['ms'],'csm',d['soft_mask_C']['ms'],d['soft_mask_C']['roofline']['frac'],'vox',d['cfg4']['voxelgrid']['ms'],'m2s',d['cfg4']['mesh_to_spc']['ms'],'rt',d['raytrace']['ms'])"
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-extra --no-p2m > $OUT/cfg5.json 2> $OUT/cfg5.err
python -c "import json;d=json.load(open('$OUT/cfg5.json'));print('cfg5',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic'])"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 20 > $R/$OUT/bench_prof.json 2> $R/$OUT/bench_prof.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_sub -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 > $R/$OUT/bench_prof_sub.json 2> $R/$OUT/bench_prof_sub.err
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "bin_word|countorder|soft_tile|gather2|raster_tile|dot2" --output-format csv \
    -d $R/$OUT/pmcs$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2 > $R/$OUT/pmcs$n.log 2>&1
done
cd $R; python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r06z/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
# p2m face splits (dev param 28 = target workgroups: 10240 -> 20 splits of 1024 faces at cfg2)
timeout -k 10 200 python scripts/dev/p2m_ab.py 28=0 28=5000 28=16000 28=0 28=5000 28=16000 > $OUT/p2m_ab.txt 2>&1 || true
grep params $OUT/p2m_ab.txt || true
