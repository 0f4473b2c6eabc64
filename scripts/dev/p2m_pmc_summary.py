"""Summarise scripts/dev/p2m_pmc.sh's output (gpurun_out/p2m_probe.log, gpurun_out/p2mpmc*/) into the
committed p2m counter profile bench.py reads (development aid).
usage: python scripts/dev/p2m_pmc_summary.py OUT.json [label]"""
import csv
import glob
import json
import re
import sys

counters = {}
ms = []
for f in sorted(glob.glob('gpurun_out/p2mpmc*/run_counter_collection.csv')):
    per = {}
    for r in csv.DictReader(open(f)):
        if 'p2m_fwd_kernel' not in r['Kernel_Name']:
            continue
        per.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
    for k, v in per.items():
        counters[k] = int(sum(v) / len(v))
for f in sorted(glob.glob('gpurun_out/p2mpmc*/run_kernel_trace.csv')):
    for r in csv.DictReader(open(f)):
        if 'p2m_fwd_kernel' in r['Kernel_Name']:
            ms.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
probe = open('gpurun_out/p2m_probe.log').read()
rows = re.findall(r'mode=morton .*?skipped=(\d+) evaluated=(\d+).*?point_pairs=(\d+)', probe)
skipped, evaluated, point_pairs = (int(x) for x in rows[-1])
flop = 64 * (counters['SQ_INSTS_VALU_ADD_F32'] + counters['SQ_INSTS_VALU_MUL_F32'] + 2 * counters['SQ_INSTS_VALU_FMA_F32'])
kms = sorted(ms)[len(ms) // 2]
out = {
    'source': (sys.argv[2] if len(sys.argv) > 2 else 'r05') + ': rocprofv3 --pmc passes over bench.py p2m leg '
              '(scripts/dev/p2m_pmc.sh), per p2m_fwd_kernel dispatch; probe: scripts/dev/p2m_probe.hip (KL_P2M_PROBE)',
    'workload': 'cfg2: 100k N(0,1) points x 20k N(0,1) faces, f32',
    'kernel_ms_under_pmc': round(kms, 4),
    'counters': counters,
    'wave_face_pairs': {'evaluated': evaluated, 'skipped': skipped,
                        'evaluated_fraction': round(evaluated / (evaluated + skipped), 4),
                        'point_face_pairs_passing_the_wave_test': evaluated * 64,
                        'point_face_pairs_evaluated': point_pairs if point_pairs else evaluated * 64,
                        'nominal_pairs': 100000 * 20000,
                        'note': 'evaluated: (wave, face) pairs the wave-level bound keeps; point_face_pairs_evaluated: '
                                'the per-point pair queue\'s passing pairs (r05), evaluated one per lane'},
    'executed_fp32_flop': flop,
    'executed_tflops': round(flop / (kms * 1e-3) / 1e12, 2),
    'valu_insts_per_evaluated_wave_face_pair': round(counters['SQ_INSTS_VALU'] / evaluated, 1),
    'valu_insts_per_evaluated_point_face_pair': round(counters['SQ_INSTS_VALU'] * 64 / max(point_pairs, 1), 1),
    'valu_issue_busy_est': round(counters['SQ_INSTS_VALU'] * 4 / (1024 * kms * 1e-3 * 2.4e9), 3),
    'wait_any_fraction_of_wave_cycles': round(counters['SQ_WAIT_ANY'] / counters['SQ_WAVE_CYCLES'], 3),
    'note': 'VALU busy = SQ_INSTS_VALU x 4 cycles (wave64 on a 16-lane SIMD) / (1024 SIMDs x kernel cycles at 2.4 GHz); '
            'executed FLOP counts ADD/MUL as 1 and FMA as 2 per lane',
}
json.dump(out, open(sys.argv[1], 'w'), indent=1)
print(json.dumps(out, indent=1))
