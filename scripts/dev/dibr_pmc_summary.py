"""Per-dispatch means of the SQ counter passes over the DIB-R kernels (scripts/dev/cycle_r05o.sh's
pmcs* dirs) -> a profile JSON, with per-wave VALU / SALU and the LDS bank-conflict and waiting shares
(development aid).  usage: python scripts/dev/dibr_pmc_summary.py OUT.json DIR [DIR ...] -- label"""
import collections
import csv
import json
import re
import sys


def main():
    args = sys.argv[1:]
    label = ''
    if '--' in args:
        i = args.index('--')
        label = ' '.join(args[i + 1:])
        args = args[:i]
    out, dirs = args[0], args[1:]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in dirs:
        for r in csv.DictReader(open(d + '/run_counter_collection.csv')):
            k = re.sub(r'\(.*', '', r['Kernel_Name'])
            acc[k][r['Counter_Name']] += float(r['Counter_Value'])
            ids[k][r['Counter_Name']].add(r['Dispatch_Id'])
    kernels = {}
    for k, cs in acc.items():
        m = {c: v / len(ids[k][c]) for c, v in cs.items()}
        w = m.get('SQ_WAVES', 0)
        if w:
            m['valu_per_wave'] = round(m.get('SQ_INSTS_VALU', 0) / w, 1)
            m['salu_per_wave'] = round(m.get('SQ_INSTS_SALU', 0) / w, 1)
        if m.get('SQ_LDS_IDX_ACTIVE'):
            m['lds_bank_conflict_share'] = round(m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE'], 3)
        if m.get('SQ_WAVE_CYCLES'):
            m['waiting_share'] = round(m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES'], 3)
        kernels[k] = m
    json.dump({'source': label, 'note': 'per-dispatch means; SQ cycle counters in quad-cycles', 'kernels': kernels},
              open(out, 'w'), indent=1)
    for k, m in kernels.items():
        print(f"{k[:60]:60s} waves {m.get('SQ_WAVES', 0):8.0f} valu/w {m.get('valu_per_wave', 0):7.1f} "
              f"salu/w {m.get('salu_per_wave', 0):7.1f} lds-conf {m.get('lds_bank_conflict_share', 0):.3f} "
              f"wait {m.get('waiting_share', 0):.3f}")


if __name__ == '__main__':
    main()
