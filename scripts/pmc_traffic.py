"""HBM traffic per dispatch from rocprofv3 --pmc passes -> profiles/pmc_traffic.json.

traffic = 2 * FETCH_SIZE + WRITE_SIZE (both reported in KiB).  FETCH_SIZE is doubled as
/opt/skills/guides/MI355X_MICROARCH.md prescribes for gfx950 (it tallies 128-B requests at
64 B); WRITE_SIZE is exact.  bench.py reads the file to fill roofline.traffic.

usage: python scripts/pmc_traffic.py OUT.json FETCH_PASS_DIR WRITE_PASS_DIR [label]
"""
import collections
import csv
import json
import sys


def per_dispatch(d, counter):
    acc = collections.defaultdict(float)
    ids = collections.defaultdict(set)
    for r in csv.DictReader(open(d + '/run_counter_collection.csv')):
        if r['Counter_Name'] != counter:
            continue
        acc[r['Kernel_Name']] += float(r['Counter_Value'])
        ids[r['Kernel_Name']].add(r['Dispatch_Id'])
    return {k: acc[k] / len(ids[k]) for k in acc}


def main():
    out, fdir, wdir = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ''
    fetch = per_dispatch(fdir, 'FETCH_SIZE')
    write = per_dispatch(wdir, 'WRITE_SIZE')
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        kernels[k] = {'fetch_kib': round(f, 1), 'write_kib': round(w, 1),
                      'hbm_bytes': round((2 * f + w) * 1024)}
    json.dump({'source': label or f'{fdir}, {wdir}', 'formula': '1024*(2*FETCH_SIZE + WRITE_SIZE) per dispatch',
               'kernels': kernels}, open(out, 'w'), indent=1)


if __name__ == '__main__':
    main()
