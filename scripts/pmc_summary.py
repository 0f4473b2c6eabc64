"""Per-dispatch averages of rocprofv3 PMC counters over several --pmc passes.

usage: python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 ...
"""
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(d + '/run_counter_collection.csv')):
        k = r['Kernel_Name'][:60]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        cnt[k].add(r['Dispatch_Id'])
for k, v in agg.items():
    n = len(cnt[k])
    print(k, 'dispatches=%d' % n, ' '.join('%s=%.4g' % (c, x / n) for c, x in sorted(v.items())))
