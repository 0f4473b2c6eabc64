"""Print the top kernels of rocprofv3 --stats output dirs.  usage: kstats.py DIR [DIR ...]"""
import csv
import sys

for d in sys.argv[1:]:
    print('==', d)
    for r in list(csv.DictReader(open(d.rstrip('/') + '/run_kernel_stats.csv')))[:12]:
        print('  %-80s %6s %10.1f us' % (r['Name'][:80], r['Calls'], float(r['AverageNs']) / 1e3))
