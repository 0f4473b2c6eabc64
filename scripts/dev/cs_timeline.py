"""Print the kernel timeline of the last call in a rocprofv3 kernel trace (calls split at gaps
> 300 us).  usage: python scripts/dev/cs_timeline.py <run_kernel_trace.csv>  (development aid)"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
groups = [[rows[0]]]
for a, b in zip(rows, rows[1:]):
    if int(b['Start_Timestamp']) - int(a['End_Timestamp']) > 300000:
        groups.append([])
    groups[-1].append(b)
g = groups[-1]
t0 = int(g[0]['Start_Timestamp'])
for r in g:
    s = (int(r['Start_Timestamp']) - t0) / 1e3
    e = (int(r['End_Timestamp']) - t0) / 1e3
    print(f"{s:8.1f} {e - s:7.1f} {r['Kernel_Name'][:90]}")
