"""One graph step's kernel timeline from a rocprofv3 kernel trace (development aid).
usage: python scripts/dev/timeline.py gpurun_out/<run>/prof/run_kernel_trace.csv [first_kernel_substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else 'raster_bin'
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if first in r['Kernel_Name']]
i0, i1 = idx[-3], idx[-2]
t0 = int(rows[i0]['Start_Timestamp'])
for r in rows[i0 - 2:i1 + 1]:
    s = (int(r['Start_Timestamp']) - t0) / 1e3
    e = (int(r['End_Timestamp']) - t0) / 1e3
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f}  q{r['Queue_Id']} {r['Kernel_Name'][:70]}")
