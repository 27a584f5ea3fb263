"""Per kernel name: launches, and the longest launch (ms) -- for a rocprofv3
kernel trace of one configuration (e.g. the C3 index step)."""
import csv
import glob
import os
import sys
from collections import defaultdict

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    rows.extend(csv.DictReader(open(f)))
d = defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(d.items(), key=lambda kv: -max(kv[1])):
    print("%-70s n=%6d max_ms=%9.3f sum_ms=%9.3f" % (k, len(v), max(v), sum(v)))
