"""Kernel timeline of a rocprofv3 --kernel-trace csv: per dispatch, the gap
since the previous dispatch ended and its duration (us)."""
import csv
import glob
import os
import sys

path = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-12:] if len(sys.argv) < 3 else rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'][:48]:48s} gap {(s - (prev or s)) / 1e3:9.1f} us  dur {(e - s) / 1e3:9.1f} us")
    prev = e
