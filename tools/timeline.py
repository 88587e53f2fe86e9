#!/usr/bin/env python3
"""Print the last N kernels of a rocprofv3 kernel trace with gaps and durations (us).
  python tools/timeline.py gpurun_out/prof/kt/kt_kernel_trace.csv [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rs = rows[-int(sys.argv[2] if len(sys.argv) > 2 else 12):]
t0, prev = int(rs[0]['Start_Timestamp']), None
for r in rs:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1e3:9.1f} gap {((s - prev) / 1e3 if prev else 0):7.1f} dur {(e - s) / 1e3:8.1f} "
          f"{r['Kernel_Name'][:64]}")
    prev = e
