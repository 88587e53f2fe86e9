#!/usr/bin/env python3
"""Condense a tools/profile.sh run (gpurun_out/prof) into a committed summary:
per-kernel launch count / average duration (rocprofv3 --kernel-trace --stats) and the
per-dispatch average of every PMC counter collected in the separate --pmc passes.
FETCH_SIZE is reported raw and x2 (gfx950 tallies 128-B requests at 64 B:
MI355X_MICROARCH.md, HBM section); both in KB per dispatch.

  python tools/prof_summary.py gpurun_out/prof profiles/r01_cfg4_vamp.txt
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.split('(')[0]
    return name.replace('void ', '')


def main(src, dst):
    out = []
    stats = os.path.join(src, 'kt', 'kt_kernel_stats.csv')
    rows = list(csv.DictReader(open(stats)))
    out.append('# rocprofv3 --kernel-trace --stats  (bench.py --no-cpu-baseline; cfg4 VAMP)')
    out.append(f'{"kernel":44s} {"calls":>6s} {"avg_us":>9s} {"total_us":>10s} {"pct":>6s}')
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
        out.append(f'{short(r["Name"])[:44]:44s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.2f} '
                   f'{float(r["TotalDurationNs"]) / 1e3:10.1f} {float(r["Percentage"]):6.2f}')
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, '*', '*_counter_collection.csv'))):
        for r in csv.DictReader(open(f)):
            pmc[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
    out.append('')
    out.append('# PMC, average per dispatch (separate --pmc passes, bench.py --steps 1 --warmup 0)')
    for k in sorted(pmc):
        if not k.startswith('amp::'):
            continue
        cs = pmc[k]
        parts = []
        for c in sorted(cs):
            v = sum(cs[c]) / len(cs[c])
            if c == 'FETCH_SIZE':
                parts.append(f'FETCH_SIZE={v:.0f}KB (x2={2 * v:.0f}KB)')
            elif c == 'WRITE_SIZE':
                parts.append(f'WRITE_SIZE={v:.0f}KB')
            else:
                parts.append(f'{c}={v:.0f}')
        out.append(f'{k}: ' + ', '.join(parts))
    open(dst, 'w').write('\n'.join(out) + '\n')
    print('\n'.join(out))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
