#!/usr/bin/env python3
"""Condense rocprofv3 output directories into one committed text summary:
  --kt DIR    kernel-trace --stats run: per-kernel calls / average / total / share
  --pmc DIR   a --pmc run: per-kernel average of every counter over its dispatches
  python tools/kt_summary.py OUT.txt --title "..." --kt gpurun_out/x/kt_cfg2 --pmc gpurun_out/x/sq_cfg2
"""
import argparse
import collections
import csv
import glob
import os


def short(name):
    return name.split('(')[0].replace('void ', '')


def kt_lines(d):
    f = glob.glob(os.path.join(d, '*kernel_stats.csv'))[0]
    rows = list(csv.DictReader(open(f)))
    out = [f'# rocprofv3 --kernel-trace --stats  ({d})',
           f'{"kernel":52s} {"calls":>6s} {"avg_us":>9s} {"total_us":>10s} {"pct":>6s}']
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
        out.append(f'{short(r["Name"])[:52]:52s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.2f} '
                   f'{float(r["TotalDurationNs"]) / 1e3:10.1f} {float(r["Percentage"]):6.2f}')
    return out


def pmc_lines(d):
    f = glob.glob(os.path.join(d, '*counter_collection.csv'))[0]
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = short(r['Kernel_Name'])
        per[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    out = [f'# rocprofv3 --pmc  ({d}): per-dispatch average (summed over XCDs / SEs)']
    for k, cs in per.items():
        n = len(disp[k])
        out.append(f'{k[:60]}  ({n} dispatches)')
        for c, v in sorted(cs.items()):
            out.append(f'    {c:28s} {v / n:16.1f}')
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out')
    ap.add_argument('--title', default='')
    ap.add_argument('--kt', action='append', default=[])
    ap.add_argument('--pmc', action='append', default=[])
    a = ap.parse_args()
    lines = [a.title] if a.title else []
    for d in a.kt:
        lines += kt_lines(d) + ['']
    for d in a.pmc:
        lines += pmc_lines(d) + ['']
    open(a.out, 'w').write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main()
