#!/usr/bin/env python3
"""Per-phase LDS counters from a tools/ubench/lds_phase_ubench.hip PMC run.

Every phase kernel is dispatched at reps = 1 and reps = 11; the counter difference / 10 is one
phase-iteration over the 256 workgroups (the init part cancels).  Scaled by T = 20 iterations it
is the phase's share of one cfg4 `vamp_persist` launch's SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS.

  python tools/lds_phase_summary.py gpurun_out/lds [profiles/r03_lds_phases.txt]
"""
import collections
import csv
import glob
import os
import re
import sys

NAMES = {1: 'r~ build (sX/sR reads, h2_store8)', 2: 'GEMM A-plane reads (one GEMM)',
         3: 'w store (GEMM1 epilogue, h2_store_acc)', 4: 'GEMM2 epilogue (sX/sR element r/w)',
         5: 'denoiser (denoise_sections_u, 16-QAM, M = 32)'}
PER_ITER = {1: 1, 2: 2, 3: 1, 4: 1, 5: 1}   # occurrences per engine iteration (two GEMMs)


def main(src, dst=None):
    disp = collections.defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(src, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r['Dispatch_Id'])
            disp[d][r['Counter_Name']] = disp[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
            names[d] = r['Kernel_Name']
    by = collections.defaultdict(list)
    for d in sorted(disp):
        m = re.search(r'kphase<(\d+), (\d+)>', names[d])
        if m:
            by[(int(m.group(1)), int(m.group(2)))].append(disp[d])
    out = ['# LDS counters per phase-iteration (256 workgroups), tools/ubench/lds_phase_ubench.hip',
           f'{"phase":46s} {"ldx pad":>7s} {"INSTS_LDS":>10s} {"BANK_CONFL":>10s} {"confl/inst":>10s} '
           f'{"x T=20 x uses":>14s}']
    tot = collections.Counter()
    for (ph, pad), runs in sorted(by.items()):
        if len(runs) < 2:
            continue
        a, b = runs[0], runs[1]
        ins = (b.get('SQ_INSTS_LDS', 0) - a.get('SQ_INSTS_LDS', 0)) / 10
        bc = (b.get('SQ_LDS_BANK_CONFLICT', 0) - a.get('SQ_LDS_BANK_CONFLICT', 0)) / 10
        launch = bc * 20 * PER_ITER[ph]
        tot[pad] += launch
        out.append(f'{NAMES[ph]:46s} {pad:7d} {ins:10.0f} {bc:10.0f} {bc / max(ins, 1):10.3f} {launch:14.0f}')
    for pad, v in sorted(tot.items()):
        out.append(f'sum of the measured phases per launch (ldx pad {pad}): {v:.0f} conflict cycles')
    text = '\n'.join(out) + '\n'
    print(text, end='')
    if dst:
        open(dst, 'w').write(text)


if __name__ == '__main__':
    main(*sys.argv[1:])
