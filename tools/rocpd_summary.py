#!/usr/bin/env python3
"""Per-kernel summary (calls, average / total duration, VGPRs, LDS) of a rocprofv3 --kernel-trace
run written in its SQLite (rocpd) format:

  python tools/rocpd_summary.py gpurun_out/<dir>/run_results.db [top]
"""
import sqlite3
import sys


def main(db, top=25):
    c = sqlite3.connect(db)
    rows = c.execute('select name, count(*), avg(duration), sum(duration), max(vgpr_count), max(accum_vgpr_count), '
                     'max(lds_size) from kernels group by name order by sum(duration) desc').fetchall()
    tot = sum(r[3] for r in rows)
    print(f'{"kernel":60s} {"calls":>6s} {"avg_us":>9s} {"total_us":>10s} {"pct":>6s} {"vgpr":>5s} {"agpr":>5s} {"lds":>7s}')
    for name, n, avg, s, vg, ag, lds in rows[:top]:
        nm = name.split('(')[0].replace('void ', '')
        print(f'{nm[:60]:60s} {n:6d} {avg / 1e3:9.2f} {s / 1e3:10.1f} {100 * s / tot:6.2f} {vg:5d} {ag:5d} {lds:7d}')


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
