"""Timeline summary of a rocprofv3 --kernel-trace run of bench.py.

    python tools/trace_timeline.py gpurun_out/prof/<tag>/run_kernel_trace.csv [--dump N]

After the capture synthesis: demod-active time, time with only other kernels
running, GPU-idle time, and per-kernel launch durations.
"""
import collections
import csv
import sys

import numpy as np


def main(path, dump=0):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0],
                     r['Queue_Id']))
    rows.sort()
    synth = [r[1] for r in rows if 'synth' in r[2]]
    if synth:
        rows = [r for r in rows if r[0] > max(synth)]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    n = (t1 - t0) // 1000 + 1
    dem = np.zeros(n, bool)
    other = np.zeros(n, bool)
    for s, e, k, q in rows:
        a, b = (s - t0) // 1000, (e - t0) // 1000 + 1
        (dem if k == 'ldg_k_demod' else other)[a:b] = True
    print('span %.1f ms: demod active %.1f, other only %.1f, idle %.1f' % (
        (t1 - t0) / 1e6, dem.sum() / 1e3, (other & ~dem).sum() / 1e3, (~dem & ~other).sum() / 1e3))
    dm = sorted((s, e) for s, e, k, q in rows if k == 'ldg_k_demod')
    if len(dm) > 2:
        gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(dm, dm[1:])]
        print('demod-to-demod gap: median %.1f us, max %.1f us' % (np.median(gaps), max(gaps)))
    d = collections.defaultdict(list)
    for s, e, k, q in rows:
        d[k].append((e - s) / 1e3)
    for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
        print('%-30s n=%5d median %8.1f us  sum %8.1f ms' % (k, len(v), np.median(v), sum(v) / 1e3))
    if dump:
        m = len(rows) // 2
        tm = rows[m][0]
        for s, e, k, q in rows[m:m + dump]:
            print('%9.1f %9.1f q%s %s' % ((s - tm) / 1e3, (e - tm) / 1e3, q, k))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == '--dump' else 0)
