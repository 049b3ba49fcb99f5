"""Why the demod queue runs dry: host issue time vs GPU start of each demod.

    python tools/issue_lag.py gpurun_out/prof/<tag>/trace

Reads run_kernel_trace.csv and run_hip_api_trace.csv of
`rocprofv3 --kernel-trace --hip-runtime-trace` (same clock), joins them on the
correlation id, and for every ldg_k_demod after the first reports
  gap    = its start - the previous demod's end (the demod-idle time)
  late   = its host issue - the previous demod's end (> 0: the host issued it late)
  queued = its start - max(issue, previous end) (the GPU held it back)
so a gap splits into host lateness and GPU-side delay (a whole free CU needed).
"""
import csv
import os
import sys

import numpy as np


def main(d):
    kern = list(csv.DictReader(open(os.path.join(d, 'run_kernel_trace.csv'))))
    api = {}
    for r in csv.DictReader(open(os.path.join(d, 'run_hip_api_trace.csv'))):
        api[r['Correlation_Id']] = (int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function'])
    dem = []
    for r in kern:
        if r['Kernel_Name'].split('(')[0] != 'ldg_k_demod':
            continue
        a = api.get(r['Correlation_Id'])
        if a is None:
            continue
        dem.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), a[0]))
    dem.sort()
    gap, late, queued = [], [], []
    for p, c in zip(dem, dem[1:]):
        gap.append((c[0] - p[1]) / 1e3)
        late.append((c[2] - p[1]) / 1e3)
        queued.append((c[0] - max(c[2], p[1])) / 1e3)
    gap, late, queued = map(np.array, (gap, late, queued))
    print('%d demods; durations median %.1f us' % (len(dem), np.median([(e - s) / 1e3 for s, e, _ in dem])))
    for name, v in (('gap', gap), ('late', late), ('queued', queued)):
        print('%-7s median %8.1f  p10 %8.1f  p90 %8.1f  us' % (name, np.median(v), np.percentile(v, 10),
                                                              np.percentile(v, 90)))
    print('issued before the previous demod ended: %d of %d' % ((late < 0).sum(), len(late)))
    print('sum of gaps %.1f ms: host-late part %.1f ms, GPU-held part %.1f ms' % (
        gap[gap > 0].sum() / 1e3, np.clip(late, 0, None).sum() / 1e3, np.clip(queued, 0, None).sum() / 1e3))


if __name__ == '__main__':
    main(sys.argv[1])
