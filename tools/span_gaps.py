"""Demod launch timeline from LDG_SPANDUMP (unprofiled bench run).

    LDG_SPANDUMP=gpurun_out/spans.txt python bench.py ...; python tools/span_gaps.py gpurun_out/spans.txt

Prints the demod-busy fraction of the timed region and the gaps between
consecutive demod launches (device wall clock), largest first.
"""
import sys

import numpy as np


def main(path):
    s = np.loadtxt(path, ndmin=2)
    s = s[np.argsort(s[:, 0])]
    dur = s[:, 1] - s[:, 0]
    gaps = s[1:, 0] - np.maximum.accumulate(s[:-1, 1])
    total = s[-1, 1] - s[0, 0]
    print('launches %d  region %.1f ms  demod busy %.1f ms (%.1f%%)  gaps %.1f ms' %
          (len(s), total, dur.sum(), 100 * dur.sum() / total, np.clip(gaps, 0, None).sum()))
    print('span ms: median %.3f  p10 %.3f  p90 %.3f' % tuple(np.percentile(dur, [50, 10, 90])))
    print('gap ms : median %.3f  p90 %.3f  max %.3f' % tuple(np.percentile(gaps, [50, 90, 100])))
    order = np.argsort(-gaps)[:15]
    print('largest gaps (after launch i: gap ms, span of i ms):')
    for i in sorted(order):
        print('  %4d  t=%8.2f  gap %7.3f  span %6.3f' % (i, s[i, 1], gaps[i], dur[i]))


if __name__ == '__main__':
    main(sys.argv[1])
