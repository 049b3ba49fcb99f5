"""One timeline of the host's decode loop and the demod launches on the GPU.

    LDG_HOSTTRACE=h.txt LDG_SPANTABLE=s.txt python bench.py ...   # GPU box
    python tools/timeline.py h.txt s.txt [t_from_ms] [t_to_ms]

h.txt: bench.py's host events (ms from the timed region's start; header '# t0_ms').
s.txt: ldg_profile_span_table rows (start, end, issue on the device clock; issue on
the host's monotonic clock).  Demod spans are mapped onto the host clock through the
issue times (ldg_profile_enable's calibration), so both lists share one axis: ms
from the timed region's start.  Prints the merged events and, per demod launch, the
idle time before it (no demod executing) and whether the host had issued it by then.
"""
import sys

import numpy as np


def main(hpath, spath, lo=0.0, hi=1e18):
    t0 = None
    host = []
    for line in open(hpath):
        if line.startswith('# t0_ms'):
            t0 = float(line.split()[2])
            continue
        t, ev, n = line.split()
        host.append((float(t), 'host  %-8s %s' % (ev, n)))
    tab = np.loadtxt(spath, ndmin=2)
    # device ms -> host ms from the timed start: issue_host - t0 = issue_dev + shift
    shift = (tab[:, 3] - t0) - tab[:, 2]
    sh = float(np.median(shift))
    ev = list(host)
    prev_end = -1e18
    for i, (st, en, iss, _) in enumerate(tab):
        st, en, iss = st + sh, en + sh, iss + sh
        idle = st - prev_end
        late = iss - prev_end
        tag = ''
        if i and idle > 0.005:
            tag = '  idle %.3f ms before it%s' % (idle, ' (host-late %.3f)' % min(idle, late) if late > 0 else '')
        ev.append((iss, 'issue demod #%d' % i))
        ev.append((st, 'GPU   demod #%d start (%.3f ms)%s' % (i, en - st, tag)))
        ev.append((en, 'GPU   demod #%d end' % i))
        prev_end = max(prev_end, en)
    for t, what in sorted(ev):
        if lo <= t <= hi:
            print('%9.3f  %s' % (t, what))


if __name__ == '__main__':
    a = sys.argv[1:]
    main(a[0], a[1], *(float(x) for x in a[2:4]))
