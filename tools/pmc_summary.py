"""Summarise a tools/profile.sh run into profiles/: kernel stats + HBM traffic per launch.

    python tools/pmc_summary.py gpurun_out/prof/<tag> profiles/<round>_<tag>

Traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes), the gfx950
correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts half of the
bytes of wide coalesced reads, WRITE_SIZE counts 16-B stores exactly.  Both
are fabric-side L2 request counters (Infinity-Cache hits included), so the
figure is an upper estimate of DRAM bytes.
"""
import csv
import collections
import json
import os
import shutil
import sys


def main(src, dst_prefix):
    stats = os.path.join(src, 'trace', 'run_kernel_stats.csv')
    shutil.copy(stats, dst_prefix + '_kernel_stats.csv')
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.Counter()
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, 'run_counter_collection.csv')
        if not sub.startswith('pmc') or not os.path.exists(f):
            continue
        seen = collections.Counter()
        for r in csv.DictReader(open(f)):
            k, c = r['Kernel_Name'], r['Counter_Name']
            agg[k][c] += float(r['Counter_Value'])
            seen[(k, c)] += 1
        for (k, c), n in seen.items():
            launches[(k, c)] = n
    out = {}
    rows = []
    for k, cs in agg.items():
        nf = launches.get((k, 'FETCH_SIZE'), 0)
        nw = launches.get((k, 'WRITE_SIZE'), 0)
        if not nf or not nw:
            continue
        fetch = cs['FETCH_SIZE'] / nf * 1024.0
        write = cs['WRITE_SIZE'] / nw * 1024.0
        out[k.replace('ldg_k_', '')] = 2 * fetch + write
        rows.append((k, nf, fetch, write, 2 * fetch + write))
    json.dump({'unit': 'bytes per launch (2*FETCH_SIZE + WRITE_SIZE)', 'source': src, 'kernels': out},
              open(dst_prefix + '_pmc_traffic.json', 'w'), indent=1, sort_keys=True)
    with open(dst_prefix + '_pmc_traffic.txt', 'w') as fh:
        fh.write('%-32s %8s %14s %14s %14s\n' % ('kernel', 'launches', 'FETCH B', 'WRITE B', '2F+W B'))
        for r in sorted(rows, key=lambda r: -r[4]):
            fh.write('%-32s %8d %14.0f %14.0f %14.0f\n' % r)
    print(open(dst_prefix + '_pmc_traffic.txt').read())


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
