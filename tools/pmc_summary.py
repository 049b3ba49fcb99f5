"""Summarise tools/profile.sh runs into profiles/: kernel stats, HBM traffic and the
demod's issue / LDS / FP64 counters per launch.

    python tools/pmc_summary.py gpurun_out/prof/<tag> profiles/<round>_<tag> [gpurun_out/prof/<tag>sq ...]
    (then copy <prefix>_pmc_traffic.json to profiles/pmc_traffic.json for bench.py; the file
    carries the library's source hash, and bench.py uses it only for a run of that library)

Traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes), the gfx950
correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts half of the
bytes of wide coalesced reads, WRITE_SIZE counts 16-B stores exactly.  Both
are fabric-side L2 request counters (Infinity-Cache hits included), so the
figure is an upper estimate of DRAM bytes.

SQ counters are summed over the chip per dispatch; per launch means are
reported, and for the isolated demod (ldg_k_demod_iso, ldg_k_demod_iso_cut: the
shipped body) and the pipeline's ldg_k_demod the derived figures:
  issue mix       ACTIVE_INST_{LDS,VALU,ANY} and WAIT_{ANY,INST_ANY} / WAVE_CYCLES
  LDS array busy  LDS_IDX_ACTIVE / BUSY_CU_CYCLES (both per-CU cycle sums)
  bank conflicts  LDS_BANK_CONFLICT / LDS_IDX_ACTIVE (extra cycles per array cycle)
  FP64 executed   64 lanes * (2 FMA_F64 + MUL_F64 + ADD_F64) wave instructions
  VALU issue      INSTS_VALU * 4 cycles / (1024 SIMDs * GRBM_GUI_ACTIVE / 8 XCDs)
                  (a wave64 VALU instruction holds its SIMD 4 cycles; FP64 FMA included)
  LDS bytes       64 * (LDS_LOAD_BANDWIDTH + LDS_STORE_BANDWIDTH)
"""
import collections
import csv
import json
import os
import shutil
import sys


def counters(src):
    """{kernel: {counter: mean per dispatch}} over every pmc* pass under src."""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(collections.Counter)
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, 'run_counter_collection.csv')
        if not sub.startswith('pmc') or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k, c = r['Kernel_Name'], r['Counter_Name']
            agg[k][c] += float(r['Counter_Value'])
            n[k][c] += 1
    return {k: {c: v / n[k][c] for c, v in cs.items()} for k, cs in agg.items()}


def short(k):
    return k.replace('ldg_k_', '')


def derived(c):
    d = {}
    wc = c.get('SQ_WAVE_CYCLES')
    if wc:
        for key in ('SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_ANY',
                    'SQ_WAIT_INST_ANY', 'SQ_WAIT_INST_LDS'):
            if key in c:
                d[key.lower().replace('sq_', '') + '_per_wave_cycle'] = c[key] / wc
    if c.get('SQ_BUSY_CU_CYCLES') and 'SQ_LDS_IDX_ACTIVE' in c:
        d['lds_array_busy_frac'] = c['SQ_LDS_IDX_ACTIVE'] / c['SQ_BUSY_CU_CYCLES']
    if c.get('SQ_LDS_IDX_ACTIVE') and 'SQ_LDS_BANK_CONFLICT' in c:
        d['lds_conflict_cycles_per_active'] = c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']
    if 'SQ_INSTS_VALU_FMA_F64' in c:
        d['fp64_flops_per_launch'] = 64 * (2 * c['SQ_INSTS_VALU_FMA_F64'] + c.get('SQ_INSTS_VALU_MUL_F64', 0) +
                                           c.get('SQ_INSTS_VALU_ADD_F64', 0))
    if 'SQ_INSTS_VALU' in c and c.get('GRBM_GUI_ACTIVE'):
        d['valu_issue_frac'] = c['SQ_INSTS_VALU'] * 4 / (1024 * c['GRBM_GUI_ACTIVE'] / 8)
        d['gpu_cycles_per_xcd'] = c['GRBM_GUI_ACTIVE'] / 8
    if 'SQ_INSTS_VALU_FMA_F64' in c and 'SQ_INSTS_VALU' in c:
        d['fp64_share_of_valu_insts'] = (c['SQ_INSTS_VALU_FMA_F64'] + c.get('SQ_INSTS_VALU_MUL_F64', 0) +
                                         c.get('SQ_INSTS_VALU_ADD_F64', 0)) / c['SQ_INSTS_VALU']
    if 'SQ_INSTS_LDS_LOAD_BANDWIDTH' in c:
        d['lds_load_bytes'] = 64 * c['SQ_INSTS_LDS_LOAD_BANDWIDTH']
        d['lds_store_bytes'] = 64 * c.get('SQ_INSTS_LDS_STORE_BANDWIDTH', 0)
        d['lds_bytes'] = d['lds_load_bytes'] + d['lds_store_bytes']
    if 'SQ_INSTS_LDS' in c and 'SQ_INSTS_VALU' in c:
        d['lds_insts_per_valu_inst'] = c['SQ_INSTS_LDS'] / max(c['SQ_INSTS_VALU'], 1)
    return d


def lib_stamp():
    """The source hash libldgpu.so was built from (its build stamp, build.py source_hash), so
    bench.py attaches these counters only to a run of that same library."""
    stamp = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ld-decode_amd', 'ldgpu',
                         'libldgpu.so.sha256')
    return open(stamp).read().strip() if os.path.exists(stamp) else None


def main(src, dst_prefix, *sq_srcs):
    stats = os.path.join(src, 'trace', 'run_kernel_stats.csv')
    if os.path.exists(stats):
        shutil.copy(stats, dst_prefix + '_kernel_stats.csv')
    cs = counters(src)
    for sq_src in sq_srcs:
        for k, v in counters(sq_src).items():
            cs.setdefault(k, {}).update(v)
    out, rows = {}, []
    for k, c in cs.items():
        if 'FETCH_SIZE' not in c or 'WRITE_SIZE' not in c:
            continue
        fetch, write = c['FETCH_SIZE'] * 1024.0, c['WRITE_SIZE'] * 1024.0
        out[short(k)] = 2 * fetch + write
        rows.append((short(k)[:40], fetch, write, 2 * fetch + write))
    res = {'unit': 'bytes per launch (2*FETCH_SIZE + WRITE_SIZE)', 'source': src, 'kernels': out,
           'lib_source_sha256': lib_stamp()}
    for k, c in cs.items():
        if short(k) in ('demod_iso', 'demod_iso_cut', 'demod') and any(x.startswith('SQ_') for x in c):
            res[short(k) + '_sq'] = {'per_launch': {x: v for x, v in sorted(c.items())}, 'derived': derived(c)}
    json.dump(res, open(dst_prefix + '_pmc_traffic.json', 'w'), indent=1, sort_keys=True)
    with open(dst_prefix + '_pmc_traffic.txt', 'w') as fh:
        fh.write('%-40s %14s %14s %14s\n' % ('kernel', 'FETCH B', 'WRITE B', '2F+W B'))
        for r in sorted(rows, key=lambda r: -r[3]):
            fh.write('%-40s %14.0f %14.0f %14.0f\n' % r)
        for name in ('demod_iso_sq', 'demod_iso_cut_sq', 'demod_sq'):
            if name in res:
                fh.write('\n%s (per launch)\n' % name)
                for x, v in res[name]['per_launch'].items():
                    fh.write('  %-34s %16.1f\n' % (x, v))
                for x, v in res[name]['derived'].items():
                    fh.write('  %-34s %16.4f\n' % (x, v))
    print(open(dst_prefix + '_pmc_traffic.txt').read())


if __name__ == '__main__':
    main(*sys.argv[1:])
