"""Diagnostics: print the read-cache misses of a GPU decode (speculation planner)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))
from ldgpu.decoder import GPUDecoder  # noqa: E402

dec = GPUDecoder(system='NTSC', batch=int(sys.argv[2]) if len(sys.argv) > 2 else 64)
n = int(40e6 * float(sys.argv[1] if len(sys.argv) > 1 else 3))
dec.ctx.synth(n, fmt=0, first_frame=1, seed=1)
dec.use_resident_capture(0, n)
orig_note, orig_plan = dec._note_miss, dec._plan
plans = []
plans_trace = []


def plan(*a):
    dec.trace = []
    new, chain = orig_plan(*a)
    plans_trace.append(dec.trace)
    dec.trace = None
    plans.append((a[0], a[1], a[2], list(new), list(chain)))
    return new, chain


def note(key):
    print('MISS', key, 'last_framenr', dec.last_framenr)
    nxt, mtf, lfr, new, chain = plans[-1]
    print('  chain', chain[:6])
    for t in plans_trace[-1][:8]:
        print('   step', t)
    print('  new', new[:8])
    for k in chain[:6]:
        inf = dec.cache[k][1] if k in dec.cache else None
        if inf is not None:
            print('   chain info', k, 'status', inf.status, 'top', inf.istop, 'fnr', inf.vbi_framenr, 'nfo', inf.nextfieldoffset)
    print('  last plan from', nxt, mtf, 'fr', lfr, 'planned near:', [k for k in new if abs(k[0] - key[0]) < 5000])
    print('  planned mtfs:', [k[1] for k in new][:40])
    for f in dec.field_log[-4:]:
        print('  field', f.readsample, f.mtf_level, 'valid', f.valid, 'top', f.istop,
              'fnr', f.vbi['framenr'] if f.vbi else None, 'next', f.nextsample)
    orig_note(key)


dec._note_miss, dec._plan = note, plan
nf = dec.decode(sink=None)
print('frames', nf, dec.stats)
