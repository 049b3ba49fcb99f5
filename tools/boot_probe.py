"""The decoder's first launches (boot): each launch's read starts, and the first launches'
records (start, status, next start, istop).  GPU box: python tools/boot_probe.py [PAL|NTSC]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ld-decode_amd'))


def main():
    from ldgpu import native
    from ldgpu.decoder import GPUDecoder
    from ldgpu.synth import make_capture
    system = sys.argv[1] if len(sys.argv) > 1 else 'PAL'
    if system == 'PAL':
        data = np.frombuffer(make_capture(int(40e6 * 1.0), 'u8', system='PAL', clv=True, first_frame=3000,
                                          seed=20181018), np.uint8)
    else:
        data = np.frombuffer(make_capture(int(40e6 * 2.0), 'u8', system='NTSC', first_frame=1, seed=20181017),
                             np.uint8)
    dec = GPUDecoder(system=system, batch=96)
    dec.set_capture(data, 0)
    orig_async, orig_wait = dec.ctx.decode_reads_async, dec.ctx.decode_reads_wait
    launches = []

    def la(starts, mtfs, slots, full=None):
        launches.append(list(starts))
        return orig_async(starts, mtfs, slots, full)

    def wa():
        infos = orig_wait()
        if len(launches) <= 3:
            print('records:', [(int(i.readsample), int(i.status), int(i.readsample + i.nextfieldoffset), int(i.istop))
                               for i in infos][:10], flush=True)
        return infos
    dec.ctx.decode_reads_async, dec.ctx.decode_reads_wait = la, wa
    dec.decode(sink=None)
    for k, l in enumerate(launches[:4]):
        print('launch %d: %d reads %s' % (k, len(l), l[:12]))
    print({k: dec.stats.get(k) for k in ('reads', 'reads_used', 'batches', 'probes', 'probe_moved')})


if __name__ == '__main__':
    main()
