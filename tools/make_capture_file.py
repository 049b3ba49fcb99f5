"""Write a synthetic NTSC capture file (the benchmark's GPU signal model, ldgpu/synth.py)
for end-to-end CLI runs:  python tools/make_capture_file.py PATH SECONDS [fmt 0..3] [--clv]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    from ldgpu import native
    from ldgpu.formats import bytes_for_samples
    path, seconds = sys.argv[1], float(sys.argv[2])
    fmt = int(sys.argv[3]) if len(sys.argv) > 3 and not sys.argv[3].startswith('-') else 0
    n = int(40e6 * seconds)
    t0 = time.perf_counter()
    ctx = native.Context('NTSC', 0, max_reads=8)
    ctx.synth(n, fmt=fmt, first_frame=1, clv='--clv' in sys.argv, seed=20181015)
    nbytes = bytes_for_samples(fmt, n)
    with open(path, 'wb') as fh:
        step = 1 << 28
        for off in range(0, nbytes, step):
            fh.write(ctx.capture_download(off, min(step, nbytes - off)))
    ctx.close()
    print('%s: %d samples, %d bytes, %.1f s' % (path, n, nbytes, time.perf_counter() - t0), flush=True)


if __name__ == '__main__':
    main()
