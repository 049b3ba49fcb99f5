#!/usr/bin/env python3
"""cx-expander (cx-expander.cxx) as a stdin -> stdout filter over the native
library's ldg_cx_process (host code: one sequential chain, no GPU needed).

    python ld-decode_amd/cx_expander.py < in.pcm > out.pcm

Reads 16-bit stereo frames as the reference does (unsigned, minus 32768) in
blocks of 1024 frames; a short final block ends the stream unprocessed
(:105-113), as in the reference.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BLOCK_BYTES = 1024 * 4


def main():
    from ldgpu.native import CXExpander
    cx = CXExpander()
    fin, fout = sys.stdin.buffer, sys.stdout.buffer
    while True:
        buf = fin.read(64 * BLOCK_BYTES)          # whole blocks; read() returns short only at EOF
        nblk = len(buf) // BLOCK_BYTES
        if nblk:
            import numpy as np
            a = np.frombuffer(buf[:nblk * BLOCK_BYTES], dtype='<u2')
            fout.write(cx.process(a).astype('<u2').tobytes())
        if len(buf) < 64 * BLOCK_BYTES:
            break
    fout.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
