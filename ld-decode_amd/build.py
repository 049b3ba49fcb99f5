"""Build libldgpu.so for gfx950 in-tree (explicit hipcc, no JIT cache).

    python ld-decode_amd/build.py [--force]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, 'ldgpu', 'libldgpu.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-shared',
         # IEEE-faithful scalar arithmetic on the parity-critical paths (numpy does not
         # contract a*b+c); FFT butterflies use explicit __fma_rn where they want it.
         '-ffp-contract=off',
         # the machine scheduler's max-ILP strategy (no kernel spills; the demod stays at
         # 121 VGPRs): 2-step bench -1.3% time in 3/3 interleaved rounds and -0.3% in 2/4, 20 sustained
         # steps -0.15% in 2/3 (profiles/r02_s84_*, r02_s85_*, r02_s91_*)
         '-mllvm', '--amdgpu-sched-strategy=max-ilp']


def sources():
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(('.hip', '.hpp', '.inc'))] + \
        [os.path.join(os.path.dirname(HERE), 'include', 'ldgpu.h'), os.path.abspath(__file__)]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in sources())


def build_variant(out, defines=(), verbose=True):
    """A profiling build (e.g. defines=('LDG_STAMPS',)) at another path; load it with LDGPU_LIB."""
    cmd = [HIPCC] + FLAGS + ['-D' + d for d in defines] + [os.path.join(CSRC, 'ldgpu.hip'), '-o', out]
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    return out


def build(force=False, verbose=True):
    if not force and up_to_date():
        if verbose:
            print('libldgpu.so up to date')
        return OUT
    cmd = [HIPCC] + FLAGS + [os.path.join(CSRC, 'ldgpu.hip'), '-o', OUT + '.tmp']
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
