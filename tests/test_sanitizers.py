"""Sanitizer runs (CPU only): the oracle's C++ comb restatements and libldgpu's
host-only C++ under AddressSanitizer + UndefinedBehaviorSanitizer, built by
tests/san/Makefile (libldgpu_asan.so: the library with its host side instrumented).
The comb drivers put strong chroma on the frame's last lines, where the reference's
Split2D reads past the frame (comb-ntsc.cxx:299,303: row l + 2 = 525 for l = 523).
Any report (heap / stack / global overflow, use-after-free, leak, UB) fails the run."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, 'oracle', '_build', 'san')
ENV = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:halt_on_error=1',
           UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1',
           LSAN_OPTIONS='suppressions=' + os.path.join(HERE, 'san', 'lsan.supp'))


@pytest.fixture(scope='module')
def built():
    if shutil.which('make') is None or not os.path.exists('/opt/rocm/llvm/bin/clang++'):
        pytest.skip('no toolchain')
    r = subprocess.run(['make', '-s', '-C', os.path.join(HERE, 'san'), '-j3'], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return OUT


@pytest.mark.parametrize('prog', ['comb_san', 'combpal_san', 'host_san'])
def test_clean_under_asan_ubsan(built, prog):
    r = subprocess.run([os.path.join(built, prog)], capture_output=True, text=True, timeout=600, env=ENV)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert '%s ok' % prog in r.stdout
    for bad in ('AddressSanitizer', 'LeakSanitizer', 'runtime error:'):
        assert bad not in out, out[-4000:]
