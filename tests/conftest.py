import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'ld-decode_amd')
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through libldgpu.so)')
    config.addinivalue_line('markers', 'slow: longer oracle runs')


@pytest.fixture(scope='session')
def capture_u8_short():
    """0.2 s of synthetic NTSC CAV RF, u8 (deterministic)."""
    from ldgpu.synth import make_capture
    return make_capture(int(40e6 * 0.2), 'u8')


def gpu_available():
    try:
        from ldgpu import native
        lib = native.load()
        return lib.ldg_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope='session')
def gpu_ctx_ntsc():
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    rf = RFTables('NTSC')
    ctx = native.Context('NTSC', 0, max_reads=8)
    ctx.set_filters(rf.params(), rf.tables)
    return ctx, rf


@pytest.fixture(scope='session')
def gpu_ctx_pal():
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    rf = RFTables('PAL')
    ctx = native.Context('PAL', 0, max_reads=8)
    ctx.set_filters(rf.params(), rf.tables)
    return ctx, rf
