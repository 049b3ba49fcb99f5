"""The C-ABI library loads on CPU and exports every entry point include/ldgpu.h declares."""
import ctypes
import os
import re
import subprocess

import pytest

from ldgpu import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'ldgpu.h')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(ldg_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_expected_api():
    fns = declared_functions()
    for f in ['ldg_create', 'ldg_destroy', 'ldg_set_filters', 'ldg_set_capture', 'ldg_decode_reads',
              'ldg_field_audio', 'ldg_assemble_frames', 'ldg_comb_ntsc', 'ldg_debug_read']:
        assert f in fns


def test_library_exports_every_declared_symbol():
    if not os.path.exists(native.LIB_PATH):
        pytest.skip('libldgpu.so not built')
    out = subprocess.run(['nm', '-D', '--defined-only', native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r'\bT (ldg_[a-z0-9_]+)', out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_without_gpu_and_binds_signatures():
    if not os.path.exists(native.LIB_PATH):
        pytest.skip('libldgpu.so not built')
    lib = native.load()
    assert lib.ldg_version().decode().startswith('ldgpu')
    for f in native.EXPORTS:
        assert hasattr(lib, f)
    # invalid-argument paths never touch the device
    assert lib.ldg_create(None, None) == -1
    assert lib.ldg_destroy(None) == -1
    assert lib.ldg_last_error(None) == b'null context'


def test_struct_layout_matches_header(tmp_path):
    """ctypes mirrors == the C compiler's view of include/ldgpu.h."""
    src = tmp_path / 'sz.c'
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "ldgpu.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(ldg_field_info), '
                   'offsetof(ldg_field_info, vsync), offsetof(ldg_field_info, vbi_framenr), sizeof(ldg_params), '
                   'sizeof(ldg_filters), sizeof(ldg_config));return 0;}')
    exe = tmp_path / 'sz'
    subprocess.run(['gcc', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    F = native.FieldInfo
    assert got == [ctypes.sizeof(F), F.vsync.offset, F.vbi_framenr.offset, ctypes.sizeof(native.Params),
                   ctypes.sizeof(native.Filters), ctypes.sizeof(native.Config)]


def test_no_cpu_fallback():
    """Creating a context without a GPU must fail loudly (no silent CPU path)."""
    if not os.path.exists(native.LIB_PATH):
        pytest.skip('libldgpu.so not built')
    if native.load().ldg_device_count() > 0:
        pytest.skip('GPU present')
    with pytest.raises(native.LDGError):
        native.Context('NTSC', 0, max_reads=1)


def test_status_and_flag_constants_match_header():
    """The host's mirrors of the LDG_FS_* status codes and log flags equal the header's
    (FS_MIGRATED: the demod's per-CU park was left by a migrated workgroup; the host
    decodes that read again)."""
    hdr = open(os.path.join(ROOT, 'include', 'ldgpu.h')).read()
    consts = {k: int(v, 0) for k, v in re.findall(r'#define (LDG_FS_[A-Z_]+)\s+([0-9]+)', hdr)}
    assert native.FS_MIGRATED == consts['LDG_FS_MIGRATED'] == 8
    assert re.search(r'#define LDG_LOG_NO_VSYNC \(1 << 16\)', hdr) and native.LOG_NO_VSYNC == 1 << 16
    for name, v in consts.items():
        short = name[len('LDG_'):]
        if hasattr(native, short):
            assert getattr(native, short) == v, name
