"""bench.py's argument checks (CPU, no device): the streamed / host-buffer modes belong to
the NTSC capture workload only, and are refused before anything touches a GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize('extra', [['--system', 'PAL', '--stream-file', '/tmp/x'], ['--sharded', '--host-io'],
                                   ['--sharded', '--stream-file', '/tmp/x']])
def test_bench_refuses_io_modes_outside_the_capture_workload(extra):
    env = dict(os.environ, WORLD_SIZE='1')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *extra], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 2
    assert 'the NTSC capture workload' in r.stderr


def test_bench_refuses_stream_file_on_a_sharded_launch():
    env = dict(os.environ, WORLD_SIZE='2', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--stream-file', '/tmp/x'],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and 'the NTSC capture workload' in r.stderr
