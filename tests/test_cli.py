"""lddecode.py CLI (lddecode.py:16-107 semantics) on the GPU decoder."""
import hashlib
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CLI = os.path.join(ROOT, 'ld-decode_amd', 'lddecode.py')


def run_cli(*args):
    return subprocess.run([sys.executable, CLI, *map(str, args)], capture_output=True, text=True, timeout=600)


def test_cli_rejects_pal_and_ntsc(tmp_path):
    r = run_cli('-p', '-n', tmp_path / 'x.u8', tmp_path / 'out')
    assert 'ERROR: Can only be PAL or NTSC' in r.stdout and r.returncode == 1


def test_cli_help_lists_reference_options():
    r = run_cli('-h')
    for opt in ('--start', '--seek', '--end', '--length', '--pal', '--ntsc', '--cut'):
        assert opt in r.stdout


def _golden_capture(tmp_path, case='ntsc_cav_u8_0p2s', ext='u8'):
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    data = make_golden.build_capture(case)
    path = tmp_path / ('cap.' + ext)
    path.write_bytes(bytes(data))
    with open(os.path.join(HERE, 'golden', case + '.json')) as fh:
        return path, json.load(fh)


@pytest.mark.gpu
def test_cli_decode_matches_golden(tmp_path):
    cap, gold = _golden_capture(tmp_path)
    out = tmp_path / 'out'
    r = run_cli(cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    frames = np.fromfile(str(out) + '.tbc', dtype=np.uint16).reshape(-1, 525, 910)
    meta = json.load(open(str(out) + '.json'))
    assert len(frames) == len(gold['frames']) == len(meta)
    for m, g in zip(meta, gold['frames']):
        assert m == g['meta']
    pcm = np.fromfile(str(out) + '.pcm', dtype=np.int16)
    assert pcm.size == sum(g['pcm_len'] for g in gold['frames'])
    printed = [l for l in r.stdout.splitlines() if l.startswith('frame ')]
    assert printed == ['frame  %s' % g['meta']['vbi']['framenr'] for g in gold['frames']]
    exact = sum(hashlib.sha256(f.tobytes()).hexdigest() == g['tbc_sha256'] for f, g in zip(frames, gold['frames']))
    print('CLI: %d/%d frames bit-identical' % (exact, len(frames)))


# field reads of this capture start at 0, 1052829, 1721434, ..., 4390767: a 15,000-sample
# dropout 20,000 samples into the third read breaks both vsync votes of two reads ("vsync vote
# needed"), one 30,000 samples into the eighth leaves it one vsync ("no/corrupt VSYNC found"),
# and frame 203 is lost; the first read (mid-field) is 'not valid'
DROPOUT_CAPTURE = dict(first_frame=200, seed=31, dropouts=((1741434, 15000), (4420767, 15000)))


@pytest.mark.gpu
def test_cli_log_and_invalid_fields_match_oracle(tmp_path):
    """The CLI's stdout after the argument line is the reference's: per field the
    Field / FieldNTSC messages and readframe's `sample nextsample True istop`, then
    `frame N` (lddecode_core.py:620,918,1175,1263; lddecode.py:92) -- on a capture with
    dropouts that make fields invalid; frames +-1 LSB, audio bit-exact, metadata exact."""
    import contextlib
    import io
    from ldgpu.synth import make_capture
    from oracle.capture import FMT_U8
    from oracle.framer import decode_capture
    data = make_capture(int(40e6 * 0.3), 'u8', **DROPOUT_CAPTURE)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        frames, pcm, meta = decode_capture(data, FMT_U8, log=print)
    want = buf.getvalue().splitlines()
    assert 'vsync vote needed 0' in want and 'no/corrupt VSYNC found, jumping forward' in want
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    out = tmp_path / 'out'
    r = run_cli(cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.splitlines()[1:] == want
    got = np.fromfile(str(out) + '.tbc', dtype=np.uint16).reshape(-1, 525 * 910)
    assert len(got) == len(frames)
    for g, f in zip(got, frames):
        assert np.abs(g.astype(np.int64) - f.astype(np.int64)).max() <= 1
    assert np.array_equal(np.fromfile(str(out) + '.pcm', dtype=np.int16), np.concatenate(pcm))
    assert json.load(open(str(out) + '.json')) == meta


@pytest.mark.gpu
def test_cli_length_and_comb(tmp_path):
    cap, gold = _golden_capture(tmp_path)
    out = tmp_path / 'out'
    r = run_cli('-l', 2, '--comb', cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    frames = np.fromfile(str(out) + '.tbc', dtype=np.uint16).reshape(-1, 525, 910)
    rgb = np.fromfile(str(out) + '.rgb', dtype=np.uint16).reshape(-1, 480, 744, 3)
    assert len(frames) == 2 and len(rgb) == 2
    from oracle.comb import Comb2D
    o = Comb2D().process(frames)
    assert np.abs(o.astype(np.int64) - rgb.astype(np.int64)).max() <= 1


def _oracle_findframe(data, target, nextsample=0):
    """oracle.framer.findframe (lddecode_core.py:1338-1378): (sample, framenr trail, messages)."""
    from oracle.capture import FMT_U8, Capture
    from oracle.demod import RFDemod
    from oracle.framer import findframe
    logs = []
    r = findframe(Capture(bytes(data), FMT_U8), RFDemod(system='NTSC'), target, nextsample,
                  log=lambda *a: logs.append(a))
    return r, _seek_trail(logs)


def _seek_trail(logs):
    """The VBI frame numbers findframe logs (first loop: (rv, vbi); second loop: (vbi,))
    and its SEEK messages; the readframe progress lines are ignored."""
    trail = [a[-1]['framenr'] for a in logs if len(a) in (1, 2) and isinstance(a[-1], dict)]
    msgs = [a[0] for a in logs if len(a) == 1 and isinstance(a[0], str)]
    return trail, msgs


SEEK_CASES = {
    # picture numbers on the first field of each frame only: the reference's CAV framing in
    # findframe (lddecode_core.py:1273-1275) needs a field without one
    'cav': dict(first_frame=100, seed=11, code_fields=(0,)),
    # a cut disc: frames from the 16th on are numbered 5 lower (110.. again), so seeking
    # frame 120 lands on 115 first and needs the retry loop (:1366-1372)
    'cav_retry': dict(first_frame=100, seed=11, code_fields=(0,), frame_skip=(15, -5)),
    # frames 115..129 missing: seeking 120 oscillates 135 / 105 and ends in SEEK WARNING (:1375-1376)
    'cav_warning': dict(first_frame=100, seed=11, code_fields=(0,), frame_skip=(15, 15)),
    # CLV time codes: tolerance 1 (:1356-1357)
    'clv': dict(first_frame=5399, seed=12, clv=True),
}


@pytest.mark.gpu
@pytest.mark.parametrize('case,target', [('cav', 105), ('cav_retry', 120), ('cav_warning', 120), ('clv', 5405),
                                         ('clv', 5420)])
def test_findframe_matches_oracle(case, target):
    """GPU findframe (ldgpu/decoder.py) against the oracle's restatement of the reference's:
    the same returned sample, the same trail of VBI frame numbers through the retries, the
    same SEEK WARNING."""
    from ldgpu.decoder import GPUDecoder
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 1.0), 'u8', **SEEK_CASES[case])
    want, (trail, msgs) = _oracle_findframe(data, target)
    dec = GPUDecoder(system='NTSC', batch=8)
    dec.set_capture(data, 0)
    logs = []
    got = dec.findframe(target, 0, log=lambda *a: logs.append(a))
    assert got == want
    assert _seek_trail(logs) == (trail, msgs)
    if case == 'cav_retry':
        assert trail[-2:] == [115, 120]
    if case == 'cav_warning':
        assert msgs == ['SEEK WARNING: seeked to frame 135 instead of 120']


@pytest.mark.gpu
def test_cli_seek_and_cut(tmp_path):
    """-S seeks by VBI frame number (findframe); -c writes the raw slice between two frames
    as .r16 (lddecode.py:60-81), with both bounds from the oracle's findframe."""
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.5), 'u8', **SEEK_CASES['cav'])
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    out = tmp_path / 'seek'
    r = run_cli('-S', 105, '-l', 2, cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    meta = json.load(open(str(out) + '.json'))
    assert [m['vbi']['framenr'] for m in meta] == [105, 106]
    first, _ = _oracle_findframe(data, 105)
    assert meta[0]['fields'][0]['readsample'] == first
    out = tmp_path / 'cut'
    r = run_cli('-c', '-S', 103, '-E', 106, cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    r16 = np.fromfile(str(out) + '.r16', dtype=np.int16)
    from ldgpu.rfparams import RFTables
    spf = RFTables('NTSC').samples_per_frame          # lddecode.py:41
    first, _ = _oracle_findframe(data, 103)
    last, _ = _oracle_findframe(data, 106, first)
    last += int(spf * .25)
    raw = np.frombuffer(bytes(data), dtype=np.uint8).astype(np.int16)
    assert np.array_equal(r16, raw[first:last])


@pytest.mark.gpu
def test_cli_sharded_two_ranks_equal_single(tmp_path):
    """torch.distributed.run with 2 ranks (field-group sharding) writes the same
    .tbc / .pcm / .json, and with --comb the same .rgb (the comb's burst-level EMA
    handed across the shard boundary), as the single-process CLI."""
    import socket
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.6), 'u8', first_frame=500, seed=13)
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    r = run_cli('--comb', cap, tmp_path / 'one')
    assert r.returncode == 0, r.stderr[-2000:]
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                        '--master-addr', '127.0.0.1', '--master-port', str(port), CLI, '--comb', str(cap),
                        str(tmp_path / 'two')], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    for ext in ('.tbc', '.pcm', '.rgb'):
        assert (tmp_path / ('one' + ext)).read_bytes() == (tmp_path / ('two' + ext)).read_bytes(), ext
    assert json.load(open(tmp_path / 'one.json')) == json.load(open(tmp_path / 'two.json'))


@pytest.mark.gpu
def test_cli_sharded_comb_3d_equals_single(tmp_path):
    """The 3D comb (comb-ntsc -d 3 -F: --comb --comb-3d) on a sharded decode: 2 and 3 ranks
    (each combing its own frames with its neighbours' boundary frames and the exact
    burst-level EMA, ldgpu/shard.py comb3d_sharded) write the same .rgb -- every frame
    but the capture's first and last -- as one process, byte for byte."""
    import socket
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.6), 'u8', first_frame=700, seed=19)
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    r = run_cli('--comb', '--comb-3d', cap, tmp_path / 'one')
    assert r.returncode == 0, r.stderr[-2000:]
    one = (tmp_path / 'one.rgb').read_bytes()
    nfr = len((tmp_path / 'one.tbc').read_bytes()) // 955500
    assert nfr >= 8 and len(one) == (nfr - 2) * 744 * 480 * 3 * 2
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    for n in (2, 3):
        with socket.socket() as sk:
            sk.bind(('127.0.0.1', 0))
            port = sk.getsockname()[1]
        out = tmp_path / ('r%d' % n)
        r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
                            '--master-addr', '127.0.0.1', '--master-port', str(port), CLI, '--comb', '--comb-3d',
                            str(cap), str(out)], capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
        assert (tmp_path / ('r%d.rgb' % n)).read_bytes() == one, n
        assert (tmp_path / ('r%d.tbc' % n)).read_bytes() == (tmp_path / 'one.tbc').read_bytes()


@pytest.mark.gpu
def test_cli_sharded_pal_equal_single(tmp_path):
    """PAL sharded too: 3 ranks on a PAL CLV capture write the same .tbc /
    .pcm / .json and, with --comb, the same PAL Y/C .rgb as one process (the Y/C decoder's
    burst-level chain is at its fixed point from the first line, so ranks comb on their own);
    and 2 ranks with --epoch-frames too."""
    import socket
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.8), 'u8', system='PAL', clv=True, first_frame=4200, seed=17)
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    r = run_cli('-p', '--comb', cap, tmp_path / 'one')
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    for name, extra, n in (('three', [], 3), ('ep', ['--epoch-frames', '5'], 2)):
        with socket.socket() as sk:
            sk.bind(('127.0.0.1', 0))
            port = sk.getsockname()[1]
        r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
                            '--master-addr', '127.0.0.1', '--master-port', str(port), CLI, '-p', '--comb'] + extra +
                           [str(cap), str(tmp_path / name)], capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
        for ext in ('.tbc', '.pcm', '.rgb'):
            assert (tmp_path / ('one' + ext)).read_bytes() == (tmp_path / (name + ext)).read_bytes(), (name, ext)
        assert json.load(open(tmp_path / 'one.json')) == json.load(open(tmp_path / (name + '.json'))), name


@pytest.mark.gpu
def test_cli_sharded_fused_comb_recombs_only_the_first_frames(tmp_path):
    """Three ranks with --comb on a 2 s capture: each rank combs its frames in HBM as they
    are decoded (ldg_output_async) from a "not initialised" burst-level EMA, then re-combs
    only its first frames with the exact state handed across the ranks (comb-ntsc.cxx:560-566;
    ldgpu/shard.py comb_fix): the .rgb is byte-identical to one process's, and ranks 1 and 2
    re-combed fewer frames than they hold."""
    import re
    import socket
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 2.0), 'u8', first_frame=900, seed=15)
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    r = run_cli('--comb', cap, tmp_path / 'one')
    assert r.returncode == 0, r.stderr[-2000:]
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '3',
                        '--master-addr', '127.0.0.1', '--master-port', str(port), CLI, '--comb', str(cap),
                        str(tmp_path / 'three')], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    for ext in ('.tbc', '.pcm', '.rgb'):
        assert (tmp_path / ('one' + ext)).read_bytes() == (tmp_path / ('three' + ext)).read_bytes(), ext
    redo = {int(a): int(b) for a, b in re.findall(r'rank (\d+): comb re-combed (\d+) frame', r.stdout)}
    nfr = len(json.load(open(tmp_path / 'one.json')))
    assert redo.get(0) == 0 and 0 < redo[1] < nfr // 3 and 0 < redo[2] < nfr // 3, (redo, nfr)


@pytest.mark.gpu
def test_cli_epochs_resume_after_a_fault(tmp_path):
    """--epoch-frames 7 --manifest: the decode runs as epochs that each start from the exact
    chain state after the previous one's last frame (read position, MTF, frame number, the
    EOF guard's read, 48 kHz offset, the comb's burst level): byte-identical to one decode.
    A run killed after its second epoch (LDG_FAULT_AFTER_EPOCHS) resumes from the manifest
    and ends with the same bytes; two ranks per epoch too."""
    import socket
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 1.0), 'u8', first_frame=400, seed=16)
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    r = run_cli('--comb', cap, tmp_path / 'one')
    assert r.returncode == 0, r.stderr[-2000:]
    man = tmp_path / 'm.json'
    env = dict(os.environ, LDG_FAULT_AFTER_EPOCHS='2')
    r = subprocess.run([sys.executable, CLI, '--comb', '--epoch-frames', '7', '--manifest', str(man), str(cap),
                        str(tmp_path / 'ep')], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 3 and 'fault injected after epoch 2' in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
    m = json.load(open(man))
    assert m['epoch'] == 2 and m['frames'] == 14 and not m['complete']
    r = run_cli('--comb', '--epoch-frames', '7', '--manifest', man, cap, tmp_path / 'ep')
    assert r.returncode == 0 and 'resuming after epoch 2' in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
    assert json.load(open(man))['complete']
    for ext in ('.tbc', '.pcm', '.rgb'):
        assert (tmp_path / ('one' + ext)).read_bytes() == (tmp_path / ('ep' + ext)).read_bytes(), ext
    assert json.load(open(tmp_path / 'one.json')) == json.load(open(tmp_path / 'ep.json'))
    # a rerun on the complete manifest is a no-op; another frame range is refused
    r = run_cli('--comb', '--epoch-frames', '7', '--manifest', man, cap, tmp_path / 'ep')
    assert r.returncode == 0 and 'already complete' in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
    r = run_cli('--comb', '-s', '1', '--epoch-frames', '7', '--manifest', man, cap, tmp_path / 'ep')
    assert r.returncode == 1 and 'belongs to another decode' in r.stdout
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                        '--master-addr', '127.0.0.1', '--master-port', str(port), CLI, '--comb', '--epoch-frames', '9',
                        str(cap), str(tmp_path / 'two')], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    for ext in ('.tbc', '.pcm', '.rgb'):
        assert (tmp_path / ('one' + ext)).read_bytes() == (tmp_path / ('two' + ext)).read_bytes(), ext
    assert json.load(open(tmp_path / 'one.json')) == json.load(open(tmp_path / 'two.json'))
    # every epoch's windows hold O(epoch) samples, the last rank's too (not the rest of the capture)
    wins = [(int(a), int(b)) for a, b in re.findall(r'capture window samples \[(\d+), (\d+)\)', r.stdout)]
    spf = 1334668
    assert len(wins) >= 2 * 3 and max(b - a for a, b in wins) <= 11 * spf + 1000001 + 2 * 16384 + 2048, wins


@pytest.mark.gpu
def test_cli_sharded_rccl_halo_equal_single(tmp_path):
    """With a GPU per rank the capture-window halo travels between the GPUs' capture buffers
    over RCCL (lddecode.py load_window, ldgpu/shard.py exchange_halo): two ranks on two GPUs
    write the same .tbc / .pcm / .json as one process.  Needs two visible devices."""
    import socket
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip('needs 2 GPUs (the RCCL halo path); a 1-GPU box runs the gloo variant above')
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.6), 'u8', first_frame=700, seed=14)
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(data))
    r = run_cli(cap, tmp_path / 'one')
    assert r.returncode == 0, r.stderr[-2000:]
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                        '--master-addr', '127.0.0.1', '--master-port', str(port), CLI, str(cap),
                        str(tmp_path / 'two')], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert 'halo from rank 1 over RCCL' in r.stdout
    for ext in ('.tbc', '.pcm'):
        assert (tmp_path / ('one' + ext)).read_bytes() == (tmp_path / ('two' + ext)).read_bytes(), ext
    assert json.load(open(tmp_path / 'one.json')) == json.load(open(tmp_path / 'two.json'))


COMB_CLI = os.path.join(ROOT, 'ld-decode_amd', 'comb_ntsc.py')


def test_comb_cli_rejects_wide_with_optical_flow():
    r = subprocess.run([sys.executable, COMB_CLI, '-d', '3', '-W'], capture_output=True, text=True, timeout=120,
                       stdin=subprocess.DEVNULL)
    assert r.returncode == 1 and 'use -d 3 -F -W' in r.stderr


@pytest.mark.gpu
def test_comb_cli_3d_optical_flow_encode_script_form(tmp_path):
    """`comb -d 3 -I 0` as encode-ntsc:4 / encode-ralf:6 run it (3D with optical flow, the
    reference's default): the stream filter against the oracle's restatement (build-defined
    Farneback, oracle/farneback.py) within +-1 LSB, chunked across calls."""
    sys.path.insert(0, HERE)
    from test_comb import frames_3d
    from oracle.comb import Comb3DFlow
    fr = frames_3d(seed=5, n=5)
    r = subprocess.run([sys.executable, COMB_CLI, '--chunk', '2', '-d', '3', '-I', '0'], input=fr.tobytes(),
                       capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    exp = Comb3DFlow(black_ire=0.0).process(fr)
    got = np.frombuffer(r.stdout, dtype=np.uint16).reshape(-1, 480, 744, 3)
    assert got.shape == exp.shape == (3, 480, 744, 3)
    assert np.abs(got.astype(np.int64) - exp.astype(np.int64)).max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize('dim', [2, 3])
def test_comb_cli_stream_matches_oracle(tmp_path, dim):
    """comb_ntsc.py as comb-ntsc's stdin/stdout filter (2D default, or -d 3 -F), with a
    trailing partial frame that ends the stream (comb-ntsc.cxx:1102-1116)."""
    sys.path.insert(0, HERE)
    from test_comb import frames_3d
    from oracle.comb import Comb2D, Comb3D
    fr = frames_3d(seed=5, n=5)
    data = fr.tobytes() + b'\x01' * 1000
    args = [sys.executable, COMB_CLI, '--chunk', '2'] + (['-d', '3', '-F'] if dim == 3 else [])
    r = subprocess.run(args, input=data, capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.frombuffer(r.stdout, dtype=np.uint16).reshape(-1, 480, 744, 3)
    exp = Comb2D().process(fr) if dim == 2 else Comb3D().process(fr)
    assert got.shape == exp.shape
    assert np.abs(got.astype(np.int64) - exp.astype(np.int64)).max() <= 1


@pytest.mark.gpu
def test_cli_comb_3d(tmp_path):
    cap, gold = _golden_capture(tmp_path)
    out = tmp_path / 'out'
    r = run_cli('--comb', '--comb-3d', cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    frames = np.fromfile(str(out) + '.tbc', dtype=np.uint16).reshape(-1, 525, 910)
    rgb = np.fromfile(str(out) + '.rgb', dtype=np.uint16).reshape(-1, 480, 744, 3)
    assert len(rgb) == len(frames) - 2
    from oracle.comb import Comb3D
    o = Comb3D().process(frames)
    assert np.abs(o.astype(np.int64) - rgb.astype(np.int64)).max() <= 1


@pytest.mark.gpu
def test_cli_comb_3d_flow(tmp_path):
    """lddecode.py --comb --comb-3d-flow: the decoded frames through the 3D comb with optical
    flow (build-defined, oracle/comb.py Comb3DFlow), +-1 LSB."""
    cap, gold = _golden_capture(tmp_path)
    out = tmp_path / 'out'
    r = run_cli('--comb', '--comb-3d-flow', cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    frames = np.fromfile(str(out) + '.tbc', dtype=np.uint16).reshape(-1, 525, 910)
    rgb = np.fromfile(str(out) + '.rgb', dtype=np.uint16).reshape(-1, 480, 744, 3)
    assert len(rgb) == len(frames) - 2 >= 1
    from oracle.comb import Comb3DFlow
    o = Comb3DFlow().process(frames)
    assert np.abs(o.astype(np.int64) - rgb.astype(np.int64)).max() <= 1


@pytest.mark.gpu
def test_cli_pal_comb(tmp_path):
    """lddecode.py -p --comb: PAL .tbc through the build-defined PAL Y/C decoder, against
    its oracle on the same frames (+-1 LSB)."""
    cap, gold = _golden_capture(tmp_path, case='pal_clv_u8_0p2s')
    out = tmp_path / 'out'
    r = run_cli('-p', '--comb', cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    frames = np.fromfile(str(out) + '.tbc', dtype=np.uint16).reshape(-1, 625, 1135)
    rgb = np.fromfile(str(out) + '.rgb', dtype=np.uint16).reshape(-1, 576, 1057, 3)
    assert len(frames) >= 1 and len(rgb) == len(frames)
    from oracle.comb import CombPAL
    o = CombPAL().process(frames)
    assert np.abs(o.astype(np.int64) - rgb.astype(np.int64)).max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize('args,opts,dim', [(['-I', '0', '-N', '1', '-v'], dict(black_ire=0.0, nr_c=1.0, linesout=525), 2),
                                           (['-d', '3', '-F', '-I', '0', '-b', '200'],
                                            dict(black_ire=0.0, brightness=200.0), 3),
                                           (['-d', '3', '-B', '-n', '0', '-Q', '-L'],
                                            dict(bw=True, nr_y=0.0, colorlpf_hq=False, colorlpf=False), 2),
                                           (['-W', '-I', '0'], dict(wide=True, black_ire=0.0), 2),
                                           (['-W', '-W'], dict(), 2)])
def test_comb_cli_options_match_oracle(args, opts, dim):
    """comb_ntsc.py with the reference's option letters (the encode scripts' `-I 0`, CNR, -v,
    -b, -B forcing dim 2, the LPF toggles) against the oracle with the same options."""
    sys.path.insert(0, HERE)
    from test_comb import frames_3d
    from oracle.comb import Comb2D, Comb3D
    fr = frames_3d(seed=8, n=5)
    r = subprocess.run([sys.executable, COMB_CLI, '--chunk', '2'] + args, input=fr.tobytes(), capture_output=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    exp = Comb2D(**opts).process(fr) if dim == 2 else Comb3D(**opts).process(fr)
    got = np.frombuffer(r.stdout, dtype=np.uint16).reshape(exp.shape)
    assert np.abs(got.astype(np.int64) - exp.astype(np.int64)).max() <= 1


@pytest.mark.gpu
def test_comb_cli_8bit_pulldown_and_images(tmp_path):
    """-8 writes the high bytes (:710-716); -p pairs fields by the line-0 flag word px 13 and
    the frame code px 14/15 (PostProcess :894-938): a CAV_ODD frame holds its odd rows, the
    next frame's even rows complete it (written with the held frame code), a CAV_EVEN frame
    is written whole, a frame without flags writes nothing; -f -o write <base><code>.rgb."""
    sys.path.insert(0, HERE)
    from test_comb import frames_3d
    from oracle.comb import Comb2D
    fr = frames_3d(seed=9, n=4).copy()
    fr[:, 0, 13:16] = 0
    fr[0, 0, 13], fr[0, 0, 15] = 0x8, 11          # CAV_ODD, code 11
    fr[1, 0, 13], fr[1, 0, 15] = 0x4, 12          # CAV_EVEN, code 12
    fr[2, 0, 13], fr[2, 0, 15] = 0x0, 13          # no flags: nothing written
    fr[3, 0, 13], fr[3, 0, 15] = 0x200, 14        # WHITE_EVEN: written whole
    rgb = Comb2D().process(fr)
    r = subprocess.run([sys.executable, COMB_CLI, '-8'], input=fr.tobytes(), capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got8 = np.frombuffer(r.stdout, dtype=np.uint8).reshape(rgb.shape)
    assert np.abs(got8.astype(np.int64) - (rgb >> 8).astype(np.int64)).max() <= 1
    mix = rgb[0].copy()
    mix[0::2] = rgb[1][0::2]
    exp = [(11, mix), (12, rgb[1]), (14, rgb[3])]
    r = subprocess.run([sys.executable, COMB_CLI, '-p'], input=fr.tobytes(), capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.frombuffer(r.stdout, dtype=np.uint16).reshape(-1, 480, 744, 3)
    assert got.shape[0] == 3
    for g, (_, e) in zip(got, exp):
        assert np.abs(g.astype(np.int64) - e.astype(np.int64)).max() <= 1
    base = str(tmp_path / 'img')
    r = subprocess.run([sys.executable, COMB_CLI, '-p', '-f', '-o', base], input=fr.tobytes(), capture_output=True,
                       timeout=600)
    assert r.returncode == 0 and r.stdout == b''
    for code, e in exp:
        g = np.fromfile(base + '%d.rgb' % code, dtype=np.uint16).reshape(480, 744, 3)
        assert np.abs(g.astype(np.int64) - e.astype(np.int64)).max() <= 1


@pytest.mark.gpu
def test_cli_comb_args(tmp_path):
    """lddecode.py --comb --comb-args '-I 0 -N 1 -v': the fused comb with comb-ntsc's options,
    against the oracle comb with the same options on the written .tbc frames."""
    cap, gold = _golden_capture(tmp_path)
    out = tmp_path / 'out'
    r = run_cli('-l', 3, '--comb', '--comb-args', '-I 0 -N 1 -v', cap, out)
    assert r.returncode == 0, r.stderr[-2000:]
    frames = np.fromfile(str(out) + '.tbc', dtype=np.uint16).reshape(-1, 525, 910)
    rgb = np.fromfile(str(out) + '.rgb', dtype=np.uint16).reshape(-1, 525, 744, 3)
    assert len(frames) == 3 and len(rgb) == 3
    from oracle.comb import Comb2D
    o = Comb2D(black_ire=0.0, nr_c=1.0, linesout=525).process(frames)
    assert np.abs(o.astype(np.int64) - rgb.astype(np.int64)).max() <= 1
