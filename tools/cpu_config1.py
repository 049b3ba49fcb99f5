"""BASELINE.json configs[0] on this container's CPU: 10 s of synthetic 40 MSPS 8-bit NTSC
RF through the oracle (the numpy restatement of lddecode.py's CPU path) -> .tbc, one
core (BASELINE.md §3 mode (i)).  Writes a JSON record to the path given.

    python tools/cpu_config1.py profiles/r03_cpu_config1.json [seconds]
"""
import contextlib
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))

from threadpoolctl import threadpool_limits  # noqa: E402


def main(out, seconds=10.0):
    import threading
    done = threading.Event()
    t_start = time.perf_counter()

    def beat():                    # a heartbeat on stderr (long CPU phases print nothing)
        while not done.wait(30.0):
            print('[cpu_config1] %.0f s' % (time.perf_counter() - t_start), file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    from ldgpu.synth import make_capture
    from oracle.capture import FMT_U8
    from oracle.framer import decode_capture
    t0 = time.perf_counter()
    data = make_capture(int(40e6 * seconds), 'u8', seed=20181016)
    synth_s = time.perf_counter() - t0
    with threadpool_limits(limits=1), contextlib.redirect_stdout(sys.stderr):
        t0 = time.perf_counter()
        frames, pcm, meta = decode_capture(data, FMT_U8)
        dt = time.perf_counter() - t0
    consumed = meta[-1]['nextsample'] if meta else 0
    tbc = b''.join(f.tobytes() for f in frames)
    rec = {'config': 'BASELINE configs[0]: %g s synthetic 40 MSPS 8-bit NTSC RF -> .tbc (oracle CPU path)' % seconds,
           'cpu_model': next((l.split(':', 1)[1].strip() for l in open('/proc/cpuinfo') if l.startswith('model name')),
                             'unknown'),
           'cores': 1, 'frames': len(frames), 'rf_samples_consumed': consumed, 'decode_s': round(dt, 2),
           'rf_msamples_per_s': consumed / dt / 1e6, 'fields_per_s': 2 * len(frames) / dt,
           'x_realtime': consumed / dt / 40e6, 'synth_s': round(synth_s, 1),
           'tbc_bytes': len(tbc), 'tbc_sha256': hashlib.sha256(tbc).hexdigest(),
           'framenrs': [m['vbi']['framenr'] for m in meta][:5] + ['...']}
    done.set()
    with open(out, 'w') as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 10.0)
