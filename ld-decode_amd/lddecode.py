#!/usr/bin/env python3
"""lddecode.py on the MI355X: the reference CLI (lddecode.py:16-107) with the RF
decode, TBC and (optionally) the 2D NTSC comb on the GPU.

    python ld-decode_amd/lddecode.py [-s N] [-S N] [-E N] [-l N] [-p|-n] [-c] infile outfile

Same arguments, loader selection by extension (.lds / .r30 / .r16, else 8-bit),
the same frame accounting (samples_per_frame = int(fs/FPS)+1, the 10-bit
bytes_per_frame and the fd.tell() + 1.05 frame EOF guard), `frame <n>` lines,
and the same outputs: <outfile>.tbc (native uint16 frames) and <outfile>.pcm
(int16 stereo, 48 kHz); cut mode (-c) writes <outfile>.r16.  Additions:
<outfile>.json (per-frame VBI and per-field metadata, one JSON list) and
--comb (<outfile>.rgb: comb-ntsc's default rgb48 744x480 frames; --comb-3d:
comb-ntsc -d 3 -F's).  The comb alone, on a .tbc stream: comb_ntsc.py.
"""
import argparse
import json
import os
import queue
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from ldgpu.decoder import GPUDecoder  # noqa: E402
from ldgpu.formats import fmt_from_path, read_samples, samples_in_bytes  # noqa: E402


class Writer:
    """The decode's outputs written on a thread of their own, in order: the reference's
    loop writes each frame and prints its lines between decodes (lddecode.py:88-98);
    here the decode thread queues those writes and goes on decoding.  The frames it
    queues are views of the decoder's pinned output rings: drain() (the decoder's
    before_ring_reuse hook) returns once every queued write is done, before a ring is
    filled again."""

    def __init__(self):
        self.q = queue.Queue()
        self.err = None
        self.busy_s = self.drain_s = 0.0
        self.t = threading.Thread(target=self._run, name='ldg-writer', daemon=True)
        self.t.start()

    def _run(self):
        while True:
            fn = self.q.get()
            try:
                if fn is None:
                    return
                if self.err is None:
                    t0 = time.perf_counter()
                    fn()
                    self.busy_s += time.perf_counter() - t0
            except BaseException as e:     # reported on the decode thread
                self.err = e
            finally:
                self.q.task_done()

    def put(self, fn):
        if self.err is not None:
            raise self.err
        self.q.put(fn)

    def drain(self):
        t0 = time.perf_counter()
        self.q.join()
        self.drain_s += time.perf_counter() - t0
        if self.err is not None:
            raise self.err

    def close(self):
        if self.t.is_alive():
            self.q.put(None)
            self.t.join()
        if self.err is not None:
            raise self.err


def parse(argv=None):
    p = argparse.ArgumentParser(description='Extracts audio and video from raw RF laserdisc captures')
    p.add_argument('infile', metavar='infile', type=str, help='source file')
    p.add_argument('outfile', metavar='outfile', type=str, help='base name for destination files')
    p.add_argument('-s', '--start', metavar='start', type=int, default=0,
                   help='rough jump to frame n of capture (default is 0)')
    p.add_argument('-S', '--seek', metavar='seek', type=int, default=-1, help='seek to frame n of capture')
    p.add_argument('-E', '--end', metavar='end', type=int, default=-1, help='cutting: last frame')
    p.add_argument('-l', '--length', metavar='length', type=int, help='limit length to n frames')
    p.add_argument('-p', '--pal', dest='pal', action='store_true', help='source is in PAL format')
    p.add_argument('-n', '--ntsc', dest='ntsc', action='store_true', help='source is in NTSC format')
    p.add_argument('-c', '--cut', dest='cut', action='store_true', help='cut (to r16) instead of decode')
    # MI355X additions
    p.add_argument('--device', type=int, default=0, help='HIP device')
    p.add_argument('--batch', type=int, default=128, help='field reads per GPU launch')
    p.add_argument('--comb', action='store_true',
                   help='also write <outfile>.rgb through the 2D NTSC comb (PAL: the build-defined PAL Y/C '
                        'decoder, 1057x576 rgb48)')
    p.add_argument('--comb-3d', action='store_true',
                   help='with --comb: the 3D comb without optical flow (comb-ntsc -d 3 -F); '
                        'every frame but the first and the last')
    p.add_argument('--comb-3d-flow', action='store_true',
                   help='with --comb: the 3D comb with optical flow (comb-ntsc -d 3; the flow is this build\'s '
                        'restatement of OpenCV\'s Farneback, build-defined); every frame but the first and the last')
    p.add_argument('--comb-3d-core', type=float, default=-1.0, help='comb-ntsc -c (IRE, default 1.25; 0 with flow)')
    p.add_argument('--comb-3d-range', type=float, default=-1.0, help='comb-ntsc -r (IRE, default 5.5; 0.5 with flow)')
    p.add_argument('--comb-args', default='',
                   help="comb-ntsc options for --comb (NTSC), e.g. '-I 0 -N 1 -v' (comb_ntsc.py's -I -b -n -N "
                        "-B -a -L -Q -v -l -W)")
    p.add_argument('--no-json', action='store_true', help='do not write <outfile>.json')
    p.add_argument('--stats-json', default=None,
                   help='one process: write a timing breakdown of the run (read, decode, write) to this file')
    p.add_argument('--window-mb', type=int, default=2048,
                   help='one process: the capture streams from the file through a ring of this many MiB of HBM '
                        '(device memory independent of the capture length); 0: upload the whole capture')
    p.add_argument('--epoch-frames', type=int, default=0,
                   help='decode in epochs of N frames, each a complete (sharded) decode whose outputs are final '
                        'before the next starts; with --manifest a crashed run resumes at the last finished epoch')
    p.add_argument('--manifest', default=None,
                   help='JSON progress manifest (epoch, frames and bytes written, the exact chain state): '
                        'written after every epoch, read to resume')
    return p.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    print(args)
    filename, outname = args.infile, args.outfile
    firstframe, req_frames = args.start, args.length
    if args.pal and args.ntsc:
        print("ERROR: Can only be PAL or NTSC")
        return 1
    system = 'PAL' if args.pal else 'NTSC'
    if args.comb_3d_flow:
        args.comb_3d = True
    if args.comb and system != 'NTSC' and args.comb_3d:
        print("ERROR: --comb-3d is NTSC only")
        return 1

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rccl = False
    if world > 1:
        # one process per GPU (python -m torch.distributed.run --nproc-per-node N lddecode.py ...):
        # field-group sharding of the capture (ldgpu/shard.py).  The capture-window halo
        # travels GPU to GPU over RCCL when every rank has its own GPU; the small summary
        # exchange (all_gather_object) goes over gloo.
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        local = int(os.environ.get('LOCAL_RANK', '0'))
        rccl = ndev >= world
        if rccl:
            torch.cuda.set_device(local)
        dist.init_process_group('cpu:gloo,cuda:nccl' if rccl else 'gloo')
        if rccl:
            # the RCCL communicator made by a collective every rank joins: the first device
            # operation after this is the halo's batched send / receive, which only
            # neighbouring ranks join (torch requires every rank in a first batched P2P call)
            dist.all_reduce(torch.zeros(1, device='cuda'))
        args.device = local % max(1, ndev)
        if args.comb and args.comb_3d_flow:
            print("ERROR: a sharded decode runs the 2D / 3D (-F) comb (NTSC) or the PAL Y/C decoder: the optical "
                  "flow's estimate chains over every frame")
            return 1
    dec = GPUDecoder(system=system, device=args.device, batch=args.batch)
    if args.comb_args:
        import shlex
        import comb_ntsc
        ca = comb_ntsc.parse(shlex.split(args.comb_args))
        if isinstance(ca, int) or ca.write8 or ca.pulldown or ca.images or ca.oneframe or ca.dim != 2 or \
                system != 'NTSC':
            print("ERROR: --comb-args takes comb-ntsc's arithmetic options (-I -b -n -N -B -a -L -Q -v -l), NTSC")
            return 1
        if args.comb_3d_flow:
            ca.opts['opticalflow'] = True
        dec.ctx.comb_set_opts(**ca.opts)
    elif args.comb_3d_flow:
        dec.ctx.comb_set_opts(opticalflow=True)
    samples_per_frame = dec.rf.samples_per_frame                 # int(fs / FPS) + 1
    bytes_per_frame = samples_per_frame * 5 // 4                 # for 10-bit packed files
    infile_size = os.path.getsize(filename)
    if (infile_size // bytes_per_frame - firstframe) < 2:
        print('Error: start frame is past end of file')
        return 1

    fmt = fmt_from_path(filename)
    raw = np.memmap(filename, dtype=np.uint8, mode='r')
    if world == 1 and args.window_mb > 0:
        # streamed from storage through an HBM ring, the read overlapped with the decode
        dec.open_stream(filename, fmt, args.window_mb << 20, first_sample=firstframe * dec.rf.samples_per_frame)
    elif world == 1 or args.seek >= 0 or args.cut:
        dec.set_capture(raw, fmt)
    else:
        dec.cap_bytes, dec.cap_nsamples, dec.fmt = infile_size, samples_in_bytes(fmt, infile_size), fmt

    if args.seek >= 0:
        nextsample = dec.findframe(args.seek, firstframe * samples_per_frame)
    else:
        nextsample = firstframe * samples_per_frame

    if args.cut:
        print(args.seek, args.end)
        lastsample = dec.findframe(args.end, nextsample)
        lastsample += int(samples_per_frame * .25)
        total = samples_in_bytes(fmt, infile_size)
        with open(outname + '.r16', 'wb') as out:
            for i in range(nextsample, lastsample, 16384):
                n = min(16384, lastsample - i, max(0, total - i))
                out.write(read_samples(raw, fmt, i, n).astype(np.int16).tobytes())
        return 0

    num_frames = req_frames if req_frames is not None else infile_size // bytes_per_frame - firstframe
    if world > 1 or args.epoch_frames or args.manifest:
        if args.comb and args.comb_3d and (args.epoch_frames or args.manifest):
            print("ERROR: an epoch-wise decode runs the 2D comb (NTSC) or the PAL Y/C decoder only")
            return 1
        if dec.ctx.comb_width != 744:
            print("ERROR: a sharded or epoch-wise decode does not hand comb-ntsc -W's Y-NR history across pieces")
            return 1
        return sharded(args, dec, outname, firstframe, num_frames, nextsample, req_frames, raw, fmt, rccl, world)
    tbc = open(outname + '.tbc', 'wb')
    pcm = open(outname + '.pcm', 'wb')
    rgb = open(outname + '.rgb', 'wb') if args.comb else None
    meta_all = []
    w = Writer()
    # the .rgb (2.2 MB per frame, more than twice the .tbc) on a writer of its own: the
    # two files' writes proceed in parallel (a file's buffered writes are serialised)
    w_rgb = Writer() if rgb else None

    def sink(frame, audio, meta):
        def write():
            print('frame ', meta['vbi']['framenr'])
            tbc.write(np.ascontiguousarray(frame))
            pcm.write(np.ascontiguousarray(audio))
            meta_all.append(meta)
        w.put(write)

    def comb_sink(r):
        w_rgb.put(lambda: rgb.write(np.ascontiguousarray(r)))

    def frame_log(lines):
        w.put(lambda: print('\n'.join(lines)))   # the reference's per-field lines

    def drain():
        w.drain()
        if w_rgb:
            w_rgb.drain()

    dec.frame_log = frame_log
    dec.before_ring_reuse = drain
    t0 = time.perf_counter()
    try:
        n = dec.decode(start_frame=firstframe, length=num_frames, sink=sink, comb=args.comb,
                       comb_sink=comb_sink if rgb else None, start_sample=nextsample,
                       comb3d=(args.comb_3d_core, args.comb_3d_range) if args.comb_3d else None)
        t_dec = time.perf_counter() - t0
    finally:
        dec.before_ring_reuse = None
        w.close()
        if w_rgb:
            w_rgb.close()
    if req_frames is not None and n < req_frames:
        print('Warning: end of file reached before requested number of frames were decoded')
    tbc.close()
    pcm.close()
    if rgb:
        rgb.close()
    if not args.no_json:
        with open(outname + '.json', 'w') as fh:
            fh.write(json.dumps(meta_all))     # the C encoder, one write: 5x json.dump's pace
    t_all = time.perf_counter() - t0
    if args.stats_json:
        write_stats(args.stats_json, dec, n, meta_all, t_dec, t_all, w, w_rgb)
    return 0


def write_stats(path, dec, n, metas, t_dec, t_all, w, w_rgb=None):
    """The run's timing breakdown (one process): where the wall time went between
    reading the file, the decode, and writing the outputs."""
    first = metas[0]['fields'][0]['readsample'] if metas else 0
    consumed = (metas[-1]['nextsample'] - first) if metas else 0
    st = dec.stats
    out = {'frames': n, 'rf_samples_consumed': consumed, 'decode_wall_s': round(t_dec, 4),
           'total_wall_s': round(t_all, 4),
           'rf_msamples_per_s': round(consumed / t_all / 1e6, 3) if t_all else None,
           'fields_per_s': round(2 * n / t_all, 1) if t_all else None,
           'decode_thread_s': {k: round(st.get(k, 0.0), 4) for k in ('plan_s', 'gpu_s', 'replay_s', 'flush_s',
                                                                       'wait_s')},
           'writer': {'busy_s': round(w.busy_s, 4), 'decode_waited_s': round(w.drain_s, 4)},
           'rgb_writer': ({'busy_s': round(w_rgb.busy_s, 4), 'decode_waited_s': round(w_rgb.drain_s, 4)}
                          if w_rgb else None),
           'reads_decoded': st.get('reads'), 'reads_used': st.get('reads_used'),
           'stream_seeks': st.get('stream_seeks', 0)}
    if dec.stream:
        s = dec.ctx.stream_stats()
        out['stream'] = dict(s, read_gbs=round(s['bytes_read'] / max(s['read_s'], 1e-9) / 1e9, 3))
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1)


def load_window(dec, raw, fmt, rank, world, start, rccl, start_frame=0, length=None):
    """This rank's capture window in HBM: its own samples read from storage, the tail
    halo from the next rank (ldgpu/shard.py exchange_halo: RCCL between the capture
    buffers, or gloo through host memory).  Returns what must stay alive."""
    import torch
    from ldgpu.shard import decode_bounds, exchange_halo, sample_byte, shard_windows, torch_p2p
    nbytes = raw.size
    bounds = decode_bounds(dec.cap_nsamples, dec.cap_bytes, dec.rf.samples_per_frame, world, start_frame,
                           length, start)[0]
    windows = shard_windows(bounds, dec.rf.samples_per_frame, dec.cap_nsamples)
    lo, cut, hi = windows[rank]
    end_b = lambda s: nbytes if s >= dec.cap_nsamples else sample_byte(fmt, s)   # noqa: E731
    bl, bc, bh = sample_byte(fmt, lo), end_b(cut), end_b(hi)
    if rccl:
        buf = torch.empty(bh - bl, dtype=torch.uint8, device='cuda')
        buf[:bc - bl].copy_(torch.from_numpy(np.ascontiguousarray(raw[bl:bc])))
    else:
        buf = torch.empty(bh - bl, dtype=torch.uint8)
        buf[:bc - bl].numpy()[:] = raw[bl:bc]
    got = exchange_halo(buf, rank, windows, fmt, torch_p2p)
    if not got and bh > bc:                         # halo not held by the next rank: from storage
        src = torch.from_numpy(np.ascontiguousarray(raw[bc:bh]))
        buf[bc - bl:].copy_(src)
    if rccl:
        torch.cuda.synchronize()
        dec.set_capture(None, fmt, device_ptr=buf.data_ptr(), nsamples=hi - lo, first_sample=lo,
                        total_bytes=nbytes)
    else:
        dec.set_capture(buf.numpy(), fmt, first_sample=lo, total_bytes=nbytes)
    print('rank %d: capture window samples [%d, %d), halo %s' % (rank, lo, hi,
          'from rank %d over %s' % (rank + 1, 'RCCL' if rccl else 'gloo') if got else 'from storage'))
    return buf


def widen_window(dec, raw, fmt, rccl, sample, keep):
    """A resumed decode (the last rank reading on past the decode's nominal end over
    skipped fields) needs samples past its window: make [a frame before `sample`, eight
    frames and a read after it) resident from storage.  keep: holds the buffer alive."""
    import torch
    from ldgpu.shard import sample_byte, widen_window as window_at
    lo, hi = window_at(sample, dec.rf.samples_per_frame, dec.cap_nsamples)
    nbytes = raw.size
    bl, bh = sample_byte(fmt, lo), (nbytes if hi >= dec.cap_nsamples else sample_byte(fmt, hi))
    src = torch.from_numpy(np.ascontiguousarray(raw[bl:bh]))
    if rccl:
        buf = src.to('cuda')
        torch.cuda.synchronize()
        dec.set_capture(None, fmt, device_ptr=buf.data_ptr(), nsamples=hi - lo, first_sample=lo, total_bytes=nbytes)
    else:
        buf = src
        dec.set_capture(buf.numpy(), fmt, first_sample=lo, total_bytes=nbytes)
    keep[:] = [buf]
    print('capture window widened to samples [%d, %d)' % (lo, hi))


def system_of(dec):
    return dec.sysp.name


def write_manifest(path, man):
    """Replace the manifest atomically and durably: the temp file's bytes, the rename
    and the directory entry reach storage before the next epoch starts."""
    tmp = path + '.tmp'
    with open(tmp, 'w') as fh:
        json.dump(man, fh)
        fh.flush()
        os.fsync(fh.fileno())
    os.replace(tmp, path)
    d = os.open(os.path.dirname(os.path.abspath(path)), os.O_RDONLY)
    try:
        os.fsync(d)
    finally:
        os.close(d)


def sharded(args, dec, outname, firstframe, num_frames, nextsample, req_frames, raw, fmt, rccl, world):
    """This rank's share of a field-group sharded decode (any world size), in epochs of
    --epoch-frames frames (default: one epoch).  Every rank writes its frames at their
    global offsets in the .tbc / .pcm (/ .rgb); rank 0 writes the .json.  An epoch is a
    complete decode: the next starts from the exact chain state after its last frame
    (ShardedDecode.end_state), so the result equals one decode; with --manifest the
    state is saved after every epoch and a rerun resumes after the last finished one."""
    from ldgpu.shard import comb3d_sharded, decode_sharded
    comb3d = bool(args.comb and args.comb_3d)      # after the decode, on the rank's frames
    if world > 1:
        import torch.distributed as dist
        rank = dist.get_rank()

        def allgather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
        barrier = dist.barrier
    else:
        rank = 0

        def allgather(obj):
            return [obj]

        def barrier():
            pass

    def whole():
        print('rank %d: a read left the capture window; using the whole capture' % rank)
        dec.set_capture(raw, fmt)

    exts = ('.tbc', '.pcm', '.rgb') if args.comb else ('.tbc', '.pcm')
    parts = outname + '.json.part'             # one JSON line of frame metadata per finished epoch
    st = os.stat(args.infile)
    # what makes the manifest this decode's: the input (path, size, mtime), the frame
    # range and every option that changes the outputs or the chain state it carries
    ident = {'infile': os.path.abspath(args.infile), 'infile_size': st.st_size, 'infile_mtime_ns': st.st_mtime_ns,
             'exts': list(exts), 'num_frames': num_frames, 'firstframe': firstframe, 'seek': args.seek,
             'start_sample': int(nextsample), 'system': dec.sysp.name, 'comb': bool(args.comb),
             'comb_args': args.comb_args, 'no_json': bool(args.no_json)}
    man = None
    if args.manifest and os.path.exists(args.manifest):
        with open(args.manifest) as fh:
            man = json.load(fh)
        if any(man.get(k) != v for k, v in ident.items()):
            print('ERROR: %s belongs to another decode' % args.manifest)
            return 1
        if man.get('complete'):
            if rank == 0:
                print('%s: the decode is already complete (%d frames)' % (args.manifest, man['frames']))
            if world > 1:
                import torch.distributed as dist
                dist.destroy_process_group()
            return 0
        if rank == 0:
            print('resuming after epoch %d (%d frames written)' % (man['epoch'], man['frames']))
    if man is None:
        man = dict(ident, epoch=0, frames=0, pcm_bytes=0, state=None, nextsample=int(nextsample), complete=False)
        if rank == 0:
            for ext in exts:
                open(outname + ext, 'wb').close()
            open(parts, 'w').close()
    elif rank == 0:
        # drop a metadata line written after the manifest's last epoch (a crash in between);
        # a part file lost with nothing in it yet (epoch 0) starts empty
        lines = []
        if os.path.exists(parts):
            with open(parts) as fh:
                lines = fh.readlines()[:man['epoch']]
        elif man['epoch'] and not args.no_json:
            print('ERROR: %s is missing; the metadata of the finished epochs is lost' % parts)
            return 1
        with open(parts, 'w') as fh:
            fh.writelines(lines)
    barrier()
    frame_bytes = dec.sysp.outlinelen * dec.sysp.frame_lines * 2
    rgb_bytes = (1057 * 576 if system_of(dec) == 'PAL' else dec.ctx.comb_width * dec.ctx.comb_lines) * 3 * 2
    epoch_frames = args.epoch_frames or num_frames
    stats = {}
    while not man['complete'] and man['frames'] < num_frames:
        n = min(epoch_frames, num_frames - man['frames'])
        keep = []
        widen = None
        if world > 1:
            keep = [load_window(dec, raw, fmt, rank, world, man['nextsample'], rccl, firstframe, n)]
            widen = lambda s, keep=keep: widen_window(dec, raw, fmt, rccl, s, keep)   # noqa: E731
        ep = {}
        # the rank's frames (and with --comb their rgb48, combed in HBM as they are decoded)
        # wait in spill files beside the outputs until their global offsets are known
        # (bounded host memory for any capture length)
        res = decode_sharded(dec, rank, world, allgather, start_frame=firstframe, length=n,
                             start_sample=man['nextsample'], whole_capture=whole,
                             spill_dir=os.path.dirname(os.path.abspath(outname)), comb=args.comb and not comb3d,
                             stats=stats,
                             init=man['state'], epoch_end=ep, widen=widen)
        sizes = allgather((len(res), sum(r[2].nbytes for r in res)))
        first = man['frames'] + sum(k for k, _ in sizes[:rank])
        pcm_off = man['pcm_bytes'] + sum(b for _, b in sizes[:rank])
        with open(outname + '.tbc', 'r+b') as tbc, open(outname + '.pcm', 'r+b') as pcm:
            tbc.seek(first * frame_bytes)
            pcm.seek(pcm_off)
            for r in res:
                print('frame ', r[3]['vbi']['framenr'])
                tbc.write(r[1].tobytes())
                pcm.write(r[2].tobytes())
            for fh in (tbc, pcm):         # on storage before the manifest claims the epoch
                fh.flush()
                os.fsync(fh.fileno())
        if comb3d:
            # the 3D comb (-d 3 -F) over the rank's frames with its neighbours' boundary
            # frames and the exact burst-level EMA (ldgpu/shard.py comb3d_sharded); output
            # index = global frame - 1 (the capture's first and last frames have no rgb48)
            outs = comb3d_sharded(dec, rank, allgather, [r[1] for r in res], first, args.comb_3d_core,
                                  args.comb_3d_range, stats)
            with open(outname + '.rgb', 'r+b') as fh:
                for k, rgb in outs:
                    fh.seek(k * rgb_bytes)
                    fh.write(np.ascontiguousarray(rgb).tobytes())
                fh.flush()
                os.fsync(fh.fileno())
        elif args.comb:
            # combed in HBM during the decode; the burst-level EMA (comb-ntsc.cxx:560-566,
            # global over every frame) was handed across the ranks and the first frames
            # re-combed with it (ldgpu/shard.py comb_fix)
            if system_of(dec) == 'NTSC':
                print('rank %d: comb re-combed %d frame(s) with the exact burst-level state' %
                      (rank, stats.get('comb_recombed_frames', 0)))
            with open(outname + '.rgb', 'r+b') as fh:
                fh.seek(first * rgb_bytes)
                for r in res:
                    fh.write(np.ascontiguousarray(r[4]).tobytes())
                fh.flush()
                os.fsync(fh.fileno())
        metas = allgather([r[3] for r in res])
        total = sum(k for k, _ in sizes)
        barrier()                                    # every rank's bytes of this epoch are written
        man['epoch'] += 1
        man['frames'] += total
        man['pcm_bytes'] += sum(b for _, b in sizes)
        man['state'] = ep or None
        man['nextsample'] = ep.get('nextsample', man['nextsample'])
        if total == 0 or not ep or total < n:
            man['complete'] = True                   # end of the capture (the EOF guard or the limit)
        if rank == 0:
            with open(parts, 'a') as fh:
                fh.write(json.dumps([m for part in metas for m in part]) + '\n')
                fh.flush()
                os.fsync(fh.fileno())
            if args.manifest:
                write_manifest(args.manifest, man)
        barrier()
        if int(os.environ.get('LDG_FAULT_AFTER_EPOCHS', '0') or 0) == man['epoch']:
            print('rank %d: fault injected after epoch %d (LDG_FAULT_AFTER_EPOCHS)' % (rank, man['epoch']), flush=True)
            os._exit(3)
    if rank == 0:
        if req_frames is not None and man['frames'] < req_frames:
            print('Warning: end of file reached before requested number of frames were decoded')
        if not args.no_json:
            with open(parts) as fh:
                allm = [m for line in fh for m in json.loads(line)]
            with open(outname + '.json', 'w') as fh:
                fh.write(json.dumps(allm))
        if args.manifest:
            # complete before the part file goes: a rerun then finds the decode done
            man['complete'] = True
            write_manifest(args.manifest, man)
        os.remove(parts)
    barrier()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
