"""ldgpu -- MI355X-native LaserDisc RF -> .tbc decode (drop-in for ld-decode's lddecode.py path).

Host side mirrors the reference interface (RFDecode / Field / Framer /
findframe, lddecode_core.py) over the C ABI of libldgpu.so (include/ldgpu.h);
all per-sample and per-line work runs as HIP kernels on gfx950.
"""

import os as _os

# A context drives 10 HIP streams (two demod streams, read setup, audio, records,
# frame output, comb, synchronous output and 2 field-chain sub-streams,
# INTEGRATION.md "Buffers and threading").  HIP maps streams onto
# GPU_MAX_HW_QUEUES hardware queues (default 4); fewer queues than streams put
# unrelated streams behind each other -- the two demod streams' launches stop
# overlapping: 20-step bench 23,134 RF MS/s with 12 queues, 21,924 with the box's
# 4 (every demod launch then starts after a gap, profiles/r06_f_bench.json) -- so
# ask for 12 before the HIP runtime initialises (the first HIP call in the process).
if int(_os.environ.get('GPU_MAX_HW_QUEUES', '0') or 0) < 12:
    _os.environ['GPU_MAX_HW_QUEUES'] = '12'
