"""ldgpu -- MI355X-native LaserDisc RF -> .tbc decode (drop-in for ld-decode's lddecode.py path).

Host side mirrors the reference interface (RFDecode / Field / Framer /
findframe, lddecode_core.py) over the C ABI of libldgpu.so (include/ldgpu.h);
all per-sample and per-line work runs as HIP kernels on gfx950.
"""

# A context drives 10 HIP streams (two demod streams, read setup, audio, records,
# frame output, comb, synchronous output and 2 field-chain sub-streams,
# INTEGRATION.md "Buffers and threading") over HIP's hardware queues
# (GPU_MAX_HW_QUEUES, default 4).  8 / 12 / 16 queues measured level with 4 on the
# NTSC and PAL benches, so the process's setting is left as it is.
