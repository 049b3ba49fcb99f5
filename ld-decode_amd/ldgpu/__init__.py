"""ldgpu -- MI355X-native LaserDisc RF -> .tbc decode (drop-in for ld-decode's lddecode.py path).

Host side mirrors the reference interface (RFDecode / Field / Framer /
findframe, lddecode_core.py) over the C ABI of libldgpu.so (include/ldgpu.h);
all per-sample and per-line work runs as HIP kernels on gfx950.
"""
