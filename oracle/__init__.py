"""ORACLE — CPU restatement of the reference decode path. TEST INFRASTRUCTURE ONLY.

This package is the checker the HIP path is compared against.  It restates,
function by function, the reference ld-decode snapshot's RF -> TBC path
(``lddecode_core.py``, ``lddutils.py``, ``lddecode.py``) in numpy/scipy with
numpy-1.x scalar semantics pinned, plus a C++ restatement of the
2D NTSC comb (``comb-ntsc.cxx`` dim=2, built from ``oracle/comb2d.cpp``).

Rules (DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import anything from here, and only as the
    checker / CPU baseline -- never as the thing measured or shipped.
  * The product (``ld-decode_amd/ldgpu``) never imports this package.

PARITY UNPINNED (against the reference itself).  Running the reference was denied in this environment
(binding), and the reference ships no tests, fixtures or golden
vectors.  The restatement is therefore pinned by analytic
known-answer tests derived from the reference source formulas (tests/
test_oracle_kat.py) and by scipy cross-checks; outputs on the synthetic
captures are committed as golden fixtures under tests/golden/.
"""
