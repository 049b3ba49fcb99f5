"""ORACLE -- test infrastructure only.  Pure-Python restatement of the CX
expander (cx-expander.cxx:9-117) used as the checker for ldg_cx_process.
PARITY UNPINNED against the reference binary (running it is denied, SURVEY §8
C1); pinned by the known-answer tests in tests/test_cx.py (silence, the
unity-gain region below the threshold, the 2:1 expansion above it).

Stage map:
  Filter f_left/f_right(f_a500_48k), f_left30/f_right30(f_a40h_48k)   :18-19,
      deemp.h:541-575, Filter::feed DF-I order ld-decoder.h:167-214
  Process (peak followers, gain, 0.4 output scale, clamp)             :34-92
  main (1024-frame blocks, a short final block ends the stream)       :95-117
"""

A500_B = [9.180235494788952e-01, -3.672094197915581e+00, 5.508141296873371e+00, -3.672094197915581e+00,
          9.180235494788952e-01]
A500_A = [1.000000000000000e+00, -3.828986095665020e+00, 5.501429593307183e+00, -3.515193865291172e+00,
          8.427672373989403e-01]
A40H_B = [9.931821905998739e-01, -3.972728762399496e+00, 5.959093143599244e+00, -3.972728762399496e+00,
          9.931821905998739e-01]
A40H_A = [1.000000000000000e+00, -3.986317712211590e+00, 5.959046661447476e+00, -3.959139812214155e+00,
          9.864108637247646e-01]
M14DB = 0.199526231496888
FACTOR = 6500.0
BLOCK = 1024


class _Filter:
    """Filter(vector b, vector a)::feed: y0 = sum (b[o]/a0) x[o] - sum_{o>=1} (a[o]/a0) y[o]."""

    def __init__(self, b, a):
        self.b, self.a = b, a
        self.x = [0.0] * len(b)
        self.y = [0.0] * len(a)

    def feed(self, v):
        self.x = [v] + self.x[:-1]
        self.y = [0.0] + self.y[:-1]
        a0 = self.a[0]
        y0 = 0.0
        for o in range(len(self.b)):
            y0 += (self.b[o] / a0) * self.x[o]
        for o in range(1, len(self.a)):
            y0 -= (self.a[o] / a0) * self.y[o]
        self.y[0] = y0
        return y0


def _u16(v):
    c = v + 32768
    c = 0.0 if c < 0 else (65535.0 if c > 65535 else c)
    return int(c)                    # double -> uint16_t truncates


class CX:
    """One cx-expander process; process() continues the stream."""

    def __init__(self):
        self.fl, self.fr = _Filter(A500_B, A500_A), _Filter(A500_B, A500_A)
        self.fl30, self.fr30 = _Filter(A40H_B, A40H_A), _Filter(A40H_B, A40H_A)
        self.slow = self.fast = 0.0

    def process(self, pairs):
        """pairs: iterable of (left_u16, right_u16) -> list of (left_u16, right_u16)."""
        out = []
        for lu, ru in pairs:
            left, right = float(int(lu) - 32768), float(int(ru) - 32768)
            ol, orr = left, right
            left, right = self.fl.feed(left), self.fr.feed(right)
            mx = max(abs(left), abs(right))
            self.fast = self.fast * .9998
            if mx > self.fast:
                self.fast = min(mx, self.fast + (mx * .040))
            self.slow = self.slow * .999985
            if mx > self.slow:
                self.slow = min(mx, self.slow + (mx * .0020))
            val = max(self.fast, self.slow * 1.00) - (FACTOR * M14DB)
            if val < 0:
                val = 0.0
            left, right = ol * M14DB, orr * M14DB
            left *= 1 + (val / (FACTOR * M14DB))
            right *= 1 + (val / (FACTOR * M14DB))
            left, right = self.fl30.feed(left), self.fr30.feed(right)
            left *= .4
            right *= .4
            out.append((_u16(left), _u16(right)))
        return out


def stream(data):
    """cx-expander's main on a byte string: whole 1024-frame blocks only."""
    import numpy as np
    nblk = len(data) // (BLOCK * 4)
    a = np.frombuffer(data[:nblk * BLOCK * 4], dtype='<u2').reshape(-1, 2)
    return np.array(CX().process(a.tolist()), dtype='<u2').reshape(-1, 2)
