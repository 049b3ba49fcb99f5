"""ORACLE (test infrastructure only): the dense optical flow of the reference
comb's 3D mode with flow (comb-ntsc.cxx:600-662 OpticalFlow3D, called from
Process :851-858), i.e. OpenCV's calcOpticalFlowFarneback(prev, next, flow,
0.5, 4, 60, 3, 7, 1.5, flags) -- OpenCV 3.x / 4.x CPU path,
modules/video/src/optflowgf.cpp (FarnebackPrepareGaussian, FarnebackPolyExp,
FarnebackUpdateMatrices, FarnebackUpdateFlow_Blur, and the pyramid loop of
FarnebackOpticalFlowImpl::calc), with getGaussianKernel / GaussianBlur
(BORDER_REFLECT_101) and resize (INTER_LINEAR, INTER_AREA) as that loop uses
them.

PARITY UNPINNED: OpenCV is not installed here (`import cv2` fails, SURVEY §8
C2) and the reference may not be run (C1), so no output of the real
calcOpticalFlowFarneback pins this.  The steps, parameters, border rules and
quirks are restated from the published algorithm (Farneback 2003) and OpenCV's
implementation as documented above; the ARITHMETIC IS BUILD-DEFINED: float64
throughout (OpenCV keeps images in float32 and accumulates the blurs in
double).  The GPU path (csrc/flow.hip) follows this restatement; the tests pin
this oracle by closed-form known answers (tests/test_flow.py: zero flow for
identical images, the shift of a translated pattern).

Kept from the reference's call: the images are 252 x 840 uint16 fields of the
comb's luma (rows 23 + field + 2 y, columns 70..909; rows past 524 -- the
reference reads past its 525-row buffer there -- are 0 here), the first
argument is the NEW field and the second the previous one, and from the third
call on the last flow is the initial estimate (OPTFLOW_USE_INITIAL_FLOW).
"""
import math

import numpy as np

PYR_SCALE, LEVELS, WINSIZE, ITERATIONS, POLY_N, POLY_SIGMA = 0.5, 4, 60, 3, 7, 1.5
MIN_SIZE = 32
SMALL_GAUSSIAN = {1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
                  7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}


def cv_round(x):
    """cvRound: round half to even."""
    return int(np.rint(x))


def gaussian_kernel(ksize, sigma):
    """getGaussianKernel(ksize, sigma) (fixed tables for ksize <= 7 and sigma <= 0)."""
    if ksize % 2 == 1 and ksize <= 7 and sigma <= 0:
        return np.array(SMALL_GAUSSIAN[ksize], dtype=np.float64)
    sig = sigma if sigma > 0 else ((ksize - 1) * 0.5 - 1) * 0.3 + 0.8
    s2 = -0.5 / (sig * sig)
    x = np.arange(ksize, dtype=np.float64) - (ksize - 1) * 0.5
    t = np.exp(s2 * x * x)
    return t / t.sum()


def reflect101(i, n):
    """BORDER_REFLECT_101 index (gfedcb|abcdefgh|gfedcba)."""
    if n == 1:
        return 0
    while i < 0 or i >= n:
        i = -i if i < 0 else 2 * n - 2 - i
    return i


def gaussian_blur(img, ksize, sigma):
    """GaussianBlur(img, Size(ksize, ksize), sigma, sigma): separable, rows then columns."""
    k = gaussian_kernel(ksize, sigma)
    r = ksize // 2
    h, w = img.shape
    ix = np.array([[reflect101(x + j - r, w) for j in range(ksize)] for x in range(w)])
    iy = np.array([[reflect101(y + j - r, h) for j in range(ksize)] for y in range(h)])
    tmp = np.zeros_like(img)
    for j in range(ksize):
        tmp += k[j] * img[:, ix[:, j]]
    out = np.zeros_like(img)
    for j in range(ksize):
        out += k[j] * tmp[iy[:, j], :]
    return out


def resize_linear(img, w, h):
    """resize(INTER_LINEAR) to w x h: source coordinate (d + 0.5) * ratio - 0.5, the
    integer part and weights clamped at the borders (replicate)."""
    H, W = img.shape[:2]

    def axis(n_dst, n_src):
        r = n_src / n_dst
        f = (np.arange(n_dst, dtype=np.float64) + 0.5) * r - 0.5
        i0 = np.floor(f).astype(np.int64)
        a = f - i0
        a = np.where(i0 < 0, 0.0, a)
        i0 = np.where(i0 < 0, 0, i0)
        i1 = np.minimum(i0 + 1, n_src - 1)
        a = np.where(i0 >= n_src - 1, 0.0, a)
        i0 = np.minimum(i0, n_src - 1)
        return i0, i1, a

    x0, x1, ax = axis(w, W)
    y0, y1, ay = axis(h, H)
    ax = ax.reshape((1, -1) + (1,) * (img.ndim - 2))
    ay = ay.reshape((-1, 1) + (1,) * (img.ndim - 2))
    top = img[y0][:, x0] * (1 - ax) + img[y0][:, x1] * ax
    bot = img[y1][:, x0] * (1 - ax) + img[y1][:, x1] * ax
    return top * (1 - ay) + bot * ay


def resize_area_int(img, w, h):
    """resize(INTER_AREA) by an integer factor: the mean of each block."""
    H, W = img.shape[:2]
    fy, fx = H // h, W // w
    assert fy * h == H and fx * w == W
    return img.reshape(h, fy, w, fx, *img.shape[2:]).mean(axis=(1, 3))


def prepare_gaussian(n, sigma):
    """FarnebackPrepareGaussian: g, x g, x^2 g over -n..n and the four entries of the
    inverse moment matrix the expansion uses."""
    if sigma < 1.1920929e-07:
        sigma = n * 0.3
    x = np.arange(-n, n + 1, dtype=np.float64)
    g = np.exp(-x * x / (2 * sigma * sigma))
    g = g / g.sum()
    xg, xxg = x * g, x * x * g
    G = np.zeros((6, 6))
    gy, gx = np.meshgrid(g, g, indexing='ij')
    yy, xx = np.meshgrid(x, x, indexing='ij')
    G[0, 0] = (gy * gx).sum()
    G[1, 1] = (gy * gx * xx * xx).sum()
    G[3, 3] = (gy * gx * xx ** 4).sum()
    G[5, 5] = (gy * gx * xx * xx * yy * yy).sum()
    G[2, 2] = G[0, 3] = G[0, 4] = G[3, 0] = G[4, 0] = G[1, 1]
    G[4, 4] = G[3, 3]
    G[3, 4] = G[4, 3] = G[5, 5]
    iG = np.linalg.inv(G)
    return g, xg, xxg, iG[1, 1], iG[0, 3], iG[3, 3], iG[5, 5]


def poly_exp(src, n=POLY_N, sigma=POLY_SIGMA):
    """FarnebackPolyExp: per pixel the 5 expansion coefficients [r_y, r_x, r_yy, r_xx, r_xy]
    (separable Gaussian-weighted least squares; replicate borders)."""
    g, xg, xxg, ig11, ig03, ig33, ig55 = prepare_gaussian(n, sigma)
    h, w = src.shape
    # vertical part: row[x] = (sum g p, sum xg (below - above), sum xxg p)
    r0 = src * g[n]
    r1 = np.zeros_like(src)
    r2 = np.zeros_like(src)
    for k in range(1, n + 1):
        up = src[np.maximum(np.arange(h) - k, 0)]
        dn = src[np.minimum(np.arange(h) + k, h - 1)]
        p = up + dn
        r0 = r0 + g[n + k] * p
        r1 = r1 + xg[n + k] * (dn - up)
        r2 = r2 + xxg[n + k] * p
    # horizontal part (replicated edge pixels)
    idx = lambda d: np.clip(np.arange(w) + d, 0, w - 1)   # noqa: E731
    b1 = r0 * g[n]
    b2 = np.zeros_like(src)
    b3 = r1 * g[n]
    b4 = np.zeros_like(src)
    b5 = r2 * g[n]
    b6 = np.zeros_like(src)
    for k in range(1, n + 1):
        pr, mr = idx(k), idx(-k)
        tg = r0[:, pr] + r0[:, mr]
        b1 = b1 + tg * g[n + k]
        b4 = b4 + tg * xxg[n + k]
        b2 = b2 + (r0[:, pr] - r0[:, mr]) * xg[n + k]
        b3 = b3 + (r1[:, pr] + r1[:, mr]) * g[n + k]
        b6 = b6 + (r1[:, pr] - r1[:, mr]) * xg[n + k]
        b5 = b5 + (r2[:, pr] + r2[:, mr]) * g[n + k]
    out = np.empty((h, w, 5))
    out[..., 1] = b2 * ig11
    out[..., 0] = b3 * ig11
    out[..., 3] = b1 * ig03 + b4 * ig33
    out[..., 2] = b1 * ig03 + b5 * ig33
    out[..., 4] = b6 * ig55
    return out


BORDER = np.array([0.14, 0.14, 0.4472, 0.4472, 0.4472])


def update_matrices(R0, R1, flow):
    """FarnebackUpdateMatrices: per pixel (G11, G12, G22, h1, h2) from the expansion of
    the first image and the second's, bilinearly sampled at x + flow."""
    h, w = flow.shape[:2]
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing='ij')
    dx, dy = flow[..., 0], flow[..., 1]
    fx, fy = xx + dx, yy + dy
    x1, y1 = np.floor(fx).astype(np.int64), np.floor(fy).astype(np.int64)
    ax, ay = fx - x1, fy - y1
    inside = (x1 >= 0) & (x1 < w - 1) & (y1 >= 0) & (y1 < h - 1)
    xc, yc = np.clip(x1, 0, w - 2), np.clip(y1, 0, h - 2)
    a00, a01 = (1 - ax) * (1 - ay), ax * (1 - ay)
    a10, a11 = (1 - ax) * ay, ax * ay
    s = (a00[..., None] * R1[yc, xc] + a01[..., None] * R1[yc, xc + 1] + a10[..., None] * R1[yc + 1, xc] +
         a11[..., None] * R1[yc + 1, xc + 1])
    r2 = np.where(inside, s[..., 0], 0.0)
    r3 = np.where(inside, s[..., 1], 0.0)
    r4 = np.where(inside, (R0[..., 2] + s[..., 2]) * 0.5, R0[..., 2])
    r5 = np.where(inside, (R0[..., 3] + s[..., 3]) * 0.5, R0[..., 3])
    r6 = np.where(inside, (R0[..., 4] + s[..., 4]) * 0.25, R0[..., 4] * 0.5)
    r2 = (R0[..., 0] - r2) * 0.5
    r3 = (R0[..., 1] - r3) * 0.5
    r2 = r2 + r4 * dy + r6 * dx
    r3 = r3 + r6 * dy + r5 * dx
    bx = np.ones(w)
    by = np.ones(h)
    B = len(BORDER)
    for i in range(B):
        if i < w:
            bx[i] *= BORDER[i]
            bx[w - 1 - i] *= BORDER[i]
        if i < h:
            by[i] *= BORDER[i]
            by[h - 1 - i] *= BORDER[i]
    sc = by[:, None] * bx[None, :]
    r2, r3, r4, r5, r6 = r2 * sc, r3 * sc, r4 * sc, r5 * sc, r6 * sc
    M = np.empty((h, w, 5))
    M[..., 0] = r4 * r4 + r6 * r6
    M[..., 1] = (r4 + r5) * r6
    M[..., 2] = r5 * r5 + r6 * r6
    M[..., 3] = r4 * r2 + r6 * r3
    M[..., 4] = r6 * r2 + r5 * r3
    return M


def box_sum(M, m):
    """FarnebackUpdateFlow_Blur's running sums: per pixel the sum over rows and columns
    [-m, m] around it, borders replicated (2m + 1 = block_size + 1 taps each way)."""
    h, w = M.shape[:2]
    iy = np.clip(np.arange(h)[:, None] + np.arange(-m, m + 1)[None, :], 0, h - 1)
    ix = np.clip(np.arange(w)[:, None] + np.arange(-m, m + 1)[None, :], 0, w - 1)
    v = M[iy].sum(axis=1)
    return v[:, ix].sum(axis=2)


def update_flow(M, block_size=WINSIZE):
    """FarnebackUpdateFlow_Blur's solve: the box-blurred G and h (scale 1 / block_size^2),
    flow = G^-1 h with the 1e-3 regulariser."""
    m = block_size // 2
    S = box_sum(M, m) * (1.0 / (block_size * block_size))
    g11, g12, g22, h1, h2 = (S[..., i] for i in range(5))
    idet = 1.0 / (g11 * g22 - g12 * g12 + 1e-3)
    flow = np.empty(M.shape[:2] + (2,))
    flow[..., 0] = (g11 * h2 - g12 * h1) * idet
    flow[..., 1] = (g22 * h1 - g12 * h2) * idet
    return flow


def farneback(prev0, next0, flow0=None):
    """calcOpticalFlowFarneback(prev0, next0, flow0, 0.5, 4, 60, 3, 7, 1.5,
    OPTFLOW_USE_INITIAL_FLOW if flow0 is given): the flow (h, w, 2) in pixels, float64."""
    img = [np.asarray(prev0, dtype=np.float64), np.asarray(next0, dtype=np.float64)]
    H, W = img[0].shape
    scale, levels = 1.0, 0
    for k in range(LEVELS):
        scale *= PYR_SCALE
        if W * scale < MIN_SIZE or H * scale < MIN_SIZE:
            break
        levels = k + 1
    prev_flow = None
    flow = None
    for k in range(levels, -1, -1):
        scale = PYR_SCALE ** k
        sigma = (1.0 / scale - 1) * 0.5
        smooth = max(cv_round(sigma * 5) | 1, 3)
        w, h = cv_round(W * scale), cv_round(H * scale)
        if prev_flow is None:
            if flow0 is not None:
                flow = resize_area_int(np.asarray(flow0, dtype=np.float64), w, h) * scale
            else:
                flow = np.zeros((h, w, 2))
        else:
            flow = resize_linear(prev_flow, w, h) * (1.0 / PYR_SCALE)
        R = []
        for i in range(2):
            f = gaussian_blur(img[i], smooth, sigma)
            I = f if (w, h) == (W, H) else resize_linear(f, w, h)
            R.append(poly_exp(I))
        M = update_matrices(R[0], R[1], flow)
        for it in range(ITERATIONS):
            flow = update_flow(M)
            if it < ITERATIONS - 1:
                M = update_matrices(R[0], R[1], flow)
        prev_flow = flow
    return flow


FIELD_ROWS, FIELD_COLS, FIELD_Y0, FIELD_X0 = 252, 840, 23, 70


def field_images(ybuf):
    """The two 252 x 840 uint16 fields OpticalFlow3D hands to the flow (comb-ntsc.cxx:
    617-624): luma rows 23 + field + 2 y, columns 70..909, as uint16_t (C conversion of
    a double: toward zero, low 16 bits); rows past 524 are 0 (build-defined)."""
    y = np.asarray(ybuf, dtype=np.float64)
    out = np.zeros((2, FIELD_ROWS, FIELD_COLS), dtype=np.uint16)
    for f in range(2):
        for r in range(FIELD_ROWS):
            src = FIELD_Y0 + f + 2 * r
            if src < y.shape[0]:
                v = np.trunc(y[src, FIELD_X0:FIELD_X0 + FIELD_COLS]).astype(np.int64)
                out[f, r] = (v & 0xffff).astype(np.uint16)
    return out


def combk_from_flow(flow0, flow1, core, rng):
    """OpticalFlow3D's 3D weight (comb-ntsc.cxx:633-650): per field pixel
    c = 1 - clamp((|(fy, 2 fx)| - core) / range, 0, 1) (core / range the -c / -r values
    times irescale), the smaller of the two fields', for frame rows 2 y and 2 y + 1 at
    columns 70..909 of a 525 x 910 map (0 elsewhere)."""
    def c_of(fl):
        r = np.sqrt(fl[..., 1] * fl[..., 1] + (fl[..., 0] * 2) * (fl[..., 0] * 2))
        return 1 - np.clip((r - core) / rng, 0, 1)
    c = np.minimum(c_of(flow0), c_of(flow1))
    k = np.zeros((525, 910))
    k[0:2 * FIELD_ROWS:2, FIELD_X0:FIELD_X0 + FIELD_COLS] = c
    k[1:2 * FIELD_ROWS:2, FIELD_X0:FIELD_X0 + FIELD_COLS] = c
    return k


def _selfcheck():   # pragma: no cover - quick manual check
    rng = np.random.default_rng(1)
    a = np.kron(rng.uniform(0, 60000, (32, 105)), np.ones((8, 8)))[:252, :840]
    b = np.roll(a, 3, axis=1)
    f = farneback(b, a)
    print(np.median(f[40:-40, 60:-60, 0]), np.median(f[40:-40, 60:-60, 1]), math.nan)


if __name__ == '__main__':
    _selfcheck()
