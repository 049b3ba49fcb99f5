// ORACLE -- TEST INFRASTRUCTURE ONLY.  C++ restatement of the reference NTSC
// comb filter's default path (comb-ntsc.cxx, dim = 2, no pulldown, 16-bit
// output) and of its non-optical-flow 3D path (-d 3 -F), used as the checker
// for the GPU comb.  PARITY UNPINNED against the
// reference binary itself (running it is denied; it also needs
// OpenCV, absent here); pinned by known-answer tests in tests/test_comb.py.
//
// Built with -ffp-contract=off (oracle/Makefile): the reference's clang build
// contracts or not depending on the compiler version, so the GPU tolerance is
// +-1 LSB.  Stage map (reference file:line):
//   Comb::Process (dim 2)           comb-ntsc.cxx:834-892
//   Split1D                         :246-288   (clp0; its filtered tc1f is dim 1 only)
//   Split2D                         :294-367   (clp1, combk)
//   SplitIQ                         :414-483   (held I / Q samples)
//   AdjustY                         :735-763
//   FilterIQ                        :212-243   (fresh colorlpi IIR per line, HQ)
//   VBI copy                        :870-877
//   DoYNR                           :523-553   (persistent f_nr FIR across lines + frames)
//   DoCNR                           :485-521   (persistent f_nrc FIRs on I and Q, -N)
//   ToRGB / RGB::conv / u16_to_ire  :555-598, :124-147, :116-121
//   PostProcess + WriteFrame        :894-938, :704-733 (rows 38..517, x 78..821)
//   3D (-d 3 -F): Process with f = 1 :837,851-866 (no output for the first two
//   frames; frame k is combed with frames k-1 and k+1 once k+1 arrives),
//   Split3D(opt_flow = false)       :369-412   (clp2, combk2 from the lp_3d-filtered
//                                               frame difference; combk1 = 1 - combk2)
//   p_3dcore / p_3drange defaults   :1077-1082 (1.25 / 5.5 IRE, times irescale)
//   Build-defined (parity unpinned): Split3D reads _k[4] and _k[832..835],
//   which it never writes (uninitialised stack in the reference); here 0.
//   Filter::feed (DF-I order)       ld-decoder.h:167-214
//   f_nr, f_nrc, f_colorlpi/q       deemp.h:367-380, :412-423, :425-441
// Options (main's getopt, comb-ntsc.cxx:972-1091), struct Opts: -I black_ire,
// -b brightness, -n nr_y, -N nr_c, -B b&w, -a (adaptive 2D off), -L (no colour
// LPF), -Q (Q through colorlpq), -v (linesout 525: firstline 20, the VBI copy
// shows), -l (debug line blacked out), -W (910-wide output from x 0: PostProcess's
// rout_x / roffset, :898-899; DoYNR's cross-line FIR history then reaches x 40..51).
// Output frames are 744 (910 with -W) x linesout.
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

constexpr int IN_X = 910, IN_Y = 525;
constexpr int OUT_W = 744, OUT_X0 = 78;
constexpr double IRESCALE = 358.4, IREBASE = 1024.0;
constexpr double P_2DRANGE = 45 * IRESCALE;  // Split2D sets it per pixel

// deemp.h f_nr (25-tap high pass used by DoYNR)
const double NR_B[25] = {
    1.141291975113614e-04, -1.857019211291029e-03, -4.499636864042073e-03, -5.577680979937061e-03,
    -4.423694440267179e-04, 1.309163063177155e-02,  2.861211356202848e-02,  3.029931283148555e-02,
    1.098965697652802e-03,  -6.398130386469833e-02, -1.492080690537196e-01, -2.223459379380252e-01,
    7.479077367478024e-01,  -2.223459379380252e-01, -1.492080690537196e-01, -6.398130386469833e-02,
    1.098965697652803e-03,  3.029931283148557e-02,  2.861211356202848e-02,  1.309163063177156e-02,
    -4.423694440267185e-04, -5.577680979937061e-03, -4.499636864042074e-03, -1.857019211291030e-03,
    1.141291975113614e-04};
// Split3D's lp_3d (fir1(16, 0.1), comb-ntsc.cxx:379)
const double LP3D_B[17] = {0.005719569452904, 0.009426612841315, 0.019748592575455, 0.036822680065252,
                           0.058983880135427, 0.082947830292278, 0.104489989820068, 0.119454688318951,
                           0.124812312996699, 0.119454688318952, 0.104489989820068, 0.082947830292278,
                           0.058983880135427, 0.036822680065252, 0.019748592575455, 0.009426612841315,
                           0.005719569452904};
// deemp.h f_colorlpi (1-pole IIR; the HQ default uses it for I and Q) and f_colorlpq (-Q: Q)
constexpr double LPI_B0 = 2.267438981796600e-01, LPI_B1 = 2.267438981796600e-01;
constexpr double LPI_A1 = -5.465122036406802e-01;
constexpr double LPQ_B0 = 1.169303716013410e-01, LPQ_B1 = 1.169303716013410e-01;
constexpr double LPQ_A1 = -7.661392567973181e-01;
// deemp.h f_nrc (17-tap high pass used by DoCNR)
const double NRC_B[17] = {
    -3.148569668063267e-03, -4.941974513425438e-03, -9.929538598536455e-03, -1.787793973911701e-02,
    -2.783702315543740e-02, -3.829928032339736e-02, -4.750186865627083e-02, -5.380281552534787e-02,
    9.469899799540406e-01,  -5.380281552534787e-02, -4.750186865627083e-02, -3.829928032339737e-02,
    -2.783702315543740e-02, -1.787793973911701e-02, -9.929538598536455e-03, -4.941974513425442e-03,
    -3.148569668063267e-03};

// the options main() sets before Process runs (values as typed on the command line)
struct Opts {
  double black_ire = 7.5, brightness = 236, nr_y = 1.0, nr_c = 0.0;
  int bw = 0, adaptive2d = 1, colorlpf = 1, colorlpf_hq = 1, linesout = 480, debugline = -1000, wide = 0;
  double nr_min = 0;   // raw: the 3D flow path's DoYNR / DoCNR(..., 4) raise both clips to 4 (:487-488,527-529)
  int out_w() const { return wide ? IN_X : OUT_W; }
  int out_x0() const { return wide ? 0 : OUT_X0; }
};

struct YIQ { double y = 0, i = 0, q = 0; };

double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

// u16_to_ire of a double passed where the reference takes uint16_t: the
// implicit conversion truncates toward zero (x86: to int32, then the low 16 bits).
double u16_to_ire_of(double v) {
  const uint16_t level = (uint16_t)(int32_t)v;
  if (level == 0) return -100;
  return -40 + ((double)level - IREBASE) / IRESCALE;
}

// Filter::feed of an FIR (a = {1}): y = sum_o (b[o] / 1.0) * x[o], history across calls
template <int N>
struct Fir {
  const double* b;
  double x[N] = {0};
  double feed(double v) {
    std::memmove(&x[1], &x[0], sizeof(double) * (N - 1));
    x[0] = v;
    double y0 = 0;
    for (int o = 0; o < N; o++) y0 += (b[o] / 1.0) * x[o];
    return y0;
  }
};

struct Comb {
  double aburstlev = -1;          // EMA of the burst level, global across frames
  Opts o;
  // f_hpy, f_hpi, f_hpq (the Comb members DoYNR / DoCNR feed; never reset)
  Fir<25> hpy{NR_B};
  Fir<17> hpi{NRC_B}, hpq{NRC_B};
  int firstline() const { return (o.linesout == IN_Y) ? 20 : 38; }
  double nr_y() const { return std::max(o.nr_y * IRESCALE, o.nr_min); }   // main(): nr_y *= irescale
  double nr_c() const { return std::max(o.nr_c * IRESCALE, o.nr_min); }

  // prev / next: the frames before and after `raw` for the 3D path (-d 3 -F),
  // null for 2D; core / range: p_3dcore / p_3drange (already times irescale).
  // kmap (3D with optical flow, Split3D(f, true) :395-407): combk[2] per pixel (525 x 910,
  // from the flow of OpticalFlow3D, oracle/farneback.py), clp2 = next - raw; prev unused.
  // luma_out: instead of colour, the flow path's luma (AdjustY + DoYNR of the 2D
  // decode, comb-ntsc.cxx:851-856) as 525 x 910 doubles (rgb unused).
  void process(const uint16_t* raw, uint16_t* rgb, const uint16_t* prev = nullptr, const uint16_t* next = nullptr,
               double core = 0, double range = 1, const double* kmap = nullptr, double* luma_out = nullptr) {
    // ---- Split1D: clp0 (lines 44..524), combk0 = 1 there
    static double clp0[IN_Y + 2][IN_X], clp1[IN_Y][IN_X], k0[IN_Y][IN_X], k1[IN_Y][IN_X];
    std::memset(clp0, 0, sizeof(clp0));
    std::memset(clp1, 0, sizeof(clp1));
    std::memset(k0, 0, sizeof(k0));
    std::memset(k1, 0, sizeof(k1));
    for (int l = 44; l < IN_Y; l++) {
      const uint16_t* line = raw + l * IN_X;
      for (int h = 4; h < 840; h++) {
        const int avg = ((int)line[h + 2] + (int)line[h - 2]) / 2;   // integer /2
        clp0[l][h] = (double)(avg - (int)line[h]);
        k0[l][h] = 1;
      }
    }
    // ---- Split2D (lines 36..524; 2D values for l < 524; n1line of l = 523
    //      is row 525, which the reference reads as the zeroed next plane)
    for (int l = 36; l < IN_Y; l++) {
      const double* p1 = clp0[l - 2];
      const double* c1 = clp0[l];
      const double* n1 = clp0[l + 2];
      if (l >= 4 && l < 524) {
        for (int h = 18; h < 840; h++) {
          double kp = std::fabs(std::fabs(c1[h]) - std::fabs(p1[h]));
          kp += std::fabs(std::fabs(c1[h - 1]) - std::fabs(p1[h - 1]));
          kp -= (std::fabs(c1[h]) + std::fabs(c1[h - 1])) * .10;
          double kn = std::fabs(std::fabs(c1[h]) - std::fabs(n1[h]));
          kn += std::fabs(std::fabs(c1[h - 1]) - std::fabs(n1[h - 1]));
          kn -= (std::fabs(c1[h]) + std::fabs(n1[h - 1])) * .10;
          kp /= 2;
          kn /= 2;
          kp = clampd(1 - (kp / P_2DRANGE), 0, 1);
          kn = clampd(1 - (kn / P_2DRANGE), 0, 1);
          if (!o.adaptive2d) kn = kp = 1.0;
          double sc = 1.0;
          if (kn != 0 || kp != 0) {
            if (kn > (3 * kp)) kp = 0;
            else if (kp > (3 * kn)) kn = 0;
            sc = (2.0 / (kn + kp));
            if (sc < 1.0) sc = 1.0;
          } else if ((std::fabs(std::fabs(p1[h]) - std::fabs(n1[h])) - std::fabs((n1[h] + p1[h]) * .2)) <= 0) {
            kn = kp = 1;
          }
          double tc1 = ((c1[h] - p1[h]) * kp * sc);
          tc1 += ((c1[h] - n1[h]) * kn * sc);
          tc1 /= (2 * 2);
          clp1[l][h] = tc1;
          k1[l][h] = 1.0;
        }
      }
      for (int h = 4; h < 840; h++) {
        // combk[1] *= 1 - combk[2] (combk[2] = 0 in 2D); combk[0] = 1 - combk[2] - combk[1]
        k0[l][h] = 1 - 0.0 - k1[l][h];
      }
    }
    // ---- Split3D (opt_flow = false; lines 36..524, h 4..839): Frame[0] = next,
    //      Frame[1] = raw, Frame[2] = prev
    static double clp2[IN_Y][IN_X], k2[IN_Y][IN_X];
    std::memset(clp2, 0, sizeof(clp2));
    std::memset(k2, 0, sizeof(k2));
    if (kmap) {
      for (int l = 36; l < IN_Y; l++) {
        for (int h = 4; h < 840; h++) {
          const int adr = l * IN_X + h;
          clp2[l][h] = (double)((int)next[adr] - (int)raw[adr]);
          k2[l][h] = kmap[adr];
          if (l >= 2 && l <= 523) k1[l][h] = 1 - k2[l][h];
          k0[l][h] = 1 - k2[l][h] - k1[l][h];
        }
      }
    } else if (prev) {
      for (int l = 36; l < IN_Y; l++) {
        const int o = l * IN_X;
        double x[IN_X] = {0}, kk[IN_X] = {0};   // __k fed at h = 13..839; _k[4], _k[832..835] stay 0
        for (int h = 4; h < 840; h++) {
          const int adr = o + h;
          double k = std::abs((int)next[adr] - (int)prev[adr]);
          k += std::abs(((int)raw[adr] - (int)prev[adr]) - ((int)raw[adr] - (int)next[adr]));
          if (h > 12) x[h] = k;
          if (h >= 836) kk[h] = k;
        }
        for (int j = 5; j <= 831; j++) {       // _k[h - 8] = lp_3d.feed(__k(h)), h = 13..839
          double y0 = 0;
          // the filter's history before its first feed is zero: taps reaching before x[0]
          // (j + 8 - t < 0 for j = 5..7) add 0 (an out-of-bounds read before tests/san's ASan run)
          for (int t = 0; t < 17; t++) y0 += (LP3D_B[t] / 1.0) * (j + 8 - t >= 0 ? x[j + 8 - t] : 0.0);
          kk[j] = y0;
        }
        for (int h = 4; h < 840; h++) {
          const int adr = o + h;
          clp2[l][h] = (double)((((int)next[adr] + (int)prev[adr]) / 2) - (int)raw[adr]);
          k2[l][h] = clampd(1 - ((kk[h] - core) / range), 0, 1);
          if (l >= 2 && l <= 523) k1[l][h] = 1 - k2[l][h];
          k0[l][h] = 1 - k2[l][h] - k1[l][h];
        }
      }
    }
    // ---- SplitIQ -> cbuf (lines 36..524; everything else zero)
    static YIQ cb[IN_Y][IN_X];
    std::memset(cb, 0, sizeof(cb));
    for (int l = 36; l < IN_Y; l++) {
      const uint16_t* line = raw + l * IN_X;
      const bool invertphase = (line[0] == 16384);
      double si = 0, sq = 0;
      for (int h = 4; h < 840; h++) {
        double cavg = 0;
        cavg += clp2[l][h] * k2[l][h];   // clpbuffer[2] * combk[2] (0 in 2D)
        cavg += clp1[l][h] * k1[l][h];
        cavg += clp0[l][h] * k0[l][h];
        cavg /= 2;
        if (!invertphase) cavg = -cavg;
        switch (h % 4) {
          case 0: si = cavg; break;
          case 1: sq = -cavg; break;
          case 2: si = -cavg; break;
          case 3: sq = cavg; break;
        }
        cb[l][h].y = line[h];
        cb[l][h].i = si;
        cb[l][h].q = sq;
        if (o.bw) cb[l][h].i = cb[l][h].q = 0;
      }
    }
    const int FL = firstline();
    // ---- AdjustY (lines firstline..524): p[h] = p[h + 2] with y += +-I / +-Q
    for (int l = FL; l < IN_Y; l++) {
      const bool invertphase = (raw[l * IN_X] == 16384);
      for (int h = 2; h < 842; h++) {
        YIQ y = cb[l][h + 2];
        double comp = 0;
        switch (h % 4) {
          case 0: comp = y.i; break;
          case 1: comp = -y.q; break;
          case 2: comp = -y.i; break;
          case 3: comp = y.q; break;
        }
        if (invertphase) comp = -comp;
        y.y += comp;
        cb[l][h] = y;
      }
    }
    if (luma_out) {
      // the flow path: AdjustY above, then DoYNR with its taps inside the row (h >= 70 is
      // all the flow reads), no FilterIQ / VBI copy; rows below firstline keep SplitIQ's Y
      const double NRY = nr_y();
      for (int l = 0; l < IN_Y; l++)
        for (int h = 0; h < IN_X; h++) {
          double y = cb[l][h].y;
          if (l >= FL && NRY > 0 && h >= 40 && h + 12 <= 843) {
            double y0 = 0;
            for (int q = 0; q < 25; q++) y0 += (NR_B[q] / 1.0) * cb[l][h + 12 - q].y;
            double a = y0;
            if (std::fabs(a) > NRY) a = (a > 0) ? NRY : -NRY;
            y = cb[l][h].y - a;
          }
          luma_out[l * IN_X + h] = y;
        }
      return;
    }
    // ---- FilterIQ (lines 44..524, f_colorlpf): fresh colorlpi for I and for Q (colorlpq
    //      without HQ) per line, output 2 px back
    const double qb0 = o.colorlpf_hq ? LPI_B0 : LPQ_B0, qb1 = o.colorlpf_hq ? LPI_B1 : LPQ_B1;
    const double qa1 = o.colorlpf_hq ? LPI_A1 : LPQ_A1;
    for (int l = 44; o.colorlpf && l < IN_Y; l++) {
      double xi[2] = {0, 0}, yi[2] = {0, 0}, xq[2] = {0, 0}, yq[2] = {0, 0};
      auto feed = [](double* x, double* y, double v, double b0, double b1, double a1) {
        x[1] = x[0]; y[1] = y[0];
        x[0] = v;
        double y0 = 0;
        y0 += (b0 / 1.0) * x[0];
        y0 += (b1 / 1.0) * x[1];
        y0 -= (a1 / 1.0) * y[1];
        y[0] = y0;
        return y0;
      };
      double filti = 0, filtq = 0;
      for (int h = 4; h < 840; h++) {
        switch (h % 4) {
          case 0: case 2: filti = feed(xi, yi, cb[l][h].i, LPI_B0, LPI_B1, LPI_A1); break;
          case 1: case 3: filtq = feed(xq, yq, cb[l][h].q, qb0, qb1, qa1); break;
        }
        cb[l][h - 2].i = filti;
        cb[l][h - 2].q = filtq;
      }
    }
    // ---- VBI copy: rows 0..23 <- raw lines 20..43 (Y, h 4..839; reaches the output with -v)
    for (int l = 20; l < 44; l++)
      for (int h = 4; h < 840; h++) cb[l - 20][h].y = raw[l * IN_X + h];
    // ---- DoYNR (lines firstline..524, nr_y > 0): persistent FIR fed h = 40..843, output at h + 12
    const double NRY = nr_y();
    for (int l = FL; NRY > 0 && l < IN_Y; l++) {
      double hp[IN_X + 32] = {0};
      for (int h = 40; h <= 843; h++) hp[h] = hpy.feed(cb[l][h].y);
      for (int h = 40; h < 843; h++) {
        double a = hp[h + 12];
        if (std::fabs(a) > NRY) a = (a > 0) ? NRY : -NRY;
        cb[l][h].y -= a;
      }
    }
    // ---- DoCNR (lines firstline..524, nr_c > 0): persistent FIRs fed h = 60..842, output at h + 12
    const double NRC = nr_c();
    for (int l = FL; NRC > 0 && l < IN_Y; l++) {
      YIQ hp[IN_X + 32];
      for (int h = 60; h <= 842; h++) {
        hp[h].i = hpi.feed(cb[l][h].i);
        hp[h].q = hpq.feed(cb[l][h].q);
      }
      for (int h = 60; h < 842; h++) {
        double ai = hp[h + 12].i, aq = hp[h + 12].q;
        if (std::fabs(ai) > NRC) ai = (ai > 0) ? NRC : -NRC;
        if (std::fabs(aq) > NRC) aq = (aq > 0) ? NRC : -NRC;
        cb[l][h].i -= ai;
        cb[l][h].q -= aq;
      }
    }
    // ---- ToRGB + PostProcess: rows firstline.., x 78..821 (0..909 with -W); rows past
    //      524 - firstline stay 0 (-v)
    const double m = o.brightness * 256 / 100;
    const int out_h = o.linesout;
    const int W = o.out_w(), X0 = o.out_x0();
    for (int l = FL; l < IN_Y; l++) {
      const double burstlev = raw[l * IN_X + 1] / IRESCALE;
      if (burstlev > 3) {
        if (aburstlev < 0) aburstlev = burstlev;
        aburstlev = (aburstlev * .99) + (burstlev * .01);
      }
      const int row = l - FL;
      if (row >= out_h) continue;
      for (int h = X0; h < X0 + W; h++) {
        YIQ yiq = cb[l][h];
        yiq.i *= (10 / aburstlev);
        yiq.q *= (10 / aburstlev);
        double y = u16_to_ire_of(yiq.y);
        y = (y - o.black_ire) * (100 / (100 - o.black_ire));
        const double q = +(yiq.i) / IRESCALE;
        const double i = +(yiq.q) / IRESCALE;
        double r = y + (.956 * i) + (.621 * q);
        double g = y - (.272 * i) - (.647 * q);
        double b = y - (1.106 * i) + (1.703 * q);
        r = clampd(r * m, 0, 65535);
        g = clampd(g * m, 0, 65535);
        b = clampd(b * m, 0, 65535);
        if (l == (o.debugline + 25)) r = g = b = 0;     // -l: the debug line is blacked out
        uint16_t* op = rgb + ((size_t)row * W + (h - X0)) * 3;
        op[0] = (uint16_t)r;
        op[1] = (uint16_t)g;
        op[2] = (uint16_t)b;
      }
    }
  }
};

}  // namespace

extern "C" {
void* comb2d_create() { return new Comb(); }
void comb2d_destroy(void* c) { delete static_cast<Comb*>(c); }
// the comb-ntsc options (doubles: black_ire, brightness, nr_y, nr_c; ints: bw, adaptive2d,
// colorlpf, colorlpf_hq, linesout, debugline, wide)
void comb2d_set_opts(void* c, const double* d, const int* i) {
  Opts& o = static_cast<Comb*>(c)->o;
  o.black_ire = d[0]; o.brightness = d[1]; o.nr_y = d[2]; o.nr_c = d[3];
  o.bw = i[0]; o.adaptive2d = i[1]; o.colorlpf = i[2]; o.colorlpf_hq = i[3]; o.linesout = i[4]; o.debugline = i[5];
  o.wide = i[6];
}
// n frames of 910 x 525 uint16 -> n frames of 744 (910 with -W) x linesout x 3 uint16 (rgb48)
void comb2d_process(void* c, int n, const uint16_t* frames, uint16_t* rgb) {
  Comb* cb = static_cast<Comb*>(c);
  for (int f = 0; f < n; f++)
    cb->process(frames + (size_t)f * IN_X * IN_Y, rgb + (size_t)f * cb->o.out_w() * cb->o.linesout * 3);
}
double comb2d_aburstlev(void* c) { return static_cast<Comb*>(c)->aburstlev; }
// the 3D comb with optical flow, one output frame: raw (the frame) with next and its
// weight map (525 x 910 doubles); state (aburstlev, FIR histories) as any frame
void comb2d_process_of(void* c, const uint16_t* raw, const uint16_t* next, const double* kmap, uint16_t* rgb) {
  static_cast<Comb*>(c)->process(raw, rgb, raw, next, 0, 1, kmap);
}
// the flow path's luma of a frame (525 x 910 doubles; no state touched)
void comb2d_flow_luma(void* c, const uint16_t* raw, double* luma) {
  Comb tmp = *static_cast<Comb*>(c);
  tmp.process(raw, nullptr, nullptr, nullptr, 0, 1, nullptr, luma);
}
void comb2d_set_nr_min(void* c, double v) { static_cast<Comb*>(c)->o.nr_min = v; }

// One reference process in -d 3 -F mode: its own Comb state plus the last two
// input frames.  Feeds n frames and writes one rgb48 frame per frame that now
// has both neighbours (n + history - 2 of them, >= 0); returns that count.
struct Comb3 {
  Comb c;
  std::vector<uint16_t> hist;   // up to 2 frames, oldest first
  int nhist = 0;
};
void* comb3d_create() { return new Comb3(); }
void comb3d_set_opts(void* c, const double* d, const int* i) { comb2d_set_opts(&static_cast<Comb3*>(c)->c, d, i); }
void comb3d_destroy(void* c) { delete static_cast<Comb3*>(c); }
int comb3d_process(void* h, int n, const uint16_t* frames, uint16_t* rgb, double core_ire, double range_ire) {
  Comb3* c = static_cast<Comb3*>(h);
  const size_t F = (size_t)IN_X * IN_Y;
  const double core = (core_ire < 0 ? 1.25 : core_ire) * IRESCALE;
  const double range = (range_ire < 0 ? 5.5 : range_ire) * IRESCALE;
  std::vector<uint16_t> win((size_t)(c->nhist + n) * F);
  std::copy(c->hist.begin(), c->hist.begin() + (size_t)c->nhist * F, win.begin());
  std::copy(frames, frames + (size_t)n * F, win.begin() + (size_t)c->nhist * F);
  const int L = c->nhist + n;
  int out = 0;
  for (int k = 1; k + 1 < L; k++) {
    c->c.process(&win[(size_t)k * F], rgb + (size_t)out * c->c.o.out_w() * c->c.o.linesout * 3, &win[(size_t)(k - 1) * F],
                 &win[(size_t)(k + 1) * F], core, range);
    out++;
  }
  const int keep = L < 2 ? L : 2;
  c->hist.assign(win.begin() + (size_t)(L - keep) * F, win.end());
  c->nhist = keep;
  return out;
}
double comb3d_aburstlev(void* c) { return static_cast<Comb3*>(c)->c.aburstlev; }
}
