// ORACLE -- TEST INFRASTRUCTURE ONLY.  C++ restatement of a PAL Y/C decoder
// for the 1135 x 625 .tbc frames (SURVEY §8 f, row F2): the dim = 2 path of
// the reference's only PAL comb, attic2/comb-pal.cxx (a prototype written for
// 1052 x 610 frames from the older tbc-pal), adapted to the current geometry.
// BUILD-DEFINED AND PARITY UNPINNED: the reference has no PAL comb for this
// geometry (comb-pal.README points to an external project), so the adaptation
// choices below are this build's, pinned only by the KATs in
// tests/test_combpal.py and checked against the GPU kernels.
//
// Stage map (attic2/comb-pal.cxx):
//   Process (dim 2, no colour LPF: f_colorlpf = false)   :820-877
//   Split1D (h +-2)                                      :234-274
//   Split2D (lines +-4, adaptive weights)                :280-353
//   SplitIQ (held U / V samples)                         :400-467
//   AdjustY (p[h] = p[h + 2], chroma re-added)           :790-817
//   DoYNR (persistent f_nr FIR, nr_y = 1 IRE)            :507-537, main :110
//   ToRGB: burst angle per line, frame phase, rotation   :539-654
//          to 135 degrees, V-switch flip, RGB::conv        :118-140
//   PostProcess (no pulldown)                            :879-917
// Adaptation (build-defined): IN_X 1135, IN_Y 625; active rows 44..619
// (lineoffset 44: 576 rows of the 625-line frame); burst-angle window
// h 100..131 (8 subcarrier cycles from 5.6 us after the line start at 4fsc);
// output 1057 x 576 (the reference's in_x - 78 crop).  Reads past a line's end
// (AdjustY's p[h + 2], DoYNR's p[in_x]) see the next line's untouched p[0..1],
// zero as in the reference's contiguous cline_t array.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr int IN_X = 1135, IN_Y = 625;
constexpr int FIRST_LINE = 44, LINES_OUT = 576, OUT_X0 = 78, OUT_W = IN_X - 78;
constexpr int BURST_H0 = 100, BURST_H1 = 132;
constexpr double IRESCALE = 376.32, IREBASE = 0.0;
constexpr double BLACK_IRE = 0.0, BRIGHTNESS = 240.0;
constexpr double NR_Y = 1.0 * IRESCALE;
constexpr double P_2DRANGE = 45 * IRESCALE;
const double NR_B[25] = {
    1.141291975113614e-04, -1.857019211291029e-03, -4.499636864042073e-03, -5.577680979937061e-03,
    -4.423694440267179e-04, 1.309163063177155e-02,  2.861211356202848e-02,  3.029931283148555e-02,
    1.098965697652802e-03,  -6.398130386469833e-02, -1.492080690537196e-01, -2.223459379380252e-01,
    7.479077367478024e-01,  -2.223459379380252e-01, -1.492080690537196e-01, -6.398130386469833e-02,
    1.098965697652803e-03,  3.029931283148557e-02,  2.861211356202848e-02,  1.309163063177156e-02,
    -4.423694440267185e-04, -5.577680979937061e-03, -4.499636864042074e-03, -1.857019211291030e-03,
    1.141291975113614e-04};

struct YUV { double y = 0, i = 0, q = 0; };

double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

double u16_to_ire_pal(double v) {      // u16_to_ire(uint16_t) of clamp(y, 0, 65535): truncation
  const uint16_t level = (uint16_t)v;
  if (level == 0) return -100;
  return -43.122874 + ((double)(level - IREBASE) / IRESCALE);
}

double atan2deg(double y, double x) {  // ld-decoder.h:73-78 (M_PIl product rounded to double)
  double rv = (double)((long double)std::atan2(y, x) * (180 / 3.141592653589793238462643383279502884L));
  if (rv < 0) rv += 360;
  return rv;
}

struct CombPAL {
  double aburstlev = -1;
  double nr_x[25] = {0};

  double nr_feed(double v) {
    std::memmove(&nr_x[1], &nr_x[0], sizeof(double) * 24);
    nr_x[0] = v;
    double y0 = 0;
    for (int o = 0; o < 25; o++) y0 += (NR_B[o] / 1.0) * nr_x[o];
    return y0;
  }

  void process(const uint16_t* raw, uint16_t* rgb) {
    static double clp0[IN_Y + 4][IN_X], clp1[IN_Y][IN_X], k0[IN_Y][IN_X], k1[IN_Y][IN_X];
    std::memset(clp0, 0, sizeof(clp0));
    std::memset(clp1, 0, sizeof(clp1));
    std::memset(k0, 0, sizeof(k0));
    std::memset(k1, 0, sizeof(k1));
    // Split1D (lines 24.., h 4..IN_X-5)
    for (int l = 24; l < IN_Y; l++) {
      const uint16_t* line = raw + l * IN_X;
      for (int h = 4; h < IN_X - 4; h++) {
        const int avg = ((int)line[h + 2] + (int)line[h - 2]) / 2;
        clp0[l][h] = (double)(avg - (int)line[h]);
        k0[l][h] = 1;
      }
    }
    // Split2D (lines +-4; rows past the frame read as zero)
    for (int l = 24; l < IN_Y; l++) {
      const double* p1 = clp0[l - 4];
      const double* c1 = clp0[l];
      const double* n1 = clp0[l + 4];
      if (l >= 4 && l <= IN_Y - 4) {
        for (int h = 18; h < IN_X - 4; h++) {
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
      for (int h = 4; h < IN_X - 4; h++) k0[l][h] = 1 - 0.0 - k1[l][h];
    }
    // SplitIQ (lines 24..; cb rows padded by one so p[IN_X..IN_X+1] reads the next row's zeros)
    static YUV cb[IN_Y + 1][IN_X];
    std::memset(cb, 0, sizeof(cb));
    for (int l = 24; l < IN_Y; l++) {
      const uint16_t* line = raw + l * IN_X;
      const bool invertphase = (line[0] == 16384);
      double si = 0, sq = 0;
      for (int h = 4; h < IN_X - 4; h++) {
        double cavg = 0;
        cavg += 0.0 * 0.0;
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
      }
    }
    // (Process's VBI copy into cbuf (:837-844) is undone by the second SplitIQ's memset)
    // AdjustY (lines FIRST_LINE..; h 2..IN_X-1, p[h + 2] past the end = next row's p[0..1])
    for (int l = FIRST_LINE; l < IN_Y; l++) {
      const bool invertphase = (raw[l * IN_X] == 16384);
      for (int h = 2; h < IN_X; h++) {
        const YUV y = (h + 2 < IN_X) ? cb[l][h + 2] : cb[l + 1][h + 2 - IN_X];
        YUV o = y;
        double comp = 0;
        switch (h % 4) {
          case 0: comp = y.i; break;
          case 1: comp = -y.q; break;
          case 2: comp = -y.i; break;
          case 3: comp = y.q; break;
        }
        if (invertphase) comp = -comp;
        o.y += comp;
        cb[l][h] = o;
      }
    }
    // DoYNR (lines FIRST_LINE..; persistent FIR fed h = 40..IN_X, output at h + 12)
    for (int l = FIRST_LINE; l < IN_Y; l++) {
      double hp[IN_X + 32] = {0};
      for (int h = 40; h <= IN_X; h++) hp[h] = nr_feed(h < IN_X ? cb[l][h].y : cb[l + 1][0].y);
      for (int h = 40; h < IN_X - 12; h++) {
        double a = hp[h + 12];
        if (std::fabs(a) > NR_Y) a = (a > 0) ? NR_Y : -NR_Y;
        cb[l][h].y -= a;
      }
    }
    // ToRGB: burst angle per line (lines 10..), frame phase, rotation, flip, conversion
    double angle[IN_Y] = {0};
    for (int l = 10; l < IN_Y; l++) {
      double i = 0, q = 0;
      for (int h = BURST_H0; h < BURST_H1; h++) { i += cb[l][h].i; q += cb[l][h].q; }
      angle[l] = atan2deg(q, i);
    }
    int phasecount = 0, tot = 0;
    for (int l = 20; l < (IN_Y - 4); l += 4, tot++)
      if (std::fabs(angle[l + 1] - angle[l]) < 20) phasecount++;
    const bool phase = phasecount > (tot / 2);
    const double m = BRIGHTNESS * 255 / 100;
    for (int l = FIRST_LINE; l < IN_Y - 2; l++) {
      const double burstlev = 8;
      if (burstlev > 5) {
        if (aburstlev < 0) aburstlev = burstlev;
        aburstlev = (aburstlev * .99) + (burstlev * .01);
      }
      const int row = l - FIRST_LINE;
      if (row >= LINES_OUT) continue;
      const double angleadj = 135 - angle[l];
      for (int x = 0; x < OUT_W; x++) {
        const int h = x + OUT_X0;
        YUV yiq = cb[l][h];
        const double mag = std::sqrt((yiq.i * yiq.i) + (yiq.q * yiq.q));
        const double ang = (double)((long double)std::atan2(yiq.q, yiq.i) +
                                    (long double)((angleadj + 0) / 180.0) * 3.141592653589793238462643383279502884L);
        yiq.i = std::cos(ang) * mag;
        yiq.q = std::sin(ang) * mag;
        yiq.i *= (10 / aburstlev);
        yiq.q *= (10 / aburstlev);
        const double i = yiq.i, q = yiq.q;
        const int rotate = l % 4;
        bool flip = (rotate == 1) || (rotate == 2);
        if (phase) flip = !flip;
        if (flip) {
          yiq.i = -q;
          yiq.q = -i;
        }
        double y = u16_to_ire_pal(clampd(yiq.y, 0, 65535));
        y = (y - BLACK_IRE) * (100 / (100 - BLACK_IRE));
        const double u = +(yiq.i) / IRESCALE;
        const double v = +(yiq.q) / IRESCALE;
        double r = y + (1.13983 * v);
        double g = y - (0.58060 * v) - (u * 0.39465);
        double b = y + (u * 2.032);
        r = clampd(r * m, 0, 65535);
        g = clampd(g * m, 0, 65535);
        b = clampd(b * m, 0, 65535);
        uint16_t* o = rgb + ((size_t)row * OUT_W + x) * 3;
        o[0] = (uint16_t)r;
        o[1] = (uint16_t)g;
        o[2] = (uint16_t)b;
      }
    }
  }
};

}  // namespace

extern "C" {
void* combpal_create() { return new CombPAL(); }
void combpal_destroy(void* c) { delete static_cast<CombPAL*>(c); }
// n frames of 1135 x 625 uint16 -> n frames of 1057 x 576 x 3 uint16 (rgb48)
void combpal_process(void* c, int n, const uint16_t* frames, uint16_t* rgb) {
  CombPAL* cb = static_cast<CombPAL*>(c);
  for (int f = 0; f < n; f++)
    cb->process(frames + (size_t)f * IN_X * IN_Y, rgb + (size_t)f * OUT_W * LINES_OUT * 3);
}
double combpal_aburstlev(void* c) { return static_cast<CombPAL*>(c)->aburstlev; }
}
