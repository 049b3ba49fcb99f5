// ASan / UBSan driver for the oracle's 2D / 3D NTSC comb restatement (test infrastructure,
// SURVEY §5 sanitizers; built by tests/san/Makefile, run by tests/test_sanitizers.py).
// The reference's Split2D reads row l + 2 = 525 of a 525-row frame for l = 523
// (comb-ntsc.cxx:299,303); the restatement zero-pads that row.  These frames put strong
// chroma on the last lines so every frame-edge read is exercised, over the option paths,
// the 3D comb (-d 3 -F) and the flow-weighted 3D comb.
#include "../../oracle/comb2d.cpp"

#include <cstdio>
#include <random>

static void make_frames(std::vector<uint16_t>& fr, int n, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::normal_distribution<double> noise(0.0, 60.0);
  fr.assign((size_t)n * IN_X * IN_Y, 0);
  for (int f = 0; f < n; f++)
    for (int l = 0; l < IN_Y; l++) {
      uint16_t* row = &fr[((size_t)f * IN_Y + l) * IN_X];
      const double amp = l >= 500 ? 90.0 : 30.0;            // strongest chroma on the last lines
      for (int h = 0; h < IN_X; h++) {
        const double ire = 40.0 + 30.0 * std::sin(h / 37.0 + f) + amp * ((h + l + f) % 4 < 2 ? 1 : -1) * 0.5;
        row[h] = (uint16_t)std::max(0.0, std::min(65535.0, (ire + 40.0) * 358.4 + 1024 + noise(rng)));
      }
      row[0] = ((l + f) & 1) ? 16384 : 32768;               // the TBC's burst-phase flag
      row[1] = (uint16_t)(5000 + 100 * (l % 7));            // burst level
    }
}

int main() {
  std::vector<uint16_t> fr;
  make_frames(fr, 4, 20181015);
  double sum = 0;
  struct Case { double d[4]; int i[7]; } cases[] = {
      {{7.5, 236, 1.0, 0.0}, {0, 1, 1, 1, 480, -1000, 0}},   // defaults
      {{7.5, 236, 1.0, 2.0}, {0, 1, 1, 1, 480, -1000, 0}},   // -N (chroma NR)
      {{0.0, 200, 0.0, 0.0}, {1, 0, 0, 0, 525, -1000, 0}},   // -I 0 -b -n -l -v
      {{7.5, 236, 1.0, 0.0}, {0, 1, 1, 0, 525, 300, 1}},     // -Q -v -L -W
  };
  for (const Case& c : cases) {
    void* h = comb2d_create();
    comb2d_set_opts(h, c.d, c.i);
    const Opts o = static_cast<Comb*>(h)->o;
    std::vector<uint16_t> rgb((size_t)4 * o.out_w() * o.linesout * 3);
    comb2d_process(h, 4, fr.data(), rgb.data());
    for (uint16_t v : rgb) sum += v;
    std::vector<double> kmap((size_t)IN_X * IN_Y);
    std::mt19937_64 rng(7);
    for (double& k : kmap) k = (rng() % 1000) / 1000.0;
    comb2d_process_of(h, &fr[0], &fr[(size_t)IN_X * IN_Y], kmap.data(), rgb.data());
    std::vector<double> luma((size_t)IN_X * IN_Y);
    comb2d_flow_luma(h, &fr[0], luma.data());
    for (double v : luma) sum += v;
    comb2d_destroy(h);
    void* h3 = comb3d_create();
    comb3d_set_opts(h3, c.d, c.i);
    int got = comb3d_process(h3, 3, fr.data(), rgb.data(), -1, -1);
    got += comb3d_process(h3, 1, &fr[(size_t)3 * IN_X * IN_Y], rgb.data() + (size_t)got * o.out_w() * o.linesout * 3, 0.5, 2);
    if (got != 2) { std::printf("comb3d: %d frames\n", got); return 1; }
    comb3d_destroy(h3);
  }
  std::printf("comb_san ok %.6e\n", sum);
  return 0;
}
