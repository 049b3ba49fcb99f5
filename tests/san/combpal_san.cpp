// ASan / UBSan driver for the oracle's PAL Y/C restatement (test infrastructure; see
// comb_san.cpp): full-amplitude chroma on the last rows, whose line +-4 neighbours the
// restatement pads (oracle/combpal.cpp).
#include "../../oracle/combpal.cpp"

#include <cstdio>
#include <random>

int main() {
  std::mt19937_64 rng(20181018);
  std::normal_distribution<double> noise(0.0, 60.0);
  const int n = 3;
  std::vector<uint16_t> fr((size_t)n * IN_X * IN_Y);
  for (int f = 0; f < n; f++)
    for (int l = 0; l < IN_Y; l++)
      for (int h = 0; h < IN_X; h++) {
        const double amp = l >= 600 ? 60.0 : 25.0;
        const double ire = 50.0 + amp * std::sin(h * 1.5707963 * 1.0034 + l * 0.7 + f);
        fr[((size_t)f * IN_Y + l) * IN_X + h] =
            (uint16_t)std::max(0.0, std::min(65535.0, (ire + 42.857) * 376.32 + 256 + noise(rng)));
      }
  std::vector<uint16_t> rgb((size_t)n * OUT_W * LINES_OUT * 3);
  void* h = combpal_create();
  combpal_process(h, n, fr.data(), rgb.data());
  double sum = 0;
  for (uint16_t v : rgb) sum += v;
  std::printf("combpal_san ok %.6e %.6f\n", sum, combpal_aburstlev(h));
  combpal_destroy(h);
  return 0;
}
