// ASan / UBSan driver for libldgpu's host-only C++ (test infrastructure): linked
// against libldgpu_asan.so, the library built with the host side instrumented
// (ld-decode_amd/build.py build_asan).  Runs without a GPU: the CX expander (csrc/cx.inc)
// over streams fed whole and in pieces, the audio-offset recurrence (ldg_audio_offsets),
// and every context entry point's argument checks with a null context (no device touched).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/ldgpu.h"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      return 1;                                                    \
    }                                                              \
  } while (0)

int main() {
  // ---- CX expander: one call over the stream == the same stream in ragged pieces
  std::mt19937_64 rng(20181015);
  const int64_t n = 48000 * 3;
  std::vector<uint16_t> in(2 * n), a(2 * n), b(2 * n);
  for (int64_t i = 0; i < n; i++) {
    const double t = i / 48000.0, env = (i / 12000) % 2 ? 0.9 : 0.05;   // loud / quiet: both followers
    in[2 * i] = (uint16_t)(32768 + 30000 * env * std::sin(2 * M_PI * 1000 * t) + (int)(rng() % 64) - 32);
    in[2 * i + 1] = (uint16_t)(32768 + 30000 * env * std::sin(2 * M_PI * 440 * t));
  }
  ldg_cx* cx = nullptr;
  CHECK(ldg_cx_create(&cx) == LDG_OK);
  CHECK(ldg_cx_process(cx, n, in.data(), a.data()) == LDG_OK);
  CHECK(ldg_cx_destroy(cx) == LDG_OK);
  CHECK(ldg_cx_create(&cx) == LDG_OK);
  for (int64_t i = 0, k = 1; i < n; k = k * 7 % 1009 + 1) {
    const int64_t m = std::min<int64_t>(k, n - i);
    CHECK(ldg_cx_process(cx, m, in.data() + 2 * i, b.data() + 2 * i) == LDG_OK);
    i += m;
  }
  CHECK(ldg_cx_process(cx, 0, nullptr, nullptr) == LDG_OK);
  CHECK(std::memcmp(a.data(), b.data(), a.size() * 2) == 0);
  CHECK(ldg_cx_process(cx, 5, nullptr, b.data()) == LDG_EINVAL);
  CHECK(ldg_cx_process(nullptr, 5, in.data(), b.data()) == LDG_EINVAL);
  CHECK(ldg_cx_destroy(cx) == LDG_OK);
  CHECK(ldg_cx_create(nullptr) == LDG_EINVAL);

  // ---- audio offsets (lddecode_core.py:432-484): the chain over NTSC field line counts
  std::vector<double> lc(2000), out(2001);
  for (size_t k = 0; k < lc.size(); k++) lc[k] = (k & 1) ? 263 : 262;
  CHECK(ldg_audio_offsets(0.0, (int64_t)lc.size(), lc.data(), 63.555555555555557, out.data()) == LDG_OK);
  for (size_t k = 0; k < out.size(); k++) CHECK(out[k] >= -1.0 / 48000 && out[k] < 1.0 / 48000 + 1e-12);
  CHECK(ldg_audio_offsets(0.0, 0, nullptr, 63.5, out.data()) == LDG_OK);
  CHECK(ldg_audio_offsets(0.0, 3, nullptr, 63.5, out.data()) == LDG_EINVAL);

  // ---- argument checks: a null context is refused, nothing dereferenced
  int64_t i64[4] = {0, 0, 0, 0};
  double d[16] = {0};
  int32_t s32[4] = {0, 1, 2, 3};
  uint8_t f8[4] = {0, 0, 0, 0};
  CHECK(ldg_destroy(nullptr) != LDG_OK);
  CHECK(ldg_set_capture(nullptr, in.data(), 16, 0, 0, 0) != LDG_OK);
  CHECK(ldg_stream_open(nullptr, "/dev/null", 0, 1 << 20, 0) != LDG_OK);
  CHECK(ldg_stream_release(nullptr, 0) != LDG_OK);
  CHECK(ldg_stream_seek(nullptr, 0) != LDG_OK);
  CHECK(ldg_stream_window(nullptr, i64) != LDG_OK);
  CHECK(ldg_stream_stats(nullptr, d, 16) < 0);
  CHECK(ldg_stream_close(nullptr) != LDG_OK);
  CHECK(ldg_decode_reads_async2(nullptr, 1, i64, d, s32, f8) != LDG_OK);
  CHECK(ldg_decode_reads_wait(nullptr, nullptr) != LDG_OK);
  CHECK(ldg_set_video_cut(nullptr, 0) != LDG_OK);
  CHECK(ldg_field_audio_async(nullptr, 1, s32, d) != LDG_OK);
  CHECK(ldg_assemble_frames(nullptr, 1, s32, s32, nullptr, 0) != LDG_OK);
  CHECK(ldg_comb_set_state(nullptr, 1.0) != LDG_OK);
  CHECK(ldg_sync(nullptr) != LDG_OK);
  CHECK(ldg_output_wait(nullptr) != LDG_OK);
  CHECK(ldg_demod_isolated_ex(nullptr, 1, s32, 1, 0, d) != LDG_OK);
  CHECK(ldg_capture_download(nullptr, d, 0, 8) < 0);
  CHECK(ldg_version() != nullptr && std::strlen(ldg_version()) > 0);
  std::printf("host_san ok (devices visible: %d)\n", ldg_device_count());
  return 0;
}
