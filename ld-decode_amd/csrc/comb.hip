// 2D NTSC comb filter (comb-ntsc.cxx dim=2) -- placeholder until the kernel lands.
#include <hip/hip_runtime.h>
#include "common.hpp"

struct ldg_ctx;
void ldg_comb_free(ldg_ctx*) {}
extern "C" int ldg_comb_ntsc(ldg_ctx*, int, const uint16_t*, uint16_t*, int) { return -4; }
extern "C" int ldg_comb_reset(ldg_ctx*) { return 0; }
