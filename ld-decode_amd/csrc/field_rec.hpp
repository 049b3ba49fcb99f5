// Device view of the public per-read record + the per-read line-array layout.
#pragma once
#include "../../include/ldgpu.h"
#include "common.hpp"

namespace ldg {

using FieldRec = ldg_field_info;
constexpr int VBI_NONE = LDG_VBI_NONE;

// lines[slot][LINES_STRIDE]: one MAX_LINES run per array
enum LineArr { LL1 = 0, LL2 = 1, LL3 = 2, LL4 = 3, LLF = 4, PAVG0 = 5, PAVG1 = 6, NLINEARR = 7 };
constexpr int LINES_STRIDE = NLINEARR * MAX_LINES;

}  // namespace ldg
