// libldgpu unity build: all device code + the C ABI in one translation unit.
#include "demod.hip"
#include "fft8k_h.hpp"    // the 512-thread demod's layout (host tables: bin_of)
#ifdef LDG_WITH_DEMOD2     // the experimental 512-thread demod (LDG_DEMOD2=1), a variant build:
#include "demod2.hip"      // its kernels in the default library moved ldg_k_demod's code and cost ~2%
#endif
#include "field.hip"
#include "tbc.hip"
#include "comb.hip"
#include "flow.hip"
#include "combpal.hip"
#include "synth.hip"
#include "abi.inc"
#include "cx.inc"
