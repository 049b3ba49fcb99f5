// libldgpu unity build: all device code + the C ABI in one translation unit.
#include "demod.hip"
#include "field.hip"
#include "tbc.hip"
#include "comb.hip"
#include "combpal.hip"
#include "synth.hip"
#include "abi.inc"
#include "cx.inc"
