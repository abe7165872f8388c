// The 16x16x4 fp32 forward / input-gradient GEMM lives in the library (nerf-sys_amd/csrc/gemm.hpp: gemm_nt16_kernel);
// its weight-gradient counterpart, measured slower, in gemm_wgrad16.hpp.
#pragma once
#include "gemm_wgrad16.hpp"
