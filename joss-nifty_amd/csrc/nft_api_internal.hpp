// Internal cross-file declarations of the nifty_amd C-ABI library.
#pragma once
#include "nft_common.hpp"
#include "fft_core.hpp"

namespace nft {
const char* last_error();
int get_twiddles(int n, int dtype, const void** out);
FftPlanDev make_plan(int n);
int scale_real(void* x, long long n, int dtype, double scale, hipStream_t s);
}  // namespace nft
