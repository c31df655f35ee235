// One key comb window's verify kernels (k_verify / k_slow_prep / k_slow_tail for both message modes).
// Built once per window: -DNW_WA=8, 9, 12, 13, 16, 20 (Makefile).
#include "nw_verify_kernels.h"

#ifndef NW_WA
#error "compile with -DNW_WA=<key window>"
#endif

namespace nw {
template hipError_t launch_vs_wa<NW_WA>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
template hipError_t launch_slow_tail_wa<NW_WA>(const VerifyParams&, const FinalizeParams&, int, hipStream_t);
}  // namespace nw
