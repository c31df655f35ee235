// One key comb window's latency-mode verify kernel (k_verify_split, both message modes).
// Built once per window: -DNW_WA=8, 9, 12, 13, 16, 20 (Makefile).
#include "nw_verify_split.h"

#ifndef NW_WA
#error "compile with -DNW_WA=<key window>"
#endif

namespace nw {
template hipError_t launch_split_wa<NW_WA>(const VerifyParams&, int, hipStream_t);
}  // namespace nw
