// Issue-cost microbenchmark for the gfx950 integer instructions a GF(2^255-19) multiplier can be
// built from.  Each kernel runs a loop of UNROLL x 8 independent inline-asm instructions (8
// independent destination registers per lane, so no dependency stalls) with WAVES waves resident
// per SIMD; every wave stamps s_memtime around the loop.  Cycles per wave64 instruction per SIMD =
// median wave elapsed / (waves per SIMD x instructions per wave).
//
// Build: hipcc -O3 --offload-arch=gfx950 tools/isa_rates.hip -o tools/isa_rates
// Output: one JSON line per instruction.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

#define EXP8(I) I("%0", "%8") I("%1", "%8") I("%2", "%8") I("%3", "%8") I("%4", "%8") I("%5", "%8") I("%6", "%8") I("%7", "%8")


// 32-bit destination, two 32-bit sources
#define K2(NAME, ASM)                                                                            \
__global__ void __launch_bounds__(256) NAME(uint64_t* cyc, uint32_t* sink, uint32_t b) {         \
    uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,  \
             x6 = x0 + 6, x7 = x0 + 7;                                                          \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                            \
    for (int it = 0; it < ITERS; ++it) {                                                         \
        _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                          \
            asm volatile(EXP8(ASM) : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) \
                         : "v"(b) : "vcc", "s40", "s41");                                          \
        }                                                                                        \
    }                                                                                            \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                            \
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;                                  \
    if ((threadIdx.x & 63) == 0) cyc[gid >> 6] = t1 - t0;                                        \
    sink[gid] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                                           \
}

// 64-bit destination (register pair)
#define K64(NAME, ASM)                                                                           \
__global__ void __launch_bounds__(256) NAME(uint64_t* cyc, uint32_t* sink, uint32_t b) {         \
    uint64_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,  \
             x6 = x0 + 6, x7 = x0 + 7;                                                          \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                            \
    for (int it = 0; it < ITERS; ++it) {                                                         \
        _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                          \
            asm volatile(EXP8(ASM) : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) \
                         : "v"(b) : "vcc", "s40", "s41");                                          \
        }                                                                                        \
    }                                                                                            \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                            \
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;                                  \
    if ((threadIdx.x & 63) == 0) cyc[gid >> 6] = t1 - t0;                                        \
    sink[gid] = (uint32_t)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7);                               \
}

#define I_k_add_u32(D, B) "v_add_u32 " D ", " D ", " B "\n\t"
K2(k_add_u32, I_k_add_u32)
#define I_k_add3_u32(D, B) "v_add3_u32 " D ", " D ", " B ", " D "\n\t"
K2(k_add3_u32, I_k_add3_u32)
#define I_k_mul_lo_u32(D, B) "v_mul_lo_u32 " D ", " D ", " B "\n\t"
K2(k_mul_lo_u32, I_k_mul_lo_u32)
#define I_k_mul_hi_u32(D, B) "v_mul_hi_u32 " D ", " D ", " B "\n\t"
K2(k_mul_hi_u32, I_k_mul_hi_u32)
#define I_k_mad_u32_u24(D, B) "v_mad_u32_u24 " D ", " D ", " B ", " D "\n\t"
K2(k_mad_u32_u24, I_k_mad_u32_u24)
#define I_k_mul_hi_u32_u24(D, B) "v_mul_hi_u32_u24 " D ", " D ", " B "\n\t"
K2(k_mul_hi_u32_u24, I_k_mul_hi_u32_u24)
#define I_k_mul_u32_u24(D, B) "v_mul_u32_u24 " D ", " D ", " B "\n\t"
K2(k_mul_u32_u24, I_k_mul_u32_u24)
#define I_k_mad_u32_u16(D, B) "v_mad_u32_u16 " D ", " D ", " B ", " D "\n\t"
K2(k_mad_u32_u16, I_k_mad_u32_u16)
#define I_k_dot2_u32_u16(D, B) "v_dot2_u32_u16 " D ", " D ", " B ", " D "\n\t"
K2(k_dot2_u32_u16, I_k_dot2_u32_u16)
#define I_k_dot4_u32_u8(D, B) "v_dot4_u32_u8 " D ", " D ", " B ", " D "\n\t"
K2(k_dot4_u32_u8, I_k_dot4_u32_u8)
#define I_k_alignbit(D, B) "v_alignbit_b32 " D ", " D ", " B ", 26\n\t"
K2(k_alignbit, I_k_alignbit)
#define I_k_lshl_add_u32(D, B) "v_lshl_add_u32 " D ", " D ", 4, " B "\n\t"
K2(k_lshl_add_u32, I_k_lshl_add_u32)
#define I_k_addc_co(D, B) "v_add_co_u32 " D ", vcc, " D ", " B "\n\tv_addc_co_u32 " D ", vcc, " D ", " B ", vcc\n\t"
K2(k_addc_co, I_k_addc_co)
#define I_k_mad_u64_u32(D, B) "v_mad_u64_u32 " D ", vcc, " B ", " B ", " D "\n\t"
K64(k_mad_u64_u32, I_k_mad_u64_u32)
#define I_k_mad_u64_u32_nc(D, B) "v_mad_u64_u32 " D ", s[40:41], " B ", " B ", " D "\n\t"
K64(k_mad_u64_u32_nc, I_k_mad_u64_u32_nc)
#define I_k_lshl_add_u64(D, B) "v_lshl_add_u64 " D ", " D ", 0, " D "\n\t"
K64(k_lshl_add_u64, I_k_lshl_add_u64)
#define I_k_lshrrev_b64(D, B) "v_lshrrev_b64 " D ", 7, " D "\n\t"
K64(k_lshrrev_b64, I_k_lshrrev_b64)
#define I_k_fma_f64(D, B) "v_fma_f64 " D ", " D ", " D ", " D "\n\t"
K64(k_fma_f64, I_k_fma_f64)
#define I_k_pk_fma_f32(D, B) "v_pk_fma_f32 " D ", " D ", " D ", " D "\n\t"
K64(k_pk_fma_f32, I_k_pk_fma_f32)
#define I_k_pk_mul_f32(D, B) "v_pk_mul_f32 " D ", " D ", " D "\n\t"
K64(k_pk_mul_f32, I_k_pk_mul_f32)
#define I_k_pk_add_f32(D, B) "v_pk_add_f32 " D ", " D ", " D "\n\t"
K64(k_pk_add_f32, I_k_pk_add_f32)
#define I_k_mul_f64(D, B) "v_mul_f64 " D ", " D ", " D "\n\t"
K64(k_mul_f64, I_k_mul_f64)

#define I_k_and(D, B) "v_and_b32 " D ", " D ", " B "\n\t"
K2(k_and, I_k_and)
#define I_k_xor(D, B) "v_xor_b32 " D ", " D ", " B "\n\t"
K2(k_xor, I_k_xor)
#define I_k_sub(D, B) "v_sub_u32 " D ", " D ", " B "\n\t"
K2(k_sub, I_k_sub)
#define I_k_lshl(D, B) "v_lshlrev_b32 " D ", 3, " D "\n\t"
K2(k_lshl, I_k_lshl)
#define I_k_lshr(D, B) "v_lshrrev_b32 " D ", 3, " D "\n\t"
K2(k_lshr, I_k_lshr)
#define I_k_mov(D, B) "v_mov_b32 " D ", " B "\n\t"
K2(k_mov, I_k_mov)
#define I_k_cndmask(D, B) "v_cndmask_b32 " D ", " D ", " B ", vcc\n\t"
K2(k_cndmask, I_k_cndmask)
#define I_k_add_f32(D, B) "v_add_f32 " D ", " D ", " B "\n\t"
K2(k_add_f32, I_k_add_f32)
#define I_k_fma_f32(D, B) "v_fma_f32 " D ", " D ", " B ", " D "\n\t"
K2(k_fma_f32, I_k_fma_f32)
#define I_k_max_u32(D, B) "v_max_u32 " D ", " D ", " B "\n\t"
K2(k_max_u32, I_k_max_u32)
#define I_k_bfi(D, B) "v_bfi_b32 " D ", " B ", " D ", " B "\n\t"
K2(k_bfi, I_k_bfi)
#define I_k_and_e64(D, B) "v_and_b32_e64 " D ", " D ", " B "\n\t"
K2(k_and_e64, I_k_and_e64)
#define I_k_add_e64(D, B) "v_add_u32_e64 " D ", " D ", " B "\n\t"
K2(k_add_e64, I_k_add_e64)
#define I_k_mul_u24_e64(D, B) "v_mul_u32_u24_e64 " D ", " D ", " B "\n\t"
K2(k_mul_u24_e64, I_k_mul_u24_e64)
#define I_k_mov64(D, B) "v_mov_b64 " D ", " D "\n\t"
K64(k_mov64, I_k_mov64)

typedef void (*kfn)(uint64_t*, uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    struct { const char* name; kfn f; int per_instr; } ks[] = {
        {"v_add_u32", k_add_u32, 1}, {"v_add3_u32", k_add3_u32, 1}, {"v_mul_lo_u32", k_mul_lo_u32, 1},
        {"v_mul_hi_u32", k_mul_hi_u32, 1}, {"v_mad_u32_u24", k_mad_u32_u24, 1},
        {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 1}, {"v_mul_u32_u24", k_mul_u32_u24, 1},
        {"v_mad_u32_u16", k_mad_u32_u16, 1}, {"v_dot2_u32_u16", k_dot2_u32_u16, 1},
        {"v_dot4_u32_u8", k_dot4_u32_u8, 1}, {"v_alignbit_b32", k_alignbit, 1},
        {"v_lshl_add_u32", k_lshl_add_u32, 1}, {"v_add_co_u32+v_addc_co_u32", k_addc_co, 2},
        {"v_mad_u64_u32", k_mad_u64_u32, 1}, {"v_mad_u64_u32(sgpr carry)", k_mad_u64_u32_nc, 1},
        {"v_lshl_add_u64", k_lshl_add_u64, 1}, {"v_lshrrev_b64", k_lshrrev_b64, 1},
        {"v_fma_f64", k_fma_f64, 1}, {"v_pk_fma_f32", k_pk_fma_f32, 1}, {"v_pk_mul_f32", k_pk_mul_f32, 1},
        {"v_pk_add_f32", k_pk_add_f32, 1}, {"v_mul_f64", k_mul_f64, 1},
        {"v_and_b32", k_and, 1}, {"v_xor_b32", k_xor, 1}, {"v_sub_u32", k_sub, 1}, {"v_lshlrev_b32", k_lshl, 1},
        {"v_lshrrev_b32", k_lshr, 1}, {"v_mov_b32", k_mov, 1}, {"v_cndmask_b32", k_cndmask, 1},
        {"v_add_f32", k_add_f32, 1}, {"v_fma_f32", k_fma_f32, 1}, {"v_max_u32", k_max_u32, 1},
        {"v_bfi_b32", k_bfi, 1}, {"v_and_b32_e64", k_and_e64, 1}, {"v_add_u32_e64", k_add_e64, 1},
        {"v_mul_u32_u24_e64", k_mul_u24_e64, 1}, {"v_mov_b64", k_mov64, 1},
    };
    for (int waves : {8}) {
        const int blocks = cus * waves;   // 4 waves per block -> `waves` waves per SIMD
        const int nw = blocks * 4;
        uint64_t* dc;
        uint32_t* ds;
        CHECK(hipMalloc(&dc, nw * 8));
        CHECK(hipMalloc(&ds, (size_t)blocks * 256 * 4));
        std::vector<uint64_t> h(nw);
        for (auto& k : ks) {
            for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, dc, ds, 3u);
            hipEvent_t e0, e1;
            CHECK(hipEventCreate(&e0));
            CHECK(hipEventCreate(&e1));
            CHECK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, dc, ds, 3u);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            CHECK(hipMemcpy(h.data(), dc, nw * 8, hipMemcpyDeviceToHost));
            std::sort(h.begin(), h.end());
            const double med = (double)h[nw / 2];
            const double instrs = (double)ITERS * 32 * k.per_instr;   // per wave
            const double cyc = med / (waves * instrs);
            const double clk = med / (ms * 1e-3) / 1e9;               // shader GHz (stamp / wall)
            printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_wave_instr\": %.3f, \"ms\": %.4f, "
                   "\"stamp_ghz\": %.3f}\n", k.name, waves, cyc, ms, clk);
            fflush(stdout);
            CHECK(hipEventDestroy(e0));
            CHECK(hipEventDestroy(e1));
        }
        CHECK(hipFree(dc));
        CHECK(hipFree(ds));
    }
    return 0;
}
