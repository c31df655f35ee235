// VALU integer-throughput microbenchmark for gfx950 (MI355X).
//
// Purpose: pin the peak issue rate of the instructions the Ed25519 field
// arithmetic is built from, so that (1) the limb radix is chosen from
// measurements rather than folklore and (2) bench.py's roofline "peak" for
// the verify kernel (u32xu32->u64 multiply-accumulates per second) is a number
// measured on the box ("The peak is measured by a gfx950
// microbenchmark on the box").
//
// Each kernel runs CHAINS independent dependency chains per lane so the
// measurement is throughput-, not latency-bound.  Output: one JSON line per
// instruction with ops/s over the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <string>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int CHAINS = 16;
constexpr int ITERS = 2048;

// v_mad_u64_u32: acc = lo(acc) * b + acc
__global__ void __launch_bounds__(256) k_mad_u64_u32(uint64_t* out, uint32_t b) {
    uint64_t acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 7919u + c;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) acc[c] = (uint64_t)(uint32_t)acc[c] * b + acc[c];
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= acc[c];
    if (s == 0x12345) out[0] = s;
}

// v_mul_lo_u32
__global__ void __launch_bounds__(256) k_mul_lo_u32(uint64_t* out, uint32_t b) {
    uint32_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 7919u + c + 1;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = x[c] * b;
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= x[c];
    if (s == 0x12345) out[0] = s;
}

// v_mul_hi_u32
__global__ void __launch_bounds__(256) k_mul_hi_u32(uint64_t* out, uint32_t b) {
    uint32_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 7919u + c + 1;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __umulhi(x[c], b) ^ b;
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= x[c];
    if (s == 0x12345) out[0] = s;
}

// v_mad_u32_u24
__global__ void __launch_bounds__(256) k_mad_u24(uint64_t* out, uint32_t b) {
    uint32_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 7919u + c + 1;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __umul24(x[c], b) + x[c];
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= x[c];
    if (s == 0x12345) out[0] = s;
}

// v_fma_f64
__global__ void __launch_bounds__(256) k_fma_f64(uint64_t* out, double b) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 0.5 + c;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __fma_rn(x[c], b, 0.25);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.0) out[0] = 1;
}

// 64-bit add (v_add_co_u32 + v_addc_co_u32): counted as ONE 64-bit add
__global__ void __launch_bounds__(256) k_add_u64(uint64_t* out, uint64_t b) {
    uint64_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 7919u + c + 1;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = x[c] + b;
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= x[c];
    if (s == 0x12345) out[0] = s;
}

// plain 32-bit VALU op (v_xad_u32 / v_add3 style); counted as 1 op per statement
__global__ void __launch_bounds__(256) k_xor_u32(uint64_t* out, uint32_t b) {
    uint32_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 7919u + c + 1;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = (x[c] ^ b) + 0x9e3779b9u;   // v_xad_u32 (1 instr)
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= x[c];
    if (s == 0x12345) out[0] = s;
}

// 64-bit rotate (2x v_alignbit_b32)
__global__ void __launch_bounds__(256) k_rot64(uint64_t* out, uint32_t b) {
    uint64_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 7919u + c + 1;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = ((x[c] >> 19) | (x[c] << 45)) ^ b;
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s ^= x[c];
    if (s == 0x12345) out[0] = s;
}

template <typename K, typename A>
static int run(const char* name, K kern, A arg, double ops_per_stmt, uint64_t* dout, int ncu) {
    const int threads = 256;
    const int blocks = ncu * 8;   // 8 blocks of 256 = 32 waves per CU
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, dout, arg);   // warmup
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, dout, arg);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    double ops = (double)blocks * threads * ITERS * CHAINS * ops_per_stmt;
    double rate = ops / (best * 1e-3);
    // per CU per clock at 2.4 GHz (lane-ops)
    double per_cu_clk = rate / ncu / 2.4e9;
    printf("{\"instr\": \"%s\", \"ms\": %.4f, \"lane_ops_per_s\": %.4e, \"lane_ops_per_cu_per_clk_at_2.4GHz\": %.2f}\n",
           name, best, rate, per_cu_clk);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    printf("{\"device\": \"%s\", \"arch\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n",
           p.name, p.gcnArchName, p.multiProcessorCount, p.clockRate);
    uint64_t* d;
    CHECK(hipMalloc(&d, 64));
    int ncu = p.multiProcessorCount;
    run("v_mad_u64_u32", k_mad_u64_u32, 0x9e3779b9u, 1.0, d, ncu);
    run("v_mul_lo_u32", k_mul_lo_u32, 0x9e3779b9u, 1.0, d, ncu);
    run("v_mul_hi_u32(+xor)", k_mul_hi_u32, 0x9e3779b9u, 1.0, d, ncu);
    run("v_mad_u32_u24", k_mad_u24, 0x00e3779bu, 1.0, d, ncu);
    run("v_fma_f64", k_fma_f64, 0.999999, 1.0, d, ncu);
    run("v_lshl_add_u64 (64-bit add)", k_add_u64, (uint64_t)0x9e3779b97f4a7c15ull, 1.0, d, ncu);
    run("xor+add_u32 (2 instr)", k_xor_u32, 0x9e3779b9u, 2.0, d, ncu);
    run("rot64+xor (4 instr)", k_rot64, 0x9e3779b9u, 4.0, d, ncu);
    CHECK(hipFree(d));
    return 0;
}
