// First-use cost of the host-to-device copy path (host_fed's first round): with
// L = 1, 2, 4, 8 streams copying at once (64 x 256 KiB pinned -> device each, one host thread issuing),
// the first and the second run of each level.  A first run much slower than the second marks lazy
// state in the runtime's copy path.  SMALL=1: the same with 64 KiB per stream (does a tiny warm-up
// suffice?).  Usage: tools/first_copy_probe [piece_KiB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    const size_t piece = (size_t)(argc > 1 ? atoi(argv[1]) : 256) << 10, npc = 64, per = piece * npc;
    std::vector<hipStream_t> st(8);
    std::vector<void*> h(8), d(8);
    for (int k = 0; k < 8; ++k) {
        if (hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking) != hipSuccess) return 1;
        if (hipHostMalloc(&h[k], per, hipHostMallocDefault) != hipSuccess || hipMalloc(&d[k], per) != hipSuccess)
            return 2;
        memset(h[k], k, per);
    }
    // SPIN=1: wait by polling hipEventQuery on each stream's end event instead of hipDeviceSynchronize;
    // the GPU-side span (first stream's start event -> each stream's end event) is printed beside the wall time
    const bool spin = getenv("SPIN") && atoi(getenv("SPIN"));
    std::vector<hipEvent_t> e0(8), e1(8);
    for (int k = 0; k < 8; ++k)
        if (hipEventCreate(&e0[k]) != hipSuccess || hipEventCreate(&e1[k]) != hipSuccess) return 3;
    auto run = [&](int L, float& gpu_ms) {
        (void)hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < L; ++k) (void)hipEventRecord(e0[k], st[k]);
        for (size_t c = 0; c < npc; ++c)
            for (int k = 0; k < L; ++k)
                (void)hipMemcpyAsync((char*)d[k] + c * piece, (char*)h[k] + c * piece, piece, hipMemcpyHostToDevice,
                                     st[k]);
        for (int k = 0; k < L; ++k) (void)hipEventRecord(e1[k], st[k]);
        if (spin) {
            for (int k = 0; k < L; ++k)
                while (hipEventQuery(e1[k]) == hipErrorNotReady) {}
        } else {
            (void)hipDeviceSynchronize();
        }
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
        gpu_ms = 0;
        for (int k = 0; k < L; ++k) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0[0], e1[k]);
            gpu_ms = ms > gpu_ms ? ms : gpu_ms;
        }
        return wall;
    };
    for (int L : {1, 2, 4, 8}) {
        float ga, gb, gc;
        const double a = run(L, ga), b = run(L, gb), c = run(L, gc);
        printf("streams %d x %zu KiB: wall %.2f / %.2f / %.2f ms, GPU events %.2f / %.2f / %.2f ms%s\n", L, per >> 10, a, b,
               c, ga, gb, gc, spin ? " (spin wait)" : "");
    }
    return 0;
}
