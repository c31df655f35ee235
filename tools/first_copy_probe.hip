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
    auto run = [&](int L) {
        (void)hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (size_t c = 0; c < npc; ++c)
            for (int k = 0; k < L; ++k)
                (void)hipMemcpyAsync((char*)d[k] + c * piece, (char*)h[k] + c * piece, piece, hipMemcpyHostToDevice,
                                     st[k]);
        (void)hipDeviceSynchronize();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
    };
    for (int L : {1, 2, 4, 8}) {
        const double a = run(L), b = run(L), c = run(L);
        printf("streams %d x %zu KiB: first %.2f ms, second %.2f, third %.2f ms\n", L, per >> 10, a, b, c);
    }
    return 0;
}
