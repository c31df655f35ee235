// Per-stream H2D rate: 32 streams created in order; each times 64 x 4 MiB
// hipMemcpyAsync pieces from one pinned buffer, alone, then pairs of consecutive streams copy at once.
// A stream whose copies land on a slower copy path shows up as a slow row.  Usage: tools/stream_copy_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

int main() {
    const size_t chunk = 4u << 20, nch = 64, n = chunk * nch;
    void *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, 2 * n) != hipSuccess || hipHostMalloc(&h, 2 * n, hipHostMallocDefault) != hipSuccess) return 1;
    std::vector<hipStream_t> st(32);
    for (auto& s : st)
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
    auto run = [&](std::vector<int> ids) {
        (void)hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (size_t c = 0; c < nch; ++c)
            for (size_t k = 0; k < ids.size(); ++k)
                (void)hipMemcpyAsync((char*)d + k * n + c * chunk, (char*)h + k * n + c * chunk, chunk,
                                     hipMemcpyHostToDevice, st[ids[k]]);
        (void)hipDeviceSynchronize();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    run({0});
    printf("alone:");
    for (int s = 0; s < 32; ++s) printf(" s%d %.1f", s, n / run({s}) / 1e9);
    printf(" GB/s\npairs:");
    for (int s = 0; s < 32; s += 1) printf(" s%d+%d %.1f", s, (s + 1) % 32, 2 * n / run({s, (s + 1) % 32}) / 1e9);
    printf(" GB/s (both streams' bytes)\n");
    return 0;
}
