// Staging pipeline probe (worker-window bimodality): the library's host-buffer
// upload path rebuilt outside it -- 8 threads memcpy 4 MiB chunks of a pageable source into a pinned
// buffer while the calling thread issues each chunk's hipMemcpyAsync as soon as it is staged -- with
// the source first-touched on node S and the threads bound to node T (-1: unbound).  Prints the
// wall time per 512 MiB window and the rate.  Usage: tools/stage_probe [MiB]
#include <hip/hip_runtime.h>
#include <numaif.h>
#include <sched.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static void bind_node(int node) {
    cpu_set_t s;
    CPU_ZERO(&s);
    if (node < 0) {
        for (int c = 0; c < 256; ++c) CPU_SET(c, &s);
    } else {
        for (int c = node * 64; c < node * 64 + 64; ++c) CPU_SET(c, &s);
    }
    sched_setaffinity(0, sizeof(s), &s);
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 512;
    const size_t n = mib << 20, chunk = 4u << 20, nch = n / chunk;
    void *d = nullptr, *h = nullptr;
    hipStream_t st;
    if (hipMalloc(&d, n) != hipSuccess || hipHostMalloc(&h, n, hipHostMallocDefault) != hipSuccess ||
        hipStreamCreate(&st) != hipSuccess)
        return 1;
    memset(h, 0, n);
    for (int src_node : {0, 1}) {
        char* src = nullptr;
        std::thread([&] {
            bind_node(src_node);
            src = (char*)malloc(n);
            memset(src, 7, n);
        }).join();
        for (int thr_node : {-1, 0, 1, -1, 0, 1}) {
            double best = 1e9, worst = 0;
            for (int rep = 0; rep < 3; ++rep) {
                std::atomic<size_t> next{0};
                std::vector<std::atomic<int>> ready(nch);
                for (auto& r : ready) r.store(0);
                auto take = [&]() {
                    const size_t c = next.fetch_add(1);
                    if (c >= nch) return false;
                    memcpy((char*)h + c * chunk, src + c * chunk, chunk);
                    ready[c].store(1, std::memory_order_release);
                    return true;
                };
                (void)hipStreamSynchronize(st);
                bind_node(thr_node);
                auto t0 = std::chrono::steady_clock::now();
                std::vector<std::thread> pool;
                for (int t = 0; t < 7; ++t) pool.emplace_back([&] { bind_node(thr_node); while (take()) {} });
                for (size_t sent = 0; sent < nch;) {
                    if (ready[sent].load(std::memory_order_acquire)) {
                        (void)hipMemcpyAsync((char*)d + sent * chunk, (char*)h + sent * chunk, chunk,
                                             hipMemcpyHostToDevice, st);
                        ++sent;
                    } else if (!take()) {
                        std::this_thread::yield();
                    }
                }
                for (auto& t : pool) t.join();
                const double ts = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                (void)hipStreamSynchronize(st);
                const double tt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                best = tt < best ? tt : best;
                worst = tt > worst ? tt : worst;
                if (rep == 2)
                    printf("src node%d threads %-7s staged %.1f ms, done %.1f ms (%.1f GB/s); best %.1f worst %.1f ms\n",
                           src_node, thr_node < 0 ? "unbound" : (thr_node ? "node1" : "node0"), ts * 1e3, tt * 1e3,
                           n / tt / 1e9, best * 1e3, worst * 1e3);
            }
        }
        free(src);
    }
    return 0;
}
