// Pinned-buffer NUMA placement vs H2D DMA rate: for pinned buffers allocated
// and first touched by a thread bound to node 0, node 1, or unbound, print the NUMA node of their
// pages (get_mempolicy) and the H2D rate of 4 MiB hipMemcpyAsync pieces from them; plus the GPU's
// PCI NUMA node.  Usage: tools/pinned_probe [MiB]
#include <hip/hip_runtime.h>
#include <numaif.h>
#include <pthread.h>
#include <sched.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>

static int page_node(void* p) {
    int node = -1;
    if (get_mempolicy(&node, nullptr, 0, p, MPOL_F_NODE | MPOL_F_ADDR) != 0) return -2;
    return node;
}

static void bind_node(int node) {
    if (node < 0) return;
    cpu_set_t s;
    CPU_ZERO(&s);
    for (int c = node * 64; c < node * 64 + 64; ++c) CPU_SET(c, &s);
    sched_setaffinity(0, sizeof(s), &s);
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 256;
    const size_t n = mib << 20, piece = 4u << 20;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), 0) == hipSuccess) {
        std::string b(bus);
        for (auto& c : b) c = (char)tolower(c);
        std::ifstream f("/sys/bus/pci/devices/" + b + "/numa_node");
        int nn = -9;
        f >> nn;
        printf("gpu %s numa_node %d\n", bus, nn);
    }
    void* d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess) return 1;
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 1;
    for (int mode : {-1, 0, 1, -1, 0, 1}) {
        void* h = nullptr;
        std::thread t([&] {
            bind_node(mode);
            if (hipHostMalloc(&h, n, hipHostMallocDefault) != hipSuccess) h = nullptr;
            if (h) memset(h, 1, n);
        });
        t.join();
        if (!h) return 2;
        int nodes[2] = {0, 0}, other = 0;
        for (size_t off = 0; off < n; off += n / 16) {
            const int nd = page_node((char*)h + off);
            if (nd == 0 || nd == 1) ++nodes[nd]; else ++other;
        }
        double best = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipStreamSynchronize(st);
            auto t0 = std::chrono::steady_clock::now();
            for (size_t off = 0; off < n; off += piece)
                hipMemcpyAsync((char*)d + off, (char*)h + off, piece, hipMemcpyHostToDevice, st);
            hipStreamSynchronize(st);
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (n / s / 1e9 > best) best = n / s / 1e9;
        }
        printf("alloc thread %-8s pages on node0 %2d node1 %2d other %d   H2D %.1f GB/s\n",
               mode < 0 ? "unbound" : (mode == 0 ? "node0" : "node1"), nodes[0], nodes[1], other, best);
        hipHostFree(h);
    }
    return 0;
}
