// calib_store.hip -- what HBM store rate does the binned scatter's shape allow?
// 16 GiB destination (far beyond L2 + MALL); every store is a 64-bit word per
// lane (global_store_dwordx2), as in k_bin_scatter_lds.
//   seq      : wave instruction = 512 contiguous bytes, grid-stride sweep
//   seq16    : 16 B per lane (dwordx4), 1 KiB per instruction
//   run L    : 64/L runs of L consecutive words per instruction, each run at a
//              random word offset (L = 1 .. 64); "run L a64": runs 64-B aligned,
//              "run L a32": 32-B aligned (is the memory's write atom 32 or 64 B?)
//   rw       : seq stores with a 1/3-size coalesced read stream interleaved
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/calib_store tools/calib_store.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void k_seq(uint64_t* p, uint64_t n_words) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += stride) p[i] = i;
}

__global__ void k_seq16(uint4* p, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        p[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

template <int L, int A>  // A: run alignment in words (1, 4 or 8)
__global__ void k_run(uint64_t* p, uint64_t n_words, uint64_t iters) {
    const int lane = threadIdx.x & 63;
    uint64_t h = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63) + 1) * 0x9E3779B97F4A7C15ull;
    for (uint64_t it = 0; it < iters; ++it) {
        h ^= h >> 29;
        h *= 0xBF58476D1CE4E5B9ull;
        // run r = lane / L gets its own random offset: mix r into the hash
        uint64_t g = (h + (uint64_t)(lane / L) * 0xD6E8FEB86659FD93ull);
        g ^= g >> 32;
        g *= 0x9E3779B97F4A7C15ull;
        uint64_t base = (g >> 20) % (n_words - 64);
        base &= ~(uint64_t)(A - 1);
        p[base + (lane % L)] = h;
    }
}

__global__ void k_rw(uint64_t* p, uint64_t n_words, const uint64_t* q, uint64_t n_read, unsigned* sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += stride) {
        p[i] = i;
        if (i % 3 == 0 && i / 3 < n_read) acc ^= q[i / 3];
    }
    if (acc == 0x1234567ull) *sink = 1;
}

int main() {
    const uint64_t bytes = 16ull << 30;
    const uint64_t words = bytes / 8;
    uint64_t *p = nullptr, *q = nullptr;
    unsigned* sink = nullptr;
    if (hipMalloc((void**)&p, bytes) != hipSuccess || hipMalloc((void**)&q, bytes / 3) != hipSuccess ||
        hipMalloc((void**)&sink, 4) != hipSuccess)
        return 1;
    hipMemset(p, 0, bytes);
    hipMemset(q, 1, bytes / 3);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, double wbytes, auto&& launch) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a, 0);
            launch();
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("%-14s %8.3f ms  %6.2f TB/s stored\n", name, ms, wbytes / (ms * 1e-3) / 1e12);
        }
    };
    for (int grid : {2048, 4096}) {
        printf("grid %d x 256\n", grid);
        timeit("seq", (double)bytes, [&] { hipLaunchKernelGGL(k_seq, dim3(grid), dim3(256), 0, 0, p, words); });
        timeit("seq16", (double)bytes,
               [&] { hipLaunchKernelGGL(k_seq16, dim3(grid), dim3(256), 0, 0, (uint4*)p, bytes / 16); });
        timeit("rw(+1/3 read)", (double)bytes,
               [&] { hipLaunchKernelGGL(k_rw, dim3(grid), dim3(256), 0, 0, p, words, q, words / 3, sink); });
        const uint64_t iters = words / ((uint64_t)grid * 256);
        const double wb = (double)iters * grid * 256 * 8;
#define RUN(L)                                                                                                 \
        timeit("run " #L, wb, [&] { hipLaunchKernelGGL((k_run<L, 1>), dim3(grid), dim3(256), 0, 0, p, words, iters); }); \
        timeit("run " #L " a32", wb, [&] { hipLaunchKernelGGL((k_run<L, 4>), dim3(grid), dim3(256), 0, 0, p, words, iters); }); \
        timeit("run " #L " a64", wb, [&] { hipLaunchKernelGGL((k_run<L, 8>), dim3(grid), dim3(256), 0, 0, p, words, iters); });
        RUN(1) RUN(4) RUN(8) RUN(16) RUN(32) RUN(64)
    }
    hipFree(p);
    hipFree(q);
    return 0;
}
