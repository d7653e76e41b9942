// calib_runs.hip -- random-run READ rate (the read side of a chunk-major slot
// layout): every wave-instruction reads 64/L runs of L consecutive 8-B words,
// each run at a random word offset of a 16 GiB array (a64: 64-B aligned runs).
// Also the sequential read rate for reference.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/calib_runs tools/calib_runs.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void k_seq_read(const uint64_t* p, uint64_t n_words, unsigned* sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += stride) acc ^= p[i];
    if (acc == 0x1234567ull) *sink = 1;
}

template <int L, bool A64, int U>
__global__ void k_run_read(const uint64_t* p, uint64_t n_words, uint64_t iters, unsigned* sink) {
    const int lane = threadIdx.x & 63;
    uint64_t h = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63) + 1) * 0x9E3779B97F4A7C15ull;
    uint64_t acc = 0;
    for (uint64_t it = 0; it < iters; it += U) {
        uint64_t x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            h ^= h >> 29;
            h *= 0xBF58476D1CE4E5B9ull;
            uint64_t g = (h + (uint64_t)(lane / L) * 0xD6E8FEB86659FD93ull);
            g ^= g >> 32;
            g *= 0x9E3779B97F4A7C15ull;
            uint64_t base = (g >> 20) % (n_words - 64);
            if (A64) base &= ~7ull;
            x[u] = p[base + (lane % L)];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= x[u];
    }
    if (acc == 0x1234567ull) *sink = 1;
}

int main() {
    const uint64_t bytes = 16ull << 30;
    const uint64_t words = bytes / 8;
    uint64_t* p = nullptr;
    unsigned* sink = nullptr;
    if (hipMalloc((void**)&p, bytes) != hipSuccess || hipMalloc((void**)&sink, 4) != hipSuccess) return 1;
    hipMemset(p, 1, bytes);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, double rbytes, auto&& launch) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a, 0);
            launch();
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("%-16s %8.3f ms  %6.2f TB/s useful read\n", name, ms, rbytes / (ms * 1e-3) / 1e12);
        }
    };
    for (int grid : {2048, 4096}) {
        printf("grid %d x 256\n", grid);
        timeit("seq", (double)bytes, [&] { hipLaunchKernelGGL(k_seq_read, dim3(grid), dim3(256), 0, 0, p, words, sink); });
        const uint64_t iters = (words / 2) / ((uint64_t)grid * 256) / 4 * 4;
        const double rb = (double)iters * grid * 256 * 8;
#define RUN(L)                                                                                                     \
        timeit("run " #L, rb, [&] { hipLaunchKernelGGL((k_run_read<L, false, 4>), dim3(grid), dim3(256), 0, 0, p, words, iters, sink); }); \
        timeit("run " #L " a64", rb, [&] { hipLaunchKernelGGL((k_run_read<L, true, 4>), dim3(grid), dim3(256), 0, 0, p, words, iters, sink); });
        RUN(1) RUN(4) RUN(8) RUN(16) RUN(32) RUN(64)
    }
    hipFree(p);
    return 0;
}
