// calib_l2.hip -- random 8-B accesses into XCD-local regions: what does a
// random 64-bit atomicOr / store / load cost when the region a workgroup
// touches is owned by its XCD (blockIdx % 8) and small enough for that XCD's
// 4 MB L2?  Measures G ops/s for region sizes from 1 MB to 2 GB per XCD.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/calib_l2 tools/calib_l2.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int OP>  // 0 atomicOr, 1 store, 2 load
__global__ void k_rand(uint64_t* t, uint64_t region_words, uint64_t ops_per_thread, unsigned* sink) {
    const uint32_t xcd = blockIdx.x & 7;
    uint64_t* base = t + (uint64_t)xcd * region_words;
    uint64_t h = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1) * 0x9E3779B97F4A7C15ull;
    uint64_t acc = 0;
    for (uint64_t i = 0; i < ops_per_thread; ++i) {
        h ^= h >> 29;
        h *= 0xBF58476D1CE4E5B9ull;
        const uint64_t idx = (h >> 11) % region_words;
        if (OP == 0) atomicOr((unsigned long long*)(base + idx), (unsigned long long)(1ull << (h & 63)));
        else if (OP == 1) base[idx] = h;
        else acc ^= base[idx];
    }
    if (OP == 2 && acc == 0x12345ull) *sink = 1;
}

int main() {
    const uint64_t total = 16ull << 30;  // 16 GiB table
    uint64_t* t = nullptr;
    unsigned* sink = nullptr;
    if (hipMalloc((void**)&t, total) != hipSuccess || hipMalloc((void**)&sink, 4) != hipSuccess) return 1;
    hipMemset(t, 0, total);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[3] = {"atomicOr", "store", "load"};
    const uint64_t regions_mb[] = {1, 2, 3, 4, 8, 32, 256, 2048};
    const int grid = 2048, block = 256;
    for (uint64_t rmb : regions_mb) {
        const uint64_t rw = (rmb << 20) / 8;
        for (int op = 0; op < 3; ++op) {
            const uint64_t per = 256;
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a, 0);
                if (op == 0) hipLaunchKernelGGL(k_rand<0>, dim3(grid), dim3(block), 0, 0, t, rw, per, sink);
                if (op == 1) hipLaunchKernelGGL(k_rand<1>, dim3(grid), dim3(block), 0, 0, t, rw, per, sink);
                if (op == 2) hipLaunchKernelGGL(k_rand<2>, dim3(grid), dim3(block), 0, 0, t, rw, per, sink);
                hipEventRecord(b, 0);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (rep == 1)
                    printf("region %5llu MB/XCD  %-8s  %7.2f G ops/s  (%.3f ms)\n", (unsigned long long)rmb, names[op],
                           (double)grid * block * per / (ms * 1e-3) / 1e9, ms);
            }
        }
    }
    hipFree(t);
    return 0;
}
