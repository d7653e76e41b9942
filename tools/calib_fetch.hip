// calib_fetch.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access shapes of the gossip kernels (MI355X_MICROARCH.md: only 16-B/lane
// streams are calibrated there).  Each kernel touches a known number of bytes;
// run under `rocprofv3 --pmc FETCH_SIZE` (and WRITE_SIZE) and divide.
//   k_stream16 : 16 B/lane coalesced read of N bytes           (guide: FETCH = N/2)
//   k_stream4  : 4 B/lane coalesced read (col[] reads)
//   k_gather8  : one random 8-B read per lane from a 2 GiB table (nw[u] gathers)
//   k_store8   : 8 B/lane coalesced store (seen/nx writes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_stream16(const uint4* p, uint64_t n, unsigned* sink) {
    uint4 acc{0, 0, 0, 0};
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = p[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345u) *sink = 1;
}
__global__ void k_stream4(const unsigned* p, uint64_t n, unsigned* sink) {
    unsigned acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345u) *sink = 1;
}
__global__ void k_gather8(const uint64_t* t, uint64_t mask, uint64_t reads, unsigned* sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < reads; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        acc ^= t[h & mask];
    }
    if (acc == 0x12345ull) *sink = 1;
}
__global__ void k_store8(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = i;
}

int main() {
    const uint64_t bytes = 2ull << 30;  // 2 GiB: beyond the 256 MiB Infinity Cache
    void* buf;
    unsigned* sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc((void**)&sink, 4) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    const uint64_t reads = 1ull << 28;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms;
    auto run = [&](const char* name, auto&& launch, double touched) {
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("%-10s bytes_touched=%.0f ms=%.3f GB/s=%.1f\n", name, touched, ms, touched / ms / 1e6);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("stream16", [&] { hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, sink); }, (double)bytes);
        run("stream4", [&] { hipLaunchKernelGGL(k_stream4, dim3(4096), dim3(256), 0, 0, (const unsigned*)buf, bytes / 4, sink); }, (double)bytes);
        run("gather8", [&] { hipLaunchKernelGGL(k_gather8, dim3(4096), dim3(256), 0, 0, (const uint64_t*)buf, bytes / 8 - 1, reads, sink); }, (double)reads * 8);
        run("store8", [&] { hipLaunchKernelGGL(k_store8, dim3(4096), dim3(256), 0, 0, (uint64_t*)buf, bytes / 8); }, (double)bytes);
    }
    hipDeviceSynchronize();
    printf("reads=%llu\n", (unsigned long long)reads);
    return 0;
}
