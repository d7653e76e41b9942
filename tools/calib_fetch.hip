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
__global__ void k_gather8_nt(const uint64_t* t, uint64_t mask, uint64_t reads, unsigned* sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < reads; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        acc ^= __builtin_nontemporal_load(t + (h & mask));
    }
    if (acc == 0x12345ull) *sink = 1;
}
__global__ void k_gather8_sc1(const uint64_t* t, uint64_t mask, uint64_t reads, unsigned* sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < reads; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        acc ^= __hip_atomic_load(t + (h & mask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 0x12345ull) *sink = 1;
}
// 4 independent gathers per thread per iteration (more memory-level parallelism)
__global__ void k_gather8_x4(const uint64_t* t, uint64_t mask, uint64_t reads, unsigned* sink) {
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < reads / 4; i += stride) {
        uint64_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint64_t h = (i * 4 + k + 1) * 0x9E3779B97F4A7C15ull;
            h ^= h >> 29;
            v[k] = t[h & mask];
        }
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x12345ull) *sink = 1;
}
// gathers confined to a 32 MiB window (Infinity-Cache resident)
__global__ void k_gather8_mall(const uint64_t* t, uint64_t reads, unsigned* sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < reads; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        acc ^= t[h & ((32ull << 20) / 8 - 1)];
    }
    if (acc == 0x12345ull) *sink = 1;
}
// gathers confined to a 2 MiB window (L2 resident on every XCD)
__global__ void k_gather8_l2(const uint64_t* t, uint64_t reads, unsigned* sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < reads; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        acc ^= t[h & ((2ull << 20) / 8 - 1)];
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
        run("gather8nt", [&] { hipLaunchKernelGGL(k_gather8_nt, dim3(4096), dim3(256), 0, 0, (const uint64_t*)buf, bytes / 8 - 1, reads, sink); }, (double)reads * 8);
        run("gather8sc1", [&] { hipLaunchKernelGGL(k_gather8_sc1, dim3(4096), dim3(256), 0, 0, (const uint64_t*)buf, bytes / 8 - 1, reads, sink); }, (double)reads * 8);
        run("gather8x4", [&] { hipLaunchKernelGGL(k_gather8_x4, dim3(4096), dim3(256), 0, 0, (const uint64_t*)buf, bytes / 8 - 1, reads, sink); }, (double)reads * 8);
        run("gather8mall", [&] { hipLaunchKernelGGL(k_gather8_mall, dim3(4096), dim3(256), 0, 0, (const uint64_t*)buf, reads, sink); }, (double)reads * 8);
        run("gather8l2", [&] { hipLaunchKernelGGL(k_gather8_l2, dim3(4096), dim3(256), 0, 0, (const uint64_t*)buf, reads, sink); }, (double)reads * 8);
    }
    hipDeviceSynchronize();
    printf("reads=%llu\n", (unsigned long long)reads);
    return 0;
}
