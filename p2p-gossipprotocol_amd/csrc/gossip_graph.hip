// gossip_graph.hip -- device-side overlay generator (powerlaw model).
//
// Replaces the seed bootstrap + selectAndConnectPeers (peer.cpp:63-72,
// 161-253; seed.cpp:109-129): every peer draws k from the reference's power
// law k = floor(L * U^(1/2.5)) (peer.cpp:219-222, evaluated with exact integer
// thresholds), picks k of its L i.i.d. skewed candidates, skips itself
// (peer.cpp:230), and the edge set is symmetrised, deduplicated
// (connectedPeers map overwrite, peer.cpp:242) and row-sorted.
//
// Pipeline (all on the ctx stream): count keys -> emit 64-bit keys
// (row_local << 32 | col) for the owned rows -> radix sort -> unique ->
// row bounds -> exclusive scan -> extract col.  Deterministic: the CSR is a
// pure function of (n, list_len, seed), identical on every rank and to the
// CPU restatement.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <string>

#include "gossip_internal.hpp"
#include "philox.hpp"

namespace gossip {

typedef unsigned __int128 u128;

static bool thr_ok(uint64_t x, uint32_t j, uint32_t L) {
    const u128 l5 = (u128)L * L * L * L * L;
    const u128 j5 = (u128)j * j * j * j * j;
    return (u128)x * x * l5 >= (j5 << 64);
}

uint64_t pick_threshold(uint32_t j, uint32_t L) {
    if (j >= L) return 1ull << 32;
    if (j == 0) return 0;
    // start from a double estimate, then settle on the exact smallest x
    double r = (double)j / (double)L;
    double est = r * r * __builtin_sqrt(r) * 4294967296.0;
    uint64_t x = (uint64_t)est;
    if (x > (1ull << 32)) x = 1ull << 32;
    while (x > 0 && thr_ok(x - 1, j, L)) --x;
    while (!thr_ok(x, j, L)) ++x;
    return x;
}

namespace {

struct ThrTable {
    uint32_t t[64];  // t[j] for 1 <= j < L
    uint32_t L;
};

__device__ __forceinline__ uint32_t draw_count(uint32_t x, const ThrTable& tt) {
    uint32_t k = 0;
    for (uint32_t j = 1; j < tt.L; ++j) k += x >= tt.t[j];
    return k;
}

__device__ __forceinline__ unsigned long long wsum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    return x;
}

// Visit every kept directed draw u -> c of peer u.
template <class F>
__device__ __forceinline__ void draws_of(uint32_t u, uint64_t n, uint32_t seed, const ThrTable& tt, F&& f) {
    const uint32_t k = draw_count(philox4x32_10(P_DEGREE, 0, 0, 0, seed, u).x, tt);
    for (uint32_t i = 0; i < k; i += 4) {
        const u32x4 r = philox4x32_10(P_TARGET, 0, i >> 2, 0, seed, u);
        for (uint32_t j = 0; j < 4 && i + j < k; ++j) {
            const uint32_t c = skew_pick(lane_of(r, j), n);
            if (c != u) f(c);
        }
    }
}

__global__ __launch_bounds__(256) void k_gen_count(uint64_t n, uint64_t begin, uint64_t end, uint32_t seed,
                                                   ThrTable tt, unsigned long long* total) {
    unsigned long long mine = 0;
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (uint64_t)gridDim.x * blockDim.x) {
        const bool own_u = u >= begin && u < end;
        draws_of((uint32_t)u, n, seed, tt, [&](uint32_t c) { mine += (unsigned)own_u + (unsigned)(c >= begin && c < end); });
    }
    mine = wsum(mine);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(total, mine);
}

__global__ __launch_bounds__(256) void k_gen_fill(uint64_t n, uint64_t begin, uint64_t end, uint32_t seed,
                                                  ThrTable tt, unsigned long long* keys, unsigned long long* cursor) {
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // uniform trip count per wave so the wave-level append stays converged
    const uint64_t first = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
    for (uint64_t base = first; base < n; base += stride) {
        const uint64_t u = base + lane;
        const bool valid = u < n;
        const bool own_u = valid && u >= begin && u < end;
        unsigned cnt = 0;
        if (valid)
            draws_of((uint32_t)u, n, seed, tt, [&](uint32_t c) { cnt += (unsigned)own_u + (unsigned)(c >= begin && c < end); });
        unsigned incl = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        const unsigned total = __shfl(incl, 63);
        unsigned long long at = 0;
        if (lane == 0 && total) at = atomicAdd(cursor, (unsigned long long)total);
        at = __shfl(at, 0) + (incl - cnt);
        if (valid && cnt) {
            draws_of((uint32_t)u, n, seed, tt, [&](uint32_t c) {
                if (own_u) keys[at++] = ((unsigned long long)(u - begin) << 32) | c;
                if (c >= begin && c < end) keys[at++] = ((unsigned long long)(c - begin) << 32) | (uint32_t)u;
            });
        }
    }
}

__global__ void k_row_bounds(const unsigned long long* keys, uint64_t m, unsigned long long* start,
                             unsigned long long* stop) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = keys[e] >> 32;
        if (e == 0 || (keys[e - 1] >> 32) != r) start[r] = e;
        if (e + 1 == m || (keys[e + 1] >> 32) != r) stop[r] = e + 1;
    }
}

__global__ void k_row_len(unsigned long long* start, const unsigned long long* stop, uint64_t n) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (uint64_t)gridDim.x * blockDim.x)
        start[v] = v < n ? stop[v] - start[v] : 0ull;
}

__global__ void k_extract_col(const unsigned long long* keys, uint64_t m, uint32_t* col) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x)
        col[e] = (uint32_t)keys[e];
}

unsigned gridn(uint64_t items) {
    uint64_t g = (items + 255) / 256;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    return (unsigned)g;
}

}  // namespace

#define GCHECK(x)                                                                     \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            if (err) *err = std::string(#x ": ") + hipGetErrorString(e_);             \
            goto fail;                                                                \
        }                                                                             \
    } while (0)

hipError_t build_powerlaw_device(uint64_t n, uint64_t begin, uint64_t end, uint32_t list_len, uint32_t seed,
                                 uint64_t** rp_out, uint32_t** col_out, uint64_t* n_edges, hipStream_t s,
                                 std::string* err) {
    ThrTable tt{};
    tt.L = list_len;
    for (uint32_t j = 1; j < list_len; ++j) tt.t[j] = (uint32_t)pick_threshold(j, list_len);
    const uint64_t n_local = end - begin;
    unsigned long long *d_cnt = nullptr, *keys_a = nullptr, *keys_b = nullptr, *start = nullptr, *stop = nullptr;
    long long* d_nsel = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0, need = 0;
    uint64_t* rp = nullptr;
    uint32_t* col = nullptr;
    unsigned long long n_keys = 0;
    long long n_unique = 0;
    int end_bit = 32;
    hipError_t last = hipSuccess;

    GCHECK(hipMallocAsync((void**)&d_cnt, 2 * sizeof(unsigned long long), s));
    GCHECK(hipMemsetAsync(d_cnt, 0, 2 * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_gen_count, dim3(gridn(n)), dim3(256), 0, s, n, begin, end, seed, tt, d_cnt);
    GCHECK(hipGetLastError());
    GCHECK(hipMemcpyAsync(&n_keys, d_cnt, sizeof(n_keys), hipMemcpyDeviceToHost, s));
    GCHECK(hipStreamSynchronize(s));

    GCHECK(hipMalloc((void**)&keys_a, (n_keys + 1) * sizeof(unsigned long long)));
    GCHECK(hipMalloc((void**)&keys_b, (n_keys + 1) * sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_gen_fill, dim3(gridn(n)), dim3(256), 0, s, n, begin, end, seed, tt, keys_a, d_cnt + 1);
    GCHECK(hipGetLastError());

    while ((1ull << (end_bit - 32)) < n_local) ++end_bit;
    GCHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, need, keys_a, keys_b, (size_t)n_keys, 0, end_bit, s));
    temp_bytes = need;
    GCHECK(hipcub::DeviceSelect::Unique(nullptr, need, keys_b, keys_a, d_nsel, (int64_t)n_keys, s));
    if (need > temp_bytes) temp_bytes = need;
    GCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, start, rp, n_local + 1, s));
    if (need > temp_bytes) temp_bytes = need;
    GCHECK(hipMalloc(&temp, temp_bytes + 16));
    GCHECK(hipMalloc((void**)&d_nsel, sizeof(long long)));

    need = temp_bytes;
    GCHECK(hipcub::DeviceRadixSort::SortKeys(temp, need, keys_a, keys_b, (size_t)n_keys, 0, end_bit, s));
    need = temp_bytes;
    GCHECK(hipcub::DeviceSelect::Unique(temp, need, keys_b, keys_a, d_nsel, (int64_t)n_keys, s));
    GCHECK(hipMemcpyAsync(&n_unique, d_nsel, sizeof(n_unique), hipMemcpyDeviceToHost, s));
    GCHECK(hipStreamSynchronize(s));
    GCHECK(hipFree(keys_b));
    keys_b = nullptr;

    GCHECK(hipMalloc((void**)&start, (n_local + 1) * sizeof(unsigned long long)));
    GCHECK(hipMalloc((void**)&stop, (n_local + 1) * sizeof(unsigned long long)));
    GCHECK(hipMemsetAsync(start, 0, (n_local + 1) * sizeof(unsigned long long), s));
    GCHECK(hipMemsetAsync(stop, 0, (n_local + 1) * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_row_bounds, dim3(gridn((uint64_t)n_unique)), dim3(256), 0, s, keys_a, (uint64_t)n_unique,
                       start, stop);
    GCHECK(hipGetLastError());
    hipLaunchKernelGGL(k_row_len, dim3(gridn(n_local + 1)), dim3(256), 0, s, start, stop, n_local);
    GCHECK(hipGetLastError());
    GCHECK(hipMalloc((void**)&rp, (n_local + 1) * sizeof(uint64_t)));
    need = temp_bytes;
    GCHECK(hipcub::DeviceScan::ExclusiveSum(temp, need, (const unsigned long long*)start,
                                            (unsigned long long*)rp, n_local + 1, s));
    GCHECK(hipMalloc((void**)&col, ((uint64_t)n_unique + 1) * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_extract_col, dim3(gridn((uint64_t)n_unique)), dim3(256), 0, s, keys_a, (uint64_t)n_unique,
                       col);
    GCHECK(hipGetLastError());
    GCHECK(hipStreamSynchronize(s));

    hipFree(keys_a);
    hipFree(start);
    hipFree(stop);
    hipFree(temp);
    hipFree(d_nsel);
    hipFreeAsync(d_cnt, s);
    *rp_out = rp;
    *col_out = col;
    *n_edges = (uint64_t)n_unique;
    return hipSuccess;

fail:
    last = hipGetLastError();
    (void)last;
    hipStreamSynchronize(s);
    if (keys_a) hipFree(keys_a);
    if (keys_b) hipFree(keys_b);
    if (start) hipFree(start);
    if (stop) hipFree(stop);
    if (temp) hipFree(temp);
    if (d_nsel) hipFree(d_nsel);
    if (d_cnt) hipFree(d_cnt);
    if (rp) hipFree(rp);
    if (col) hipFree(col);
    return hipErrorUnknown;
}

}  // namespace gossip
