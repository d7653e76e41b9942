// Unit test of the LDS record staging protocol (p2p-gossipprotocol_amd/csrc/gossip_stage.hpp) on the GPU:
// every workgroup stages pseudo-random records (unique ids) into kNB bins of kB records, flushing full
// buffers to per-bin global regions; the host checks every id arrives exactly once, in its own bin.
// usage: stage_test <bins> <records per workgroup> <skew 0|1>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../p2p-gossipprotocol_amd/csrc/gossip_stage.hpp"

using namespace gossip;

constexpr int kBlockT = 1024;
constexpr uint32_t kB = 64;
constexpr uint32_t kMaxBins = 96;

__device__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <bool kNoGlobal>
__global__ __launch_bounds__(kBlockT) void k_stage(uint32_t nb, uint32_t per_wg, uint32_t skew, uint32_t* out_id,
                                                   unsigned long long* out_w, uint32_t* cur, uint64_t cap_per_bin,
                                                   uint32_t* err) {
    __shared__ uint32_t tk_s[kMaxBins], wr_s[kMaxBins], dn_s[kMaxBins];
    __shared__ uint16_t bd_s[kMaxBins * kB];
    __shared__ unsigned long long bw_s[kMaxBins * kB];
    for (uint32_t i = threadIdx.x; i < kMaxBins; i += kBlockT) tk_s[i] = wr_s[i] = dn_s[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    auto reserve = [&](uint32_t f) { return atomicAdd(&cur[f], kB); };
    auto flush = [&](uint32_t f, uint32_t pos) {
        const uint16_t dv = bd_s[f * kB + lane];
        const unsigned long long wv = bw_s[f * kB + lane];
        lds_fence();
        if (lane == 0) stage_release(wr_s, dn_s, f);
        if (kNoGlobal) return;
        if ((uint64_t)pos + kB <= cap_per_bin) {
            out_id[f * cap_per_bin + pos + lane] = dv == 0xFFFFu ? 0xFFFFFFFFu : (uint32_t)(wv >> 32);
            out_w[f * cap_per_bin + pos + lane] = wv;
        } else if (lane == 0) {
            atomicOr(err, 2u);
        }
    };
    constexpr int kU = 4;
    for (uint32_t i0 = (uint32_t)wave * 64 * kU; i0 < per_wg; i0 += kBlockT * kU) {
        uint32_t k[kU], d[kU];
        unsigned long long w[kU];
        bool pend[kU];
        for (int j = 0; j < kU; ++j) {
            const uint32_t i = i0 + j * 64 + lane;
            const uint32_t id = blockIdx.x * per_wg + i;
            pend[j] = i < per_wg;
            const uint32_t h = hash32(id);
            k[j] = skew ? (h % 8 == 0 ? h % nb : 0u) : h % nb;
            d[j] = k[j];
            w[j] = ((unsigned long long)id << 32) | k[j];
        }
        if (kNoGlobal) stage<kU, kB>(tk_s, wr_s, dn_s, bd_s, bw_s, k, d, w, pend, [](uint32_t) { return 0u; }, flush, err);
        else stage<kU, kB>(tk_s, wr_s, dn_s, bd_s, bw_s, k, d, w, pend, reserve, flush, err);
    }
    __syncthreads();
    for (uint32_t f = wave; f < nb; f += kBlockT / 64) {
        const uint32_t c = stage_open(tk_s, f, kB);
        if (lane == 0) { atomicAdd(&err[2], c); atomicMax(&err[3], c); atomicAdd(&err[4], wr_s[f]); }
        if (!c) continue;
        if ((uint32_t)lane >= c) {
            bd_s[f * kB + lane] = 0xFFFFu;
            bw_s[f * kB + lane] = 0ull;
        }
        lds_fence();
        uint32_t pos = 0;
        if (lane == 0) pos = reserve(f);
        flush(f, (uint32_t)__shfl((int)pos, 0));
    }
}

int main(int argc, char** argv) {
    const uint32_t nb = argc > 1 ? atoi(argv[1]) : 1, per_wg = argc > 2 ? atoi(argv[2]) : 20000,
                   skew = argc > 3 ? atoi(argv[3]) : 0;
    const uint32_t grid = argc > 4 ? atoi(argv[4]) : 512;
    const uint64_t total = (uint64_t)grid * per_wg;
    const uint64_t cap = total + (uint64_t)grid * kB;  // per bin, worst case
    uint32_t *out_id, *cur, *err;
    unsigned long long* out_w;
    hipMalloc(&out_id, cap * nb * 4);
    hipMalloc(&out_w, cap * nb * 8);
    hipMalloc(&cur, nb * 4);
    hipMalloc(&err, 32);
    hipMemset(cur, 0, nb * 4);
    hipMemset(err, 0, 32);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int noglobal = argc > 5 ? atoi(argv[5]) : 0;
    if (noglobal) {
        hipLaunchKernelGGL(k_stage<true>, dim3(grid), dim3(kBlockT), 0, 0, nb, per_wg, skew, out_id, out_w, cur, cap, err);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_stage<true>, dim3(grid), dim3(kBlockT), 0, 0, nb, per_wg, skew, out_id, out_w, cur, cap, err);
        hipEventRecord(e1);
        hipDeviceSynchronize();
        float t = 0;
        hipEventElapsedTime(&t, e0, e1);
        printf("bins %u per_wg %u grid %u, no global flush: %.3f ms (%.2f G records/s)\n", nb, per_wg, grid, t,
               (double)grid * per_wg / t * 1e-6);
        return 0;
    }
    hipLaunchKernelGGL(k_stage<false>, dim3(grid), dim3(kBlockT), 0, 0, nb, per_wg, skew, out_id, out_w, cur, cap, err);
    hipDeviceSynchronize();
    hipMemset(cur, 0, nb * 4);
    hipMemset(err, 0, 32);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_stage<false>, dim3(grid), dim3(kBlockT), 0, 0, nb, per_wg, skew, out_id, out_w, cur, cap, err);
    hipEventRecord(e1);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint32_t> hc(nb), hid;
    std::vector<unsigned long long> hw;
    uint32_t herr = 0, hx[8];
    hipMemcpy(hc.data(), cur, nb * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hx, err, 32, hipMemcpyDeviceToHost);
    herr = hx[0];
    printf("flushed non-pad %u, drained cnt sum %u max %u, drained wr sum %u\n", hx[1], hx[2], hx[3], hx[4]);
    std::vector<uint8_t> seen(total, 0);
    uint64_t got = 0, bad = 0, dup = 0;
    for (uint32_t f = 0; f < nb; ++f) {
        hid.resize(hc[f]);
        hw.resize(hc[f]);
        hipMemcpy(hid.data(), out_id + f * cap, hc[f] * 4, hipMemcpyDeviceToHost);
        hipMemcpy(hw.data(), out_w + f * cap, hc[f] * 8, hipMemcpyDeviceToHost);
        for (uint32_t i = 0; i < hc[f]; ++i) {
            if (hid[i] == 0xFFFFFFFFu) continue;
            if (hid[i] >= total || (uint32_t)(hw[i] & 0xFFFFFFFFu) != f) { ++bad; continue; }
            if (seen[hid[i]]++) ++dup;
            ++got;
        }
    }
    printf("bins %u per_wg %u skew %u grid %u: %.3f ms (%.2f G records/s), err %u, records %llu of %llu, bad %llu, dup %llu -> %s\n", nb, per_wg,
           skew, grid, ms, total / ms * 1e-6, herr, (unsigned long long)got, (unsigned long long)total, (unsigned long long)bad,
           (unsigned long long)dup, (!herr && got == total && !bad && !dup) ? "OK" : "FAIL");
    return (!herr && got == total && !bad && !dup) ? 0 : 1;
}
