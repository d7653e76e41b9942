// stage_selftest.hip -- GPU test of the LDS record-staging protocol of the blocked rounds
// (p2p-gossipprotocol_amd/csrc/gossip_stage.hpp), loaded by tests/test_gpu_stage.py through ctypes.
// Test infrastructure only: the product library does not link it.
//
// Every workgroup (1024 threads, 4 records per lane per call, as k_pb_scatter / k_pb_split) stages
// pseudo-random records with unique ids into nb bins of kB records per half and flushes whole
// generations into its own segment of each bin at place generation * kB, the segments sized from the
// records' counts (as build_pb sizes the blocked rounds' segments from the overlay's edges).  The host then checks every id arrived exactly once, in its own bin.  With skew, 7 of 8
// records go to bin 0: one bin hot in every wave at once (round 3's hang: a retried reservation wrapped
// its counter under contention and handed out a place twice; one bin lost 256 of 576 records).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../p2p-gossipprotocol_amd/csrc/gossip_stage.hpp"

using namespace gossip;

namespace {

constexpr int kBlockT = 1024;
constexpr uint32_t kMaxBins = 160;  // as kPbCoarseMax; 100 in level 2's geometry (kb = 64), as kPbFineMax

__device__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

uint32_t bin_of(uint32_t id, uint32_t nb, uint32_t skew) {  // host copy of the kernel's draw
    uint32_t h = id;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return skew ? (h % 8 == 0 ? h % nb : 0u) : h % nb;
}

template <uint32_t kB, uint32_t kH, class TD, uint32_t kNB>
__global__ __launch_bounds__(kBlockT) void k_stage(uint32_t nb, uint32_t per_wg, uint32_t skew, uint32_t* out_id,
                                                   unsigned long long* out_w, const uint64_t* seg_base,
                                                   const uint32_t* seg_cap, uint32_t* err) {
    __shared__ uint32_t tk_s[kNB], wr_s[kH * kNB], gn_s[kH * kNB];
    __shared__ uint64_t base_s[kNB];  // this workgroup's segment of each bin
    __shared__ uint32_t cap_s[kNB];
    __shared__ TD bd_s[kNB * kH * kB];
    __shared__ unsigned long long bw_s[kNB * kH * kB];
    stage_init<kH>(tk_s, wr_s, gn_s, kNB, threadIdx.x, kBlockT);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t f = threadIdx.x; f < nb; f += kBlockT) {
        base_s[f] = seg_base[(uint64_t)blockIdx.x * nb + f];
        cap_s[f] = seg_cap[(uint64_t)blockIdx.x * nb + f];
    }
    __syncthreads();
    auto flush = [&](uint32_t f, uint32_t g) {
        const uint32_t i = lane & (kB - 1);
        const uint32_t hb = stage_at<kB, kH>(f, g, 0);
        const TD dv = bd_s[hb + i];
        const unsigned long long wv = bw_s[hb + i];
        lds_fence();
        if (lane == 0) stage_release<kH>(wr_s, gn_s, f, g);
        if ((uint64_t)g * kB + kB > cap_s[f]) {  // the segment would overflow
            if (lane == 0) atomicOr(err, 2u);
            return;
        }
        const uint64_t at = base_s[f] + (uint64_t)g * kB + i;
        // (kB = 64: one lane per record, both stores; kB = 32: lanes 0-31 destinations, 32-63 words)
        if (kB == 64 || lane < (int)kB) out_id[at] = (TD)~dv == 0 ? 0xFFFFFFFFu : (uint32_t)(wv >> 32);
        if (kB == 64 || (lane >= (int)kB && lane < 2 * (int)kB)) out_w[at] = wv;
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
        stage<kU, kB, kH>(tk_s, wr_s, gn_s, bd_s, bw_s, k, d, w, pend, flush, err);
    }
    __syncthreads();
    for (uint32_t f = wave; f < nb; f += kBlockT / 64) {
        uint32_t g = 0;
        const uint32_t c = stage_open(tk_s, f, kB, &g);
        if (lane == 0) atomicAdd(&err[1], stage_len(tk_s, f, kB));
        if (!c) continue;
        if ((uint32_t)lane >= c && lane < (int)kB) {
            const uint32_t s = stage_at<kB, kH>(f, g, lane);
            bd_s[s] = (TD)~0u;
            bw_s[s] = 0ull;
        }
        lds_fence();
        flush(f, g);
    }
}

}  // namespace

// Runs one staging test; out[0] = 1 iff every record arrived once in its bin, out[1] records found,
// out[2] records expected, out[3] misplaced, out[4] duplicates, out[5] error flags (bit 4: a stuck wave),
// out[6] = Σ of the segments' lengths (stage_len: whole generations), out[7] = the same from the host
// (the segments' capacities).
// kb: 32 (32-bit destinations, two buffers per bin: level 1's geometry), 64 (16-bit destinations, two
// buffers per bin: level 2's) or 16 (32-bit destinations, two buffers: the protocol at another size).
// Returns 0, or -1 on a HIP error / bad argument.
extern "C" int stage_selftest(uint32_t nb, uint32_t per_wg, uint32_t skew, uint32_t grid, uint32_t kb,
                              uint64_t* out) {
    if (!out || nb < 1 || nb > (kb == 64 ? 100u : kMaxBins) || (kb != 16 && kb != 32 && kb != 64) || !grid)
        return -1;
    const uint64_t total = (uint64_t)grid * per_wg;
    // segments: (workgroup, bin) pairs in bin-major order, each its records rounded up to whole generations
    std::vector<uint64_t> base((uint64_t)grid * nb);
    std::vector<uint32_t> cap((uint64_t)grid * nb, 0);
    for (uint32_t b = 0; b < grid; ++b)
        for (uint32_t i = 0; i < per_wg; ++i) ++cap[(uint64_t)b * nb + bin_of(b * per_wg + i, nb, skew)];
    uint64_t slots = 0;
    for (uint32_t f = 0; f < nb; ++f)
        for (uint32_t b = 0; b < grid; ++b) {
            uint32_t& c = cap[(uint64_t)b * nb + f];
            c = (c + kb - 1) / kb * kb;
            base[(uint64_t)b * nb + f] = slots;
            slots += c;
        }
    uint32_t *out_id = nullptr, *err = nullptr, *d_cap = nullptr;
    unsigned long long* out_w = nullptr;
    uint64_t* d_base = nullptr;
    auto cleanup = [&] {
        (void)hipFree(out_id);
        (void)hipFree(out_w);
        (void)hipFree(err);
        (void)hipFree(d_cap);
        (void)hipFree(d_base);
    };
    const uint64_t segs = (uint64_t)grid * nb;
    if (hipMalloc(&out_id, (slots + 1) * 4) != hipSuccess || hipMalloc(&out_w, (slots + 1) * 8) != hipSuccess ||
        hipMalloc(&err, 32) != hipSuccess || hipMalloc(&d_cap, segs * 4) != hipSuccess ||
        hipMalloc(&d_base, segs * 8) != hipSuccess ||
        hipMemset(out_id, 0xFF, (slots + 1) * 4) != hipSuccess ||  // unwritten slots read as padding
        hipMemset(err, 0, 32) != hipSuccess ||
        hipMemcpy(d_cap, cap.data(), segs * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_base, base.data(), segs * 8, hipMemcpyHostToDevice) != hipSuccess) {
        cleanup();
        return -1;
    }
    if (kb == 16)
        hipLaunchKernelGGL((k_stage<16, 2, uint32_t, kMaxBins>), dim3(grid), dim3(kBlockT), 0, 0, nb, per_wg, skew, out_id,
                           out_w, d_base, d_cap, err);
    else if (kb == 32)
        hipLaunchKernelGGL((k_stage<32, 2, uint32_t, kMaxBins>), dim3(grid), dim3(kBlockT), 0, 0, nb, per_wg, skew, out_id,
                           out_w, d_base, d_cap, err);
    else
        hipLaunchKernelGGL((k_stage<64, 2, uint16_t, 100>), dim3(grid), dim3(kBlockT), 0, 0, nb, per_wg, skew, out_id,
                           out_w, d_base, d_cap, err);
    uint32_t hx[8] = {};
    std::vector<uint32_t> hid(slots + 1);
    std::vector<unsigned long long> hw(slots + 1);
    const bool ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
                    hipMemcpy(hx, err, 32, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(hid.data(), out_id, slots * 4, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(hw.data(), out_w, slots * 8, hipMemcpyDeviceToHost) == hipSuccess;
    cleanup();
    if (!ok) return -1;
    std::vector<uint8_t> seen(total, 0);
    uint64_t got = 0, bad = 0, dup = 0;
    for (uint32_t f = 0; f < nb; ++f)
        for (uint32_t b = 0; b < grid; ++b) {
            const uint64_t s0 = base[(uint64_t)b * nb + f], s1 = s0 + cap[(uint64_t)b * nb + f];
            for (uint64_t at = s0; at < s1; ++at) {
                if (hid[at] == 0xFFFFFFFFu) continue;  // padding
                const uint32_t id = hid[at];
                if (id >= total || id / per_wg != b || (uint32_t)(hw[at] & 0xFFFFFFFFu) != f ||
                    (uint32_t)(hw[at] >> 32) != id) {
                    ++bad;
                    continue;
                }
                if (seen[id]++) ++dup;
                ++got;
            }
        }
    out[0] = (!hx[0] && got == total && !bad && !dup && hx[1] == slots) ? 1 : 0;
    out[1] = got;
    out[2] = total;
    out[3] = bad;
    out[4] = dup;
    out[5] = hx[0];
    out[6] = hx[1];
    out[7] = slots;
    return 0;
}
