// gossip_device.hpp -- device helpers shared by the round kernels of libgossip_hip
// (gossip_kernels.hip, gossip_blocked.hip): stat accumulation and its block flush,
// the bits a peer can still learn, wave reductions.
#pragma once
#include <hip/hip_runtime.h>

#include "gossip_internal.hpp"

namespace gossip {
namespace {

constexpr int kWavesPerBlock = kBlock / 64;
constexpr unsigned kMaxGrid = 2048;  // 256 CUs x 8 blocks of 256 threads

__device__ __forceinline__ bool bit_alive(const uint32_t* bits, uint32_t v) { return (bits[v >> 5] >> (v & 31)) & 1u; }

// source chunk c of a bin layout: global peers [bin_chunk_vb, bin_chunk_ve) (BinArgs.seg / .cps)
__device__ __forceinline__ uint64_t bin_chunk_vb(const BinArgs& b, uint64_t c) {
    return (c / b.cps) * b.seg + (c % b.cps) * b.chunk;
}
// (a chunk of the last segment can start past n: empty, not negative)
__device__ __forceinline__ uint64_t bin_chunk_ve(const BinArgs& b, uint64_t c, uint64_t n) {
    const uint64_t vb = bin_chunk_vb(b, c);
    return max(vb, min(min(vb + b.chunk, (c / b.cps + 1) * b.seg), n));
}

// Checked-index build (`make checked`: -DGOSSIP_CHECKED, build/checked/libgossip_hip.so).  GOSSIP_IDX(a, site,
// i, bound) is i in the product build; the checked build records the first index at or past its bound in a.chk
// ({trips, site, index, bound}) and substitutes 0, so the access stays inside the buffer and the run ends with
// GOSSIP_EBOUNDS naming the site instead of a fault that depends on what the allocator placed after the buffer.
#ifdef GOSSIP_CHECKED
__device__ __forceinline__ uint64_t chk_idx(unsigned long long* chk, uint32_t site, uint64_t i, uint64_t bound) {
    if (i < bound) return i;
    if (chk && atomicAdd(&chk[0], 1ull) == 0ull) {
        chk[1] = site;
        chk[2] = i;
        chk[3] = bound;
    }
    return 0;
}
#define GOSSIP_IDX(a, site, i, bound) chk_idx((a).chk, (site), (uint64_t)(i), (uint64_t)(bound))
constexpr bool kChecked = true;
#else
#define GOSSIP_IDX(a, site, i, bound) ((uint64_t)(i))
constexpr bool kChecked = false;
#endif

// the bits a peer can still learn: messages injected so far (at P = 1 the ones whose origin was alive to
// inject them -- a never-injected message kept every row of config 5 scanning to its end)
__device__ __forceinline__ uint64_t injm_full(const RoundArgs& a, int w) {
    return a.inj_live ? a.inj_mask[w] & a.inj_live[w] : a.inj_mask[w];
}
// ... and of those, this round: only bits that are in some new word (P = 1: in_flight, the previous
// round's receipts with this round's injections -- a bit outside it kept config 5's hubs and needy
// rows scanning to their ends: a message injected at an isolated peer is never in flight)
__device__ __forceinline__ uint64_t injm(const RoundArgs& a, int w) {
    return injm_full(a, w) & (a.use_flight ? a.in_flight[w] : ~0ull);
}
__device__ __forceinline__ uint64_t sgpr64(uint64_t x) {  // a wave-uniform value, kept in scalar registers
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}
// Both masks of a round, read once at a kernel's start (round 6).  Read where they were used, inside a
// sweep or a finish loop, inj_live is a global load the compiler cannot hoist past the loop's stores to
// seen and nx, and the wait for it (vmcnt(0)) also waited for every load the loop had put in flight ahead:
// k_pull_rows's next-tile prefetch, the binned apply's whole-bin seen loads.
template <int W>
struct InjMasks {
    uint64_t full[W], cur[W];
    __device__ __forceinline__ explicit InjMasks(const RoundArgs& a) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            full[w] = sgpr64(injm_full(a, w));
            cur[w] = sgpr64(injm(a, w));
        }
    }
    // word i % W's mask for a lane-varying i (a select chain: no register-array indexing)
    __device__ __forceinline__ uint64_t cur_at(uint32_t wi) const {
        uint64_t m = cur[0];
#pragma unroll
        for (int w = 1; w < W; ++w)
            if (wi == (uint32_t)w) m = cur[w];
        return m;
    }
};

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    return x;
}

__device__ __forceinline__ uint32_t lane_rank(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

struct Acc {
    unsigned long long frontier = 0, trav = 0, deliv = 0, undeliv = 0, fresh = 0, digest = 0, covered = 0, died = 0,
                       reports = 0, removals = 0, injected = 0, htrav = 0, checked = 0,
                       activated = 0, pulled = 0, gathered = 0, reconnects = 0, rejoined = 0, atomics = 0,
                       diag = 0, dead_cov = 0;
    unsigned long long fresh_or[kMaxWords] = {};  // OR of the receipts (only the words a kernel touches stay)
};

// The next round's source side, booked where a peer is activated (RoundArgs.st_pre): per wave, one
// atomic per nonzero field into a line of st_pre.  Every lane of the wave must call it.
struct PreAcc {
    unsigned long long frontier = 0, trav = 0, deliv = 0, digest = 0, covered = 0;
};

__device__ __forceinline__ void flush_pre(const PreAcc& p, DevStats* st) {
    if (!st) return;
    const unsigned long long v[5] = {wave_sum(p.frontier), wave_sum(p.trav), wave_sum(p.deliv), wave_sum(p.digest),
                                     wave_sum(p.covered)};
    if ((threadIdx.x & 63) != 0) return;
    DevStats* l = st + (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % kStatLines;
    unsigned long long* f[5] = {&l->frontier, &l->traversals, &l->deliveries, &l->digest, &l->covered};
#pragma unroll
    for (int i = 0; i < 5; ++i)
        if (v[i]) atomicAdd(f[i], v[i]);
}

// Appends v (lanes with app) to a.lst_out: one counter atomic per wave.  Every lane of the wave must call it.
__device__ __forceinline__ void list_push(const RoundArgs& a, bool app, uint32_t v) {
    const unsigned long long b = __ballot(app);
    if (!b) return;
    const int lead = __builtin_ctzll(b);
    uint32_t base = 0;
    if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(a.lst_n, (uint32_t)__popcll(b));
    base = (uint32_t)__shfl((int)base, lead);
    if (app) {
        const uint32_t i = base + lane_rank(b);
        if (i < a.lst_cap) a.lst_out[i] = v;  // past the cap: counted only (overflow)
    }
}

// Appends a wave's n <= 64 staged rows (LDS, s[0..n)) to a.lst_out with one counter atomic.
__device__ __forceinline__ void list_flush(const RoundArgs& a, const uint32_t* s, uint32_t n) {
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(a.lst_n, n);
    base = (uint32_t)__shfl((int)base, 0);
    if ((uint32_t)lane < n && base + lane < a.lst_cap) a.lst_out[base + lane] = s[lane];
}

// Block-level flush: wave sums -> LDS -> one atomic per nonzero field per
// block, into stat line blockIdx % kStatLines of the round.  Same-line device
// atomics serialise (~9 ns each measured); one line per round hit by every
// wave cost ~0.65 ms per pull round at 2^20 peers.  Must be reached by every
// wave of the block (it holds a barrier).
// flush_into: the same with caller-provided LDS scratch (kWaves * kStatFields words).
template <int kWaves>
__device__ __forceinline__ void flush_into(Acc& acc, DevStats* st, unsigned long long (*red)[kStatFields]);

template <int kWaves = kWavesPerBlock>
__device__ __forceinline__ void flush(Acc& acc, DevStats* st) {
    __shared__ unsigned long long red[kWaves][kStatFields];
    flush_into<kWaves>(acc, st, red);
}

template <int kWaves>
__device__ __forceinline__ void flush_into(Acc& acc, DevStats* st, unsigned long long (*red)[kStatFields]) {
    constexpr int kF = kStatFields;
    static_assert(sizeof(DevStats) == kF * 8, "one u64 per stat field");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // DevStats field order
    const unsigned long long v[kF] = {acc.frontier, acc.trav,     acc.deliv,   acc.undeliv, acc.fresh,  acc.injected,
                                      acc.died,     acc.reports,  acc.removals, acc.digest, acc.covered, acc.htrav,
                                      acc.checked,  acc.activated, acc.pulled,  acc.gathered, acc.reconnects,
                                      acc.rejoined, acc.atomics, acc.diag, acc.dead_cov,
                                      acc.fresh_or[0], acc.fresh_or[1], acc.fresh_or[2], acc.fresh_or[3],
                                      acc.fresh_or[4], acc.fresh_or[5], acc.fresh_or[6], acc.fresh_or[7]};
#pragma unroll
    for (int f = 0; f < kF; ++f) {
        unsigned long long s_ = v[f];
        if (f < kStatSums) {
            s_ = wave_sum(s_);
        } else {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) s_ |= __shfl_xor(s_, off);
        }
        if (lane == 0) red[wave][f] = s_;
    }
    __syncthreads();
    if (threadIdx.x < kF) {
        unsigned long long s_ = 0;
        const bool sum = threadIdx.x < kStatSums;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s_ = sum ? s_ + red[w][threadIdx.x] : s_ | red[w][threadIdx.x];
        unsigned long long* f = reinterpret_cast<unsigned long long*>(st + blockIdx.x % kStatLines) + threadIdx.x;
        if (s_) {
            if (sum) atomicAdd(f, s_);
            else atomicOr(f, s_);
        }
    }
}

// Source lane of edge position p within a tile: the number of rows whose
// inclusive end is <= p (incl = in-wave inclusive scan of row lengths).
__device__ __forceinline__ int src_lane(uint32_t incl, uint32_t p) {
    int s = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
        const uint32_t val = __shfl(incl, s + step - 1);
        if (val <= p) s += step;
    }
    return s;
}

inline unsigned grid_for(uint64_t items, uint64_t per_block) {
    uint64_t g = (items + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > kMaxGrid) g = kMaxGrid;
    return (unsigned)g;
}

}  // namespace
}  // namespace gossip
