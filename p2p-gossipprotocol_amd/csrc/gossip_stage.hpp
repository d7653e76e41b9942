// gossip_stage.hpp -- workgroup-level record staging in LDS (propagation-blocked
// push rounds, gossip_blocked.hip; tested on the GPU by tests/gpu_support/stage_selftest.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>

namespace gossip {

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Stages up to kU records per lane -- bin k[j], destination d[j], word w[j], for the j with pend[j] --
// into the workgroup's LDS buffers: per bin kH parts ("halves") of kB records each (bd / bw hold bin b's
// part h at [(b kH + h) kB, (b kH + h + 1) kB)).  Every record takes a ticket t from tick[bin] (an LDS
// atomic that never fails): generation g = t / kB, part g % kH, slot t % kB.  A record is written once
// its part is open for generation g (gen[bin kH + g % kH] == g: generation g - kH has gone out); the
// write that completes generation g (wr[bin kH + part] reaching kB) makes its wave flush it: flush(bin, g)
// reads the kB records, releases the part for generation g + kH (stage_release) and writes them at
// place g * kB of the bin's own output segment, so flushes need no global atomics.  Lanes whose part is
// still busy wait (they hold their tickets: nothing is retried, no counter runs past the records).
// Wave-uniform.
// Round 3 had one part per bin: a ticket of generation g + 1 waited until every record of g was written
// and flushed, and a k_pb_split wave spent 51 of 102 us in here (gpurun_out/pbdbg.out).  Two parts of
// half the size in the same LDS cost more than they saved (config 4 round 4: level 1 5.4 -> 6.2 ms,
// level 2 3.9 -> 4.1: twice the flushes, each half as wide); level 2 has the LDS for two whole-size parts.
// (A first version reserved places with an atomic that failed past kB and retried: under contention the
// failed increments wrapped the 32-bit counter and handed out a place twice.)  Bounded: after kStageSpin
// passes it drops what is left and flags err (bit 4, GOSSIP_ESTALL at the host), so a wave never spins
// forever (the protocol always progresses: the lowest unflushed generation's part is open, and every one
// of its tickets can be written).
constexpr uint32_t kStageSpin = 1u << 24;

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDS state of nb bins: tick[nb], wr[kH nb], gen[kH nb]
template <uint32_t kH>
__device__ __forceinline__ void stage_init(uint32_t* tick, uint32_t* wr, uint32_t* gen, uint32_t nb, uint32_t tid,
                                           uint32_t nthreads) {
    for (uint32_t i = tid; i < kH * nb; i += nthreads) {
        if (i < nb) tick[i] = 0;
        wr[i] = 0;
        gen[i] = i % kH;  // part h first takes generation h
    }
}

// buffer slot of generation g's record s (of kB) in bin's parts
template <uint32_t kB, uint32_t kH>
__device__ __forceinline__ uint32_t stage_at(uint32_t bin, uint32_t g, uint32_t s) {
    return (bin * kH + g % kH) * kB + s;
}

// end of a flush of generation g (one lane, after the records were read): the part takes generation g + kH
template <uint32_t kH>
__device__ __forceinline__ void stage_release(uint32_t* wr, uint32_t* gen, uint32_t bin, uint32_t g) {
    const uint32_t h = bin * kH + g % kH;
    lds_store(&wr[h], 0u);
    lds_fence();
    lds_store(&gen[h], g + kH);
}

template <int kU, uint32_t kB, uint32_t kH, class TD, class FlushF>
__device__ __forceinline__ void stage(uint32_t* tick, uint32_t* wr, uint32_t* gen, TD* bd, unsigned long long* bw,
                                      const uint32_t (&k)[kU], const uint32_t (&d)[kU],
                                      const unsigned long long (&w)[kU], bool (&pend)[kU], FlushF&& flush,
                                      uint32_t* err) {
    // the records' values are in registers before any ticket is taken: a wave holding tickets must never
    // wait on memory, or every later ticket of its bins waits with it (measured: waves took their tickets,
    // then waited on their loads and on the previous flushes' stores -- vmcnt counts both -- and convoys
    // of waiting waves made a 16-wave workgroup move about one generation per global round trip)
#pragma unroll
    for (int j = 0; j < kU; ++j) asm volatile("" ::"v"(d[j]), "v"(w[j]));  // (waits for exactly these loads)
    uint32_t t[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) t[j] = pend[j] ? atomicAdd(&tick[k[j]], 1u) : 0u;
    for (uint32_t pass = 0;; ++pass) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < kU; ++j) any |= pend[j];
        if (!__ballot(any)) return;
        if (pass == kStageSpin) {
            if ((threadIdx.x & 63) == 0) {
                atomicOr(err, 4u);
                printf("gossip stage: wave %u of block %u stuck\n", threadIdx.x >> 6, blockIdx.x);
            }
            return;
        }
        bool go[kU];
#pragma unroll
        for (int j = 0; j < kU; ++j)
            go[j] = pend[j] && lds_load(&gen[k[j] * kH + (t[j] / kB) % kH]) == t[j] / kB;
#pragma unroll
        for (int j = 0; j < kU; ++j)
            if (go[j]) {
                const uint32_t s = stage_at<kB, kH>(k[j], t[j] / kB, t[j] % kB);
                bd[s] = (TD)d[j];
                bw[s] = w[j];
            }
        lds_fence();  // the records are in LDS before they are counted
        uint32_t full = 0;
        bool left = false;
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            if (go[j]) {
                pend[j] = false;
                if (atomicAdd(&wr[k[j] * kH + (t[j] / kB) % kH], 1u) == kB - 1) full |= 1u << j;
            }
            left |= pend[j];
        }
#pragma unroll
        for (int j = 0; j < kU; ++j)
            for (unsigned long long m = __ballot((full >> j) & 1u); m; m &= m - 1) {
                const int src = __builtin_ctzll(m);
                flush((uint32_t)__shfl((int)k[j], src), (uint32_t)__shfl((int)(t[j] / kB), src));
            }
        if (__ballot(left)) __builtin_amdgcn_s_sleep(1);  // another wave is completing that generation
    }
}

// After the workgroup's last stage (behind a barrier): bin's open generation *g and its record count
// (slots [0, n) of its part; the caller pads the rest of the part and flushes it).  Every earlier
// generation is full and has gone out.
__device__ __forceinline__ uint32_t stage_open(const uint32_t* tick, uint32_t bin, uint32_t kB, uint32_t* g) {
    const uint32_t t = lds_load(&tick[bin]);
    *g = t / kB;
    return t % kB;
}

// records a bin's segment received (whole generations, the last one padded)
__device__ __forceinline__ uint32_t stage_len(const uint32_t* tick, uint32_t bin, uint32_t kB) {
    return (lds_load(&tick[bin]) + kB - 1) / kB * kB;
}

}  // namespace gossip
