// gossip_stage.hpp -- workgroup-level record staging in LDS (propagation-blocked
// push rounds, gossip_blocked.hip; tested on the GPU by tests/gpu_support/stage_selftest.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>

namespace gossip {

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Stages up to kU records per lane -- bin k[j], destination d[j], word w[j], for the j with pend[j] --
// into the workgroup's LDS buffers: per bin two halves of kB records each (bd / bw hold bin b's halves
// at [b * 2kB, b * 2kB + kB) and [b * 2kB + kB, (b + 1) * 2kB)).  Every record takes a ticket t from
// tick[bin] (an LDS atomic that never fails): generation g = t / kB, half g & 1, slot t % kB.  A record
// is written once half (g & 1) is open for generation g (gen[2 bin + h] == g: generation g - 2 has
// gone out); the write that completes generation g (wr[2 bin + h] reaching kB) makes its wave flush it:
// flush(bin, g) reads the kB records, releases the half for generation g + 2 (stage_release) and writes
// them at place g * kB of the bin's own output segment, so flushes need no global atomics.  Lanes whose
// half is still busy wait (they hold their tickets: nothing is retried, no counter runs past the records).
// Wave-uniform.
// Round 3 had one buffer per bin: a ticket of generation g + 1 waited until every record of g was written
// and flushed, and a k_pb_split wave spent 51 of 102 us in here (gpurun_out/pbdbg.out); with two halves a
// wave waits only when it is two generations ahead.  (A first version reserved places with an atomic that
// failed past kB and retried: under contention the failed increments wrapped the 32-bit counter and
// handed out a place twice.)  Bounded: after kStageSpin passes it drops what is left and flags err (bit 4,
// GOSSIP_ESTALL at the host), so a wave never spins forever (the protocol always progresses: the lowest
// unflushed generation's half is open, and every one of its tickets can be written).
constexpr uint32_t kStageSpin = 1u << 24;

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDS state of nb bins: tick[nb], wr[2 nb], gen[2 nb]
__device__ __forceinline__ void stage_init(uint32_t* tick, uint32_t* wr, uint32_t* gen, uint32_t nb, uint32_t tid,
                                           uint32_t nthreads) {
    for (uint32_t i = tid; i < 2 * nb; i += nthreads) {
        if (i < nb) tick[i] = 0;
        wr[i] = 0;
        gen[i] = i & 1;  // half h first takes generation h
    }
}

// end of a flush of generation g (one lane, after the records were read): the half takes generation g + 2
__device__ __forceinline__ void stage_release(uint32_t* wr, uint32_t* gen, uint32_t bin, uint32_t g) {
    const uint32_t h = 2 * bin + (g & 1);
    lds_store(&wr[h], 0u);
    lds_fence();
    lds_store(&gen[h], g + 2u);
}

// slot of ticket t in bin's buffers
template <uint32_t kB>
__device__ __forceinline__ uint32_t stage_slot(uint32_t bin, uint32_t t) {
    return bin * 2 * kB + ((t / kB) & 1) * kB + t % kB;
}

template <int kU, uint32_t kB, class TD, class FlushF>
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
            go[j] = pend[j] && lds_load(&gen[2 * k[j] + ((t[j] / kB) & 1)]) == t[j] / kB;
#pragma unroll
        for (int j = 0; j < kU; ++j)
            if (go[j]) {
                const uint32_t s = stage_slot<kB>(k[j], t[j]);
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
                if (atomicAdd(&wr[2 * k[j] + ((t[j] / kB) & 1)], 1u) == kB - 1) full |= 1u << j;
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
// (slots [0, n) of half *g & 1; the caller pads the rest of the half and flushes it).  Every earlier
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
