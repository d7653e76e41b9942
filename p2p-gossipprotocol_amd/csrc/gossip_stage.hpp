// gossip_stage.hpp -- workgroup-level record staging in LDS (propagation-blocked
// push rounds, gossip_blocked.hip; unit-tested by tools/stage_test.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>

namespace gossip {

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Stages up to kU records per lane -- bin k[j], destination d[j], word w[j], for the j with pend[j] --
// into the workgroup's LDS buffers of kB records per bin (one buffer per bin).  Every record takes a
// ticket t from tick[bin] (an LDS atomic that never fails): generation t / kB, slot t % kB.  A record
// is written once its generation is the bin's current one (done[bin]); the write that completes a
// generation (wr[bin] reaching kB) makes its wave flush the bin: flush(bin) reads the kB records,
// releases the buffer (stage_release: wr reset, done advanced) and writes them out -- generation g of
// a bin at place g * kB of the bin's own output segment, so flushes need no global atomics (measured,
// tools/stage_test: 57 bins, 2 workgroups per CU, 90 G records/s without the global part against 13-18
// with a global atomic per flush on the critical path).  Lanes whose generation is not current yet wait
// (they hold their tickets: nothing is retried, no counter runs past the records).  Wave-uniform.
// (A first version reserved places with an atomic that failed past kB and retried: under contention
// the failed increments wrapped the 32-bit counter and handed out a place twice -- tools/stage_test.)
// Bounded: after kStageSpin passes it drops what is left and flags err (bit 4), so a wave never spins
// forever (the protocol always progresses: the lowest open generation's tickets can all be written).
constexpr uint32_t kStageSpin = 1u << 24;

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// end of a flush (one lane): the generation's slots may be reused
__device__ __forceinline__ void stage_release(uint32_t* wr, uint32_t* done, uint32_t bin) {
    lds_store(&wr[bin], 0u);
    lds_fence();
    lds_store(&done[bin], lds_load(&done[bin]) + 1u);
}

template <int kU, uint32_t kB, class TD, class FlushF>
__device__ __forceinline__ void stage(uint32_t* tick, uint32_t* wr, uint32_t* done, TD* bd, unsigned long long* bw,
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
        for (int j = 0; j < kU; ++j) go[j] = pend[j] && t[j] / kB == lds_load(&done[k[j]]);
#pragma unroll
        for (int j = 0; j < kU; ++j)
            if (go[j]) {
                bd[k[j] * kB + t[j] % kB] = (TD)d[j];
                bw[k[j] * kB + t[j] % kB] = w[j];
            }
        lds_fence();  // the records are in LDS before they are counted
        uint32_t full = 0;
        bool left = false;
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            if (go[j]) {
                pend[j] = false;
                if (atomicAdd(&wr[k[j]], 1u) == kB - 1) full |= 1u << j;
            }
            left |= pend[j];
        }
#pragma unroll
        for (int j = 0; j < kU; ++j)
            for (unsigned long long m = __ballot((full >> j) & 1u); m; m &= m - 1)
                flush((uint32_t)__shfl((int)k[j], __builtin_ctzll(m)));
        if (__ballot(left)) __builtin_amdgcn_s_sleep(1);  // another wave is completing that generation
    }
}

// After the workgroup's last stage (behind a barrier): the records of bin's open generation, if any
// (slots [0, n)); the caller pads the rest of the buffer and flushes it.
__device__ __forceinline__ uint32_t stage_open(const uint32_t* tick, uint32_t bin, uint32_t kB) {
    return lds_load(&tick[bin]) % kB;
}

}  // namespace gossip
