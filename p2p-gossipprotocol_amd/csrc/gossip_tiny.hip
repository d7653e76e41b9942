// gossip_tiny.hip -- a whole run of a small overlay in ONE launch.
//
// On small overlays (BASELINE config 1: the reference's 8 peers on loopback,
// 47 rounds) a round is a few hundred edge deliveries, and the launch-per-phase
// engine paid ~27 us per round in launches and the stats read-back that decides
// termination.  Here one workgroup runs round after round of the round contract
// (DESIGN.md section 2), phases separated by workgroup barriers, and decides
// termination itself; the host reads every round's stats once at the end:
//   1. kills, then churn (philox({seed,v},{4,r,0,0}).x < threshold): a dead
//      peer stops receiving, forwarding and pinging; its pending new words go
//      (the reference's Ctrl+C, README.md:6);
//   2. liveness on ping rounds (pingLoop peer.cpp:320-355): every unmasked
//      out-edge of a live peer is pinged; a live target resets the miss
//      counter, a dead one increments it, and at max_missed the edge is
//      dropped (connectedPeers.erase, peer.cpp:388), a report (r, u, v) is
//      emitted and the seed registry drops v on its first report
//      (SeedNode::handleDeadNode, seed.cpp:158-167);
//   3. injection (messageGenerationLoop, peer.cpp:357-379);
//   4. push-start statistics (frontier, digest and covered of seen);
//   5. push (broadcastMessage, peer.cpp:310-316 -> handleClient's dedup,
//      peer.cpp:277-285) as a 64-bit test-and-set per delivered word;
//   6. advance: new <- next; finished after a round with no new receipts and
//      no pending injection, once min_rounds have run, or at max_rounds.
// Only overlays whose whole run fits one workgroup's pass per phase take this
// path (gossip_engine.hip: tiny_ok), and only the features listed above:
// re-bootstrap, join churn and coverage history use the round-by-round engine.
#include <hip/hip_runtime.h>

#include "gossip_internal.hpp"
#include "philox.hpp"

namespace gossip {

namespace {

__device__ __forceinline__ bool tbit(const uint32_t* bits, uint32_t v) { return (bits[v >> 5] >> (v & 31)) & 1u; }

// one round's sums, in gossip_round_stats order from frontier on
enum { kTFrontier, kTTrav, kTDeliv, kTUndeliv, kTFresh, kTInjected, kTDied, kTReports, kTRemovals, kTDigest,
       kTCovered, kTFields };

template <int kB>
__device__ __forceinline__ void tiny_reduce(unsigned long long (&v)[kTFields], unsigned long long (*red)[kTFields],
                                            unsigned long long* tot) {
    constexpr int kWaves = kB / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if constexpr (kB == 64) {
        // one wave: the lanes' values through LDS (field-major rows padded by two words, so the summing
        // lanes' 16-B reads fall in different banks), then lane f sums row f with four accumulators, its
        // loads in flight together.  Shuffle trees waited for every permute of every field (66 round trips,
        // ~3 us of a 4 us round); LDS atomics into one word per field serialised the lanes (0.17 ms a run).
        constexpr int kRow = 66;
        __shared__ unsigned long long tr[kTFields * kRow];
#pragma unroll
        for (int f = 0; f < kTFields; ++f) {
            tr[f * kRow + lane] = v[f];
            v[f] = 0;
        }
        __syncthreads();
        if (lane < kTFields) {
            const unsigned long long* row = tr + lane * kRow;
            unsigned long long a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
            for (int i = 0; i < 64; i += 4) {
                a0 += row[i];
                a1 += row[i + 1];
                a2 += row[i + 2];
                a3 += row[i + 3];
            }
            tot[lane] = (a0 + a1) + (a2 + a3);
        }
        __syncthreads();
        return;
    }
#pragma unroll
    for (int f = 0; f < kTFields; ++f) {
        unsigned long long s = v[f];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
        if (lane == 0) red[wave][f] = s;
        v[f] = 0;
    }
    __syncthreads();
    if (threadIdx.x < kTFields) {
        unsigned long long s = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += red[w][threadIdx.x];
        tot[threadIdx.x] = s;
    }
    __syncthreads();
}

// overlays this small keep their whole state in LDS for the run (copied in and out).  The body reads
// and writes it through pointers the compiler can see are LDS pointers (picked by the template flag,
// never merged with global ones), so it emits ds_* instructions: through generic pointers every access
// was a flat instruction that waits for all outstanding memory operations (~4 us per round).
constexpr uint32_t kLdsWords = 4096;  // n * Wp words (seen, new, next each)
constexpr uint32_t kLdsEdges = 4096;
constexpr uint32_t kLdsPeers = 4096;
constexpr uint32_t kLdsSched = 512;   // injections (<= 512 messages) and kills (+ a sentinel) held in LDS
constexpr uint32_t kStatRing = 64;    // rounds of stats buffered in LDS between writes to the host

template <int W, int kB, bool kLds>
__global__ __launch_bounds__(kB) void k_tiny_run(TinyArgs t) {
    __shared__ unsigned long long red[kB / 64][kTFields];
    __shared__ unsigned long long tot[kTFields];
    __shared__ uint32_t done;
    __shared__ gossip_round_stats ring[kStatRing];
    __shared__ uint64_t l_seen[kLds ? kLdsWords : 1], l_nw[kLds ? kLdsWords : 1], l_nx[kLds ? kLdsWords : 1];
    __shared__ uint32_t l_col[kLds ? kLdsEdges : 1], l_erow[kLds ? kLdsEdges : 1];
    __shared__ uint32_t l_alive[kLds ? kLdsPeers / 32 : 1], l_reg[kLds ? kLdsPeers / 32 : 1];
    __shared__ uint8_t l_miss[kLds ? kLdsEdges : 1];
    __shared__ uint32_t l_io[kLds ? kLdsSched : 1], l_im[kLds ? kLdsSched : 1], l_ir[kLds ? kLdsSched : 1];
    __shared__ uint32_t l_kp[kLds ? kLdsSched : 1], l_kr[kLds ? kLdsSched : 1];
    if (kLds) {
        for (uint32_t i = threadIdx.x; i < t.n * W; i += kB) {
            l_seen[i] = t.seen[i];
            l_nw[i] = t.nw[i];
            l_nx[i] = t.nx[i];
        }
        for (uint32_t e = threadIdx.x; e < t.n_edges; e += kB) {
            l_col[e] = t.col[e];
            l_erow[e] = t.erow[e];
            l_miss[e] = t.miss ? t.miss[e] : 0;
        }
        for (uint32_t i = threadIdx.x; i < (t.n + 31) / 32; i += kB) {
            l_alive[i] = t.alive[i];
            l_reg[i] = t.registered[i];
        }
        for (uint32_t i = threadIdx.x; i < t.n_inj; i += kB) {
            l_io[i] = t.inj_origin[i];
            l_im[i] = t.inj_msg[i];
            l_ir[i] = t.inj_round[i];
        }
        for (uint32_t i = threadIdx.x; i <= t.n_kill; i += kB) {  // (kill_round holds a sentinel past the end)
            l_kp[i] = i < t.n_kill ? t.kill_peer[i] : 0u;
            l_kr[i] = t.kill_round[i];
        }
        __syncthreads();
    }
    // the state: LDS or global, fixed at compile time
    uint64_t* const seen = kLds ? l_seen : t.seen;
    uint64_t* nw = kLds ? l_nw : t.nw;
    uint64_t* nx = kLds ? l_nx : t.nx;
    uint32_t* const col = kLds ? l_col : t.col;
    const uint32_t* const erow = kLds ? l_erow : t.erow;
    uint32_t* const alive = kLds ? l_alive : t.alive;
    uint32_t* const reg = kLds ? l_reg : t.registered;
    uint8_t* const miss = kLds ? l_miss : t.miss;
    const uint32_t* const inj_origin = kLds ? l_io : t.inj_origin;
    const uint32_t* const inj_msg = kLds ? l_im : t.inj_msg;
    const uint32_t* const inj_round = kLds ? l_ir : t.inj_round;
    const uint32_t* const kill_peer = kLds ? l_kp : t.kill_peer;
    const uint32_t* const kill_round = kLds ? l_kr : t.kill_round;
    unsigned long long v[kTFields] = {};
    uint32_t kp = 0, ip = 0;  // kill / injection cursors (sorted by round)
    while (kp < t.n_kill && kill_round[kp] < t.start) ++kp;
    while (ip < t.n_inj && inj_round[ip] < t.start) ++ip;
    uint32_t r = t.start;
    for (;; ++r) {
        // 1. kills, then churn
        uint32_t k1 = kp;
        while (k1 < t.n_kill && kill_round[k1] == r) ++k1;
        for (uint32_t i = kp + threadIdx.x; i < k1; i += kB) {
            const uint32_t p = kill_peer[i], bit = 1u << (p & 31);
            if (atomicAnd(&alive[p >> 5], ~bit) & bit) {
                v[kTDied]++;
#pragma unroll
                for (int w = 0; w < W; ++w) nw[(uint64_t)p * W + w] = 0ull;
            }
        }
        kp = k1;
        if (t.churn) {
            __syncthreads();
            for (uint32_t p = threadIdx.x; p < t.n; p += kB) {
                if (!tbit(alive, p)) continue;
                if (lane_of(philox4x32_10(P_CHURN, r, 0, 0, t.seed, p >> 2), p & 3) >= t.churn) continue;
                atomicAnd(&alive[p >> 5], ~(1u << (p & 31)));
                v[kTDied]++;
#pragma unroll
                for (int w = 0; w < W; ++w) nw[(uint64_t)p * W + w] = 0ull;
            }
        }
        __syncthreads();
        // 2. liveness
        const bool ping = t.ping_every && r % t.ping_every == 0;
        if (ping) {
            for (uint32_t e = threadIdx.x; e < t.n_edges; e += kB) {
                const uint32_t u = erow[e];
                if (!tbit(alive, u)) continue;
                const uint32_t c = col[e];
                if (c & kMaskedEdge) continue;
                if (tbit(alive, c)) {
                    miss[e] = 0;
                    continue;
                }
                const uint32_t m = miss[e] + (miss[e] < 255u ? 1u : 0u);
                miss[e] = (uint8_t)m;
                if (m < t.max_missed) continue;
                col[e] = c | kMaskedEdge;
                v[kTReports]++;
                const unsigned long long i = atomicAdd(t.n_reports, 1ull);
                if (i < t.report_cap) t.reports[i] = DeadReport{r, u, c};
                const uint32_t bit = 1u << (c & 31);
                if (atomicAnd(&reg[c >> 5], ~bit) & bit) v[kTRemovals]++;
            }
            __syncthreads();
        }
        // 3. injection
        uint32_t i1 = ip;
        while (i1 < t.n_inj && inj_round[i1] == r) ++i1;
        for (uint32_t i = ip + threadIdx.x; i < i1; i += kB) {
            const uint32_t o = inj_origin[i], m = inj_msg[i];
            if (!tbit(alive, o)) continue;
            const unsigned long long b = 1ull << (m & 63);
            atomicOr(reinterpret_cast<unsigned long long*>(seen) + (uint64_t)o * W + (m >> 6), b);
            atomicOr(reinterpret_cast<unsigned long long*>(nw) + (uint64_t)o * W + (m >> 6), b);
            atomicOr(reinterpret_cast<unsigned long long*>(t.inj_live) + (m >> 6), b);
            v[kTInjected]++;
        }
        ip = i1;
        __syncthreads();
        // 4. push-start statistics
        for (uint32_t p = threadIdx.x; p < t.n; p += kB) {
            bool act = false;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint64_t x = seen[(uint64_t)p * W + w];
                act |= nw[(uint64_t)p * W + w] != 0;
                if (w < (int)t.wd) {
                    v[kTCovered] += (unsigned long long)__popcll(x);
                    v[kTDigest] += digest_weight((uint64_t)p * t.wd + w) * x;
                }
            }
            v[kTFrontier] += act;
        }
        __syncthreads();
        // 5. push
        for (uint32_t e = threadIdx.x; e < t.n_edges; e += kB) {
            const uint32_t u = erow[e];
            uint64_t m[W];
            uint32_t pc = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                m[w] = nw[(uint64_t)u * W + w];
                pc += (uint32_t)__popcll(m[w]);
            }
            if (!pc) continue;
            const uint32_t c = col[e];
            if (c & kMaskedEdge) continue;
            v[kTTrav]++;
            if (!tbit(alive, c)) {
                v[kTUndeliv] += pc;
                continue;
            }
            v[kTDeliv] += pc;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                if (!m[w]) continue;
                const unsigned long long old =
                    atomicOr(reinterpret_cast<unsigned long long*>(seen) + (uint64_t)c * W + w, (unsigned long long)m[w]);
                const unsigned long long fr = m[w] & ~old;
                if (!fr) continue;
                atomicOr(reinterpret_cast<unsigned long long*>(nx) + (uint64_t)c * W + w, fr);
                v[kTFresh] += (unsigned long long)__popcll(fr);
            }
        }
        __syncthreads();
        // 6. advance: the consumed words go, next becomes new
        for (uint32_t i = threadIdx.x; i < t.n * W; i += kB) nw[i] = 0ull;
        uint64_t* tmp = nw;
        nw = nx;
        nx = tmp;
        tiny_reduce<kB>(v, red, tot);
        if (threadIdx.x == 0) {
            gossip_round_stats s{};
            s.round = r;
            s.flags = ping ? 1u : 0u;
            s.frontier = tot[kTFrontier];
            s.traversals = tot[kTTrav];
            s.deliveries = tot[kTDeliv];
            s.undelivered = tot[kTUndeliv];
            s.new_receipts = tot[kTFresh];
            s.duplicates = tot[kTDeliv] - tot[kTFresh];
            s.injected = tot[kTInjected];
            s.died = tot[kTDied];
            s.reports = tot[kTReports];
            s.seed_removals = tot[kTRemovals];
            s.digest = tot[kTDigest];
            s.covered = tot[kTCovered];
            ring[(r - t.start) % kStatRing] = s;
            const bool pending = t.has_schedule && t.last_inject_round > r;
            done = (tot[kTFresh] == 0 && !pending && r + 1 >= t.min_rounds) || r + 1 >= t.max_rounds ||
                   r + 1 - t.start >= t.out_cap;
        }
        __syncthreads();
        const uint32_t k = r + 1 - t.start;
        if (done || k % kStatRing == 0) {  // the buffered rounds to the host (a store to host memory
            const uint32_t b0 = (k - 1) / kStatRing * kStatRing;  // before a barrier waits for its PCIe trip)
            for (uint32_t i = b0 + threadIdx.x; i < k; i += kB) t.out[i] = ring[i % kStatRing];
            __syncthreads();
        }
        if (done) break;
    }
    if (kLds) {  // the state back to the ctx's buffers (the new words into its nw buffer: nothing swaps)
        for (uint32_t i = threadIdx.x; i < t.n * W; i += kB) {
            t.seen[i] = seen[i];
            t.nw[i] = nw[i];
            t.nx[i] = nx[i];
        }
        for (uint32_t e = threadIdx.x; e < t.n_edges; e += kB) {
            t.col[e] = col[e];
            if (t.miss) t.miss[e] = miss[e];
        }
        for (uint32_t i = threadIdx.x; i < (t.n + 31) / 32; i += kB) {
            t.alive[i] = alive[i];
            t.registered[i] = reg[i];
        }
    }
    if (threadIdx.x == 0) {
        t.result[0] = r + 1 - t.start;                     // rounds run
        t.result[1] = kLds || nw == t.nw ? 0u : 1u;        // the new words now live in the ctx's nx buffer
    }
}

// everything gossip_reset clears, in one launch (the host part of the reset stays in gossip_reset)
__global__ __launch_bounds__(1024) void k_tiny_reset(TinyArgs t, uint64_t words, uint32_t bitwords, uint32_t n_started,
                                                     uint32_t unmask, uint64_t tact_words, uint64_t* tact0,
                                                     uint64_t* tact1, DevStats* st) {
    for (uint64_t i = threadIdx.x; i < words; i += 1024) {
        t.seen[i] = 0ull;
        t.nw[i] = 0ull;
        t.nx[i] = 0ull;
    }
    for (uint32_t i = threadIdx.x; i < bitwords; i += 1024) {
        const uint32_t lo = i * 32;
        const uint32_t all = lo + 32 <= t.n ? ~0u : (1u << (t.n - lo)) - 1u;
        const uint32_t started = lo >= n_started ? 0u : lo + 32 <= n_started ? ~0u : (1u << (n_started - lo)) - 1u;
        t.registered[i] = all;
        t.alive[i] = all & started;
    }
    for (uint32_t e = threadIdx.x; e < t.n_edges; e += 1024) {
        if (t.miss) t.miss[e] = 0;
        if (unmask) t.col[e] &= ~kMaskedEdge;
    }
    for (uint64_t i = threadIdx.x; i < tact_words; i += 1024) {
        tact0[i] = 0ull;
        tact1[i] = 0ull;
    }
    unsigned long long* s = reinterpret_cast<unsigned long long*>(st);
    for (uint32_t i = threadIdx.x; i < kStatLines * kStatFields; i += 1024) s[i] = 0ull;
    if (threadIdx.x < kMaxWords) t.inj_live[threadIdx.x] = 0ull;
    if (threadIdx.x == 0) *t.n_reports = 0ull;
}

__global__ void k_tiny_erow(const uint64_t* rp, uint32_t n, uint32_t* erow) {
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < n; u += gridDim.x * blockDim.x)
        for (uint64_t e = rp[u]; e < rp[u + 1]; ++e) erow[e] = u;
}

}  // namespace

hipError_t launch_tiny_erow(const uint64_t* rp, uint32_t n, uint32_t* erow, hipStream_t s) {
    hipLaunchKernelGGL(k_tiny_erow, dim3((n + 255) / 256), dim3(256), 0, s, rp, n, erow);
    return hipGetLastError();
}

hipError_t launch_tiny_reset(const TinyArgs& t, uint64_t words, uint32_t n_started, bool unmask, uint64_t tact_words,
                             uint64_t* tact0, uint64_t* tact1, DevStats* st, hipStream_t s) {
    hipLaunchKernelGGL(k_tiny_reset, dim3(1), dim3(1024), 0, s, t, words, (t.n + 31) / 32, n_started,
                       unmask ? 1u : 0u, tact_words, tact0, tact1, st);
    return hipGetLastError();
}

hipError_t launch_tiny_run(const TinyArgs& t, uint32_t Wp, hipStream_t s) {
    // state in LDS when it fits (one wave while the phases are short: its barriers are free), else in
    // global memory with one 16-wave workgroup
    const bool lds = t.n_edges <= kLdsEdges && t.n <= kLdsPeers && (uint64_t)t.n * Wp <= kLdsWords &&
                     t.n_inj <= kLdsSched && t.n_kill < kLdsSched;
    const bool wide = t.n_edges > 1024 || t.n > 1024;
#define GOSSIP_TINY(WW)                                                                                  \
    do {                                                                                                 \
        if (lds && wide) hipLaunchKernelGGL((k_tiny_run<WW, 1024, true>), dim3(1), dim3(1024), 0, s, t); \
        else if (lds) hipLaunchKernelGGL((k_tiny_run<WW, 64, true>), dim3(1), dim3(64), 0, s, t);        \
        else hipLaunchKernelGGL((k_tiny_run<WW, 1024, false>), dim3(1), dim3(1024), 0, s, t);            \
    } while (0)
    switch (Wp) {
        case 1: GOSSIP_TINY(1); break;
        case 2: GOSSIP_TINY(2); break;
        case 4: GOSSIP_TINY(4); break;
        default: GOSSIP_TINY(8); break;
    }
#undef GOSSIP_TINY
    return hipGetLastError();
}

}  // namespace gossip
