// gossip_kernels.hip -- round kernels of libgossip_hip for gfx950 (CDNA4).
//
// One round of the reference's recursion
//   broadcastMessage (peer.cpp:297-318) -> handleClient (peer.cpp:255-295)
// over ALL peers at once, plus liveness (peer.cpp:320-355, 381-405) and
// churn.  Everything is integer; results do not depend on atomic order.
//
// Layout: CSR rows of the owned peers (row_ptr u64,
// col u32 global ids, bit 31 = edge masked by liveness); seen/new/next as
// Wp u64 words per peer (bit m = message m); alive and registry as global
// bitsets.  Work mapping: one wave64 per tile of 64 consecutive peers with
// an in-wave prefix sum over row lengths ("edge-space expansion"), so the
// wave's lanes walk consecutive col entries of the tile -- one contiguous
// span when the tile's rows are all active; rows longer than the heavy
// threshold (RoundArgs.heavy) are cut into kHeavyChunk-edge chunks, one wave
// each, so no wave walks a long tail.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <type_traits>
#include <stdlib.h>

#include "gossip_device.hpp"
#include "gossip_internal.hpp"
#include "philox.hpp"

namespace gossip {

namespace {

// Edge-space expansion of one tile (64 rows, one wave).  deg = this lane's
// row length (0 = skip), rb = its row begin.  f(src_lane, valid, e) runs once
// per 64-edge batch in every lane (so it may shuffle); valid lanes own edge e.
template <class F>
__device__ __forceinline__ void tile_edges(uint32_t deg, uint64_t rb, F&& f) {
    const int lane = threadIdx.x & 63;
    uint32_t incl = deg;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    const uint32_t excl = incl - deg;
    const uint32_t total = __shfl(incl, 63);
    for (uint32_t base = 0; base < total; base += 64) {
        const uint32_t p = base + lane;
        int s = 0;  // number of rows whose inclusive end <= p  == source lane
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const uint32_t val = __shfl(incl, s + step - 1);
            if (val <= p) s += step;
        }
        const uint32_t ex = __shfl(excl, s);
        const uint64_t rbs = __shfl(rb, s);
        f(s, p < total, rbs + (uint64_t)(p - ex));
    }
}

// handleClient's dedup (peer.cpp:277-285) as a 64-bit test-and-set: deliver
// the source's new words m to local peer lv whose seen words were read as cur.
// The plain read first: seen only grows within a round, so a stale read can
// only cost an extra atomic, never a wrong answer.  It also keeps atomics off
// the hubs' words: without it (a blind test-and-set) config 4's round-3
// push_light took 19.5 ms instead of 3.0 for only 5 M more atomics -- the
// extra ones all land on a few hot words and serialise.
template <int W>
__device__ __forceinline__ void deliver_local(const RoundArgs& a, uint64_t lv, const uint64_t (&m)[W],
                                              const uint64_t (&cur)[W], Acc& acc) {
    unsigned long long* sp = reinterpret_cast<unsigned long long*>(a.seen) + lv * W;
    unsigned long long* np = reinterpret_cast<unsigned long long*>(a.nx) + lv * W;
    auto mark = [&] {  // the peer's tile joins the next round's frontier tiles
        const unsigned long long tb = 1ull << ((lv >> 6) & 63);
        unsigned long long* tw = reinterpret_cast<unsigned long long*>(a.tnx) + (lv >> 12);
        if (!(*tw & tb)) {  // read first: most tiles are already marked
            atomicOr(tw, tb);
            acc.atomics++;
        }
    };
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const unsigned long long u = m[w] & ~cur[w];
        if (!u) continue;  // all duplicates: dropped (peer.cpp:281)
        if (a.defer) {     // seen is the round-start set all round: one atomic, on nx
            const unsigned long long old = atomicOr(np + w, u);
            acc.atomics++;
            const unsigned long long fr = u & ~old;  // not yet received this round either
            acc.fresh_or[w] |= fr;
            if (fr) {
                acc.activated += old == 0;
                if (a.tnx && old == 0) mark();
                acc.fresh += (unsigned long long)__popcll(fr);
            }
            continue;
        }
        const unsigned long long old = atomicOr(sp + w, (unsigned long long)m[w]);
        acc.atomics++;
        const unsigned long long fr = m[w] & ~old;
        acc.fresh_or[w] |= fr;
        if (fr) {
            const unsigned long long onx = atomicOr(np + w, fr);
            acc.atomics++;
            acc.activated += onx == 0;
            if (a.tnx && onx == 0) mark();
            acc.fresh += (unsigned long long)__popcll(fr);
        }
    }
}

// A sparse push round's staging write to global peer c marks c's 64-peer tile (each staging word written in
// the round was written by an atomic that marked it: the compaction reads only marked tiles).
__device__ __forceinline__ void mark_send(const RoundArgs& a, uint32_t c) {
    if (!a.smark) return;
    unsigned long long* w = a.smark + (c >> 12);
    const unsigned long long bit = 1ull << ((c >> 6) & 63);
    if (!(*w & bit)) atomicOr(w, bit);
}

// Owned peer lv was activated (its next-round new words were zero): its 64-peer tile joins the next round's
// frontier tiles (a.tnx; read first: most tiles are already marked)
__device__ __forceinline__ void mark_tile(const RoundArgs& a, uint64_t lv, Acc& acc) {
    if (!a.tnx) return;
    const unsigned long long tb = 1ull << ((lv >> 6) & 63);
    unsigned long long* tw = reinterpret_cast<unsigned long long*>(a.tnx) + (lv >> 12);
    if (!(*tw & tb)) {
        atomicOr(tw, tb);
        acc.atomics++;
    }
}

// Appends {c, m} to destination block q's records (RoundArgs.rec_out) for every lane with want set: one
// counter atomic per wave and destination block (one word per peer)
__device__ __forceinline__ void append_records(const RoundArgs& a, bool want, uint32_t c, uint64_t m) {
    const int lane = threadIdx.x & 63;
    uint32_t q = 0;
    if (want)
        while (q + 1 < a.world && a.part[q + 1] <= c) ++q;
    for (unsigned long long todo = __ballot(want); todo;) {  // wave-uniform
        const int lead = __builtin_ctzll(todo);
        const uint32_t qq = (uint32_t)__shfl((int)q, lead);
        const unsigned long long grp = __ballot(want && q == qq);
        unsigned long long base = 0;
        if (lane == lead) base = atomicAdd(a.rec_cnt + qq, (unsigned long long)__popcll(grp));
        base = ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)(base >> 32), lead) << 32) |
               (uint32_t)__shfl((int)(uint32_t)base, lead);
        if (want && q == qq) {
            const uint64_t k = base + (uint64_t)__popcll(grp & ((1ull << lane) - 1));
            uint64_t* rec = a.rec_out + (qq * a.rec_stride + GOSSIP_IDX(a, kChkRecordOut, k, a.rec_stride)) * 2;
            rec[0] = c;
            rec[1] = m;
        }
        todo &= ~grp;
    }
}

// One delivery to global peer c (bit 31: masked edge): liveness, remote
// staging or the local test-and-set.
template <int W, bool CA, bool RM>
__device__ __forceinline__ void deliver(const RoundArgs& a, uint32_t c, const uint64_t (&m)[W], uint32_t pc,
                                        Acc& acc) {
    if (c & kMaskedEdge) return;  // connectedPeers.erase'd (peer.cpp:388)
    acc.trav++;
    if (CA && !bit_alive(a.alive, c)) {  // send() to a dead peer fails (peer.cpp:312)
        acc.undeliv += pc;
        return;
    }
    acc.deliv += pc;  // sentTo.insert (peer.cpp:314)
    if (RM && (c < a.begin || c >= a.end)) {
        if (W == 1 && a.rec_out) {  // a record of its own (deliver_batch appends them a wave at a time)
            uint32_t q = 0;
            while (q + 1 < a.world && a.part[q + 1] <= c) ++q;
            uint64_t* rec = a.rec_out + (q * a.rec_stride + atomicAdd(a.rec_cnt + q, 1ull)) * 2;
            rec[0] = c;
            rec[1] = m[0];
            return;
        }
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.send) + (uint64_t)c * W;
        bool wrote = false;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            if (!m[w]) continue;
            const unsigned long long cur = dst[w];
            if ((cur & m[w]) != m[w]) {
                atomicOr(dst + w, (unsigned long long)m[w]);
                acc.atomics++;
                wrote = true;
            }
        }
        if (wrote) mark_send(a, c);
        return;
    }
    const uint64_t lv = (uint64_t)(c - (uint32_t)a.begin);
    uint64_t cur[W];
#pragma unroll
    for (int w = 0; w < W; ++w) cur[w] = m[w] ? a.seen[GOSSIP_IDX(a, kChkPushSeen, lv * W + w, a.n_local * W)] : ~0ull;
    deliver_local<W>(a, lv, m, cur, acc);
}

// kU deliveries per lane at once (one per 64-edge batch), in phases so that
// every load of a phase is in flight together: the liveness bits, then the
// seen words, then the atomics.  A sparse push round is otherwise a chain of
// dependent round trips per batch (col -> seen -> atomic -> atomic).
template <int W, bool CA, bool RM, int kU>
__device__ __forceinline__ void deliver_batch(const RoundArgs& a, const uint32_t (&c)[kU],
                                              const uint64_t (&m)[kU][W], const uint32_t (&pc)[kU], Acc& acc) {
    bool loc[kU], rem[kU];
    uint32_t al[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
        rem[j] = false;
        const bool ok = !(c[j] & kMaskedEdge);  // invalid lanes carry a masked id
        acc.trav += ok;
        loc[j] = ok;
        if (CA) al[j] = a.alive[ok ? c[j] >> 5 : 0];
    }
#pragma unroll
    for (int j = 0; j < kU; ++j) {
        if (CA && loc[j] && !((al[j] >> (c[j] & 31)) & 1u)) {  // send() to a dead peer fails (peer.cpp:312)
            acc.undeliv += pc[j];
            loc[j] = false;
        } else if (loc[j]) {
            acc.deliv += pc[j];  // sentTo.insert (peer.cpp:314)
        }
        if (RM && loc[j] && (c[j] < a.begin || c[j] >= a.end) && W == 1 && a.rec_out) {
            rem[j] = true;  // a record, appended below
            loc[j] = false;
        } else if (RM && loc[j] && (c[j] < a.begin || c[j] >= a.end)) {
            unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.send) + (uint64_t)c[j] * W;
            bool wrote = false;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                if (!m[j][w]) continue;
                if ((dst[w] & m[j][w]) != m[j][w]) {
                    atomicOr(dst + w, (unsigned long long)m[j][w]);
                    acc.atomics++;
                    wrote = true;
                }
            }
            if (wrote) mark_send(a, c[j]);
            loc[j] = false;
        }
    }
    if (RM && W == 1 && a.rec_out) {
#pragma unroll
        for (int j = 0; j < kU; ++j) append_records(a, rem[j], c[j], m[j][0]);
    }
    // unconditional loads (lanes without a delivery read word 0): a load under a branch gets its own wait
    uint64_t cur[kU][W];
#pragma unroll
    for (int j = 0; j < kU; ++j)
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint64_t x =
                a.seen[GOSSIP_IDX(a, kChkPushSeen, loc[j] ? (uint64_t)(c[j] - (uint32_t)a.begin) * W + w : 0, a.n_local * W)];
            cur[j][w] = x | (loc[j] && m[j][w] ? 0ull : ~0ull);  // (a select would sink the load into a branch)
        }
    // the test-and-sets, every atomic of a phase issued before any result is used
    uint64_t old[kU][W];
#pragma unroll
    for (int j = 0; j < kU; ++j)
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint64_t lv = (uint64_t)(c[j] - (uint32_t)a.begin);
            const unsigned long long u = m[j][w] & ~cur[j][w];  // 0: all duplicates, dropped (peer.cpp:281)
            unsigned long long* p = reinterpret_cast<unsigned long long*>(a.defer ? a.nx : a.seen) + lv * W + w;
            old[j][w] = u ? atomicOr(p, a.defer ? u : (unsigned long long)m[j][w]) : ~0ull;
            acc.atomics += u != 0;
        }
    uint64_t fr[kU][W], onx[kU][W];
#pragma unroll
    for (int j = 0; j < kU; ++j)
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint64_t lv = (uint64_t)(c[j] - (uint32_t)a.begin);
            // defer: seen is the round-start set and nx holds the round's receipts so far
            fr[j][w] = (a.defer ? m[j][w] & ~cur[j][w] : m[j][w]) & ~old[j][w];
            onx[j][w] = a.defer ? old[j][w]
                        : fr[j][w] ? atomicOr(reinterpret_cast<unsigned long long*>(a.nx) + lv * W + w,
                                              (unsigned long long)fr[j][w])
                                   : ~0ull;
            acc.atomics += !a.defer && fr[j][w];
        }
#pragma unroll
    for (int j = 0; j < kU; ++j)
#pragma unroll
        for (int w = 0; w < W; ++w) {
            acc.fresh_or[w] |= fr[j][w];
            if (!fr[j][w]) continue;
            acc.fresh += (unsigned long long)__popcll(fr[j][w]);
            acc.activated += onx[j][w] == 0;
            if (onx[j][w] == 0) mark_tile(a, (uint64_t)(c[j] - (uint32_t)a.begin), acc);  // joins next round's tiles
        }
}

// Edge-space expansion of up to 64 rows (one per lane: deg = row length, 0 =
// skip; rb = row begin; m/pc = the row's new words and their popcount), kU
// batches of 64 edges at once, every edge delivered through deliver_batch.
template <int W, bool CA, bool RM, int kU>
__device__ __forceinline__ void expand_push(const RoundArgs& a, uint32_t deg, uint64_t rb, const uint64_t (&m)[W],
                                            uint32_t pc, Acc& acc) {
    const int lane = threadIdx.x & 63;
    uint32_t incl = deg;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    const uint32_t excl = incl - deg;
    const uint32_t total = __shfl(incl, 63);
    for (uint32_t base = 0; base < total; base += 64 * kU) {
        uint32_t c[kU], pcs[kU];
        uint64_t ms[kU][W];
        uint64_t e[kU];
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            const uint32_t p = base + j * 64 + lane;
            const int s = src_lane(incl, p);
            e[j] = __shfl(rb, s) + (uint64_t)(p - __shfl(excl, s));
            pcs[j] = __shfl(pc, s);
#pragma unroll
            for (int w = 0; w < W; ++w) ms[j][w] = __shfl(m[w], s);
            if (p >= total) pcs[j] = 0;
        }
#pragma unroll
        for (int j = 0; j < kU; ++j) c[j] = base + j * 64 + lane < total ? a.col[e[j]] : kMaskedEdge;
        deliver_batch<W, CA, RM, kU>(a, c, ms, pcs, acc);
    }
}

// ---------------------------------------------------------------------------
// push: light rows (<= kHeavyDegree).  Each wave sweeps 64-peer tiles and
// does the round's push-start bookkeeping for their active peers (frontier,
// digest and coverage increments: the new words ARE the bits added to seen
// since the last push start); it collects the active peers into a wave-private
// packet in LDS and expands 64 of them at a time (expand_push).  On a sparse
// frontier a tile holds about one active peer: expanding tile by tile left
// each wave one short chain of dependent loads at a time.
// ---------------------------------------------------------------------------
constexpr int kPushU = 4;  // 64-edge batches delivered together (W <= 2)
template <int W, bool CA, bool RM, bool COV, bool SP>  // SP: visit only the tiles marked in tcur
__global__ __launch_bounds__(kBlock) void k_push_light(RoundArgs a, uint32_t wd) {
    constexpr int kU = W <= 2 ? kPushU : 1;
    __shared__ unsigned int cov_s[COV ? 64 * W : 1];
    __shared__ uint32_t pk_v[kWavesPerBlock][128];
    __shared__ unsigned long long pk_m[kWavesPerBlock][128 * W];
    if (COV) {
        for (int i = threadIdx.x; i < 64 * W; i += kBlock) cov_s[i] = 0;
        __syncthreads();
    }
    Acc acc;
    const int lane = threadIdx.x & 63;
    uint32_t* pv = pk_v[threadIdx.x >> 6];
    unsigned long long* pm = pk_m[threadIdx.x >> 6];
    uint32_t n_pk = 0;  // wave-uniform
    const uint64_t n_tiles = (a.n_local + 63) >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // expand the packet's first min(n_pk, 64) peers; keep the rest
    auto expand = [&] {
        wave_sync();
        const uint32_t cnt = n_pk < 64 ? n_pk : 64;
        const bool have = (uint32_t)lane < cnt;
        const uint64_t v = have ? pv[lane] : 0;
        uint64_t m[W];
        uint32_t pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            m[w] = have ? pm[lane * W + w] : 0ull;
            pc += (uint32_t)__popcll(m[w]);
        }
        uint32_t deg = 0;
        uint64_t rb = 0;
        if (have) {
            rb = a.rp[v];
            const uint64_t d = a.rp[v + 1] - rb;
            deg = d <= a.heavy ? (uint32_t)d : 0u;  // heavy rows: k_push_heavy
        }
        const uint32_t rest = n_pk - cnt;
        wave_sync();
        if ((uint32_t)lane < rest) {  // entries 64.. move down (rest < 64)
            pv[lane] = pv[64 + lane];
#pragma unroll
            for (int w = 0; w < W; ++w) pm[lane * W + w] = pm[(64 + lane) * W + w];
        }
        n_pk = rest;
        expand_push<W, CA, RM, kU>(a, deg, rb, m, pc, acc);
    };
    auto load = [&](uint64_t t, uint64_t (&m)[W]) {
        const uint64_t v = (t << 6) + lane;
#pragma unroll
        for (int w = 0; w < W; ++w) m[w] = v < a.n_local ? a.nw[v * W + w] : 0ull;
    };
    auto tile = [&](uint64_t t, uint64_t (&m)[W]) {
        const uint64_t v = (t << 6) + lane;
        bool act = false;
#pragma unroll
        for (int w = 0; w < W; ++w) act |= m[w] != 0;
        const unsigned long long bal = __ballot(act);
        if (!bal) return;
        if (act) {
            acc.frontier++;
            uint32_t pc = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                pc += (uint32_t)__popcll(m[w]);
                if (w < (int)wd) acc.digest += digest_weight((a.begin + v) * wd + w) * m[w];
                a.nw[v * W + w] = 0ull;  // consumed: this buffer is next round's accumulator
                if (COV) {
                    for (uint64_t x = m[w]; x; x &= x - 1) atomicAdd(&cov_s[w * 64 + __builtin_ctzll(x)], 1u);
                }
            }
            acc.covered += pc;
            const uint32_t pos = n_pk + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            pv[pos] = (uint32_t)v;
#pragma unroll
            for (int w = 0; w < W; ++w) pm[pos * W + w] = m[w];
        }
        n_pk += (uint32_t)__popcll(bal);
        if (n_pk >= 64) expand();
    };
    const uint64_t wave0 = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if constexpr (SP) {  // only the tiles marked in tcur (64 per bitmap word), clearing the words
        const uint64_t n_words = (n_tiles + 63) >> 6;
        for (uint64_t i = wave0; i < n_words; i += nwaves) {
            const unsigned long long word = a.tcur[i];
            unsigned long long bits = ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(word >> 32)) << 32) |
                                      __builtin_amdgcn_readfirstlane((uint32_t)word);  // wave-uniform
            if (!bits) continue;
            if (lane == 0) a.tcur[i] = 0ull;
            for (; bits; bits &= bits - 1) {
                uint64_t m[W];
                load((i << 6) + (uint64_t)__builtin_ctzll(bits), m);
                tile((i << 6) + (uint64_t)__builtin_ctzll(bits), m);
            }
        }
    } else {  // (the engine clears tcur)
        // kPre tiles' words in flight per wave: a sweep over a sparse frontier is bound by load latency
        constexpr int kPre = W <= 2 ? 4 : 1;
        for (uint64_t t0 = wave0; t0 < n_tiles; t0 += kPre * nwaves) {
            uint64_t m[kPre][W];
#pragma unroll
            for (int j = 0; j < kPre; ++j) load(t0 + j * nwaves, m[j]);
#pragma unroll
            for (int j = 0; j < kPre; ++j)
                if (t0 + j * nwaves < n_tiles) tile(t0 + j * nwaves, m[j]);
        }
    }
    if (n_pk) expand();  // n_pk < 64 here
    flush(acc, a.st);
    if (COV) {
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * W; i += kBlock)
            if (cov_s[i]) atomicAdd(&a.cov[i], (unsigned long long)cov_s[i]);
    }
}

// push: heavy rows, one wave per kHeavyChunk-edge chunk; runs before
// k_push_light (which clears the new words).
template <int W, bool CA, bool RM>
__global__ __launch_bounds__(kBlock) void k_push_heavy(RoundArgs a) {
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t ci = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); ci < a.n_chunks; ci += nwaves) {
        const HeavyChunk ch = a.chunks[ci];
        uint64_t m[W];
        bool act = false;
        uint32_t pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            m[w] = a.nw[(uint64_t)ch.v * W + w];
            act |= m[w] != 0;
            pc += (uint32_t)__popcll(m[w]);
        }
        if (!act) continue;  // uniform over the wave
        constexpr int kU = W <= 2 ? kPushU : 1;
        uint64_t ms[kU][W];
        uint32_t pcs[kU];
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            pcs[j] = pc;
#pragma unroll
            for (int w = 0; w < W; ++w) ms[j][w] = m[w];
        }
        for (uint64_t e0 = ch.e0 + lane; e0 < ch.e1; e0 += 64 * kU) {
            uint32_t c[kU];
#pragma unroll
            for (int j = 0; j < kU; ++j) c[j] = e0 + j * 64 < ch.e1 ? a.col[e0 + j * 64] : kMaskedEdge;
            deliver_batch<W, CA, RM, kU>(a, c, ms, pcs, acc);
        }
    }
    acc.htrav = acc.trav;
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// pull (direction-optimised dense rounds): every peer that can still learn a
// message ORs the new words of its neighbours into a wave-private LDS
// accumulator, then applies its own test-and-set with plain stores -- no
// global atomics.  Same round contract as push: on a symmetric overlay with
// no dead peers and no masked edges, edge u->v is traversed iff u is in the
// frontier, so traversals/deliveries are summed on the source side
// (deg(u), popcount(new[u]) * deg(u)) and new_receipts on the receiving side.
// Heavy rows are pulled by k_pull_heavy (one wave per chunk, one atomicOr per
// chunk).  Gathers read nw_src: the own new words (P = 1) or the all-gathered
// words of every block, indexed by global peer (P > 1).
// ---------------------------------------------------------------------------
// Frontier bitmap for a pull round: one ballot per 64-peer tile, stored by
// the tile's own wave (no atomics).  n/8 bytes -- cache-resident at 2^28 peers.
template <int W>
__global__ __launch_bounds__(kBlock) void k_frontier_bits(RoundArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t n_tiles = (a.n_src + 63) >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); t < n_tiles; t += nwaves) {
        const uint64_t v = (t << 6) + lane;
        bool act = false;
        if (v < a.n_src) {
#pragma unroll
            for (int w = 0; w < W; ++w) act |= a.nw_src[v * W + w] != 0;
        }
        const unsigned long long bits = __ballot(act);
        if (lane == 0) a.front[t] = bits;
    }
}

// pull, light rows, as a row queue with an early exit.  Each wave sweeps 64-peer tiles: source side of the pushes, nx = 0, and every
// light row that can still learn something (need != 0) joins the wave's queue
// in LDS.  Lanes take rows from the queue and scan them kRowB edges per step,
// OR-ing the neighbours' new words into what they got; a row stops as soon as
// it got every bit it can learn (need) -- most rows need one neighbour (config
// 4, round 7: 90.1 M needy rows, 101 M gathers with the exit against 479 M
// for whole rows) -- or at its end.  Finished lanes take the next row:
// fr = (OR of the scanned neighbours) & need, and a row that stops early
// already holds all of need.
template <int W, bool COV, bool FRONT, int kRowB, int kRowQ = 128>  // kRowB: edges per lane per step; kRowQ: queue entries per wave
// (116 VGPRs, four waves per SIMD.  Launch bounds asking five or six spill to scratch and ran round 7 at
// 5.9-6.1 and 8.3-8.6 ms against 4.8-5.1: the sweep and the row state do not fit 96 or 80 registers.)
__global__ __launch_bounds__(kBlock) void k_pull_rows(RoundArgs a, uint32_t wd) {
    __shared__ unsigned int cov_s[COV ? 64 * W : 1];
    __shared__ uint32_t q_v[kWavesPerBlock][kRowQ];
    __shared__ uint32_t q_d[kWavesPerBlock][kRowQ];
    __shared__ unsigned long long q_rb[kWavesPerBlock][kRowQ];
    __shared__ unsigned long long q_f2[kWavesPerBlock][kRowQ];  // the row's first two entries (a.first2)
    __shared__ unsigned long long q_need[kWavesPerBlock][kRowQ * W];
    __shared__ uint32_t q_lst[kWavesPerBlock][128];  // rows for the next round's list (a.lst_out), staged
    if (COV) {
        for (int i = threadIdx.x; i < 64 * W; i += kBlock) cov_s[i] = 0;
        __syncthreads();
    }
    Acc acc;
    PreAcc pre;
    const InjMasks<W> im(a);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* qv = q_v[wv];
    uint32_t* lq = q_lst[wv];
    uint32_t lq_n = 0;  // wave-uniform
    uint32_t* qd = q_d[wv];
    unsigned long long* qrb = q_rb[wv];
    unsigned long long* qf2 = q_f2[wv];
    unsigned long long* qneed = q_need[wv];
    uint32_t q_head = 0, q_tail = 0;  // wave-uniform ring counters (q_tail - q_head <= kRowQ)
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // this lane's row
    bool has = false;
    uint32_t rv = 0, rd = 0, rk = 0;
    uint64_t rrb = 0, rf2 = 0, need[W], got[W];
#pragma unroll
    for (int w = 0; w < W; ++w) need[w] = got[w] = 0;
    const uint64_t n_tiles = (a.n_local + 63) >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
    // the sweep is a chain of two round trips per tile (the peer words, then the
    // row bounds of the rows that matter); each wave keeps the next tile's
    // words and row bounds in flight while it sweeps the current one
    // (unconditional loads, clamped past the end)
    struct TileIn {
        uint64_t m[W], sv[W], r0, r1, f2;
        uint32_t al;
    };
    auto load_tile = [&](uint64_t tt, TileIn& d) {
        const uint64_t v = min((tt << 6) + lane, a.n_local - 1);
#pragma unroll
        for (int w = 0; w < W; ++w) {
            d.m[w] = a.nw[v * W + w];
            d.sv[w] = a.seen[v * W + w];
        }
        d.r0 = a.rp[v];
        d.r1 = a.rp[v + 1];
        d.f2 = a.first2 ? a.first2[v] : 0ull;
        d.al = a.dead_mode ? a.alive[(uint32_t)(a.begin + v) >> 5] : ~0u;
    };
    auto sweep_tile = [&](uint64_t tt, const TileIn& d) {
        const uint64_t v = (tt << 6) + lane;
        const bool vv = v < a.n_local;
        uint64_t m[W], nd[W];
        bool act = false, needy = false;
        const bool va = vv && (!a.dead_mode || ((d.al >> ((uint32_t)(a.begin + v) & 31)) & 1u));  // dead: no receive
#pragma unroll
        for (int w = 0; w < W; ++w) {
            m[w] = vv ? d.m[w] : 0ull;
            // a.fold: the previous round's receipts (this round's new words) are not yet in seen; the
            // sweep folds them in (the peers with new words of the tile) -- before the tile's rows are
            // queued, so their own later stores come after it
            const uint64_t sv = vv ? (a.fold ? d.sv[w] | m[w] : d.sv[w]) : ~0ull;
            if (a.fold && vv && m[w]) a.seen[v * W + w] = sv;
            // nd: every bit the peer lacks (the row's final seen word is rebuilt from it); a row is queued
            // only if one of them is in flight this round
            nd[w] = va ? im.full[w] & ~sv : 0ull;
            act |= m[w] != 0;
            needy |= (nd[w] & im.cur[w]) != 0;
            // nx is written whole in a pull round; rows that learn rewrite it.  (Leaving a queued row's word to
            // its finish alone turned these whole-line stores into partial ones: round 7 5.2-5.7 against
            // 4.8-5.1 ms.)
            if (vv) a.nx[v * W + w] = 0ull;
        }
        const uint64_t rb = d.r0, d_ = d.r1 - d.r0;
        const uint64_t dg = (act || needy) ? d_ : 0ull;
        if (act && !a.src_booked) {  // source side of this peer's pushes (broadcastMessage, peer.cpp:310-316)
            uint32_t pc = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                pc += (uint32_t)__popcll(m[w]);
                if (w < (int)wd) acc.digest += digest_weight((a.begin + v) * wd + w) * m[w];
                if (COV)
                    for (uint64_t x = m[w]; x; x &= x - 1) atomicAdd(&cov_s[w * 64 + __builtin_ctzll(x)], 1u);
            }
            acc.frontier++;
            acc.covered += pc;
            // (the increments as values added once: written as two branches' own updates, the compiler merged
            // them into one store through a selected address and moved the counters to scratch memory)
            uint64_t dt = dg, dd = (uint64_t)pc * dg, du = 0;  // every edge alive and unmasked
            if (a.dead_mode) {
                dt = dd = 0;
                if (a.dgone) {  // from the per-source counters; else k_src_count books them
                    const uint32_t g = a.dgone[v], k = a.dmask[v];
                    dt = dg - k;
                    dd = (uint64_t)pc * (dg - g);
                    du = (uint64_t)pc * (g - k);
                }
            }
            acc.trav += dt;
            acc.deliv += dd;
            acc.undeliv += du;
        }
        const bool enq = needy && dg > 0 && dg <= a.heavy;  // heavy rows: k_pull_heavy
        const unsigned long long bal = __ballot(enq);
        if (enq) {
            const uint32_t pos = (q_tail + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                               (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))) %
                                 kRowQ;
            qv[pos] = (uint32_t)v;
            qd[pos] = (uint32_t)dg;
            qrb[pos] = rb;
            qf2[pos] = d.f2;
#pragma unroll
            for (int w = 0; w < W; ++w) qneed[pos * W + w] = nd[w];
        }
        q_tail += (uint32_t)__popcll(bal);
    };
    // (Round 6 measured two tiles in flight per wave, swept as pairs from two buffers: 124-147 VGPRs, so three
    // waves per SIMD or spills at four; round 7 4.94 -> 5.48 ms, tools/experiments/r06_row_pull_tile_pairs.patch.)
    TileIn nxt;
    load_tile(t, nxt);
    while (true) {
        // refill the queue while it has room for a whole tile
        while (t < n_tiles && q_tail - q_head <= (uint32_t)(kRowQ - 64)) {
            const TileIn cur = nxt;
            load_tile(t + nwaves, nxt);  // unconditional (clamped): the wait before the sweep can then count it
            sweep_tile(t, cur);
            t += nwaves;
        }
        // idle lanes take queued rows
        const unsigned long long idle = __ballot(!has);
        const uint32_t avail = q_tail - q_head;
        if (idle && avail) {
            wave_sync();
            const uint32_t r = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (!has && r < avail) {
                const uint32_t pos = (q_head + r) % kRowQ;
                has = true;
                rv = qv[pos];
                rd = qd[pos];
                rrb = qrb[pos];
                rf2 = qf2[pos];
                rk = 0;
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    need[w] = qneed[pos * W + w];
                    got[w] = 0;
                }
            }
            const uint32_t taken = min((uint32_t)__popcll(idle), avail);
            q_head += taken;
            wave_sync();  // the taken entries are read before a sweep overwrites them
        }
        if (!__any(has)) {
            if (t >= n_tiles && q_tail == q_head) break;
            continue;
        }
        // one step: kRowB edges of this lane's row, every load of the step in flight together
        uint32_t u[kRowB];
        bool ok[kRowB];
#pragma unroll
        for (int j = 0; j < kRowB; ++j) {
            ok[j] = has && rk + j < rd;
            // rows are sorted, so the scan meets the hubs first: their words are cache-hot (scanning
            // from the row's end measured 192 M gathers and 8.0-9.2 ms against 180 M, 7.3-7.5 ms at
            // config 4 round 7).  A row's first two entries may come with its queue entry (a.first2).
            const uint32_t q = rk + j;
            const bool f2 = a.first2 && q < 2;
            const uint32_t uc = a.col[ok[j] && !f2 ? rrb + q : 0];
            u[j] = f2 ? (uint32_t)(rf2 >> (32 * q)) : uc;
        }
        acc.pulled += (has ? min(kRowB, (int)(rd - rk)) : 0);
#pragma unroll
        for (int j = 0; j < kRowB; ++j) ok[j] = ok[j] && !(u[j] & kMaskedEdge);  // dead neighbour: words are zero
        if (FRONT) {
            uint64_t fb[kRowB];
#pragma unroll
            for (int j = 0; j < kRowB; ++j) fb[j] = a.front[ok[j] ? u[j] >> 6 : 0];
#pragma unroll
            for (int j = 0; j < kRowB; ++j) ok[j] = ok[j] && ((fb[j] >> (u[j] & 63)) & 1ull);  // nothing new: no gather
        }
        uint64_t x[kRowB][W];
#pragma unroll
        for (int j = 0; j < kRowB; ++j)
#pragma unroll
            for (int w = 0; w < W; ++w)  // unconditional (a select would sink the load into a branch)
                x[j][w] = a.nw_src[GOSSIP_IDX(a, kChkPullGather, (ok[j] ? (uint64_t)u[j] : 0) * W + w, a.n_src * W)] &
                          (ok[j] ? ~0ull : 0ull);
#pragma unroll
        for (int j = 0; j < kRowB; ++j) acc.gathered += ok[j];
        bool done = true;
#pragma unroll
        for (int w = 0; w < W; ++w) {
#pragma unroll
            for (int j = 0; j < kRowB; ++j) got[w] |= x[j][w] & need[w];
            done &= got[w] == (need[w] & im.cur[w]);  // every bit it can still learn this round
        }
        rk += kRowB;
        bool lacks = false;
        if (has && (done || rk >= rd)) {  // the row is finished: handleClient's test-and-set, owner stores
            bool any = false;
            uint32_t pc = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint64_t fr = got[w];  // subset of need: bits this peer had not seen
                acc.fresh_or[w] |= fr;
                // still lacking a bit in flight: the only rows that can learn later (no injections: the next
                // round's bits in flight are this round's receipts, a subset of this round's)
                lacks |= (need[w] & im.cur[w] & ~fr) != 0;
                if (fr) {
                    a.seen[(uint64_t)rv * W + w] = (im.full[w] & ~need[w]) | fr;  // within inj_mask
                    a.nx[(uint64_t)rv * W + w] = fr;
                    pc += (uint32_t)__popcll(fr);
                    if (a.st_pre && w < (int)wd) pre.digest += digest_weight(((uint64_t)a.begin + rv) * wd + w) * fr;
                    any = true;
                }
            }
            acc.fresh += pc;
            acc.activated += any;
            if (a.st_pre && any) {  // the next round's push from this peer (no deaths: every edge delivers)
                pre.frontier++;
                pre.covered += pc;
                pre.trav += rd;
                pre.deliv += (unsigned long long)pc * rd;
            }
            lacks = lacks && a.lst_out;
            has = false;
        }
        if (a.lst_out) {  // staged per wave, one counter atomic per 64 entries
            const unsigned long long lb = __ballot(lacks);
            if (lb) {
                if (lacks) lq[lq_n + lane_rank(lb)] = rv;
                lq_n += (uint32_t)__popcll(lb);
                if (lq_n >= 64) {
                    wave_sync();
                    list_flush(a, lq, 64);
                    lq_n -= 64;
                    const uint32_t mv = (uint32_t)lane < lq_n ? lq[64 + lane] : 0u;
                    wave_sync();
                    if ((uint32_t)lane < lq_n) lq[lane] = mv;
                    wave_sync();
                }
            }
        }
    }
    if (a.lst_out && lq_n) {
        wave_sync();
        list_flush(a, lq, lq_n);
    }
    flush_pre(pre, a.st_pre);
    flush(acc, a.st);
    if (COV) {
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * W; i += kBlock)
            if (cov_s[i]) atomicAdd(&a.cov[i], (unsigned long long)cov_s[i]);
    }
}

// kDefer (binned rounds, P = 1; round 6): the chunks only OR what they found into their row's hacc word, and
// k_heavy_commit applies the rows after the apply -- so the heavy rows' pull runs on a second stream beside the
// binned round's scatter (it reads seen and the new words, which the scatter does not write) instead of after
// the apply (whose whole-tile stores rewrite the heavy rows' seen and nx words).
template <int W, bool kDefer = false>
__global__ __launch_bounds__(kBlock) void k_pull_heavy(RoundArgs a) {
    Acc acc;
    PreAcc pre;
    const InjMasks<W> im(a);
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t ci = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); ci < a.n_chunks; ci += nwaves) {
        const HeavyChunk ch = a.chunks[ci];
        uint64_t need[W], part[W], pub[W];  // pub: bits this chunk has published in hacc
        bool any = false;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            pub[w] = 0;
            // one lane reads, every lane uses the same value: the branch below stays wave-uniform
            const uint64_t s0 = __shfl(a.seen[(uint64_t)ch.v * W + w], 0);
            need[w] = im.cur[w] & ~s0;
            if (a.dead_mode && !bit_alive(a.alive, (uint32_t)(a.begin + ch.v))) need[w] = 0;  // dead: no receive
            part[w] = 0;
            any |= need[w] != 0;
        }
        if (!any) continue;
        // early exit (a.heavy_exit): every kHeavyExitEvery batches the wave ORs what it
        // has; once that holds every bit the peer can still learn, the rest of the
        // chunk cannot add to part & need (hubs are satisfied after a few edges)
        uint32_t batch = 0;
        for (uint64_t e0 = ch.e0; e0 < ch.e1; e0 += 64) {
            const uint64_t e = e0 + lane;
            if (e < ch.e1) {
                const uint32_t u = a.col[e];
                acc.pulled++;
                const bool skip = (u & kMaskedEdge) ||  // the neighbour is dead, its words are zero
                                  (a.front && !((a.front[u >> 6] >> (u & 63)) & 1ull));
                if (!skip) {
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        if (need[w]) part[w] |= a.nw_src[GOSSIP_IDX(a, kChkPullGather, (uint64_t)u * W + w, a.n_src * W)] & need[w];
                }
            }
            if (a.heavy_exit && (++batch % kHeavyExitEvery) == 0 && e0 + 64 < ch.e1) {
                bool done = true;
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    uint64_t x = part[w];
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) x |= __shfl_xor(x, off);
                    // what the row's other chunks found: publish ours (it is committed to seen at
                    // this chunk's end, so every published bit reaches seen) and read theirs
                    if (a.hacc) {
                        unsigned long long* hw =
                            reinterpret_cast<unsigned long long*>(a.hacc) + (uint64_t)ch.first * W + w;
                        unsigned long long o = 0;
                        if (lane == 0)
                            o = (x & need[w] & ~pub[w]) ? atomicOr(hw, (unsigned long long)(x & need[w]))
                                                        : __hip_atomic_load(hw, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT);
                        pub[w] |= x & need[w];
                        x |= __shfl(o, 0);
                    }
                    done &= (x & need[w]) == need[w];
                }
                if (done) break;  // wave-uniform (x is the wave's OR)
            }
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) part[w] |= __shfl_xor(part[w], off);
        }
        if (kDefer) {  // the row's bits: k_heavy_commit tests them against seen after the apply
            if (lane == 0)
#pragma unroll
                for (int w = 0; w < W; ++w)
                    if (part[w] & ~pub[w])
                        atomicOr(reinterpret_cast<unsigned long long*>(a.hacc) + (uint64_t)ch.first * W + w,
                                 (unsigned long long)part[w]);
            continue;
        }
        if (lane == 0) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                if (!part[w]) continue;
                unsigned long long* sp = reinterpret_cast<unsigned long long*>(a.seen) + (uint64_t)ch.v * W + w;
                const unsigned long long fr = part[w] & ~atomicOr(sp, (unsigned long long)part[w]);
                acc.atomics += fr ? 2 : 1;
                acc.fresh_or[w] |= fr;
                if (fr) {
                    const unsigned long long onx =
                        atomicOr(reinterpret_cast<unsigned long long*>(a.nx) + (uint64_t)ch.v * W + w, fr);
                    acc.activated += onx == 0;
                    acc.fresh += (unsigned long long)__popcll(fr);
                    if (a.st_pre) {  // one word per peer: the row's chunks' fr are disjoint, its push counted once
                        const uint64_t deg = a.rp[ch.v + 1] - a.rp[ch.v];
                        const uint32_t pc = (uint32_t)__popcll(fr);
                        pre.covered += pc;
                        pre.digest += digest_weight((uint64_t)a.begin + ch.v) * fr;
                        pre.deliv += (unsigned long long)pc * deg;
                        if (onx == 0) {
                            pre.frontier++;
                            pre.trav += deg;
                        }
                    }
                }
            }
        }
    }
    acc.htrav = acc.pulled;  // heavy-row edges scanned
    acc.pulled = 0;
    flush_pre(pre, a.st_pre);
    flush(acc, a.st);
}

// After a binned round's apply: the deferred heavy rows (k_pull_heavy<W, true>), one thread per row -- handleClient's
// test-and-set of what the row's chunks found (peer.cpp:277-285).  The apply wrote the heavy rows' nx words (zero:
// their in-edges have no slots); a row's words are ORed in here.
template <int W>
__global__ __launch_bounds__(kBlock) void k_heavy_commit(RoundArgs a) {
    Acc acc;
    for (uint64_t ci = (uint64_t)blockIdx.x * kBlock + threadIdx.x; ci < a.n_chunks; ci += (uint64_t)gridDim.x * kBlock) {
        const HeavyChunk ch = a.chunks[ci];
        if (ch.first != ci) continue;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint64_t x = a.hacc[ci * W + w];
            if (!x) continue;
            const uint64_t sv = a.seen[(uint64_t)ch.v * W + w];
            const uint64_t fr = x & ~sv;
            acc.fresh_or[w] |= fr;
            if (!fr) continue;
            a.seen[(uint64_t)ch.v * W + w] = sv | fr;
            const uint64_t onx = a.nx[(uint64_t)ch.v * W + w];
            a.nx[(uint64_t)ch.v * W + w] = onx | fr;
            acc.activated += onx == 0;
            acc.fresh += (unsigned long long)__popcll(fr);
        }
    }
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// Late pull rounds over a needy list (P = 1, one word per peer, no deaths;
// DESIGN.md section 6.5).  After the dense rounds few peers still lack a
// message (config 4 round 8: 1.8 M of 2^28), yet a row-queue pull sweeps every
// peer for the source side of the round and for its needy rows.  The round
// before books this round's source side where it activates peers (st_pre) and
// lists the light rows that still lack a bit; this round pulls just those
// rows -- handleClient's test-and-set per row, the scan stopping once the row
// holds every bit in flight that it lacks -- and lists the rows that still
// lack one for the next.  Heavy rows stay k_pull_heavy's.
// ---------------------------------------------------------------------------
// nx is the buffer of the round before last's new words: only that round's list (or the heavy rows)
// can have left anything in it
__global__ __launch_bounds__(kBlock) void k_list_zero(RoundArgs a, const uint32_t* lst, uint32_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) a.nx[lst[i]] = 0ull;
    for (uint64_t ci = (uint64_t)blockIdx.x * kBlock + threadIdx.x; ci < a.n_chunks; ci += stride) {
        const HeavyChunk ch = a.chunks[ci];
        if (ch.first == ci) a.nx[ch.v] = 0ull;
    }
}

__global__ __launch_bounds__(kBlock) void k_pull_list(RoundArgs a, const uint32_t* lst, uint32_t n) {
    Acc acc;
    PreAcc pre;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t n_pad = ((uint64_t)n + 63) & ~63ull;
    const uint64_t inj_all = injm_full(a, 0), inj_now = injm(a, 0);
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n_pad; i += stride) {
        const bool in = i < n;
        const uint32_t v = in ? (uint32_t)GOSSIP_IDX(a, kChkListRow, lst[i], a.n_local) : 0u;
        const uint64_t sv = in ? a.seen[v] : ~0ull;
        const uint64_t need = inj_all & ~sv;  // every bit the peer lacks ...
        const uint64_t want = need & inj_now;  // ... and of those, the ones in some new word this round
        uint64_t r0 = 0, r1 = 0;
        if (in) {
            r0 = a.rp[v];
            r1 = a.rp[v + 1];
        }
        uint64_t got = 0;
        if (want) {
            for (uint64_t e = r0; e < r1; e += 2) {  // two neighbours' words in flight per step
                const bool two = e + 1 < r1;
                const uint32_t u0 = a.col[e], u1 = two ? a.col[e + 1] : kMaskedEdge;
                const bool ok0 = !(u0 & kMaskedEdge), ok1 = !(u1 & kMaskedEdge);  // (no deaths: none masked)
                const uint64_t x0 = a.nw_src[ok0 ? u0 : 0u] & (ok0 ? ~0ull : 0ull);
                const uint64_t x1 = a.nw_src[ok1 ? u1 : 0u] & (ok1 ? ~0ull : 0ull);
                acc.pulled += two ? 2u : 1u;
                acc.gathered += (unsigned)ok0 + (unsigned)ok1;
                got |= (x0 | x1) & want;
                if (got == want) break;  // every bit it can learn this round
            }
        }
        if (got) {  // handleClient: new -> Message-List insert (peer.cpp:281-282)
            a.seen[v] = sv | got;
            a.nx[v] = got;
            const uint32_t pc = (uint32_t)__popcll(got);
            acc.fresh += pc;
            acc.activated++;
            acc.fresh_or[0] |= got;
            if (a.st_pre) {  // the next round's push from this peer
                const uint64_t d = r1 - r0;
                pre.frontier++;
                pre.covered += pc;
                pre.digest += digest_weight((uint64_t)a.begin + v) * got;
                pre.trav += d;
                pre.deliv += (unsigned long long)pc * d;
            }
        }
        if (a.lst_out) list_push(a, in && (want & ~got) != 0 && r1 > r0, v);  // (next round: a subset in flight)
    }
    flush_pre(pre, a.st_pre);
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// binned dense rounds (layout: gossip_bins.hip).  Same round contract and the
// same source-side accounting as pull: every peer v ends with
// next[v] = (OR of new[u] over u in N(v)) & ~seen[v]; heavy destinations are
// left to k_pull_heavy.
// ---------------------------------------------------------------------------
// Phase 1 (scatter): one 16-wave workgroup per CU stages a
// source chunk's new words (kBinChunkWords words, 144 KB) in LDS and writes
// them into the slots of the chunk's binned edges, walked in bin order (the cb
// list).  The units of XCD x are a contiguous range of the chunk order, dealt
// round-robin to its workgroups: the ~32 chunks in flight on an XCD are
// consecutive, and their slot runs inside each bin are adjacent, so the lines
// of a bin fill up in that XCD's L2 from several workgroups before they are
// written back.
// Staging of one scatter unit's source chunk (every thread of the block):
// the chunk's new words into the LDS slice, the live bits of its sources and,
// in the chunk's first unit, the source side of its pushes (broadcastMessage,
// peer.cpp:310-316) unless the apply books them (BinArgs.src_stats = 0: the
// staging is then one round trip instead of a chain of dependent row-bound
// loads, ~40 us per unit).  Ends before the block barrier that publishes the
// slice.
// kCW / kSB: the slice's words and the block's threads (k_bin_stream's small-chunk instance: 4096 / 256)
template <int W, bool COV, int kCW = (int)kBinChunkWords, int kSB = kScatterBlock>
__device__ __forceinline__ void scatter_stage(const RoundArgs& a, const BinArgs& b, const BinUnit& un, uint32_t wd,
                                              unsigned long long* slice, unsigned long long* live_s,
                                              unsigned int* cov_s, Acc& acc) {
    constexpr int kSliceIt = kCW / kSB;  // slice words per lane
    static_assert(kCW % kSB == 0, "slice split");
    const int lane = threadIdx.x & 63;
    // global source chunk; words from nw_src (own words at P = 1, the all-gathered ones at P > 1)
    const uint64_t vb = bin_chunk_vb(b, un.c), ve = bin_chunk_ve(b, un.c, a.n_src);  // vb % 64 == 0
    const uint64_t nwords = (ve - vb) * W;
    // stage the slice (and the previous round's live bits): every load of
    // the lane in flight at once
    const uint64_t n_src = ve - vb;
    uint64_t r[kSliceIt];
#pragma unroll
    for (int k = 0; k < kSliceIt; ++k) {
        const uint64_t i = threadIdx.x + (uint64_t)k * kSB;
        r[k] = i < nwords ? a.nw_src[GOSSIP_IDX(a, kChkStageSrc, vb * W + i, a.n_src * W)] : 0ull;
    }
    __syncthreads();  // previous unit's readers are done with the slice
#pragma unroll
    for (int k = 0; k < kSliceIt; ++k) slice[threadIdx.x + k * kSB] = r[k];
    if (threadIdx.x < kCW / 64 / W) live_s[threadIdx.x] = b.noskip ? ~0ull : 0ull;
    __syncthreads();
    // per source (a wave covers 64 consecutive ones): live bits and, in the
    // chunk's first unit, the source side of its pushes (broadcastMessage,
    // peer.cpp:310-316) for the owned sources; row lengths loaded together
    constexpr int kSrcIt = (kCW / W + kSB - 1) / kSB;
    constexpr int kB = 5;  // sources whose row lengths are loaded together (register budget)
#pragma unroll
    for (int k0 = 0; k0 < kSrcIt; k0 += kB) {
        uint32_t pcs[kB];
#pragma unroll
        for (int kk = 0; kk < kB; ++kk) {
            const uint64_t j = threadIdx.x + (uint64_t)(k0 + kk) * kSB;
            pcs[kk] = 0;
            if (k0 + kk >= kSrcIt || j >= ((n_src + 63) & ~63ull)) continue;  // wave-uniform
            const uint64_t v = vb + j;
            const bool vv = j < n_src;
            const bool own = vv && b.src_stats && un.first && v >= a.begin && v < a.end;
            bool nz = false;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint64_t m = vv ? slice[j * W + w] : 0ull;
                nz |= m != 0;
                if (!own || !m) continue;
                pcs[kk] += (uint32_t)__popcll(m);
                if (w < (int)wd) acc.digest += digest_weight(v * wd + w) * m;
                if (COV)
                    for (uint64_t x = m; x; x &= x - 1) atomicAdd(&cov_s[w * 64 + __builtin_ctzll(x)], 1u);
            }
            const unsigned long long bits = __ballot(nz);
            if (lane == 0) live_s[j >> 6] |= bits;
        }
        uint64_t d0[kB], d1[kB];
        uint32_t dg[kB], dk[kB];  // per-source counters (dead mode); else k_src_count books them
        const bool cnt = a.dead_mode && a.dgone;
#pragma unroll
        for (int kk = 0; kk < kB; ++kk) {
            const uint64_t lv = vb + threadIdx.x + (uint64_t)(k0 + kk) * kSB - a.begin;
            d0[kk] = pcs[kk] ? a.rp[lv] : 0ull;
            d1[kk] = pcs[kk] ? a.rp[lv + 1] : 0ull;
            dg[kk] = pcs[kk] && cnt ? a.dgone[lv] : 0u;
            dk[kk] = pcs[kk] && cnt ? a.dmask[lv] : 0u;
        }
#pragma unroll
        for (int kk = 0; kk < kB; ++kk) {
            if (!pcs[kk]) continue;
            acc.frontier++;
            acc.covered += pcs[kk];
            const uint64_t d = d1[kk] - d0[kk];
            if (!a.dead_mode || cnt) {
                acc.trav += d - dk[kk];
                acc.deliv += (unsigned long long)pcs[kk] * (d - dg[kk]);
                acc.undeliv += (unsigned long long)pcs[kk] * (dg[kk] - dk[kk]);
            }
        }
    }
}

// The row loop of the scatters: member j of XCD x takes unit j of each
// row of the XCD's unit list (gossip_bins.hip), so the XCD's workgroups stage
// consecutive chunks together and write adjacent slot runs into every bin (a
// row barrier on top of that measured no gain: 71.4 against 71.3 ms per step).
template <class F>
__device__ __forceinline__ void scatter_rows(const BinArgs& b, F&& unit) {
    // rows of `members` units, row r on XCD r % 8 (gossip_bins.hip; n_units: this launch's unit count)
    const uint32_t xcd = blockIdx.x & 7, member = blockIdx.x >> 3, members = gridDim.x >> 3;
    const uint64_t rows = (b.n_units + members - 1) / members;  // (units come in rows of kScatterGrid / 8)
    for (uint64_t r = xcd; r < rows; r += 8)
        if (r * members + member < b.n_units) unit(r * members + member);
}

// Producer/consumer scatter (slot layout).  Measured on the round-1 single-role kernel: a wave that both
// loads and stores cannot keep stores in flight -- vmcnt counts loads and
// stores in issue order, and every wait for a load (the next cb entries)
// also waited for the stores issued before it (the compiled loop drained to
// vmcnt(1)-vmcnt(0) every iteration), so each wave had one batch of stores in
// flight per HBM write latency.  Here the 16 waves split the work:
//   producers (waves 0-7) load the unit's cb entries and resolve their slots
//     (cb_grp + a ballot of the run-start flags + cb_run), and hand
//     {slot, chunk-local source | active} to their consumer through an LDS
//     ring; they issue only loads, so their waits are exact;
//   consumers (waves 8-15) read the ring and the staged slice and store --
//     they issue no global loads, never wait on vmcnt, and keep as many slot
//     stores in flight as the memory system takes.
// Producer k and consumer k share a private ring of kPcRing 64-entry slots;
// each side publishes a counter in LDS (its own wave writes it, after
// s_waitcnt lgkmcnt(0) on the ring data).  Both sides walk the unit's
// 64-entry groups g0 + k, g0 + k + 8, ... in the same order, so consecutive
// groups go out through different consumer waves at about the same time.
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// kPcProd producer waves, the other 16 - kPcProd consume; consumer c serves the
// producers p = c (mod consumers) in turn.  kPcG: groups a producer resolves per
// pipeline stage; kPcRing: ring slots (64 entries each) per producer; kPcSets:
// register sets a producer rotates through -- a stage's cb entries are loaded
// kPcSets - 1 stages before its hand-over and its slots resolved (cb_run
// loads issued) (kPcSets - 1) / 2 stages before it.  Deeper rotations were
// measured and dropped (config 4, per launch, one box: 3 sets 9.2-9.4 ms, 5
// sets 9.6, 7 sets 16.0, 9 sets of one group 11.6): the 1024-thread block
// caps a wave at 128 VGPRs, and the extra sets spill (scratch 52 -> 104-208
// bytes per lane).
template <int W, bool COV, int kPcProd, int kPcG, int kPcRing, int kPcSets>
__global__ __launch_bounds__(kScatterBlock) void k_bin_scatter_pc(RoundArgs a, BinArgs b, uint32_t wd) {
    constexpr int kWaves = kScatterBlock / 64;
    constexpr int kPcCons = kWaves - kPcProd;
    static_assert(kPcProd % kPcCons == 0, "every consumer serves the same number of producers");
    static_assert(kPcRing % kPcG == 0, "a stage fills whole ring slots");
    __shared__ unsigned long long slice[kBinChunkWords];
    __shared__ unsigned long long live_s[kBinChunkWords / 64 / W];  // the chunk has kBinChunkWords / W sources
    __shared__ unsigned int cov_s[COV ? 64 * W : 1];
    // (the final stat reduction reuses the ring: LDS is 160 KB and the slice takes 144 KB)
    __shared__ __attribute__((aligned(16))) uint32_t ring_slot[kPcProd][kPcRing][64];
    __shared__ uint16_t ring_src[kPcProd][kPcRing][64];  // chunk-local source | 0x8000 = a slot to write
    __shared__ uint32_t prod_cnt[kPcProd], cons_cnt[kPcProd];  // groups handed over / taken, per pair
    if (COV) {
        for (int i = threadIdx.x; i < 64 * W; i += kScatterBlock) cov_s[i] = 0;
    }
    Acc acc;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool producer = wave < kPcProd;
    const int pair = producer ? wave : wave - kPcProd;  // producer index, or the consumer's first producer
    // hand-over counters: relaxed workgroup-scope atomics on LDS (ds_read / ds_write; a generic
    // volatile pointer compiles to flat accesses, which wait for vmcnt(0) as well)
    auto ld_prod = [&](int p) { return __hip_atomic_load(&prod_cnt[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto ld_cons = [&] { return __hip_atomic_load(&cons_cnt[pair], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    const unsigned long long below = (lane == 63 ? ~0ull : ((2ull << lane) - 1)) & ~1ull;  // lanes 1..lane
    auto run = [&](const uint64_t p0_, const uint64_t p1_) {
        // positions fit 32 bits (build_bins: fewer than kNoSlot edges)
        const uint32_t p0 = (uint32_t)p0_, p1 = (uint32_t)p1_, nb = (uint32_t)b.n_binned;
        if (p0 >= p1) return;  // block-uniform; nb >= 1 below
        const uint32_t g0 = p0 >> 6, n_groups = ((p1 - 1) >> 6) - g0 + 1;
        // producer p's groups: g0 + p + kPcProd * i, i < items(p)
        auto items = [&](int p) { return n_groups > (uint32_t)p ? (n_groups - p + kPcProd - 1) / kPcProd : 0u; };
        const uint32_t n_items = items(pair);
        if (producer) {
            const uint32_t n_grp = (nb + 63) >> 6;
            // register sets: loads of stage j+N-1 | run resolution of j+L | hand-over of j
            constexpr int N = kPcSets, L = (kPcSets - 1) / 2;
            static_assert(N >= 3, "load, resolve and hand-over each need a set");
            uint32_t sv[N][kPcG], gr[N][kPcG], rv[N][kPcG], uu[N][kPcG];
            auto load = [&](int set, uint32_t j) {  // stage j = items j*kPcG .. j*kPcG + kPcG - 1
#pragma unroll
                for (int t = 0; t < kPcG; ++t) {
                    const uint32_t i = j * kPcG + t;
                    const uint32_t g = min(g0 + pair + kPcProd * i, n_grp - 1);  // clamped past the end
                    const uint32_t q = g * 64 + lane;
                    sv[set][t] = (uint32_t)__builtin_nontemporal_load(b.cb_src + min(q, nb - 1));
                    gr[set][t] = b.cb_grp[g];
                }
            };
            auto resolve = [&](int set, uint32_t j) {
#pragma unroll
                for (int t = 0; t < kPcG; ++t) {
                    const uint32_t i = j * kPcG + t;
                    const uint32_t g = g0 + pair + kPcProd * i;
                    const uint32_t q = g * 64 + lane;
                    const uint32_t v = i < n_items && q < nb ? sv[set][t] : 0u;  // past the end: no run starts
                    const uint32_t u = v & (kRunStart - 1u);
                    const uint32_t live = (uint32_t)(live_s[u >> 6] >> (u & 63)) & 1u;
                    const uint32_t act = (uint32_t)(i < n_items) & (uint32_t)(q >= p0) & (uint32_t)(q < p1) & live;
                    uu[set][t] = u | (act << 15);
                    const unsigned long long starts = __ballot((v & kRunStart) != 0);
                    const uint32_t run = gr[set][t] + (uint32_t)__popcll(starts & below);
                    rv[set][t] = q + b.cb_run[min(run, (uint32_t)b.n_runs_m1)];  // the slot
                }
            };
            auto hand_over = [&](int set, uint32_t j) {
                const uint32_t i0 = j * kPcG;
                if (i0 >= n_items) return;  // wave-uniform
                while (i0 + kPcG - ld_cons() > (uint32_t)kPcRing) __builtin_amdgcn_s_sleep(2);  // ring full
                asm volatile("" ::: "memory");
#pragma unroll
                for (int t = 0; t < kPcG; ++t) {
                    const uint32_t i = i0 + t;
                    ring_slot[pair][i % kPcRing][lane] = rv[set][t];
                    ring_src[pair][i % kPcRing][lane] = (uint16_t)uu[set][t];
                }
                lds_wait();
                if (lane == 0)
                    __hip_atomic_store(&prod_cnt[pair], min(i0 + kPcG, n_items), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            const uint32_t n_stages = (n_items + kPcG - 1) / kPcG;
#pragma unroll
            for (int k = 0; k < N - 1; ++k) load(k, k);
#pragma unroll
            for (int k = 0; k < L; ++k) resolve(k, k);
            for (uint32_t j = 0;; j += N) {  // sets rotate with no register copies (unrolled: constant indices)
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    load((k + N - 1) % N, j + k + N - 1);
                    resolve((k + L) % N, j + k + L);
                    hand_over(k, j + k);
                    if (j + k + 1 >= n_stages) goto produced;
                }
            }
        produced:;
        } else {
            const uint32_t n_max = items(pair);  // the first producer served has the most items
            for (uint32_t i = 0; i < n_max; ++i) {
                for (int pp = pair; pp < kPcProd; pp += kPcCons) {
                    if (i >= items(pp)) break;  // wave-uniform; later producers have no more items either
                    while (ld_prod(pp) <= i) __builtin_amdgcn_s_sleep(2);  // not handed over yet
                    asm volatile("" ::: "memory");                        // the ring reads stay behind the poll
                    const uint32_t slot = ring_slot[pp][i % kPcRing][lane];
                    const uint32_t su = ring_src[pp][i % kPcRing][lane];
                    uint64_t x[W];
#pragma unroll
                    for (int w = 0; w < W; ++w) x[w] = slice[(uint64_t)(su & (kRunStart - 1u)) * W + w];
                    lds_wait();
                    if (lane == 0)  // the ring slot is free again
                        __hip_atomic_store(&cons_cnt[pp], i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (su & kRunStart) {
#pragma unroll
                        for (int w = 0; w < W; ++w) b.val[(uint64_t)slot * W + w] = x[w];
                    }
                    acc.gathered += (su & kRunStart) ? 1u : 0u;  // slots written (byte accounting)
                }
            }
        }
    };
    auto scatter_unit = [&](const uint64_t ui) {
        const BinUnit un = b.units[ui];
        if (un.p0 >= un.p1 && !un.first) return;  // padding of a row (block-uniform)
        scatter_stage<W, COV>(a, b, un, wd, slice, live_s, cov_s, acc);
        if (threadIdx.x < kPcProd) prod_cnt[threadIdx.x] = cons_cnt[threadIdx.x] = 0;
        __syncthreads();
        run(un.p0, un.p1);
    };
    scatter_rows(b, scatter_unit);
    static_assert(sizeof(ring_slot) >= kWaves * kStatFields * 8, "stat scratch fits the ring");
    __syncthreads();  // the ring is idle
    flush_into<kWaves>(acc, a.st, reinterpret_cast<unsigned long long (*)[kStatFields]>(&ring_slot[0][0][0]));
    if (COV) {
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * W; i += kScatterBlock)
            if (cov_s[i]) atomicAdd(&a.cov[i], (unsigned long long)cov_s[i]);
    }
}

// The source side of a binned round for a bin's peers (their pushes,
// broadcastMessage peer.cpp:310-316) when the scatter leaves it to the apply
// (BinArgs.src_stats = 0): per peer with new words, frontier, traversals,
// deliveries and undelivered sends from its row length (and dead-edge
// counters), digest, covered and coverage of the words -- the same sums
// scatter_stage books, read as three sequential streams (nw, deg, dgone/dmask).
template <int W, int kB>
__device__ __forceinline__ void bin_src_stats(const RoundArgs& a, const BinArgs& b, uint64_t v0, uint32_t nv,
                                              uint32_t wd, unsigned int* cov_s, Acc& acc) {
    const bool cnt = a.dead_mode && a.dgone;
    for (uint32_t i = threadIdx.x; i < nv; i += kB) {
        const uint64_t lv = v0 + i, v = a.begin + lv;
        uint32_t pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint64_t m = a.nw[lv * W + w];
            if (!m) continue;
            pc += (uint32_t)__popcll(m);
            if (w < (int)wd) acc.digest += digest_weight(v * wd + w) * m;
            if (a.cov)
                for (uint64_t x = m; x; x &= x - 1) atomicAdd(&cov_s[w * 64 + __builtin_ctzll(x)], 1u);
        }
        if (!pc) continue;
        acc.frontier++;
        acc.covered += pc;
        const uint64_t d = b.deg[lv];
        const uint32_t dg = cnt ? a.dgone[lv] : 0u, dk = cnt ? a.dmask[lv] : 0u;
        if (!a.dead_mode || cnt) {
            acc.trav += d - dk;
            acc.deliv += (unsigned long long)pc * (d - dg);
            acc.undeliv += (unsigned long long)pc * (dg - dk);
        }
    }
}

// The end of a bin (k_bin_apply, k_bin_apply_runs): handleClient's test-and-set of the bin's peers from the
// LDS accumulator (peer.cpp:277-285): fr = acc & ~seen.  Every seen word a thread tests (and, after a
// deferred push round, a.fold, its pending new word) is loaded before any is used: a loop that loads,
// tests and stores one word per iteration waited a memory round trip per word -- 18 per thread and bin at
// 18432 peers, ≈ 57 bins per CU and launch.  seen is rewritten whole for a tile where any word changes (a
// single-word store into a 64-B sector costs a read-modify-write at the memory); nx is written whole (heavy
// rows: 0 here, OR-ed by k_pull_heavy afterwards).
template <int W, int kWords, int kB>
__device__ __forceinline__ void bin_finish(const RoundArgs& a, uint64_t v0, uint32_t nv,
                                           const unsigned long long* acc_s, Acc& acc, const InjMasks<W>& im) {
    constexpr int kJ = (kWords + kB - 1) / kB;
    const uint32_t n = nv * W, n_pad = (n + 63) & ~63u;
    uint64_t sv[kJ], pv[kJ];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
        const uint32_t i = threadIdx.x + (uint32_t)j * kB;
        sv[j] = i < n ? a.seen[v0 * W + i] : 0ull;
        pv[j] = a.fold && i < n ? a.nw[v0 * W + i] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
        const uint32_t i = threadIdx.x + (uint32_t)j * kB;
        if (i >= n_pad) break;  // wave-uniform
        const bool in = i < n;
        const uint64_t p = pv[j];
        const uint64_t s = sv[j] | p;
        const bool va = in && (!a.dead_mode || bit_alive(a.alive, (uint32_t)(a.begin + v0 + i / W)));  // dead: no receive
        const uint64_t fr = va ? acc_s[i] & im.cur_at(i % W) & ~s : 0ull;
#pragma unroll
        for (int w = 0; w < W; ++w)
            if (i % W == w) acc.fresh_or[w] |= fr;  // (constant register indices)
        if (fr) {  // handleClient: new -> Message-List insert (peer.cpp:281-282)
            acc.fresh += (unsigned long long)__popcll(fr);
            acc.activated++;
        }
        const bool tile = __ballot((fr | p) != 0) != 0ull;
        if (in && tile) a.seen[v0 * W + i] = s | fr;
        if (in) a.nx[v0 * W + i] = fr;
    }
}

// Phase 2: one workgroup per bin folds the bin's slots into an LDS
// accumulator (ds_or_b64), then applies handleClient's test-and-set to the
// bin's peers with plain stores.  A bin none of whose peers can still learn
// anything skips its slots.
template <int W, int kWords, int kB>  // kWords: LDS accumulator words; kB: threads
__global__ __launch_bounds__(kB) void k_bin_apply(RoundArgs a, BinArgs b, uint32_t wd) {
    __shared__ unsigned long long acc_s[kWords];
    __shared__ unsigned int cov_s[64 * W];
    Acc acc;
    const InjMasks<W> im(a);
    const Bin bn = b.bins[blockIdx.x];
    const uint32_t nv = bn.v1 - bn.v0;
    const uint64_t v0 = bn.v0;
    if (!b.src_stats) {
        if (a.cov)
            for (uint32_t i = threadIdx.x; i < 64 * W; i += kB) cov_s[i] = 0;
        __syncthreads();
        bin_src_stats<W, kB>(a, b, v0, nv, wd, cov_s, acc);
    }
    // a.fold: the previous (deferred) push round's receipts are this round's new words and not yet
    // in seen; every peer of the bin (heavy rows included) gets seen |= nw here, before k_pull_heavy
    auto pend = [&](uint32_t i) { return a.fold ? a.nw[v0 * W + i] : 0ull; };
    bool needy = !b.needy_check;
    for (uint32_t i = threadIdx.x; i < nv * W; i += kB) {
        acc_s[i] = 0ull;
        if (!b.needy_check) continue;
        const bool va = !a.dead_mode || bit_alive(a.alive, (uint32_t)(a.begin + v0 + i / W));
        needy |= va && (im.cur_at(i % W) & ~(a.seen[v0 * W + i] | pend(i))) != 0;
    }
    auto cov_out = [&] {
        if (b.src_stats || !a.cov) return;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 64 * W; i += kB)
            if (cov_s[i]) atomicAdd(&a.cov[i], (unsigned long long)cov_s[i]);
    };
    if (!__syncthreads_or(needy)) {
        for (uint32_t i = threadIdx.x; i < nv * W; i += kB) {
            a.nx[v0 * W + i] = 0ull;
            if (const uint64_t p = pend(i)) a.seen[v0 * W + i] |= p;
        }
        flush<kB / 64>(acc, a.st);
        cov_out();
        return;
    }
    if (threadIdx.x == 0) acc.pulled = bn.s1 - bn.s0;  // slots scanned (byte accounting)
    // 8 slots per lane per step: 16 B of bdst, 64*W B of val
    for (uint64_t i = bn.s0 + (uint64_t)threadIdx.x * 8; i < bn.s1; i += (uint64_t)kB * 8) {
        const uint4 dd = *reinterpret_cast<const uint4*>(b.bdst + i);
        uint64_t x[8 * W];
        const uint4* vp = reinterpret_cast<const uint4*>(b.val + i * W);
#pragma unroll
        for (int q = 0; q < 4 * W; ++q) {
            const uint4 y = vp[q];
            x[2 * q] = ((uint64_t)y.y << 32) | y.x;
            x[2 * q + 1] = ((uint64_t)y.w << 32) | y.z;
        }
        const uint32_t dw[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t dl = (dw[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;  // padding slots hold zero words
#pragma unroll
            for (int w = 0; w < W; ++w)
                if (x[k * W + w]) atomicOr(&acc_s[dl * W + w], (unsigned long long)x[k * W + w]);
        }
    }
    __syncthreads();
    bin_finish<W, kWords, kB>(a, v0, nv, acc_s, acc, im);
    flush<kB / 64>(acc, a.st);
    cov_out();
}

// ---------------------------------------------------------------------------
// Streamed binned rounds (the default layout, gossip_bins.hip (d)): the values
// live in cb order, so the scatter is a front-to-back stream and the random
// access moves to the apply, as reads of slot runs (a read of a short run
// costs no read-modify-write of a partly written line).
// ---------------------------------------------------------------------------
// Phase 1: stage each unit's source chunk in LDS (scatter_stage), then
// val[p] = slice[cb_src[p]] for the unit's cb entries, written front to back
// in 16-B pieces with consecutive lanes on consecutive pieces, so every store
// instruction covers 1 KB of whole lines (W = 1: a piece holds two entries;
// W >= 2: an entry is W / 2 pieces).  An earlier mapping -- 8 entries per lane
// as four 16-B stores 64 B apart -- sent every lane's store to L2 as a request
// of its own (config 4: 9.7e8 write requests per launch, the TA ~92 % busy).
// Every entry is written every binned round.
// kCW / kSB: the LDS slice's words and the block's threads -- 18432 / 1024 (one workgroup per CU), or
// 4096 / 256 for layouts of small chunks (several workgroups per CU: a unit's staging and its short entry
// stream are a few dependent round trips, which one workgroup per CU leaves exposed)
template <int W, bool COV, int kCW = (int)kBinChunkWords, int kSB = kScatterBlock>
__global__ __launch_bounds__(kSB) void k_bin_stream(RoundArgs a, BinArgs b, uint32_t wd) {
    constexpr int kWaves = kSB / 64;
    constexpr int kPW = W == 1 ? 1 : W / 2;  // pieces per entry (W >= 2)
    constexpr int kU = 4;                    // pieces per lane in flight
    __shared__ unsigned long long slice[kCW];
    __shared__ unsigned long long live_s[kCW / 64 / W];
    __shared__ unsigned int cov_s[COV ? 64 * W : 1];
    if (COV) {
        for (int i = threadIdx.x; i < 64 * W; i += kSB) cov_s[i] = 0;
    }
    Acc acc;
    auto unit = [&](const uint64_t ui) {
        const BinUnit un = b.units[ui];
        if (un.p0 >= un.p1 && !un.first) return;  // padding of a row (block-uniform)
        // b.direct (a vertex block of a partitioned run): a chunk with no owned source books no stats, and
        // its few entries (1/P of a whole overlay's) read their words straight from the gather buffer (the
        // chunk's 144 KB stay in L2 after the first touch) instead of paying the chunk's staging
        const uint64_t vb = bin_chunk_vb(b, un.c);
        // (b.split_direct: a split chunk's later units, whose first unit stages the chunk and books its stats)
        const bool direct = (b.direct && !(vb < a.end && bin_chunk_ve(b, un.c, a.n_src) > a.begin)) ||
                            (b.split_direct && !un.first);  // block-uniform
        const uint64_t ve = bin_chunk_ve(b, un.c, a.n_src);  // (the checked build's bound of a source)
        (void)ve;
        if (!direct) {
            scatter_stage<W, COV, kCW, kSB>(a, b, un, wd, slice, live_s, cov_s, acc);
            __syncthreads();
        }
        if (un.p0 >= un.p1) return;
        acc.gathered += threadIdx.x == 0 ? un.p1 - un.p0 : 0;  // slots written (byte accounting)
        // the word source as a compile-time choice (a select would issue both loads)
        auto pieces = [&](auto dir) {
        constexpr bool kDirect = decltype(dir)::value;
        auto word = [&](uint64_t u) {
            return kDirect ? a.nw_src[GOSSIP_IDX(a, kChkStreamDirect, vb * W + u, ve * W)]
                           : (uint64_t)slice[GOSSIP_IDX(a, kChkStreamSlice, u, (ve - vb) * W)];
        };
        // Software-pipelined: the cb entries of a lane's next batch are loaded before the current batch's
        // words are stored.  vmcnt counts loads and stores in issue order, so a batch whose loads follow the
        // previous batch's stores waits for those stores' acknowledgements as well; issued one batch ahead,
        // the loads only wait behind one batch of stores.  (Unpipelined, and with the scheduler free to sink
        // the first piece's LDS read and its wait between the loads, a wave had about one batch in flight.)
        constexpr uint64_t kStep = (uint64_t)kSB * kU;
        if (W == 1) {
            // piece k = entries 2k, 2k + 1 (cb_src read as one u32: 4-B aligned)
            const uint64_t k0 = un.p0 >> 1, k1 = (un.p1 + 1) >> 1;
            const uint32_t* cb2 = reinterpret_cast<const uint32_t*>(b.cb_src);
            auto load = [&](uint64_t kb, uint32_t (&o)[kU]) {
#pragma unroll
                for (int j = 0; j < kU; ++j)
                    o[j] = __builtin_nontemporal_load(cb2 + min(kb + (uint64_t)j * kSB, k1 - 1));
            };
            uint32_t sv[kU], nv[kU];
            uint64_t kb = k0 + threadIdx.x;
            if (kb < k1) load(kb, sv);
            for (; kb < k1; kb += kStep) {
                load(kb + kStep, nv);  // (unconditional: clamped, and one wait count on every path)
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < kU; ++j) {
                    const uint64_t k = kb + (uint64_t)j * kSB;
                    if (k >= k1) break;
                    const uint64_t e = 2 * k;
                    // A piece cut by the unit's ends holds an entry of the neighbouring unit in cb order --
                    // another chunk's local source id (e = p0 - 1 when p0 is odd, e + 1 = p1 when p1 is odd;
                    // k in [k0, k1) keeps e + 1 >= p0 and e < p1).  Staged, that id only indexes the LDS slice
                    // (any chunk-local id is < kCW) and its word is dropped below; read directly from the
                    // gather buffer it addressed up to a chunk past this chunk's sources: past the buffer's
                    // end for the last chunk of the ids (the illegal access of test_group_dense_exchange_
                    // forms_equal_oracle[3-100003-3-direct], round 5).  Such an entry reads source 0 instead.
                    constexpr bool kMask = kDirect || kChecked;
                    const uint32_t u0 = kMask && e < un.p0 ? 0u : sv[j] & (kRunStart - 1u);
                    const uint32_t u1 = kMask && e + 1 >= un.p1 ? 0u : (sv[j] >> 16) & (kRunStart - 1u);
                    const uint64_t x0 = word(u0);
                    const uint64_t x1 = word(u1);
                    if (e >= un.p0 && e + 2 <= un.p1) {
                        u64x2 y;
                        y.x = x0;
                        y.y = x1;
                        reinterpret_cast<u64x2*>(b.val)[k] = y;
                    } else {  // a piece cut by the unit's ends
                        if (e >= un.p0 && e < un.p1) b.val[e] = x0;
                        if (e + 1 >= un.p0 && e + 1 < un.p1) b.val[e + 1] = x1;
                    }
                }
#pragma unroll
                for (int j = 0; j < kU; ++j) sv[j] = nv[j];
            }
        } else {
            const uint64_t k0 = un.p0 * kPW, k1 = un.p1 * kPW;
            auto load = [&](uint64_t kb, uint32_t (&o)[kU]) {
#pragma unroll
                for (int j = 0; j < kU; ++j) o[j] = b.cb_src[min(kb + (uint64_t)j * kSB, k1 - 1) / kPW];
            };
            uint32_t sv[kU], nv[kU];
            uint64_t kb = k0 + threadIdx.x;
            if (kb < k1) load(kb, sv);
            for (; kb < k1; kb += kStep) {
                load(kb + kStep, nv);  // (unconditional: clamped, and one wait count on every path)
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < kU; ++j) {
                    const uint64_t k = kb + (uint64_t)j * kSB;
                    if (k >= k1) break;
                    const uint32_t u = sv[j] & (kRunStart - 1u);
                    const uint32_t w0 = (uint32_t)(k % kPW) * 2;
                    u64x2 y;
                    y.x = word((uint64_t)u * W + w0);
                    y.y = word((uint64_t)u * W + w0 + 1);
                    reinterpret_cast<u64x2*>(b.val)[k] = y;  // entry k / kPW, words w0, w0 + 1
                }
#pragma unroll
                for (int j = 0; j < kU; ++j) sv[j] = nv[j];
            }
        }
        };
        if (direct) pieces(std::true_type{});
        else pieces(std::false_type{});
    };
    scatter_rows(b, unit);
    flush<kWaves>(acc, a.st);
    if (COV) {
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * W; i += kSB)
            if (cov_s[i]) atomicAdd(&a.cov[i], (unsigned long long)cov_s[i]);
    }
}

// Phase 2 (streamed layout): the bin's slots, each folded into the LDS
// accumulator of its destination.  A slot's value sits at its cb position
// q - ap_run[run], so each 64-slot group is a chain of three dependent loads:
// bdst (destination, bit 15 = a run starts here) with the group's count of
// earlier runs (ap_grp) -> the run's offset (ap_run, the run from a ballot of
// the flags) -> the value.  Unpipelined that chain made the apply latency-bound
// (config 4: 12.3 ms per launch for ~20 GB).  Here every wave keeps kS stages
// of kG groups in flight: in iteration i it issues the first loads of stage
// i+3, the offsets of i+2, the values of i+1 and folds the values of i into
// the LDS accumulator (ds_or_b64), rotating kS register sets without copies
// (loop unrolled by kS) so each wait is for loads issued an iteration earlier.
// Lanes past the bin or its groups load clamped addresses and fold nothing.
// The blocks that share an XCD (blockIdx % 8) apply consecutive bins, which read neighbouring runs of every
// chunk (rows of kApplyRow bins, dealt round-robin to the XCD groups; see the end of the kernel).  (Round 3
// measured a persistent launch that also kept each row's bins in step with a bounded per-row sync: slower,
// 10.3-11.5 against 9.6-9.8 ms.  The persistent launch here has no sync between blocks.)  The end of each
// bin is k_bin_apply's: test-and-set of its peers with plain stores (and the fold of a deferred push
// round's words, a.fold).
// Pipeline shape (kPipe, W = 1 only; others use 0): groups per stage kG, and how many iterations ahead
// each load is issued -- bdst + ap_grp LA, ap_run LB, val LC (LA > LB > LC >= 1), kS = LA + 1 register sets.
// kSeq (shapes 4-6, round 6): a wave's groups are one contiguous range of the bin instead of every kWaves-th
// group, so the runs that start before a group are the wave's running count of run-start flags (a scalar: the
// ballot's popcount), ap_grp is read once per wave and bin, and the group indices are scalars.  Strided, every
// group's ap_grp word was a vector load and a register per stage, and the destinations came only one iteration
// ahead of the run lookup that needs them (LA - LB = 1 in shapes 0, 2, 3).
template <int W, int kPipe> struct ApplyPipe {
    static constexpr int kG = W == 1 ? 4 : W == 2 ? 2 : 1, LA = 3, LB = 2, LC = 1;
    static constexpr bool kSeq = false;
};
template <> struct ApplyPipe<1, 1> { static constexpr int kG = 2, LA = 5, LB = 3, LC = 1; static constexpr bool kSeq = false; };
template <> struct ApplyPipe<1, 2> { static constexpr int kG = 2, LA = 5, LB = 4, LC = 2; static constexpr bool kSeq = false; };
template <> struct ApplyPipe<1, 3> { static constexpr int kG = 2, LA = 6, LB = 5, LC = 3; static constexpr bool kSeq = false; };
template <> struct ApplyPipe<1, 4> { static constexpr int kG = 2, LA = 5, LB = 4, LC = 2; static constexpr bool kSeq = true; };
template <> struct ApplyPipe<1, 5> { static constexpr int kG = 2, LA = 6, LB = 4, LC = 2; static constexpr bool kSeq = true; };
template <> struct ApplyPipe<1, 6> { static constexpr int kG = 2, LA = 7, LB = 5, LC = 3; static constexpr bool kSeq = true; };
template <> struct ApplyPipe<1, 7> { static constexpr int kG = 2, LA = 8, LB = 5, LC = 2; static constexpr bool kSeq = true; };
template <> struct ApplyPipe<1, 8> { static constexpr int kG = 2, LA = 7, LB = 4, LC = 2; static constexpr bool kSeq = true; };
template <> struct ApplyPipe<1, 9> { static constexpr int kG = 3, LA = 6, LB = 4, LC = 2; static constexpr bool kSeq = true; };
template <> struct ApplyPipe<1, 10> { static constexpr int kG = 3, LA = 5, LB = 3, LC = 1; static constexpr bool kSeq = true; };

template <int W, int kWords, int kB, int kPipe = 0, bool kProbe = false>  // kProbe: apply_probe's clocks
__global__ __launch_bounds__(kB) void k_bin_apply_runs(RoundArgs a, BinArgs b, uint32_t wd) {
    constexpr int kWaves = kB / 64;
    constexpr int kG = ApplyPipe<W, kPipe>::kG;                      // groups per stage
    constexpr int LA = ApplyPipe<W, kPipe>::LA, LB = ApplyPipe<W, kPipe>::LB, LC = ApplyPipe<W, kPipe>::LC;
    constexpr int kS = LA + 1;                                        // stages in flight
    constexpr bool kSeq = ApplyPipe<W, kPipe>::kSeq;
    static_assert(LA > LB && LB > LC && LC >= 1, "load lags");
    __shared__ unsigned long long acc_s[kWords];
    __shared__ unsigned int cov_s[64 * W];
    Acc acc;
    const InjMasks<W> im(a);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);  // (the same value, known wave-uniform)
    if (!b.src_stats && a.cov)
        for (uint32_t i = threadIdx.x; i < 64 * W; i += kB) cov_s[i] = 0;
    const unsigned long long upto = lane == 63 ? ~0ull : (2ull << lane) - 1;  // lanes 0..lane
    const uint32_t run_max = (uint32_t)b.n_runs_m1;
    const uint64_t t_block = kProbe ? wall_clock64() : 0;  // apply_probe: the block's lifetime
    auto apply_bin = [&](const uint32_t bi) {
        const Bin bn = b.bins[bi];
        const uint32_t nv = bn.v1 - bn.v0;
        const uint64_t v0 = bn.v0;
        __syncthreads();  // the previous bin is done with acc_s (and cov_s is initialised)
        // apply_probe (diagnostics): thread 0 clocks the phases, with a barrier after each one
        uint64_t tk = kProbe ? wall_clock64() : 0;
        auto tick = [&](int slot) {
            if (!kProbe) return;
            __syncthreads();
            if (threadIdx.x == 0) {
                const uint64_t t = wall_clock64();
                atomicAdd(&b.probe[slot], (unsigned long long)(t - tk));
                tk = t;
            }
        };
        if (!b.src_stats) bin_src_stats<W, kB>(a, b, v0, nv, wd, cov_s, acc);
        tick(kProbeSrc);
        auto pend = [&](uint32_t i) { return a.fold ? a.nw[v0 * W + i] : 0ull; };
        bool needy = !b.needy_check;
        for (uint32_t i = threadIdx.x; i < nv * W; i += kB) {
            acc_s[i] = 0ull;
            if (!b.needy_check) continue;
            const bool va = !a.dead_mode || bit_alive(a.alive, (uint32_t)(a.begin + v0 + i / W));
            needy |= va && (im.cur_at(i % W) & ~(a.seen[v0 * W + i] | pend(i))) != 0;
        }
        tick(kProbeInit);
        if (kProbe && threadIdx.x == 0) {
            atomicAdd(&b.probe[kProbeBins], 1ull);
            atomicAdd(&b.probe[kProbeSlotsN], (unsigned long long)(bn.s1 - bn.s0));
        }
        if (!__syncthreads_or(needy)) {
            for (uint32_t i = threadIdx.x; i < nv * W; i += kB) {
                a.nx[v0 * W + i] = 0ull;
                if (const uint64_t p = pend(i)) a.seen[v0 * W + i] |= p;
            }
            return;
        }
        if (threadIdx.x == 0) acc.pulled += bn.s1 - bn.s0;  // slots scanned (byte accounting)
        if (bn.s1 > bn.s0) {
            const uint64_t g_lo = bn.s0 >> 6, g_hi = ((bn.s1 - 1) >> 6) + 1;
            // this wave's groups: g_lo + wave + kWaves * t, t < n_t (kSeq: g_lo + t_lo + t, t < n_t)
            const uint64_t n_g = g_hi - g_lo;
            const uint64_t t_lo = kSeq ? n_g * (uint32_t)wave_u / kWaves : 0;
            const uint32_t n_t = kSeq ? (uint32_t)(n_g * ((uint32_t)wave_u + 1) / kWaves - t_lo)
                                 : n_g > (uint64_t)wave ? (uint32_t)((n_g - wave + kWaves - 1) / kWaves) : 0u;
            const uint32_t n_it = (n_t + kG - 1) / kG;
            uint32_t d[kS][kG], gr[kS][kG], off[kS][kG];
            uint64_t x[kS][kG][W];
            // kSeq: the runs that start before the wave's next group (scalar)
            uint32_t rc = kSeq && n_t ? __builtin_amdgcn_readfirstlane(b.ap_grp[g_lo + t_lo]) : 0u;
            auto grp = [&](uint32_t i, int j) {
                return kSeq ? g_lo + t_lo + (uint64_t)(i * kG + j) : g_lo + wave + (uint64_t)kWaves * (i * kG + j);
            };
            auto valid = [&](uint32_t i, int j) {  // lane's slot belongs to the bin (and to this wave's groups)
                const uint64_t g = grp(i, j), q = g * 64 + lane;
                return i * kG + j < n_t && q >= bn.s0 && q < bn.s1;
            };
            auto ld_a = [&](int st, uint32_t i) {  // bdst and the group's earlier runs (ap_grp holds whole groups)
#pragma unroll
                for (int j = 0; j < kG; ++j) {
                    const uint64_t g = min(grp(i, j), g_hi - 1);
                    // kSeq: the raw 32-bit word of the lane's slot pair, its half taken where it is used.  (A u16
                    // load whose flag test the compiler narrowed to a 16-bit compare kept a separate zero-extension
                    // in the load's own iteration, which waited for the load there: every iteration waited for its
                    // own destinations, whatever the lags.)
                    if (kSeq) d[st][j] = reinterpret_cast<const uint32_t*>(b.bdst)[(g * 64 + lane) >> 1];
                    else d[st][j] = b.bdst[g * 64 + lane];
                    if (!kSeq) gr[st][j] = b.ap_grp[g];
                }
            };
            auto ld_b = [&](int st, uint32_t i) {  // the run of each slot -> its offset
#pragma unroll
                for (int j = 0; j < kG; ++j) {
                    if (kSeq) d[st][j] = (d[st][j] >> ((lane & 1) * 16)) & 0xFFFFu;  // the lane's slot
                    const unsigned long long fl = __ballot((d[st][j] & kRunStart) != 0);
                    // a slot of the bin lies in a run that starts at or before it (run >= 0); others clamp
                    // (kSeq: stages come here in order, so rc counts the runs before group (i, j); a clamped
                    // group past the wave's range adds garbage that only such groups see)
                    const uint32_t g0 = kSeq ? rc : gr[st][j];
                    if (kSeq) rc += (uint32_t)__popcll(fl);
                    const uint32_t run = min(g0 + (uint32_t)__popcll(fl & upto) - 1u, run_max);
                    off[st][j] = b.ap_run[run];
                }
            };
            auto ld_c = [&](int st, uint32_t i) {  // the values
#pragma unroll
                for (int j = 0; j < kG; ++j) {
                    const uint64_t q = grp(i, j) * 64 + lane;
                    const uint64_t p = valid(i, j) ? (uint64_t)((uint32_t)q - off[st][j]) : 0;  // the slot's cb position
#pragma unroll
                    for (int w = 0; w < W; ++w) x[st][j][w] = b.val[GOSSIP_IDX(a, kChkApplyVal, p * W + w, b.n_binned * W)];
                }
            };
            auto fold = [&](int st, uint32_t i) {
#pragma unroll
                for (int j = 0; j < kG; ++j) {
                    if (!valid(i, j)) continue;
                    const uint32_t dl = d[st][j] & (kRunStart - 1u);
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        if (x[st][j][w]) atomicOr(&acc_s[dl * W + w], (unsigned long long)x[st][j][w]);  // ds_or_b64
                }
            };
            // prologue: the loads of stages 0 .. LA - 1 issued as the loop would have issued them
#pragma unroll
            for (int t = -LA; t < 0; ++t) {
                if (t + LA >= 0) ld_a((t + LA) % kS, (uint32_t)(t + LA));
                if (t + LB >= 0) ld_b((t + LB) % kS, (uint32_t)(t + LB));
                if (t + LC >= 0) ld_c((t + LC) % kS, (uint32_t)(t + LC));
            }
            for (uint32_t i0 = 0; i0 < n_it; i0 += kS) {
#pragma unroll
                for (int k = 0; k < kS; ++k) {
                    const uint32_t i = i0 + k;
                    if (i >= n_it) break;  // wave-uniform
                    ld_a((k + LA) % kS, i + LA);
                    ld_b((k + LB) % kS, i + LB);
                    ld_c((k + LC) % kS, i + LC);
                    fold(k, i);
                }
            }
        }
        __syncthreads();
        tick(kProbeSlots);
        bin_finish<W, kWords, kB>(a, v0, nv, acc_s, acc, im);
        tick(kProbeFinish);
    };
    // Rows of kApplyRow consecutive bins, row r to XCD group r % 8 (the blocks x + 8 i): member j of group x
    // applies bin (j / kApplyRow * 8 + x) * kApplyRow + j % kApplyRow.  The blocks resident on an XCD apply
    // consecutive bins, whose runs sit next to each other in every chunk (lines shared at run ends come
    // through that XCD's L2 once), and every group gets every eighth row.  (Measured at config 4, per XCD
    // group: contiguous eighths of the bins took 7.9 ms for the first and 5.5 ms for the last -- bins of
    // low peer ids hold more, shorter runs -- and the launch lasted as long as the first; single bins dealt
    // round-robin balanced the groups but every bin's slots took 114 instead of 88 us.)  With one block per
    // bin, member j is blockIdx.x / 8; persistent (b.work), the group's resident blocks take j from its
    // counter, and a block flushes its stats once.
    const uint32_t xg = blockIdx.x & 7;
    auto bin_of = [&](uint64_t j) { return ((j / kApplyRow) * 8 + xg) * kApplyRow + j % kApplyRow; };
    if (b.work) {
        __shared__ uint32_t next_s;
        while (true) {
            if (threadIdx.x == 0) next_s = atomicAdd(&b.work[xg], 1u);
            __syncthreads();  // (every thread read the previous value before apply_bin's first barrier)
            const uint64_t bi = bin_of(next_s);
            if (bi >= b.n_bins) break;  // block-uniform; later j only map further
            apply_bin((uint32_t)bi);
        }
    } else {
        const uint64_t bi = bin_of(blockIdx.x >> 3);
        if (bi < b.n_bins) apply_bin((uint32_t)bi);
    }
    if (kProbe && threadIdx.x == 0) {
        const unsigned long long life = wall_clock64() - t_block;
        atomicAdd(&b.probe[kProbeBlock], life);
        atomicAdd(&b.probe[kProbeXcd + xg], life);
        atomicAdd(&b.probe[kProbeBlocks], 1ull);
    }
    flush<kWaves>(acc, a.st);
    if (!b.src_stats && a.cov) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 64 * W; i += kB)
            if (cov_s[i]) atomicAdd(&a.cov[i], (unsigned long long)cov_s[i]);
    }
}

// ---------------------------------------------------------------------------
// Source side of a dense round with dead peers (broadcastMessage,
// peer.cpp:310-316): every unmasked out-edge of a frontier peer is a
// traversal, a delivery to a live target and an undelivered send to a dead
// one.  Reads only; the receive side is the pull / binned kernels'.
// ---------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(kBlock) void k_src_count(RoundArgs a) {
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t n_tiles = (a.n_local + 63) >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); t < n_tiles; t += nwaves) {
        const uint64_t v = (t << 6) + lane;
        uint32_t pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) pc += v < a.n_local ? (uint32_t)__popcll(a.nw[v * W + w]) : 0u;
        if (!__any(pc != 0)) continue;
        uint32_t deg = 0;
        uint64_t rb = 0;
        if (pc) {
            rb = a.rp[v];
            const uint64_t d = a.rp[v + 1] - rb;
            deg = d <= a.heavy ? (uint32_t)d : 0u;
        }
        tile_edges(deg, rb, [&](int s, bool valid, uint64_t e) {
            const uint32_t pcs = __shfl(pc, s);
            if (!valid) return;
            const uint32_t c = a.col[e];
            if (c & kMaskedEdge) return;
            acc.trav++;
            if (bit_alive(a.alive, c)) acc.deliv += pcs;
            else acc.undeliv += pcs;
        });
    }
    // heavy rows: one wave per chunk
    for (uint64_t ci = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); ci < a.n_chunks; ci += nwaves) {
        const HeavyChunk ch = a.chunks[ci];
        uint32_t pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) pc += (uint32_t)__popcll(a.nw[(uint64_t)ch.v * W + w]);
        if (!pc) continue;
        for (uint64_t e = ch.e0 + lane; e < ch.e1; e += 64) {
            const uint32_t c = a.col[e];
            if (c & kMaskedEdge) continue;
            acc.trav++;
            if (bit_alive(a.alive, c)) acc.deliv += pc;
            else acc.undeliv += pc;
        }
    }
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// liveness (pingLoop peer.cpp:328-346 -> handleDeadPeer :383-397 ->
// SeedNode::handleDeadNode seed.cpp:158-167)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ping_edge(const RoundArgs& a, bool valid, uint64_t e, bool& emit, uint32_t& dead,
                                          unsigned long long& checked) {
    emit = false;
    dead = 0;
    if (!valid) return;
    const uint32_t c = a.col[e];
    if (c & kMaskedEdge) return;
    checked++;
    if (bit_alive(a.alive, c)) {  // ping ok: failedAttempts = 0 (:340-341)
        if (a.miss[e]) a.miss[e] = 0;
        return;
    }
    uint32_t mm = a.miss[e];
    if (mm < 255) ++mm;  // failedAttempts++ (:336)
    a.miss[e] = (uint8_t)mm;
    if (mm >= a.max_missed) {  // >= 3 -> dead (:337)
        a.col[e] = c | kMaskedEdge;
        emit = true;
        dead = c;
    }
}

// Dead-node reports + registry removal.  Reports are staged per wave in LDS
// and appended with one global atomic per kRepStage entries: a per-batch
// append atomic on the single report counter serialised (~9 ns each) and cost
// ~30 ms per ping round at config 5 (2^26 peers, ~10^7 reports per round).
constexpr int kRepStage = 256;  // staged reports per wave

struct RepStage {
    DeadReport* buf;  // this wave's kRepStage LDS entries
    uint32_t n;       // staged (wave-uniform)
};

__device__ __forceinline__ void flush_reports(const RoundArgs& a, RepStage& rs) {
    if (!rs.n) return;
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(a.n_reports, (unsigned long long)rs.n);
    base = __shfl(base, 0);
    for (uint32_t i = lane; i < rs.n; i += 64)
        if (base + i < a.report_cap) a.reports[base + i] = rs.buf[i];
    rs.n = 0;
}

__device__ __forceinline__ void emit_reports(const RoundArgs& a, bool emit, uint32_t reporter, uint32_t dead,
                                             Acc& acc, RepStage& rs) {
    const unsigned long long mask = __ballot(emit);
    if (!mask) return;
    // one registry atomic per run of emitting lanes reporting the same peer (the
    // in-edges of one dead peer sit in consecutive lanes of a row walk)
    const int lane = threadIdx.x & 63;
    const unsigned long long below = mask & ((1ull << lane) - 1ull);
    const int pl = below ? 63 - __builtin_clzll(below) : lane;
    const uint32_t prev_dead = __shfl(dead, pl);
    if (emit) {
        rs.buf[rs.n + lane_rank(mask)] = DeadReport{a.round, reporter, dead};
        acc.reports++;
        if (pl == lane || prev_dead != dead) {
            const uint32_t bit = 1u << (dead & 31);
            const uint32_t old = atomicAnd(&a.registered[dead >> 5], ~bit);
            if (old & bit) acc.removals++;  // peerList.erase > 0 (seed.cpp:162)
        }
    }
    rs.n += (uint32_t)__popcll(mask);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (rs.n > kRepStage - 64) flush_reports(a, rs);
}

#define GOSSIP_REP_STAGE                                                    \
    __shared__ DeadReport rep_lds[kWavesPerBlock][kRepStage];               \
    RepStage rs{rep_lds[threadIdx.x >> 6], 0u}

__global__ __launch_bounds__(kBlock) void k_liveness_light(RoundArgs a) {
    GOSSIP_REP_STAGE;
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t n_tiles = (a.n_local + 63) >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); t < n_tiles; t += nwaves) {
        const uint64_t v = (t << 6) + lane;
        const bool act = v < a.n_local && bit_alive(a.alive, (uint32_t)(a.begin + v));
        if (!__any(act)) continue;
        uint32_t deg = 0;
        uint64_t rb = 0;
        if (act) {
            rb = a.rp[v];
            const uint64_t d = a.rp[v + 1] - rb;
            deg = d <= a.heavy ? (uint32_t)d : 0u;
        }
        const uint32_t tile_base = (uint32_t)(a.begin + (t << 6));
        tile_edges(deg, rb, [&](int s, bool valid, uint64_t e) {
            bool emit;
            uint32_t dead;
            ping_edge(a, valid, e, emit, dead, acc.checked);
            emit_reports(a, emit, tile_base + (uint32_t)s, dead, acc, rs);
        });
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    flush_reports(a, rs);
    flush(acc, a.st);
}

__global__ __launch_bounds__(kBlock) void k_liveness_heavy(RoundArgs a) {
    GOSSIP_REP_STAGE;
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t ci = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); ci < a.n_chunks; ci += nwaves) {
        const HeavyChunk ch = a.chunks[ci];
        const uint32_t u = (uint32_t)(a.begin + ch.v);
        if (!bit_alive(a.alive, u)) continue;
        for (uint64_t base = ch.e0; base < ch.e1; base += 64) {
            const uint64_t e = base + lane;
            bool emit;
            uint32_t dead;
            ping_edge(a, e < ch.e1, e, emit, dead, acc.checked);
            emit_reports(a, emit, u, dead, acc, rs);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    flush_reports(a, rs);
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// Closed-form liveness (single partition, symmetric overlay, no rejoin).
// Deaths are permanent, so an edge u->v misses exactly at the ping rounds from
// v's death on while u is alive: every alive in-neighbour of v reaches
// max_missed at the same ping round p*(v) -- the max_missed-th ping round at or
// after v's death -- and a miss counter per edge carries no information.  A
// ping round then only visits the in-edges of the peers whose p* it is (by
// symmetry, their own rows), instead of pinging every edge of every alive
// peer: same masks, reports and registry removals as pingLoop's counters
// (peer.cpp:328-346, handleDeadPeer :383-397, seed.cpp:158-167).
// The same death rounds keep two per-source counters -- dgone (out-edges to
// peers that died) and dmask (out-edges masked) -- from which the source side
// of a dense round follows without an alive test per edge:
// traversals = deg - dmask, undelivered = pc (dgone - dmask), deliveries =
// pc (deg - dgone).
// ---------------------------------------------------------------------------

// position of c in u's sorted row (mask bits stripped), or ~0
__device__ __forceinline__ uint64_t find_in_row(const RoundArgs& a, uint64_t u, uint32_t c) {
    uint64_t lo = a.rp[u], hi = a.rp[u + 1];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((a.col[mid] & ~kMaskedEdge) < c) lo = mid + 1;
        else hi = mid;
    }
    return lo < a.rp[u + 1] && (a.col[lo] & ~kMaskedEdge) == c ? lo : ~0ull;
}

// Row walks over the symmetric overlay: for each selected row v, each entry
// e (v -> u) stands for the in-edge u -> v, found at rev[e] in u's row.
enum : int {
    kRowsDead = 0,  // v died this round: one more out-edge of u points at a dead peer (dgone[u]++)
    kRowsLive = 1,  // ping round, v's p* is now: alive u masks u -> v, counts it (dmask[u]++) and reports v
    kRowsRev = 2,   // every row: rev[e] = position of v in u's row (once per overlay)
};

template <int MODE>
__device__ __forceinline__ void row_entry(const RoundArgs& a, bool valid, uint64_t e, uint32_t v, bool& emit,
                                          uint32_t& reporter, Acc& acc) {
    emit = false;
    if (!valid) return;
    const uint32_t u = a.col[e] & ~kMaskedEdge;
    reporter = u;
    if (MODE == kRowsDead) {
        atomicAdd(&a.dgone[u - a.begin], 1u);
    } else if (MODE == kRowsRev) {
        a.rev[e] = (uint32_t)find_in_row(a, u - a.begin, v);
    } else {
        acc.checked++;
        if (!bit_alive(a.alive, u)) return;  // a dead reporter stopped pinging before its count reached max_missed
        const uint64_t f = a.rev[e];
        if (a.col[f] & kMaskedEdge) return;
        a.col[f] = v | kMaskedEdge;  // connectedPeers.erase (peer.cpp:388)
        atomicAdd(&a.dmask[u - a.begin], 1u);
        emit = true;
    }
}

template <int MODE>
__device__ __forceinline__ bool row_selected(const RoundArgs& a, uint64_t lv, uint32_t lo, uint32_t hi) {
    if (MODE == kRowsRev) return true;
    const uint32_t d = a.death_r[lv];
    return d != 0xFFFFu && d >= lo && d <= hi;
}

// light rows (one wave per 64-peer tile, edge-space expansion)
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_rows_light(RoundArgs a, uint32_t lo, uint32_t hi) {
    GOSSIP_REP_STAGE;
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t n_tiles = (a.n_local + 63) >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    // (a strided sweep: the death round of the tile after next is loaded ahead)
    auto death = [&](uint64_t v) { return MODE != kRowsRev && v < a.n_local ? (uint32_t)a.death_r[v] : 0xFFFFu; };
    uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    uint32_t dn = death((t << 6) + lane);
    for (; t < n_tiles; t += nwaves) {
        const uint64_t v = (t << 6) + lane;
        const uint32_t d = dn;
        dn = death(((t + nwaves) << 6) + lane);
        const bool act = v < a.n_local && (MODE == kRowsRev || (d != 0xFFFFu && d >= lo && d <= hi));
        if (!__any(act)) continue;
        uint32_t deg = 0;
        uint64_t rb = 0;
        if (act) {
            rb = a.rp[v];
            const uint64_t d = a.rp[v + 1] - rb;
            deg = d <= a.heavy ? (uint32_t)d : 0u;
        }
        const uint32_t tile_base = (uint32_t)(a.begin + (t << 6));
        tile_edges(deg, rb, [&](int s, bool valid, uint64_t e) {
            bool emit;
            uint32_t u = 0;
            const uint32_t dv = tile_base + (uint32_t)s;
            row_entry<MODE>(a, valid, e, dv, emit, u, acc);
            if (MODE == kRowsLive) emit_reports(a, emit, u, dv, acc, rs);
        });
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (MODE == kRowsLive) flush_reports(a, rs);
    flush(acc, a.st);
}

// heavy rows (one wave per 1024-edge chunk)
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_rows_heavy(RoundArgs a, uint32_t lo, uint32_t hi) {
    GOSSIP_REP_STAGE;
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t ci = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); ci < a.n_chunks; ci += nwaves) {
        const HeavyChunk ch = a.chunks[ci];
        if (!row_selected<MODE>(a, ch.v, lo, hi)) continue;
        const uint32_t dv = (uint32_t)(a.begin + ch.v);
        for (uint64_t base = ch.e0; base < ch.e1; base += 64) {
            const uint64_t e = base + lane;
            bool emit;
            uint32_t u = 0;
            row_entry<MODE>(a, e < ch.e1, e, dv, emit, u, acc);
            if (MODE == kRowsLive) emit_reports(a, emit, u, dv, acc, rs);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (MODE == kRowsLive) flush_reports(a, rs);
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// re-bootstrap after a death: handleDeadPeer
// (peer.cpp:398-404) re-registers with the seeds and runs
// selectAndConnectPeers (:214-253) on their lists; the new connectedPeers
// entries live in per-peer overflow rows (ex_col, up to ex_cap each).
// ---------------------------------------------------------------------------
// one thread per owned peer; the wave runs max(ex_cnt) iterations so that the
// report ballot is wave-uniform
__global__ __launch_bounds__(kBlock) void k_liveness_extra(RoundArgs a) {
    GOSSIP_REP_STAGE;
    Acc acc;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t n_pad = (a.n_local + 63) & ~63ull;
    for (uint64_t u = (uint64_t)blockIdx.x * kBlock + threadIdx.x; u < n_pad; u += stride) {
        const bool vu = u < a.n_local && bit_alive(a.alive, (uint32_t)(a.begin + u));
        const uint32_t cnt = vu ? a.ex_cnt[u] : 0u;
        uint32_t kmax = cnt;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, off));
        for (uint32_t k = 0; k < kmax; ++k) {
            bool emit = false;
            uint32_t dead = 0;
            if (k < cnt) {
                const uint64_t x = u * a.ex_cap + k;
                const uint32_t c = a.ex_col[x];
                if (!(c & kMaskedEdge)) {
                    acc.checked++;
                    if (bit_alive(a.alive, c)) {  // ping ok (peer.cpp:340-341)
                        if (a.ex_miss[x]) a.ex_miss[x] = 0;
                    } else {
                        uint32_t mm = a.ex_miss[x];
                        if (mm < 255) ++mm;  // failedAttempts++ (:336)
                        a.ex_miss[x] = (uint8_t)mm;
                        if (mm >= a.max_missed) {  // >= 3 -> dead (:337)
                            a.ex_col[x] = c | kMaskedEdge;
                            emit = true;
                            dead = c;
                        }
                    }
                }
            }
            emit_reports(a, emit, (uint32_t)(a.begin + u), dead, acc, rs);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    flush_reports(a, rs);
    flush(acc, a.st);
}

// push over the overflow rows; runs before k_push_light (which consumes new[])
template <int W, bool CA, bool RM>
__global__ __launch_bounds__(kBlock) void k_push_extra(RoundArgs a) {
    Acc acc;
    for (uint64_t u = (uint64_t)blockIdx.x * kBlock + threadIdx.x; u < a.n_local; u += (uint64_t)gridDim.x * kBlock) {
        const uint32_t cnt = a.ex_cnt[u];
        if (!cnt) continue;
        uint64_t m[W];
        uint32_t pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            m[w] = a.nw[u * W + w];
            pc += (uint32_t)__popcll(m[w]);
        }
        if (!pc) continue;
        for (uint32_t k = 0; k < cnt; ++k) deliver<W, CA, RM>(a, a.ex_col[u * a.ex_cap + k], m, pc, acc);
    }
    flush(acc, a.st);
}

__global__ void k_reboot_keys(DeadReport* rep, uint64_t first, uint64_t n, uint64_t begin, unsigned long long* keys) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const DeadReport r = rep[first + i];
        keys[i] = ((unsigned long long)(r.reporter - begin) << 32) | r.dead;
    }
}

// u holds a connection to c: an unmasked entry of its sorted row or of its
// overflow row (a dropped edge is erased from connectedPeers, peer.cpp:388)
__device__ __forceinline__ bool has_out_edge(const RoundArgs& a, uint64_t u, uint32_t c) {
    uint64_t lo = a.rp[u], hi = a.rp[u + 1];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((a.col[mid] & ~kMaskedEdge) < c) lo = mid + 1;
        else hi = mid;
    }
    if (lo < a.rp[u + 1] && a.col[lo] == c) return true;  // equal and unmasked
    const uint32_t cnt = a.ex_cnt[u];
    for (uint32_t k = 0; k < cnt; ++k)
        if (a.ex_col[u * a.ex_cap + k] == c) return true;
    return false;
}

// one thread per reporter (the first of its run of sorted keys): its reports
// in dead order, each a seed response of L candidates, the first k kept
// (the power-law pick) unless self, dead (connect() fails), already connected
// (connectedPeers is a map) or the overflow row is full
__global__ __launch_bounds__(kBlock) void k_rebootstrap(RoundArgs a, RebootArgs rb, const unsigned long long* keys,
                                                        uint64_t n) {
    Acc acc;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t u = keys[i] >> 32;
        if (i > 0 && (keys[i - 1] >> 32) == u) continue;  // not the first report of u
        const uint32_t ug = (uint32_t)(a.begin + u);
        for (uint64_t j = i; j < n && (keys[j] >> 32) == u; ++j) {
            if (a.ex_cnt[u] >= a.ex_cap) break;  // row full: the remaining re-selections add nothing
            const uint32_t dead = (uint32_t)keys[j];
            const uint32_t x0 = philox4x32_10(P_REBOOT, a.round, dead, 0, rb.seed, ug).x;
            uint32_t k = 0;
            for (uint32_t t = 1; t < rb.L; ++t) k += x0 >= rb.thr[t];
            for (uint32_t c_i = 0; c_i < k; ++c_i) {
                const u32x4 r = philox4x32_10(P_REBOOT, a.round, dead, 1 + (c_i >> 2), rb.seed, ug);
                const uint32_t c = skew_pick(lane_of(r, c_i & 3), a.n_global);
                if (c == ug || !bit_alive(a.alive, c) || has_out_edge(a, u, c)) continue;
                const uint32_t cnt = a.ex_cnt[u];
                if (cnt >= a.ex_cap) continue;
                a.ex_col[u * a.ex_cap + cnt] = c;
                a.ex_miss[u * a.ex_cap + cnt] = 0;
                a.ex_cnt[u] = cnt + 1;
                acc.reconnects++;
            }
        }
    }
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// Join churn (the reference has no rejoin path).  A peer
// dead at the start of round r restarts at its address in r with probability
// threshold / 2^32 -- PeerNode::start again (peer.cpp:28-101): re-registered
// (seed.cpp:153-156), an empty Message-List, its old connections gone (its row
// is dropped) and, once the round's deaths are known, fresh out-edges from one
// seed response in its overflow row.  Runs before the round's kills and churn
// deaths; one thread per 32-peer word of the alive bitset.
// ---------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(kBlock) void k_rejoin(RoundArgs a, uint32_t wd, uint32_t seed, uint32_t thr,
                                                   uint64_t n_boot, uint32_t* list, unsigned long long* n_list) {
    Acc acc;
    const uint64_t n_words = (n_boot + 31) >> 5;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n_words; i += (uint64_t)gridDim.x * kBlock) {
        const uint32_t valid = (i + 1) * 32 <= n_boot ? ~0u : (1u << (n_boot & 31)) - 1u;
        const uint32_t word = a.alive[i];
        uint32_t back = 0;
        for (uint32_t x = ~word & valid; x; x &= x - 1) {
            const uint32_t b = (uint32_t)__builtin_ctz(x);
            if (philox4x32_10(P_REJOIN, a.round, 0, 0, seed, (uint32_t)(i * 32 + b)).x < thr) back |= 1u << b;
        }
        if (!back) continue;
        a.alive[i] = word | back;
        a.registered[i] |= back;  // one thread per word: plain stores
        for (uint32_t x = back; x; x &= x - 1) {
            const uint32_t v = (uint32_t)(i * 32 + __builtin_ctz(x));
            if (v < a.begin || v >= a.end) continue;
            const uint64_t lv = v - a.begin;
            acc.rejoined++;
            // the old Message-List is gone: its words leave the digest and coverage
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint64_t mm = a.seen[lv * W + w];
                a.seen[lv * W + w] = 0ull;
                a.nw[lv * W + w] = 0ull;
                if (!mm) continue;
                if (w < (int)wd) acc.digest -= digest_weight((uint64_t)v * wd + w) * mm;
                acc.covered -= (unsigned long long)__popcll(mm);
                if (a.cov)
                    for (uint64_t y = mm; y; y &= y - 1) atomicAdd(&a.cov[w * 64 + __builtin_ctzll(y)], ~0ull);
            }
            for (uint64_t e = a.rp[lv]; e < a.rp[lv + 1]; ++e) a.col[e] |= kMaskedEdge;  // old connections
            if (a.ex_cap) a.ex_cnt[lv] = 0;
            list[atomicAdd(n_list, 1ull)] = (uint32_t)lv;
        }
    }
    flush(acc, a.st);
}

// the restarted peers' selectAndConnectPeers (peer.cpp:214-253) once the
// round's deaths are known: one response of L candidates keyed by the round,
// self / dead / repeated candidates skipped, at most ex_cap kept
__global__ __launch_bounds__(kBlock) void k_rejoin_select(RoundArgs a, RebootArgs rb, const uint32_t* list,
                                                          const unsigned long long* n_list) {
    Acc acc;
    const uint64_t n = *n_list;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t lv = list[i];
        const uint32_t v = (uint32_t)(a.begin + lv);
        if (!bit_alive(a.alive, v)) continue;  // died again in the same round
        const uint32_t y = philox4x32_10(P_REJOIN, a.round, 0, 0, rb.seed, v).y;
        uint32_t k = 0;
        for (uint32_t t = 1; t < rb.L; ++t) k += y >= rb.thr[t];
        for (uint32_t c_i = 0; c_i < k; ++c_i) {
            const u32x4 r = philox4x32_10(P_REJOIN, a.round, 1 + (c_i >> 2), 0, rb.seed, v);
            const uint32_t c = skew_pick(lane_of(r, c_i & 3), a.n_global);
            if (c == v || !bit_alive(a.alive, c) || has_out_edge(a, lv, c)) continue;
            const uint32_t cnt = a.ex_cnt[lv];
            if (cnt >= a.ex_cap) continue;
            a.ex_col[lv * a.ex_cap + cnt] = c;
            a.ex_miss[lv * a.ex_cap + cnt] = 0;
            a.ex_cnt[lv] = cnt + 1;
            acc.reconnects++;
        }
    }
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// Measurement only (while timing is on): SURVEY.md 8(d)'s liveness term of a ping round counts the pings
// pingLoop sends (peer.cpp:328-346) -- every connected (unmasked) out-edge of every alive owned peer, the
// overflow rows included -- and those peers.  The closed-form ping round visits far fewer edges; this
// count is what its bytes are charged against.  out[0] += edges, out[1] += peers.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_live_count(RoundArgs a, unsigned long long* out) {
    unsigned long long e = 0, nv = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x; v < a.n_local; v += (uint64_t)gridDim.x * kBlock) {
        if (!bit_alive(a.alive, (uint32_t)(a.begin + v))) continue;
        ++nv;
        const uint64_t r0 = a.rp[v], r1 = a.rp[v + 1];
        if (a.dmask) {
            e += (r1 - r0) - a.dmask[v];
        } else {
            for (uint64_t i = r0; i < r1; ++i) e += !(a.col[i] & kMaskedEdge);
        }
        if (a.ex_cnt)
            for (uint32_t k = 0; k < a.ex_cnt[v]; ++k) e += !(a.ex_col[v * a.ex_cap + k] & kMaskedEdge);
    }
    e = wave_sum(e);
    nv = wave_sum(nv);
    if ((threadIdx.x & 63) == 0 && (e | nv)) {
        atomicAdd(out, e);
        atomicAdd(out + 1, nv);
    }
}

// ---------------------------------------------------------------------------
// churn / kills: a dead peer stops receiving, forwarding and pinging.  Its
// pending new words are dropped, but they are already in seen, so their
// digest/coverage contribution is booked here.
// ---------------------------------------------------------------------------
template <int W>
__device__ __forceinline__ void retire_peer(const RoundArgs& a, uint32_t v, uint32_t wd, Acc& acc) {
    if (v < a.begin || v >= a.end) return;
    acc.died++;
    const uint64_t lv = v - a.begin;
    if (a.death_r) a.death_r[lv] = (uint16_t)a.round;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const uint64_t mm = a.nw[lv * W + w];
        acc.dead_cov += (unsigned long long)__popcll(a.seen[lv * W + w] | mm);  // (a pending fold: mm not in seen)
        if (!mm) continue;
        if (w < (int)wd) acc.digest += digest_weight((uint64_t)v * wd + w) * mm;
        acc.covered += (unsigned long long)__popcll(mm);
        if (a.cov)
            for (uint64_t x = mm; x; x &= x - 1) atomicAdd(&a.cov[w * 64 + __builtin_ctzll(x)], 1ull);
        a.nw[lv * W + w] = 0ull;
    }
}

// One lane per quad of peers (P_CHURN: one Philox draw per 4 peers, lane v & 3 of it is peer v's churn
// number), so a wave covers eight words of the alive bitset: each peer alive at the start of the round is
// tested, the eight lanes of a word OR their deaths together and one of them clears the word.  The draws
// bound the kernel (VALU: ten rounds of 32-bit multiplies each); round 3 drew once per peer, in a chain of
// up to 32 per thread, and took 0.14 ms per round at config 5, one draw per peer and lane 0.2 ms.  A small
// grid strides over the quads with the next alive word loaded ahead.
template <int W>
__global__ __launch_bounds__(kBlock) void k_churn(RoundArgs a, uint32_t wd, uint32_t seed, uint32_t thr) {
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t n_quads = (a.n_global + 3) >> 2;
    const uint64_t q_pad = (n_quads + 63) & ~63ull, stride = (uint64_t)gridDim.x * kBlock;
    uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t next = q < n_quads ? a.alive[q >> 3] : 0u;
    for (; q < q_pad; q += stride) {  // (wave-uniform: q_pad and the wave's quads are 64-aligned)
        // the word of the next iteration is loaded ahead (only this wave writes it, and later)
        const uint32_t word = next;
        next = q + stride < n_quads ? a.alive[(q + stride) >> 3] : 0u;
        const uint64_t v0 = q << 2;
        uint32_t live = (word >> (v0 & 31)) & 0xFu;
        if (v0 + 4 > a.n_global) live &= v0 < a.n_global ? (1u << (uint32_t)(a.n_global - v0)) - 1u : 0u;
        uint32_t die = 0;
        if (live) {
            const u32x4 r = philox4x32_10(P_CHURN, a.round, 0, 0, seed, (uint32_t)q);
            die = (uint32_t)(r.x < thr) | (uint32_t)(r.y < thr) << 1 | (uint32_t)(r.z < thr) << 2 |
                  (uint32_t)(r.w < thr) << 3;
            die &= live;
        }
        // lanes 8k .. 8k + 7 hold the quads of one alive word
        uint32_t dw = die << (4 * (lane & 7));
        dw |= (uint32_t)__shfl_xor((int)dw, 1);
        dw |= (uint32_t)__shfl_xor((int)dw, 2);
        dw |= (uint32_t)__shfl_xor((int)dw, 4);
        if (!__ballot(die != 0)) continue;  // wave-uniform
        if ((lane & 7) == 0 && dw) a.alive[q >> 3] = word & ~dw;
        for (uint32_t m = die; m; m &= m - 1) retire_peer<W>(a, (uint32_t)(v0 + (uint32_t)__builtin_ctz(m)), wd, acc);
    }
    flush(acc, a.st);
}

template <int W>
__global__ __launch_bounds__(kBlock) void k_kills(RoundArgs a, uint32_t wd, const uint32_t* peers, uint32_t n) {
    Acc acc;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    bool died = false;
    uint32_t v = 0;
    if (i < n) {
        v = peers[i];
        const uint32_t bit = 1u << (v & 31);
        died = (atomicAnd(&a.alive[v >> 5], ~bit) & bit) != 0;
    }
    if (died) retire_peer<W>(a, v, wd, acc);
    flush(acc, a.st);
}

// messageGenerationLoop (peer.cpp:359-374): origin marks the message seen and
// will push it this round.
template <int W>
__global__ __launch_bounds__(kBlock) void k_inject(RoundArgs a, const uint32_t* origin, const uint32_t* msg_id,
                                                    uint32_t n) {
    Acc acc;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) {
        const uint32_t o = origin[i];
        if (o >= a.begin && o < a.end && bit_alive(a.alive, o)) {
            const uint32_t m = msg_id[i];
            const uint64_t idx = (uint64_t)(o - a.begin) * W + (m >> 6);
            const unsigned long long bit = 1ull << (m & 63);
            atomicOr(reinterpret_cast<unsigned long long*>(a.seen) + idx, bit);
            atomicOr(reinterpret_cast<unsigned long long*>(a.nw) + idx, bit);
            if (a.inj_live) atomicOr(reinterpret_cast<unsigned long long*>(a.inj_live) + (m >> 6), bit);
            if (a.tcur) atomicOr(reinterpret_cast<unsigned long long*>(a.tcur) + ((o - a.begin) >> 12), 1ull << (((o - a.begin) >> 6) & 63));
            acc.injected++;
        }
    }
    flush(acc, a.st);
}

// Partitioned rounds: OR the masks received from every rank into the owned
// peers (test-and-set without atomics: this kernel is the only writer); an
// activated peer marks its tile for the next round's marked-tile sweep.
template <int W>
__global__ __launch_bounds__(kBlock) void k_apply_remote(RoundArgs a, const uint64_t* recv, uint32_t world,
                                                         uint64_t stride) {
    Acc acc;
    for (uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x; v < a.n_local; v += (uint64_t)gridDim.x * kBlock) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            uint64_t inc = 0;
            for (uint32_t p = 0; p < world; ++p)
                inc |= recv[GOSSIP_IDX(a, kChkApplyRemote, ((uint64_t)p * stride + v) * W + w, (uint64_t)world * stride * W)];
            if (!inc) continue;
            const uint64_t cur = a.seen[v * W + w];
            if (a.defer) {  // seen is folded in by k_commit_nx: this round's local receipts are in nx
                const uint64_t nxc = a.nx[v * W + w];
                const uint64_t fr = inc & ~cur & ~nxc;
                if (!fr) continue;
                a.nx[v * W + w] = nxc | fr;
                acc.fresh += (unsigned long long)__popcll(fr);
                if (!nxc) mark_tile(a, v, acc);
                continue;
            }
            const uint64_t fr = inc & ~cur;
            if (!fr) continue;
            a.seen[v * W + w] = cur | fr;
            const uint64_t nxc = a.nx[v * W + w];
            a.nx[v * W + w] = nxc | fr;
            acc.fresh += (unsigned long long)__popcll(fr);
            if (!nxc) mark_tile(a, v, acc);
        }
    }
    flush(acc, a.st);
}

// ---------------------------------------------------------------------------
// Sparse exchange (push rounds of a partitioned run): the dense staging
// buffer (send, one entry per global peer, OR of everything this rank pushed
// to that peer) is compacted into per-destination-rank records
// {peer, words[W]} and cleared in the same pass, so only the touched peers
// cross xGMI.  Records of a destination stay <= its block size.  Deterministic
// and without atomics: a bitmap of each destination block's 64-peer tiles
// (k_send_bits), the exclusive prefix of their popcounts (hipcub scan), then
// every touched peer's record at its rank in its block (k_send_pack).  (Round
// 3's version took each record's place from one global counter per
// destination: millions of same-address atomics per round -- config 4 at
// P = 8, 69 ms of compaction per step.)
// ---------------------------------------------------------------------------
// block q of tile T (toff: the tiles of the blocks before each block; world is small)
__device__ __forceinline__ uint32_t send_block(const uint64_t* toff, uint32_t world, uint64_t T) {
    uint32_t q = 0;
    while (q + 1 < world && toff[q + 1] <= T) ++q;
    return q;
}

template <int W>
__global__ __launch_bounds__(kBlock) void k_send_bits(RoundArgs a, const uint64_t* part_g, const uint64_t* toff_g,
                                                      uint32_t world, uint64_t* bits) {
    __shared__ uint64_t part[kMaxWorld + 1], toff[kMaxWorld + 1];  // (a dependent global load per lookup step)
    for (uint32_t i = threadIdx.x; i <= world; i += kBlock) {
        part[i] = part_g[i];
        toff[i] = toff_g[i];
    }
    __syncthreads();
    // a wave per 64 tiles: lane l tests tile T0 + l against the round's marks (its peers span at most two
    // marked 64-peer tiles), unmarked tiles get a zero bitmap word, and the wave reads the staging words of
    // the marked ones in turn (a sparse round's send buffer is 2 GB at config 4; the marked tiles are few)
    const int lane = threadIdx.x & 63;
    const uint64_t tiles = toff[world];
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t T0 = ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; T0 < tiles;
         T0 += nwaves * 64) {
        const uint64_t T = T0 + lane;
        bool mk = false;
        if (T < tiles) {
            const uint32_t q = send_block(toff, world, T);
            const uint64_t v0 = part[q] + (T - toff[q]) * 64, end = part[q + 1];
            if (v0 < end) {
                const uint64_t g0 = v0 >> 6, g1 = (min(v0 + 64, end) - 1) >> 6;
                mk = ((a.smark[g0 >> 6] >> (g0 & 63)) | (a.smark[g1 >> 6] >> (g1 & 63))) & 1ull;
            }
            if (!mk) bits[T] = 0ull;
        }
        for (unsigned long long todo = __ballot(mk); todo; todo &= todo - 1) {  // wave-uniform
            const uint64_t Tm = T0 + (uint64_t)__builtin_ctzll(todo);
            const uint32_t q = send_block(toff, world, Tm);
            const uint64_t end = part[q + 1];
            const uint64_t v = part[q] + (Tm - toff[q]) * 64 + lane;
            bool any = false;
            if (v < end) {
#pragma unroll
                for (int w = 0; w < W; ++w) any |= a.send[v * W + w] != 0ull;
            }
            const unsigned long long b = __ballot(any);
            if (lane == 0) bits[Tm] = b;
        }
    }
}

template <int W>
__global__ __launch_bounds__(kBlock) void k_send_pack(RoundArgs a, const uint64_t* part_g, const uint64_t* toff_g,
                                                      uint32_t world, uint64_t stride, const uint64_t* bits,
                                                      const uint64_t* pos, unsigned long long* counts, uint64_t* seg) {
    __shared__ uint64_t part[kMaxWorld + 1], toff[kMaxWorld + 1];
    for (uint32_t i = threadIdx.x; i <= world; i += kBlock) {
        part[i] = part_g[i];
        toff[i] = toff_g[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t tiles = toff[world];
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (gid < world) counts[gid] = pos[toff[gid + 1]] - pos[toff[gid]];  // records per destination
    // a wave per 64 tiles: one coalesced read of their bitmap words, then the tiles with records in turn
    // (a wave per tile waited on one bitmap word per tile: 64 round trips per wave at config 4, P = 8)
    for (uint64_t T0 = ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; T0 < tiles;
         T0 += nwaves * 64) {
        const uint64_t bl = T0 + lane < tiles ? bits[T0 + lane] : 0ull;
        for (unsigned long long todo = __ballot(bl != 0); todo; todo &= todo - 1) {  // wave-uniform
            const int src = __builtin_ctzll(todo);
            const uint64_t T = T0 + (uint64_t)src;
            const uint64_t b = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(bl >> 32), src) << 32) |
                               (uint32_t)__shfl((int)(uint32_t)bl, src);
            if ((b >> lane) & 1) {
                const uint32_t q = send_block(toff, world, T);
                const uint64_t v = part[q] + (T - toff[q]) * 64 + lane;
                const uint64_t idx = pos[T] - pos[toff[q]] + (uint64_t)__popcll(b & ((1ull << lane) - 1));
                uint64_t* rec = seg + (q * stride + idx) * (1 + W);
                rec[0] = v;
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    rec[1 + w] = a.send[v * W + w];
                    a.send[v * W + w] = 0ull;
                }
            }
        }
    }
}

template <int W>
__global__ __launch_bounds__(kBlock) void k_apply_records(RoundArgs a, const uint64_t* rec, uint64_t n_rec) {
    Acc acc;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n_rec; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t* r = rec + i * (1 + W);
        const uint64_t lv = GOSSIP_IDX(a, kChkApplyRecord, r[0] - a.begin, a.n_local);
        unsigned long long* sp = reinterpret_cast<unsigned long long*>(a.seen) + lv * W;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const unsigned long long m = r[1 + w];
            if (!m || !(m & ~sp[w])) continue;
            if (a.defer) {  // as deliver: the round-start seen, one atomic on nx
                const unsigned long long u = m & ~sp[w];
                const unsigned long long old = atomicOr(reinterpret_cast<unsigned long long*>(a.nx) + lv * W + w, u);
                acc.atomics++;
                const unsigned long long fr = u & ~old;
                acc.activated += fr && old == 0;
                acc.fresh += (unsigned long long)__popcll(fr);
                if (fr && old == 0) mark_tile(a, lv, acc);
                continue;
            }
            const unsigned long long fr = m & ~atomicOr(sp + w, m);
            acc.atomics += fr ? 2 : 1;
            if (fr) {
                const unsigned long long onx = atomicOr(reinterpret_cast<unsigned long long*>(a.nx) + lv * W + w, fr);
                acc.activated += onx == 0;
                acc.fresh += (unsigned long long)__popcll(fr);
                if (onx == 0) mark_tile(a, lv, acc);
            }
        }
    }
    flush(acc, a.st);
}

// After a deferred push round: seen |= nx (nx holds exactly this round's
// fresh bits).  16-B words, streamed; seen is written only where nx is set.
__global__ __launch_bounds__(kBlock) void k_commit_nx(u64x2* seen, const u64x2* nx, uint64_t n2) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n2; i += (uint64_t)gridDim.x * kBlock) {
        const u64x2 x = __builtin_nontemporal_load(nx + i);
        if (!(x.x | x.y)) continue;
        seen[i] |= x;
    }
}

// reset: zero a word array with 16-B stores (hipMemsetAsync's fill kernel
// reached ~2.6 TB/s on the 2 GB arrays of config 4)
__global__ __launch_bounds__(kBlock) void k_zero2(u64x2* p, uint64_t n2) {
    const u64x2 z = {0ull, 0ull};
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n2; i += (uint64_t)gridDim.x * kBlock) p[i] = z;
}

template <int W>
__global__ __launch_bounds__(kBlock) void k_coverage(const uint64_t* words, uint64_t n, unsigned long long* counts) {
    __shared__ unsigned int cnt[64 * W];
    for (int i = threadIdx.x; i < 64 * W; i += kBlock) cnt[i] = 0;
    __syncthreads();
    for (uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x; v < n; v += (uint64_t)gridDim.x * kBlock) {
#pragma unroll
        for (int w = 0; w < W; ++w)
            for (uint64_t x = words[v * W + w]; x; x &= x - 1) atomicAdd(&cnt[w * 64 + __builtin_ctzll(x)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * W; i += kBlock)
        if (cnt[i]) atomicAdd(&counts[i], (unsigned long long)cnt[i]);
}

// first two entries of every row (a.first2); rows of one entry repeat it
__global__ __launch_bounds__(kBlock) void k_first2(const uint64_t* rp, const uint32_t* col, uint64_t n,
                                                   uint64_t* out) {
    for (uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x; v < n; v += (uint64_t)gridDim.x * kBlock) {
        const uint64_t b = rp[v], d = rp[v + 1] - b;
        const uint64_t c0 = d ? col[b] : 0u, c1 = d > 1 ? col[b + 1] : c0;
        out[v] = c0 | (c1 << 32);
    }
}

__global__ void k_heavy_count(const uint64_t* rp, uint64_t n, uint32_t heavy, uint32_t clen, unsigned long long* n_chunks) {
    unsigned long long mine = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t d = rp[v + 1] - rp[v];
        if (d > heavy) mine += (d + clen - 1) / clen;
    }
    mine = wave_sum(mine);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(n_chunks, mine);
}

__global__ void k_heavy_fill(const uint64_t* rp, uint64_t n, uint32_t heavy, uint32_t clen, HeavyChunk* chunks,
                             unsigned long long* cursor) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = rp[v], e = rp[v + 1];
        if (e - b <= heavy) continue;
        const uint64_t nc = (e - b + clen - 1) / clen;
        const unsigned long long at = atomicAdd(cursor, (unsigned long long)nc);
        for (uint64_t k = 0; k < nc; ++k) {
            const uint64_t e0 = b + k * clen;
            chunks[at + k] = HeavyChunk{(uint32_t)v, (uint32_t)at, e0, e0 + clen < e ? e0 + clen : e};
        }
    }
}



}  // namespace

// ---- launchers: dispatch the padded word count Wp in {1,2,4,8} ------------
#define GOSSIP_DISPATCH_W(Wp, CALL)                     \
    switch (Wp) {                                       \
        case 1: { constexpr int W = 1; CALL; } break;   \
        case 2: { constexpr int W = 2; CALL; } break;   \
        case 4: { constexpr int W = 4; CALL; } break;   \
        case 8: { constexpr int W = 8; CALL; } break;   \
        default: return hipErrorInvalidValue;           \
    }

// Wp is the padded storage stride; the digest uses the unpadded W carried in
// the upper 16 bits of the W argument (see gossip_engine.hip: pack_w).
static inline uint32_t wp_of(uint32_t w) { return w & 0xFFFFu; }
static inline uint32_t wd_of(uint32_t w) { return w >> 16; }

hipError_t launch_churn(const RoundArgs& a, uint32_t W_, uint32_t seed, uint32_t threshold, hipStream_t s) {
    const unsigned g = (unsigned)std::min<uint64_t>(grid_for((a.n_global + 3) / 4, kBlock), 2048);
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_churn<W>, dim3(g), dim3(kBlock), 0, s, a, wd_of(W_), seed,
                                                   threshold));
    return hipGetLastError();
}

hipError_t launch_kills(const RoundArgs& a, uint32_t W_, const uint32_t* peers, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    const unsigned g = (n + kBlock - 1) / kBlock;
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_kills<W>, dim3(g), dim3(kBlock), 0, s, a, wd_of(W_), peers, n));
    return hipGetLastError();
}

hipError_t launch_liveness(const RoundArgs& a, hipStream_t s, int heavy) {
    if (heavy) {
        if (!a.n_chunks) return hipSuccess;
        hipLaunchKernelGGL(k_liveness_heavy, dim3(grid_for(a.n_chunks, kWavesPerBlock)), dim3(kBlock), 0, s, a);
    } else {
        const uint64_t tiles = (a.n_local + 63) / 64;
        hipLaunchKernelGGL(k_liveness_light, dim3(grid_for(tiles, kWavesPerBlock)), dim3(kBlock), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_inject(const RoundArgs& a, uint32_t W_, const uint32_t* origin, const uint32_t* msg_id, uint32_t n,
                         hipStream_t s) {
    if (!n) return hipSuccess;
    const unsigned g = (n + kBlock - 1) / kBlock;
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_inject<W>, dim3(g), dim3(kBlock), 0, s, a, origin, msg_id, n));
    return hipGetLastError();
}

hipError_t launch_push_heavy(const RoundArgs& a, uint32_t W_, bool check_alive, bool remote, hipStream_t s) {
    if (!a.n_chunks) return hipSuccess;
    const unsigned g = grid_for(a.n_chunks, kWavesPerBlock);
#define GOSSIP_HEAVY(CA, RM) hipLaunchKernelGGL((k_push_heavy<W, CA, RM>), dim3(g), dim3(kBlock), 0, s, a)
    GOSSIP_DISPATCH_W(wp_of(W_), {
        if (check_alive) {
            if (remote) GOSSIP_HEAVY(true, true); else GOSSIP_HEAVY(true, false);
        } else {
            if (remote) GOSSIP_HEAVY(false, true); else GOSSIP_HEAVY(false, false);
        }
    });
#undef GOSSIP_HEAVY
    return hipGetLastError();
}

hipError_t launch_push_light(const RoundArgs& a, uint32_t W_, bool check_alive, bool remote, hipStream_t s) {
    const uint64_t tiles = (a.n_local + 63) / 64;
    // every wave resident at once (4 blocks per CU at <= 128 VGPRs): a sweep wave's packets carry its
    // work, and a second partial wave of blocks would only stretch the tail
    const unsigned g = std::min(grid_for(tiles, kWavesPerBlock), 1024u);
    const uint32_t wd = wd_of(W_);
    const bool cov = a.cov != nullptr;
#define GOSSIP_LIGHT(CA, RM, COV) \
    hipLaunchKernelGGL((k_push_light<W, CA, RM, COV, false>), dim3(g), dim3(kBlock), 0, s, a, wd)
    if (a.tsparse) {  // a nearly empty frontier: only the marked tiles (a vertex block's too, round 5)
        const unsigned gs = grid_for((tiles + 63) / 64, kWavesPerBlock);
#define GOSSIP_SP(CA, RM, COV) \
    hipLaunchKernelGGL((k_push_light<W, CA, RM, COV, true>), dim3(gs), dim3(kBlock), 0, s, a, wd)
        GOSSIP_DISPATCH_W(wp_of(W_), {
            if (remote) {
                if (cov) {
                    if (check_alive) GOSSIP_SP(true, true, true);
                    else GOSSIP_SP(false, true, true);
                } else {
                    if (check_alive) GOSSIP_SP(true, true, false);
                    else GOSSIP_SP(false, true, false);
                }
            } else if (cov) {
                if (check_alive) GOSSIP_SP(true, false, true);
                else GOSSIP_SP(false, false, true);
            } else {
                if (check_alive) GOSSIP_SP(true, false, false);
                else GOSSIP_SP(false, false, false);
            }
        });
#undef GOSSIP_SP
        return hipGetLastError();
    }
    GOSSIP_DISPATCH_W(wp_of(W_), {
        if (cov) {
            if (check_alive) { if (remote) GOSSIP_LIGHT(true, true, true); else GOSSIP_LIGHT(true, false, true); }
            else { if (remote) GOSSIP_LIGHT(false, true, true); else GOSSIP_LIGHT(false, false, true); }
        } else {
            if (check_alive) { if (remote) GOSSIP_LIGHT(true, true, false); else GOSSIP_LIGHT(true, false, false); }
            else { if (remote) GOSSIP_LIGHT(false, true, false); else GOSSIP_LIGHT(false, false, false); }
        }
    });
#undef GOSSIP_LIGHT
    return hipGetLastError();
}

hipError_t launch_frontier_bits(const RoundArgs& a, uint32_t W_, hipStream_t s) {
    const uint64_t tiles = (a.n_src + 63) / 64;
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_frontier_bits<W>, dim3(grid_for(tiles, kWavesPerBlock)),
                                                   dim3(kBlock), 0, s, a));
    return hipGetLastError();
}

// the workgroups of kernel f resident on the device at once (occupancy at its registers and LDS x CUs)
template <class K>
unsigned resident_blocks(K f, int block) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, block, 0) != hipSuccess || nb < 1 || cus < 1) {
        hipGetLastError();
        return kMaxGrid;
    }
    return (unsigned)(nb * cus);
}

hipError_t launch_pull_rows(const RoundArgs& a, uint32_t W_, hipStream_t s) {
    // a row queue per wave: every wave resident at once (its queue carries its work).  The grid is the
    // resident workgroups (1024 at 116 VGPRs: four per CU): kMaxGrid (2048) left half the waves to start
    // after the first half had swept its tiles -- arms alternated in one process, config 4 round 7 5.16
    // against 5.02 ms, config 5 2.36 against 2.19 (profiles/r05/ab/r05u); "row_grid" overrides it (A/B)
    const unsigned want = grid_for((a.n_local + 63) / 64, kWavesPerBlock);
    const uint32_t wd = wd_of(W_);
    auto go = [&](void (*kern)(RoundArgs, uint32_t)) {
        static std::pair<const void*, unsigned> cache[16] = {};  // (instances share the pointer type)
        unsigned res = 0;
        for (auto& e : cache) {
            if (e.first == (const void*)kern) { res = e.second; break; }
            if (!e.first) {
                e = {(const void*)kern, resident_blocks(kern, kBlock)};
                res = e.second;
                break;
            }
        }
        if (!res) res = resident_blocks(kern, kBlock);
        const unsigned g = std::min(want, a.row_grid ? a.row_grid : res);
        hipLaunchKernelGGL(kern, dim3(g), dim3(kBlock), 0, s, a, wd);
    };
#define GOSSIP_ROWS(COV, FR)                                                                        \
    do {                                                                                            \
        if (a.row_step == 1 && a.row_q == 256 && W == 1 && !COV && !FR) go(k_pull_rows<W, COV, FR, 1, 256>); \
        else if (a.row_step == 1) go(k_pull_rows<W, COV, FR, 1>);                                   \
        else go(k_pull_rows<W, COV, FR, 2>);                                                        \
    } while (0)
    GOSSIP_DISPATCH_W(wp_of(W_), {
        if (a.cov) { if (a.front) GOSSIP_ROWS(true, true); else GOSSIP_ROWS(true, false); }
        else { if (a.front) GOSSIP_ROWS(false, true); else GOSSIP_ROWS(false, false); }
    });
#undef GOSSIP_ROWS
    return hipGetLastError();
}

hipError_t launch_pull_heavy(const RoundArgs& a, uint32_t W_, hipStream_t s, bool hacc_zeroed, bool defer) {
    if (!a.n_chunks) return hipSuccess;
    if (a.hacc && !hacc_zeroed) {
        const hipError_t e = hipMemsetAsync(a.hacc, 0, a.n_chunks * wp_of(W_) * sizeof(uint64_t), s);
        if (e != hipSuccess) return e;
    }
    if (defer) {
        if (!a.hacc) return hipErrorInvalidValue;
        GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL((k_pull_heavy<W, true>),
                                                       dim3(grid_for(a.n_chunks, kWavesPerBlock)), dim3(kBlock), 0,
                                                       s, a));
    } else {
        GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_pull_heavy<W>, dim3(grid_for(a.n_chunks, kWavesPerBlock)),
                                                       dim3(kBlock), 0, s, a));
    }
    return hipGetLastError();
}

hipError_t launch_heavy_commit(const RoundArgs& a, uint32_t W_, hipStream_t s) {
    if (!a.n_chunks) return hipSuccess;
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_heavy_commit<W>, dim3(grid_for(a.n_chunks, kBlock)),
                                                   dim3(kBlock), 0, s, a));
    return hipGetLastError();
}

hipError_t launch_list_zero(const RoundArgs& a, const uint32_t* lst, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_list_zero, dim3(grid_for(std::max<uint64_t>(n, a.n_chunks), kBlock)), dim3(kBlock), 0, s, a,
                       lst, n);
    return hipGetLastError();
}

hipError_t launch_pull_list(const RoundArgs& a, const uint32_t* lst, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_pull_list, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, a, lst, n);
    return hipGetLastError();
}

hipError_t launch_apply_remote(const RoundArgs& a, uint32_t W_, const uint64_t* recv, uint32_t world,
                               uint64_t part_stride, hipStream_t s) {
    const unsigned g = grid_for(a.n_local, kBlock);
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_apply_remote<W>, dim3(g), dim3(kBlock), 0, s, a, recv, world,
                                                   part_stride));
    return hipGetLastError();
}

namespace {
struct PopOp {
    __host__ __device__ uint64_t operator()(uint64_t x) const { return (uint64_t)__builtin_popcountll(x); }
};
}  // namespace

hipError_t compact_send_scratch(uint64_t tiles, size_t* scan_bytes) {
    hipcub::TransformInputIterator<uint64_t, PopOp, const uint64_t*> it(nullptr, PopOp());
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *scan_bytes, it, (uint64_t*)nullptr, (int)(tiles + 1));
}

hipError_t launch_compact_send(const RoundArgs& a, uint32_t W_, const uint64_t* part, const uint64_t* toff,
                               uint64_t tiles, uint32_t world, uint64_t stride, unsigned long long* counts,
                               uint64_t* seg, uint64_t* bits, uint64_t* pos, void* scan_tmp, size_t scan_bytes,
                               hipStream_t s) {
    if (!a.smark) return hipErrorInvalidValue;
    const unsigned grid_b = (unsigned)std::min<uint64_t>(grid_for((tiles + 63) / 64, kWavesPerBlock), 4096);
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_send_bits<W>, dim3(grid_b), dim3(kBlock), 0, s, a, part, toff,
                                                   world, bits));
    if (hipError_t e = hipGetLastError()) return e;
    // (bits[tiles] is zero from the allocation: the scan's last element is the total)
    hipcub::TransformInputIterator<uint64_t, PopOp, const uint64_t*> it(bits, PopOp());
    size_t tb = scan_bytes;
    if (hipError_t e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, tb, it, pos, (int)(tiles + 1), s)) return e;
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_send_pack<W>, dim3(std::max(grid_b, grid_for(world, kBlock))),
                                                   dim3(kBlock), 0, s, a, part, toff, world, stride, bits, pos,
                                                   counts, seg));
    if (hipError_t e = hipGetLastError()) return e;
    return hipMemsetAsync(a.smark, 0, smark_bytes(a.n_global), s);
}

hipError_t launch_apply_records(const RoundArgs& a, uint32_t W_, const uint64_t* rec, uint64_t n_rec, hipStream_t s) {
    if (!n_rec) return hipSuccess;
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_apply_records<W>, dim3(grid_for(n_rec, kBlock)), dim3(kBlock),
                                                   0, s, a, rec, n_rec));
    return hipGetLastError();
}

hipError_t launch_bin_scatter(const RoundArgs& a, const BinArgs& b, uint32_t W_, hipStream_t s) {
    const uint32_t wd = wd_of(W_);
    if (b.stream) {
        if (b.small && b.chunk * wp_of(W_) <= kSmallChunkWords) {  // small chunks: 256-thread blocks, kSmallGrid of them
            GOSSIP_DISPATCH_W(wp_of(W_), {
                if (a.cov)
                    hipLaunchKernelGGL((k_bin_stream<W, true, kSmallChunkWords, 256>), dim3(kSmallGrid), dim3(256), 0,
                                       s, a, b, wd);
                else
                    hipLaunchKernelGGL((k_bin_stream<W, false, kSmallChunkWords, 256>), dim3(kSmallGrid), dim3(256), 0,
                                       s, a, b, wd);
            });
            return hipGetLastError();
        }
        GOSSIP_DISPATCH_W(wp_of(W_), {
            if (a.cov) hipLaunchKernelGGL((k_bin_stream<W, true>), dim3(kScatterGrid), dim3(kScatterBlock), 0, s, a, b, wd);
            else hipLaunchKernelGGL((k_bin_stream<W, false>), dim3(kScatterGrid), dim3(kScatterBlock), 0, s, a, b, wd);
        });
        return hipGetLastError();
    }
    // 8 producer waves resolving 2 groups per stage into 4-slot rings, 3 register sets (measured best:
    // DESIGN.md section 6.1)
#define GOSSIP_PC(COV) \
    hipLaunchKernelGGL((k_bin_scatter_pc<W, COV, 8, 2, 4, 3>), dim3(kScatterGrid), dim3(kScatterBlock), 0, s, a, b, wd)
    GOSSIP_DISPATCH_W(wp_of(W_), {
        if (a.cov) GOSSIP_PC(true);
        else GOSSIP_PC(false);
    });
#undef GOSSIP_PC
    return hipGetLastError();
}

hipError_t launch_bin_apply(const RoundArgs& a, const BinArgs& b, uint32_t W_, hipStream_t s) {
    if (!b.n_bins) return hipSuccess;
    const uint32_t wd = wd_of(W_);
    if (b.stream) {
        // one block per bin: every (row, member) of every group's rows (k_bin_apply_runs: bin_of)
        const uint64_t rows = (b.n_bins + kApplyRow - 1) / kApplyRow;
        unsigned sgrid = (unsigned)((rows + 7) / 8 * 8 * kApplyRow);
        if (b.work) {  // persistent: the resident blocks; b.work was zeroed before the round's scatter
            const bool wide = b.wide && b.bin_words <= kSmallBinWords;
            const unsigned resident = b.bin_words > kBinWords / 2 ? 256u
                                      : b.bin_words > kSmallBinWords || wide ? 512u
                                                                           : 2048u;
            sgrid = std::min(sgrid, resident);
        }
        if (b.bin_words > kBinWords / 2 && wp_of(W_) == 1) {  // one word: the pipeline shapes (A/B), the probe
            if (b.probe)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 2, true>), dim3(sgrid), dim3(1024), 0, s, a, b,
                                   wd);
            else if (b.apply_pipe == 0)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 0>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 1)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 1>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 2)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 2>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 3)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 3>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 4)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 4>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 5)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 5>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 6)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 6>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 7)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 7>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 8)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 8>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else if (b.apply_pipe == 9)
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 9>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
            else
                hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords, 1024, 10>), dim3(sgrid), dim3(1024), 0, s, a, b, wd);
        } else if (b.bin_words > kBinWords / 2) {
            GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL((k_bin_apply_runs<W, kBinWords, 1024>),
                                                           dim3(sgrid), dim3(1024), 0, s, a, b, wd));
        } else if (b.bin_words <= kSmallBinWords && b.wide) {
            // 16 KB accumulators, 16 waves each: a bin's slots in a quarter of the iterations (small overlays,
            // fewer bins than the chip holds workgroups)
            GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL((k_bin_apply_runs<W, kSmallBinWords, 1024>),
                                                           dim3(sgrid), dim3(1024), 0, s, a, b, wd));
        } else if (b.bin_words <= kSmallBinWords) {
            // 16 KB accumulators: eight 4-wave workgroups per CU (small bins of small overlays)
            GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL((k_bin_apply_runs<W, kSmallBinWords, 256>),
                                                           dim3(sgrid), dim3(256), 0, s, a, b, wd));
        } else if (wp_of(W_) == 1) {
            // 72 KB accumulators: two 8-wave workgroups per CU, one's per-bin phases under the other's slots
            // (one word: shape 5's contiguous groups)
            hipLaunchKernelGGL((k_bin_apply_runs<1, kBinWords / 2, 512, 5>), dim3(sgrid), dim3(512), 0, s, a, b, wd);
        } else {
            GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL((k_bin_apply_runs<W, kBinWords / 2, 512>),
                                                           dim3(sgrid), dim3(512), 0, s, a, b, wd));
        }
        return hipGetLastError();
    }
    const unsigned grid = (unsigned)b.n_bins;
    if (b.bin_words > kBinWords / 2) {  // up to 144 KB accumulators: one 16-wave workgroup per CU
        GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL((k_bin_apply<W, kBinWords, 1024>), dim3(grid), dim3(1024), 0,
                                                       s, a, b, wd));
    } else {  // 64 KB accumulators: two 4-wave workgroups per CU
        GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL((k_bin_apply<W, kBinWords / 2, kBlock>), dim3(grid),
                                                       dim3(kBlock), 0, s, a, b, wd));
    }
    return hipGetLastError();
}

hipError_t launch_liveness_extra(const RoundArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_liveness_extra, dim3(grid_for((a.n_local + 63) & ~63ull, kBlock)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_push_extra(const RoundArgs& a, uint32_t W_, bool check_alive, bool remote, hipStream_t s) {
    const unsigned g = grid_for(a.n_local, kBlock);
#define GOSSIP_EXTRA(CA, RM) hipLaunchKernelGGL((k_push_extra<W, CA, RM>), dim3(g), dim3(kBlock), 0, s, a)
    GOSSIP_DISPATCH_W(wp_of(W_), {
        if (check_alive) {
            if (remote) GOSSIP_EXTRA(true, true); else GOSSIP_EXTRA(true, false);
        } else {
            if (remote) GOSSIP_EXTRA(false, true); else GOSSIP_EXTRA(false, false);
        }
    });
#undef GOSSIP_EXTRA
    return hipGetLastError();
}

hipError_t launch_reboot_keys(const RoundArgs& a, uint64_t first, uint64_t n, unsigned long long* keys,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_reboot_keys, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, a.reports, first, n, a.begin,
                       keys);
    return hipGetLastError();
}

hipError_t launch_rebootstrap(const RoundArgs& a, const RebootArgs& r, const unsigned long long* keys, uint64_t n,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_rebootstrap, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, a, r, keys, n);
    return hipGetLastError();
}

hipError_t launch_rejoin(const RoundArgs& a, uint32_t W_, uint32_t seed, uint32_t thr, uint64_t n_boot, uint32_t* list,
                         unsigned long long* n_list, hipStream_t s) {
    const uint32_t wd = wd_of(W_);
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_rejoin<W>, dim3(grid_for((n_boot + 31) / 32, kBlock)), dim3(kBlock),
                                                   0, s, a, wd, seed, thr, n_boot, list, n_list));
    return hipGetLastError();
}

hipError_t launch_rejoin_select(const RoundArgs& a, const RebootArgs& r, const uint32_t* list,
                                const unsigned long long* n_list, uint64_t max_list, hipStream_t s) {
    if (!a.ex_cap || !max_list) return hipSuccess;
    hipLaunchKernelGGL(k_rejoin_select, dim3(grid_for(max_list, kBlock)), dim3(kBlock), 0, s, a, r, list, n_list);
    return hipGetLastError();
}

template <int MODE>
static hipError_t launch_rows(const RoundArgs& a, uint32_t lo, uint32_t hi, hipStream_t s) {
    if (a.n_chunks)
        hipLaunchKernelGGL(k_rows_heavy<MODE>, dim3(grid_for(a.n_chunks, kWavesPerBlock)), dim3(kBlock), 0, s, a, lo, hi);
    // a strided sweep (a block per 4 tiles was 262 K blocks at config 5, most of them selecting nothing)
    const unsigned g = (unsigned)std::min<uint64_t>(grid_for((a.n_local + 63) / 64, kWavesPerBlock), 8192);
    hipLaunchKernelGGL(k_rows_light<MODE>, dim3(g), dim3(kBlock), 0, s, a, lo, hi);
    return hipGetLastError();
}

hipError_t launch_dead_edges(const RoundArgs& a, uint32_t lo, uint32_t hi, hipStream_t s) {
    return launch_rows<kRowsDead>(a, lo, hi, s);
}

hipError_t launch_live_count(const RoundArgs& a, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(k_live_count, dim3(std::min<uint64_t>(grid_for(a.n_local, kBlock), 4096)), dim3(kBlock), 0, s, a,
                       out);
    return hipGetLastError();
}

hipError_t launch_liveness_window(const RoundArgs& a, uint32_t lo, uint32_t hi, hipStream_t s) {
    return launch_rows<kRowsLive>(a, lo, hi, s);
}

hipError_t launch_reverse_edges(const RoundArgs& a, hipStream_t s) { return launch_rows<kRowsRev>(a, 0, 0, s); }

hipError_t launch_src_count(const RoundArgs& a, uint32_t W_, hipStream_t s) {
    const uint64_t tiles = (a.n_local + 63) / 64;
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_src_count<W>, dim3(grid_for(tiles, kWavesPerBlock)), dim3(kBlock),
                                                   0, s, a));
    return hipGetLastError();
}

hipError_t launch_first2(const uint64_t* rp, const uint32_t* col, uint64_t n, uint64_t* out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_first2, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, rp, col, n, out);
    return hipGetLastError();
}

hipError_t launch_commit_nx(uint64_t* seen, const uint64_t* nx, uint64_t n_words, hipStream_t s) {
    const uint64_t n2 = (n_words + 1) / 2;  // the word arrays are allocated in whole pairs
    hipLaunchKernelGGL(k_commit_nx, dim3(grid_for(n2, kBlock)), dim3(kBlock), 0, s, reinterpret_cast<u64x2*>(seen),
                       reinterpret_cast<const u64x2*>(nx), n2);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_zero_batch(ZeroBatch z) {
    for (uint32_t r = 0; r < z.count; ++r) {
        uint32_t* p = z.p[r];
        uint32_t* save = z.save[r];
        for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < z.n[r]; i += gridDim.x * kBlock) {
            if (save) save[i] = p[i];
            p[i] = 0u;
        }
    }
}

hipError_t launch_zero_batch(const ZeroBatch& z, hipStream_t s) {
    uint32_t most = 0;
    for (uint32_t r = 0; r < z.count; ++r) most = std::max(most, z.n[r]);
    hipLaunchKernelGGL(k_zero_batch, dim3(grid_for(most, kBlock)), dim3(kBlock), 0, s, z);
    return hipGetLastError();
}

hipError_t launch_zero_words(uint64_t* words, uint64_t n_words, hipStream_t s, bool fill) {
    const uint64_t n2 = (n_words + 1) / 2;  // the word arrays are allocated in whole pairs
    if (!n2) return hipSuccess;
    // fill (round 6, "zero_fill"): the runtime's fill kernel, which on this image clears config 4's 2 GB in
    // 0.32 ms (the list rounds' clears) against k_zero2's 0.48
    if (fill) return hipMemsetAsync(words, 0, n2 * 2 * sizeof(uint64_t), s);
    hipLaunchKernelGGL(k_zero2, dim3(grid_for(n2, kBlock)), dim3(kBlock), 0, s, reinterpret_cast<u64x2*>(words), n2);
    return hipGetLastError();
}

hipError_t launch_coverage(const uint64_t* words, uint64_t n_local, uint32_t W_, unsigned long long* counts,
                           hipStream_t s) {
    const unsigned g = grid_for(n_local, kBlock);
    GOSSIP_DISPATCH_W(wp_of(W_), hipLaunchKernelGGL(k_coverage<W>, dim3(g), dim3(kBlock), 0, s, words, n_local,
                                                   counts));
    return hipGetLastError();
}

hipError_t launch_heavy_count(const uint64_t* rp, uint64_t n_local, uint32_t heavy, uint32_t clen,
                              unsigned long long* n_chunks, hipStream_t s) {
    hipLaunchKernelGGL(k_heavy_count, dim3(grid_for(n_local, kBlock)), dim3(kBlock), 0, s, rp, n_local, heavy, clen,
                       n_chunks);
    return hipGetLastError();
}

hipError_t launch_heavy_fill(const uint64_t* rp, uint64_t n_local, uint32_t heavy, uint32_t clen, HeavyChunk* chunks,
                             unsigned long long* cursor, hipStream_t s) {
    hipLaunchKernelGGL(k_heavy_fill, dim3(grid_for(n_local, kBlock)), dim3(kBlock), 0, s, rp, n_local, heavy, clen,
                       chunks, cursor);
    return hipGetLastError();
}

}  // namespace gossip
