// gossip_blocked.hip -- propagation-blocked push rounds of libgossip_hip (P = 1, one word per peer).
//
// A push round (broadcastMessage peer.cpp:297-318 over every peer with new
// messages, handleClient's dedup peer.cpp:277-285 at every receiver) delivers
// each frontier peer's new word along its out-edges.  The atomic push
// (k_push_light / k_push_heavy) pays one random test-and-set per delivery and
// is bound by memory-side atomics once a round carries tens of millions of
// deliveries (config 4, round 3: 53.5 M traversals in 4.2 ms); a binned round
// streams every edge of the overlay whatever the frontier (config 4, round 4:
// 17 % of the peers active, 15.6 ms).  A blocked round writes one record
// {destination, new word} per delivery and sorts the records to their
// destinations in two coalesced binning passes before one LDS-accumulated
// apply per bin, so its cost follows the round's traversals:
//   level 1 (k_pb_scatter): workgroup w owns the tiles t = w (mod kPbGrid)
//     (every part of the id space: a round's frontier is not uniform in it,
//     contiguous ranges left one workgroup 3x the mean) and the heavy chunks
//     c = w (mod kPbGrid);
//     its waves expand the frontier's rows (heavy rows by chunk, light rows 64
//     at a time from a packet, as the push does) and stage
//     each record in the workgroup's LDS buffer of its coarse bin (kPbCoarse
//     bins of about equal in-degree); a full buffer goes out whole into the
//     workgroup's own segment of that bin;
//   level 2 (k_pb_split): slice s of coarse bin k re-stages the segments of
//     kPbGrid / kPbSlices level-1 workgroups into the bin's fine bins (whole
//     tiles, <= kBinWords peers and about kPbFineIn in-degree each: the hubs'
//     tiles get bins of their own, so no fine bin is hot), destinations as
//     16-bit offsets;
//   apply (k_pb_apply): one workgroup per fine bin ORs its records into an
//     LDS accumulator (ds_or_b64), then test-and-sets the bin's peers with
//     plain stores: fr = acc & ~seen -> seen |= fr, nx = fr.
// Segments are sized at bootstrap from the overlay's edge counts, so no
// record needs a global atomic.  Source-side statistics are the push's
// (frontier, traversals, deliveries, undelivered sends to dead peers,
// digest, coverage); receive-side ones the apply's.  Results do not depend
// on the order records arrive in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "gossip_device.hpp"
#include "gossip_internal.hpp"
#include "gossip_stage.hpp"
#include "philox.hpp"

namespace gossip {

namespace {

constexpr int kPbWaves = kPbBlock / 64;
constexpr int kPbU = 4;  // 64-record batches per lane in flight

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// index i with lo[i] <= x < lo[i + 1] in a table of kN + 1 bounds padded with ~0 (lo[0] <= x)
template <uint32_t kN>
__host__ __device__ __forceinline__ uint32_t find_bin(const uint32_t* lo, uint32_t x) {
    static_assert((kN & (kN - 1)) == 0, "power of two");
    uint32_t i = 0;
#pragma unroll
    for (uint32_t step = kN / 2; step; step >>= 1) i += lo[i + step] <= x ? step : 0u;
    return i;
}

// Level 1's per-lane counters: Acc's fields, the counts held in 32 bits (a lane's share of one round stays
// far below 2^32; deliveries, undelivered sends and the digest stay 64-bit).  Acc's 64-bit counters took
// 22 of the kernel's 128 VGPRs and, with them, the staging loop spilled to scratch.
struct PbAcc {
    uint32_t frontier = 0, trav = 0, htrav = 0, covered = 0, fresh = 0, activated = 0, atomics = 0;
    unsigned long long deliv = 0, undeliv = 0, digest = 0;
    unsigned long long fresh_or[1] = {};
    __device__ Acc full() const {
        Acc f;
        f.frontier = frontier;
        f.trav = trav;
        f.htrav = htrav;
        f.covered = covered;
        f.fresh = fresh;
        f.activated = activated;
        f.atomics = atomics;
        f.deliv = deliv;
        f.undeliv = undeliv;
        f.digest = digest;
        f.fresh_or[0] = fresh_or[0];
        return f;
    }
};

// ---------------------------------------------------------------------------
// level 1: workgroup w's share of the frontier's deliveries -> coarse-bin records
// ---------------------------------------------------------------------------
// (Round 6: the expansion's next batch loaded into a second register set without copies spilled at 128 VGPRs and
// took level 1 from 5.56 to 7.99 ms per config-4 run; tools/experiments/r06_blocked_level1_expand_rotation.patch.)
template <bool CA, bool COV>
__global__ __launch_bounds__(kPbBlock) void k_pb_scatter(RoundArgs a, PbArgs p, uint32_t wd) {
    __shared__ uint32_t lo_s[kPbCoarse + 1];
    __shared__ uint8_t cmap_s[kPbMap];  // coarse bin of each id bucket's first peer (then a short walk)
    __shared__ uint32_t tk_s[kPbCoarseMax], wr_s[kPbH1 * kPbCoarseMax], gn_s[kPbH1 * kPbCoarseMax];
    __shared__ unsigned long long base_s[kPbCoarseMax];  // this workgroup's segment of each coarse bin
    __shared__ uint32_t cap_s[kPbCoarseMax];
    __shared__ uint32_t bd_s[kPbCoarseMax * kPbH1 * kPbB1];
    __shared__ unsigned long long bw_s[kPbCoarseMax * kPbH1 * kPbB1];
    __shared__ uint32_t pk_v[kPbWaves][128];
    __shared__ unsigned long long pk_m[kPbWaves][128];
    __shared__ unsigned int cov_s[COV ? 64 : 1];
    const uint32_t nc = p.n_coarse, wg = blockIdx.x;
    for (uint32_t i = threadIdx.x; i <= kPbCoarse; i += kPbBlock) lo_s[i] = i <= nc ? p.c_lo[i] : 0xFFFFFFFFu;
    stage_init<kPbH1>(tk_s, wr_s, gn_s, kPbCoarseMax, threadIdx.x, kPbBlock);
    for (uint32_t i = threadIdx.x; i < kPbCoarseMax; i += kPbBlock) {
        base_s[i] = i < nc ? p.s1_base[(uint64_t)wg * nc + i] : 0ull;
        cap_s[i] = i < nc ? p.s1_cap[(uint64_t)wg * nc + i] : 0u;
    }
    if (COV)
        for (uint32_t i = threadIdx.x; i < 64; i += kPbBlock) cov_s[i] = 0;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kPbMap; b += kPbBlock) cmap_s[b] = (uint8_t)find_bin<kPbCoarse>(lo_s, b << p.map_shift);
    __syncthreads();
    auto coarse_of = [&](uint32_t c) {
        uint32_t k = cmap_s[c >> p.map_shift];
        while (c >= lo_s[k + 1]) ++k;
        return k;
    };
    PbAcc acc;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    // generation g of coarse bin k goes to place g * kPbB1 of the workgroup's segment:
    // 32 lanes store the destinations (128 B), 32 the words (256 B)
    static_assert(2 * kPbB1 <= 64, "one wave flushes a generation");
    auto flush1 = [&](uint32_t k, uint32_t g) {
        const uint32_t pos = g * kPbB1;
        const uint32_t i = lane & (kPbB1 - 1);
        const uint32_t hb = stage_at<kPbB1, kPbH1>(k, g, 0);
        const uint32_t dv = bd_s[hb + i];
        const unsigned long long wv = bw_s[hb + i];
        lds_fence();
        if (lane == 0) stage_release<kPbH1>(wr_s, gn_s, k, g);
        if (pos + kPbB1 <= cap_s[k]) {
            const uint64_t at = base_s[k] + pos + i;
            if (lane < (int)kPbB1) p.r1_dst[at] = dv;
            else if (lane < 2 * (int)kPbB1) p.r1_w[at] = wv;
        } else if (lane == 0) {
            atomicOr(p.err, 1u);
        }
    };
    // the hubs' deliveries (c < direct_end): handleClient's test-and-set at once (k_push_*'s plain read,
    // then atomics only for new bits -- a hub holds every message after a few rounds)
    auto direct = [&](const uint32_t (&c)[kPbU], const unsigned long long (&m)[kPbU], bool (&rec)[kPbU]) {
        bool dir[kPbU];
        unsigned long long cur[kPbU];
        bool any = false;
#pragma unroll
        for (int j = 0; j < kPbU; ++j) {
            dir[j] = rec[j] && c[j] >= p.dir_lo && c[j] < p.dir_hi;
            any |= dir[j];
        }
        if (!__ballot(any)) return;  // (most batches: no hub among the destinations)
        // a.fold: the hub's own new words (nw, left for the split to clear) are not yet in seen everywhere
        unsigned long long nwc[kPbU];
        uint32_t lc[kPbU];  // local index of a direct destination
#pragma unroll
        for (int j = 0; j < kPbU; ++j) {
            lc[j] = dir[j] ? c[j] - p.dir_base : 0u;
            cur[j] = a.seen[lc[j]];
            nwc[j] = a.fold && dir[j] ? a.nw[lc[j]] : 0ull;
        }
#pragma unroll
        for (int j = 0; j < kPbU; ++j) {
            if (!dir[j]) continue;
            rec[j] = false;
            if (!(m[j] & ~(cur[j] | nwc[j]))) continue;  // all duplicates: dropped (peer.cpp:281)
            const unsigned long long fr =
                m[j] & ~nwc[j] & ~atomicOr(reinterpret_cast<unsigned long long*>(a.seen) + lc[j], m[j]);
            acc.atomics++;
            acc.fresh_or[0] |= fr;
            if (!fr) continue;
            const unsigned long long onx = atomicOr(reinterpret_cast<unsigned long long*>(a.nx) + lc[j], fr);
            acc.atomics++;
            acc.fresh += (unsigned long long)__popcll(fr);
            acc.activated += onx == 0;
            if (a.tnx && onx == 0) {  // the peer's tile joins the next round's frontier tiles
                unsigned long long* tw = reinterpret_cast<unsigned long long*>(a.tnx) + (lc[j] >> 12);
                const unsigned long long tb = 1ull << ((lc[j] >> 6) & 63);
                if (!(*tw & tb)) atomicOr(tw, tb);
            }
        }
    };
    // kPbU deliveries per lane (c: destination, bit 31 = masked or no edge): statistics, then records
    // (each delivery's message count is the popcount of its word, recomputed here: carried per record it
    // cost kPbU registers twice over and pushed the kernel past 128 VGPRs into scratch spills)
    auto emit = [&](const uint32_t (&c)[kPbU], const unsigned long long (&m)[kPbU]) {
        bool rec[kPbU];
        uint32_t k[kPbU], al[kPbU];
#pragma unroll
        for (int j = 0; j < kPbU; ++j) {
            rec[j] = !(c[j] & kMaskedEdge);  // connectedPeers.erase'd (peer.cpp:388), or no edge
            acc.trav += rec[j];
            if (CA) al[j] = a.alive[rec[j] ? c[j] >> 5 : 0];
        }
#pragma unroll
        for (int j = 0; j < kPbU; ++j) {
            if (CA && rec[j] && !((al[j] >> (c[j] & 31)) & 1u)) {  // send() to a dead peer fails (peer.cpp:312)
                acc.undeliv += (uint32_t)__popcll(m[j]);
                rec[j] = false;
            } else if (rec[j]) {
                acc.deliv += (uint32_t)__popcll(m[j]);  // sentTo.insert (peer.cpp:314)
            }
        }
        direct(c, m, rec);
#pragma unroll
        for (int j = 0; j < kPbU; ++j) k[j] = rec[j] ? coarse_of(c[j]) : 0u;
        stage<kPbU, kPbB1, kPbH1>(tk_s, wr_s, gn_s, bd_s, bw_s, k, c, m, rec, flush1, p.err);
    };

    // (1) heavy chunks wg, wg + kPbGrid, ..., one wave each (their rows' words are cleared by the split)
    {
        const uint32_t trav0 = acc.trav;
        for (uint64_t ci = wg + (uint64_t)wave * kPbGrid; ci < a.n_chunks; ci += (uint64_t)kPbGrid * kPbWaves) {
            const HeavyChunk ch = a.chunks[ci];
            const unsigned long long m = a.nw[ch.v];
            if (!m) continue;  // wave-uniform
            unsigned long long ms[kPbU];
#pragma unroll
            for (int j = 0; j < kPbU; ++j) ms[j] = m;
            for (uint64_t b = ch.e0; b < ch.e1; b += 64 * kPbU) {
                uint32_t c[kPbU];
#pragma unroll
                for (int j = 0; j < kPbU; ++j) {
                    const uint64_t e = b + j * 64 + lane;
                    c[j] = e < ch.e1 ? a.col[e] : kMaskedEdge;
                }
                emit(c, ms);
            }
        }
        acc.htrav = acc.trav - trav0;
    }
    // (2) the range's tiles: push-start statistics of their active peers, the light rows' words cleared
    // and the rows expanded 64 at a time from a wave-private packet (as k_push_light)
    {
        uint32_t* pv = pk_v[wave];
        unsigned long long* pm = pk_m[wave];
        uint32_t n_pk = 0;  // wave-uniform
        auto expand = [&] {
            wave_sync();
            const uint32_t cnt = n_pk < 64 ? n_pk : 64;
            const bool have = (uint32_t)lane < cnt;
            const uint64_t v = have ? pv[lane] : 0;
            const unsigned long long m = have ? pm[lane] : 0ull;
            uint32_t deg = 0;
            uint64_t rb = 0;
            if (have) {
                rb = a.rp[v];
                const uint64_t d = a.rp[v + 1] - rb;
                deg = d <= a.heavy ? (uint32_t)d : 0u;  // heavy rows: (1)
                // consumed: this buffer is the next round's accumulator (the hubs' words are read by
                // direct(), heavy rows' by their chunks: the split clears those)
                if (!p.clear_all && d <= a.heavy && v >= p.keep_end) a.nw[v] = 0ull;
            }
            const uint32_t rest = n_pk - cnt;
            wave_sync();
            if ((uint32_t)lane < rest) {
                pv[lane] = pv[64 + lane];
                pm[lane] = pm[64 + lane];
            }
            n_pk = rest;
            uint32_t incl = deg;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(incl, off);
                if (lane >= off) incl += y;
            }
            const uint32_t excl = incl - deg;
            const uint32_t total = __shfl(incl, 63);
            // batch base's deliveries; the next batch's col loads are issued before this one is emitted
            uint32_t c[kPbU], c2[kPbU];
            unsigned long long ms[kPbU], ms2[kPbU];
            auto batch = [&](uint32_t base, uint32_t (&c_)[kPbU], unsigned long long (&m_)[kPbU]) {
                uint64_t e[kPbU];
#pragma unroll
                for (int j = 0; j < kPbU; ++j) {
                    const uint32_t q = base + j * 64 + lane;
                    const int s = src_lane(incl, q);
                    e[j] = __shfl(rb, s) + (uint64_t)(q - __shfl(excl, s));
                    m_[j] = __shfl(m, s);
                }
#pragma unroll
                for (int j = 0; j < kPbU; ++j) c_[j] = base + j * 64 + lane < total ? a.col[e[j]] : kMaskedEdge;
            };
            if (total) batch(0, c, ms);
            for (uint32_t base = 0; base < total; base += 64 * kPbU) {
                const bool more = base + 64 * kPbU < total;  // wave-uniform
                if (more) batch(base + 64 * kPbU, c2, ms2);
                emit(c, ms);
                if (!more) break;
#pragma unroll
                for (int j = 0; j < kPbU; ++j) {
                    c[j] = c2[j];
                    ms[j] = ms2[j];
                }
            }
        };
        auto tile = [&](uint64_t t, unsigned long long m) {
            const uint64_t v = (t << 6) + lane;
            const bool act = m != 0;
            const unsigned long long bal = __ballot(act);
            if (!bal) return;
            if (act) {  // push start: the new words are the bits added to seen since the last one
                if (a.fold) {  // the previous round deferred: its receipts (m) join seen here
                    if (v < p.direct_end) atomicOr(reinterpret_cast<unsigned long long*>(a.seen) + v, m);
                    else a.seen[v] |= m;  // (only direct() writes seen during this pass, hubs only)
                }
                acc.frontier++;
                const uint32_t pc = (uint32_t)__popcll(m);
                acc.covered += pc;
                acc.digest += digest_weight((a.begin + v) * wd) * m;  // word 0 of wd
                if (COV)
                    for (unsigned long long x = m; x; x &= x - 1) atomicAdd(&cov_s[__builtin_ctzll(x)], 1u);
                const uint32_t pos = n_pk + lane_rank(bal);
                pv[pos] = (uint32_t)v;
                pm[pos] = m;
            }
            n_pk += (uint32_t)__popcll(bal);
            if (n_pk >= 64) expand();
        };
        const uint64_t n_tiles = (a.n_local + 63) >> 6;
        constexpr uint64_t kStride = (uint64_t)kPbGrid * kPbWaves;  // a wave's tiles: wg + kPbGrid (wave + 16 i)
        constexpr int kPre = 4;                                      // tiles' words in flight per wave
        // narrow rounds (p.marks, round 6): the new words of marked tiles only.  The marks of a wave's next 64
        // tiles come with one load per lane (their words lie kStride / 64 apart) at every 64th tile; unmarked
        // tiles skip their word loads.  (A separate loop over the marked tiles gave tile() a second call site,
        // which the compiler no longer inlined: 1 KB of scratch per lane, round 4 4.6 -> 24.6 ms.)
        unsigned long long mk_bits = ~0ull;  // wave-uniform
        uint32_t it = 0;
        for (uint64_t tb = wg + (uint64_t)kPbGrid * wave; tb < n_tiles; tb += kPre * kStride, it += kPre) {
            if (p.marks && (it & 63) == 0) {
                const uint64_t T = tb + (uint64_t)lane * kStride;
                mk_bits = __ballot(T < n_tiles && ((p.marks[T >> 6] >> (T & 63)) & 1ull));
            }
            unsigned long long m[kPre];
#pragma unroll
            for (int j = 0; j < kPre; ++j) {
                const uint64_t v = ((tb + j * kStride) << 6) + lane;
                m[j] = v < a.n_local && ((mk_bits >> ((it + j) & 63)) & 1ull) ? a.nw[v] : 0ull;
            }
#pragma unroll
            for (int j = 0; j < kPre; ++j)
                if (tb + j * kStride < n_tiles) tile(tb + j * kStride, m[j]);
        }
        if (n_pk) expand();  // n_pk < 64 here
    }
    // the partly filled buffers, padded to whole flushes; then the segments' lengths
    __syncthreads();
    for (uint32_t k = wave; k < nc; k += kPbWaves) {
        uint32_t g = 0;
        const uint32_t n = stage_open(tk_s, k, kPbB1, &g);
        if (!n) continue;  // wave-uniform
        if ((uint32_t)lane >= n && lane < (int)kPbB1) {
            const uint32_t s = stage_at<kPbB1, kPbH1>(k, g, lane);
            bd_s[s] = kPbPad;
            bw_s[s] = 0ull;
        }
        lds_fence();
        flush1(k, g);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nc; k += kPbBlock) p.s1_len[(uint64_t)wg * nc + k] = stage_len(tk_s, k, kPbB1);
    Acc fa = acc.full();
    flush<kPbWaves>(fa, a.st);
    if (COV) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 64; i += kPbBlock)
            if (cov_s[i]) atomicAdd(&a.cov[i], (unsigned long long)cov_s[i]);
    }
}

// ---------------------------------------------------------------------------
// level 2: slice sl of coarse bin k -- the segments of level-1 workgroups
// [sl * kPbGrid / kPbSlices, (sl + 1) * kPbGrid / kPbSlices) -> the bin's fine bins
// ---------------------------------------------------------------------------
// kRot (blocked_pipe, round 6): the next batch of records is loaded while this one is staged, into the other of
// two register sets (the loop unrolled by two, so no set is copied while its loads are in flight), from clamped
// addresses whatever the batch's end -- validity is applied where the records are used.  (Round 6's first try
// loaded `in ? record : pad` and copied the next batch's registers into the current ones at the loop's end: the
// select and the copies made every batch wait for the loads just issued, and it measured no gain.)
template <bool kRot>
__global__ __launch_bounds__(kPbBlock) void k_pb_split(PbArgs p) {
    constexpr uint32_t kN = 128;  // search table (>= kPbFineMax, a power of two)
    static_assert(kPbFineMax <= kN, "fine bins per coarse bin");
    __shared__ uint32_t flo_s[kN + 1];
    __shared__ uint32_t tk_s[kPbFineMax], wr_s[kPbH2 * kPbFineMax], gn_s[kPbH2 * kPbFineMax];
    __shared__ unsigned long long base_s[kPbFineMax];  // this slice's segment of each fine bin
    __shared__ uint32_t cap_s[kPbFineMax];
    constexpr uint32_t kSeg = kPbGrid / kPbSlices;     // the slice's level-1 segments of bin k: one
    __shared__ unsigned long long sb_s[kSeg];           // virtual array (prefix sums ps_s), so every wave
    __shared__ uint32_t ps_s[kSeg + 1];                 // stays busy however short the segments are
    __shared__ uint16_t bd_s[kPbFineMax * kPbH2 * kPbB2];
    __shared__ unsigned long long bw_s[kPbFineMax * kPbH2 * kPbB2];
    const uint32_t k = blockIdx.x / kPbSlices, sl = blockIdx.x % kPbSlices;
    const uint32_t f0 = p.c_fine[k], nf = p.c_fine[k + 1] - f0;
    for (uint32_t i = threadIdx.x; i <= kN; i += kPbBlock) flo_s[i] = i <= nf ? p.f_lo[f0 + i] : 0xFFFFFFFFu;
    stage_init<kPbH2>(tk_s, wr_s, gn_s, kPbFineMax, threadIdx.x, kPbBlock);
    for (uint32_t i = threadIdx.x; i < kPbFineMax; i += kPbBlock) {
        base_s[i] = i < nf ? p.s2_base[(uint64_t)sl * p.n_fine + f0 + i] : 0ull;
        cap_s[i] = i < nf ? p.s2_cap[(uint64_t)sl * p.n_fine + f0 + i] : 0u;
    }
    const uint32_t nc = p.n_coarse;
    const uint32_t w0 = sl * (kPbGrid / kPbSlices);
    static_assert(kSeg == 64, "one wave scans the segment lengths");
    if (threadIdx.x < 64) {
        const uint32_t i = threadIdx.x;
        sb_s[i] = p.s1_base[(uint64_t)(w0 + i) * nc + k];
        const uint32_t len = p.s1_len[(uint64_t)(w0 + i) * nc + k];
        uint32_t incl = len;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if ((int)i >= off) incl += y;
        }
        ps_s[i + 1] = incl;
        if (i == 0) ps_s[0] = 0;
    }
    if (p.clear_all) {  // a wide frontier: every new word, consumed by level 1, cleared in whole 16-B pieces
        u64x2* nw2 = reinterpret_cast<u64x2*>(p.nw);
        const uint64_t n2 = (p.n_local + 1) / 2;  // (the word arrays are allocated in whole pairs)
        for (uint64_t i = (uint64_t)blockIdx.x * kPbBlock + threadIdx.x; i < n2; i += (uint64_t)gridDim.x * kPbBlock)
            nw2[i] = u64x2{0ull, 0ull};
    } else {
        // the heavy rows' new words, consumed by level 1 (one word per row: its first chunk)
        for (uint64_t ci = (uint64_t)blockIdx.x * kPbBlock + threadIdx.x; ci < p.n_chunks;
             ci += (uint64_t)gridDim.x * kPbBlock) {
            const HeavyChunk ch = p.chunks[ci];
            if (ch.first == ci) p.nw[ch.v] = 0ull;
        }
        for (uint64_t v = (uint64_t)blockIdx.x * kPbBlock + threadIdx.x; v < p.direct_end;
             v += (uint64_t)gridDim.x * kPbBlock)
            p.nw[v] = 0ull;  // and the hubs'
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    static_assert(kPbB2 == 64, "a lane per record of a generation");
    auto flush2 = [&](uint32_t f, uint32_t g) {  // 64 destinations (128 B), 64 words (512 B)
        const uint32_t pos = g * kPbB2;
        const uint32_t hb = stage_at<kPbB2, kPbH2>(f, g, 0);
        const uint16_t dv = bd_s[hb + lane];
        const unsigned long long wv = bw_s[hb + lane];
        lds_fence();
        if (lane == 0) stage_release<kPbH2>(wr_s, gn_s, f, g);
        if (pos + kPbB2 <= cap_s[f]) {
            const uint64_t at = base_s[f] + pos + lane;
            p.r2_dst[at] = dv;
            p.r2_w[at] = wv;
        } else if (lane == 0) {
            atomicOr(p.err, 2u);
        }
    };
    if (!kRot) {
        const uint32_t n = ps_s[kSeg];
        for (uint32_t i0 = (uint32_t)wave * 64 * kPbU; i0 < n; i0 += kPbBlock * kPbU) {  // wave-uniform
            uint32_t d[kPbU], f[kPbU], dl[kPbU];
            unsigned long long x[kPbU];
            bool rec[kPbU];
#pragma unroll
            for (int j = 0; j < kPbU; ++j) {
                const uint32_t i = i0 + j * 64 + lane;
                const bool in = i < n;
                const uint32_t sg = in ? find_bin<kSeg>(ps_s, i) : 0u;  // ps_s[sg] <= i < ps_s[sg + 1]
                const uint64_t at = sb_s[sg] + (i - ps_s[sg]);
                d[j] = in ? p.r1_dst[at] : kPbPad;
                x[j] = in ? p.r1_w[at] : 0ull;
            }
#pragma unroll
            for (int j = 0; j < kPbU; ++j) {
                rec[j] = d[j] != kPbPad;
                f[j] = rec[j] ? find_bin<kN>(flo_s, d[j]) : 0u;
                dl[j] = d[j] - flo_s[f[j]];
            }
            stage<kPbU, kPbB2, kPbH2>(tk_s, wr_s, gn_s, bd_s, bw_s, f, dl, x, rec, flush2, p.err);
        }
    } else {
        const uint32_t n = ps_s[kSeg];
        constexpr uint32_t kStep = kPbBlock * kPbU;
        auto load = [&](uint32_t i0, uint32_t (&d)[kPbU], unsigned long long (&x)[kPbU]) {
#pragma unroll
            for (int j = 0; j < kPbU; ++j) {
                const uint32_t i = min(i0 + j * 64 + lane, n - 1);  // (n > 0 here) clamped: read, not used
                const uint32_t sg = find_bin<kSeg>(ps_s, i);       // ps_s[sg] <= i < ps_s[sg + 1]
                const uint64_t at = sb_s[sg] + (i - ps_s[sg]);
                d[j] = p.r1_dst[at];
                x[j] = p.r1_w[at];
            }
        };
        auto use = [&](uint32_t i0, const uint32_t (&d)[kPbU], const unsigned long long (&x)[kPbU]) {
            uint32_t f[kPbU], dl[kPbU];
            unsigned long long xv[kPbU];
            bool rec[kPbU];
#pragma unroll
            for (int j = 0; j < kPbU; ++j) {
                rec[j] = i0 + j * 64 + lane < n && d[j] != kPbPad;
                f[j] = rec[j] ? find_bin<kN>(flo_s, d[j]) : 0u;
                dl[j] = d[j] - flo_s[f[j]];
                xv[j] = x[j];
            }
            stage<kPbU, kPbB2, kPbH2>(tk_s, wr_s, gn_s, bd_s, bw_s, f, dl, xv, rec, flush2, p.err);
        };
        uint32_t dA[kPbU], dB[kPbU];
        unsigned long long xA[kPbU], xB[kPbU];
        uint32_t i0 = (uint32_t)wave * 64 * kPbU;
        if (i0 < n) load(i0, dA, xA);
        while (i0 < n) {  // wave-uniform
            load(i0 + kStep, dB, xB);  // (clamped: the last batch's prefetch reads record n - 1 again)
            use(i0, dA, xA);
            i0 += kStep;
            if (i0 >= n) break;
            load(i0 + kStep, dA, xA);
            use(i0, dB, xB);
            i0 += kStep;
        }
    }

    __syncthreads();
    for (uint32_t fb = wave; fb < nf; fb += kPbWaves) {
        uint32_t g = 0;
        const uint32_t c = stage_open(tk_s, fb, kPbB2, &g);
        if (!c) continue;
        if ((uint32_t)lane >= c) {
            const uint32_t s = stage_at<kPbB2, kPbH2>(fb, g, lane);
            bd_s[s] = 0xFFFFu;
            bw_s[s] = 0ull;
        }
        lds_fence();
        flush2(fb, g);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nf; i += kPbBlock)
        p.s2_len[(uint64_t)sl * p.n_fine + f0 + i] = stage_len(tk_s, i, kPbB2);
}

// ---------------------------------------------------------------------------
// apply: kPbApplyGrid workgroups, each looping over the fine bins f = w, w + grid, ... (whole tiles,
// <= kBinWords peers).  handleClient's test-and-set for every peer a record reached (peer.cpp:277-285):
// fr = (OR of its records) & ~seen.  A workgroup holds the 144 KB accumulator for its whole life: the
// next bin's segment table is loaded while this bin is swept, the accumulator is cleared by the sweep
// that reads it, and the statistics are flushed once (one workgroup per bin, 14.6 K of them at
// config 4, paid a launch, a clear, three dependent round trips and a flush per bin: 1.8 ms for round
// 3's 53.5 M records).
// ---------------------------------------------------------------------------
constexpr int kPbApplyGrid = 256;  // one per CU (the accumulator takes most of the LDS)
// kRot (blocked_pipe): the record loop as k_pb_split's -- two register sets in turn, clamped loads, and the
// destinations read as the 32-bit word of their pair (a u16 load compared as a 16-bit value kept a separate
// zero-extension, which waited for the load where it was issued)
template <bool kRot>
__global__ __launch_bounds__(1024) void k_pb_apply(RoundArgs a, PbArgs p) {
    __shared__ unsigned long long acc_s[kBinWords];
    __shared__ uint32_t meta_s[2][3 * kPbSlices + 2];  // per bin: s2_len[4], s2_base lo/hi [8], f_lo, f_lo + 1
    // the bin's activated tiles (a.tnx bits), gathered in LDS and OR-ed into a.tnx once per bin (round 6: a
    // read-then-atomic of the tnx word per activated tile inside the finish waited vmcnt(0) -- for the seen and
    // nx stores just issued too -- up to 18 times per wave and bin)
    constexpr uint32_t kMarkWords = (kBinWords / 64 + 63) / 64 + 1;
    __shared__ unsigned long long tmark_s[kMarkWords];
    for (uint32_t i = threadIdx.x; i < kBinWords; i += 1024) acc_s[i] = 0ull;
    if (threadIdx.x < kMarkWords) tmark_s[threadIdx.x] = 0ull;
    Acc acc;
    const int lane = threadIdx.x & 63;
    const uint64_t inj = injm(a, 0);
    constexpr int kJ = (kBinWords + 1023) / 1024;
    // the segment table of bin f into meta_s[b] (threads 0 .. 3 kPbSlices + 1)
    auto load_meta = [&](uint32_t f, int b) {
        const uint32_t t = threadIdx.x;
        if (f >= p.n_fine || t >= 3 * kPbSlices + 2) return;
        uint32_t x;
        if (t < kPbSlices) x = p.s2_len[(uint64_t)t * p.n_fine + f];
        else if (t < 3 * kPbSlices) {
            const uint32_t s = (t - kPbSlices) >> 1;
            const uint64_t base = p.s2_base[(uint64_t)s * p.n_fine + f];
            x = (t - kPbSlices) & 1 ? (uint32_t)(base >> 32) : (uint32_t)base;
        } else {
            x = p.f_lo[f + (t - 3 * kPbSlices)];
        }
        meta_s[b][t] = x;
    };
    int cb = 0;
    load_meta(blockIdx.x, 0);
    __syncthreads();
    for (uint32_t f = blockIdx.x; f < p.n_fine; f += gridDim.x, cb ^= 1) {
        const uint32_t* m = meta_s[cb];
        uint32_t ps[kPbSlices + 1];
        uint64_t sb[kPbSlices];
        ps[0] = 0;
#pragma unroll
        for (uint32_t s = 0; s < kPbSlices; ++s) {
            ps[s + 1] = ps[s] + m[s];
            sb[s] = (uint64_t)m[kPbSlices + 2 * s] | ((uint64_t)m[kPbSlices + 2 * s + 1] << 32);
        }
        const uint32_t v0 = m[3 * kPbSlices], nv = m[3 * kPbSlices + 1] - v0;
        const uint32_t total = ps[kPbSlices];
        load_meta(f + gridDim.x, cb ^ 1);  // (its own buffer: read after the barriers below)
        if (total == 0) {  // no record: nothing changes (nx is zero at a push round's start)
            __syncthreads();
            continue;
        }
        // the records of the bin's kPbSlices segments (one virtual array: prefix sums ps), kPbU per thread,
        // the next batch's loads in flight while this one is folded
        if (kRot) {
            auto pos = [&](uint32_t vi) {  // the record's position (vi < total)
                uint32_t sg = 0;
#pragma unroll
                for (uint32_t s = 1; s < kPbSlices; ++s) sg += vi >= ps[s];
                return sb[sg] + (vi - ps[sg]);
            };
            const uint32_t* r2d = reinterpret_cast<const uint32_t*>(p.r2_dst);
            auto load = [&](uint32_t v0_, uint32_t (&d)[kPbU], unsigned long long (&w)[kPbU]) {
#pragma unroll
                for (int j = 0; j < kPbU; ++j) {
                    const uint64_t at = pos(min(v0_ + j * 1024, total - 1));  // clamped: read, not used
                    d[j] = r2d[at >> 1];
                    w[j] = p.r2_w[at];
                }
            };
            auto fold = [&](uint32_t v0_, const uint32_t (&d)[kPbU], const unsigned long long (&w)[kPbU]) {
#pragma unroll
                for (int j = 0; j < kPbU; ++j) {
                    const uint32_t vi = v0_ + j * 1024;
                    const uint32_t dd = (d[j] >> ((uint32_t)(pos(min(vi, total - 1)) & 1) * 16)) & 0xFFFFu;
                    if (vi < total && dd != 0xFFFFu) atomicOr(&acc_s[dd], w[j]);  // ds_or_b64
                }
            };
            constexpr uint32_t kStep = 1024 * kPbU;
            uint32_t dA[kPbU], dB[kPbU];
            unsigned long long wA[kPbU], wB[kPbU];
            uint32_t vb = threadIdx.x;
            load(vb, dA, wA);
            while (vb < total) {
                load(vb + kStep, dB, wB);
                fold(vb, dA, wA);
                vb += kStep;
                if (vb >= total) break;
                load(vb + kStep, dA, wA);
                fold(vb, dB, wB);
                vb += kStep;
            }
        } else {
            auto load = [&](uint32_t v0_, uint16_t (&d)[kPbU], unsigned long long (&w)[kPbU]) {
#pragma unroll
                for (int j = 0; j < kPbU; ++j) {
                    const uint32_t vi = v0_ + j * 1024;
                    uint32_t sg = 0;
#pragma unroll
                    for (uint32_t s = 1; s < kPbSlices; ++s) sg += vi >= ps[s];
                    const bool in = vi < total;
                    const uint64_t at = in ? sb[sg] + (vi - ps[sg]) : 0;
                    d[j] = in ? p.r2_dst[at] : (uint16_t)0xFFFFu;
                    w[j] = in ? p.r2_w[at] : 0ull;
                }
            };
            uint16_t d[kPbU], d2[kPbU];
            unsigned long long w[kPbU], w2[kPbU];
            uint32_t vb = threadIdx.x;
            load(vb, d, w);
            while (vb < total) {
                load(vb + 1024 * kPbU, d2, w2);
#pragma unroll
                for (int j = 0; j < kPbU; ++j)
                    if (d[j] != 0xFFFFu) atomicOr(&acc_s[d[j]], w[j]);  // ds_or_b64
                vb += 1024 * kPbU;
#pragma unroll
                for (int j = 0; j < kPbU; ++j) {
                    d[j] = d2[j];
                    w[j] = w2[j];
                }
            }
        }
        __syncthreads();
        // a thread's peers i = tid + 1024 j (a wave covers one 64-peer tile): every seen word it needs
        // loaded at once; the accumulator words read are cleared for the next bin.  A tile with a record
        // reads and, if a peer of it learns, writes its seen and nx words whole (512 B each): single-word
        // stores into a 64-B sector cost a read-modify-write at the memory, and at round 4's 17 % of
        // peers learning nearly every sector gets one.  Untouched peers rewrite their own seen word and a
        // zero nx word (nx is zero at a push round's start).
        unsigned long long x[kJ], sv[kJ];
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
            const uint32_t i = threadIdx.x + 1024u * j;
            x[j] = i < nv ? acc_s[i] : 0ull;
            if (x[j]) acc_s[i] = 0ull;
            const bool tile = __ballot(x[j] != 0) != 0ull;
            sv[j] = tile && i < nv ? a.seen[v0 + i] : 0ull;
        }
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
            const uint32_t i = threadIdx.x + 1024u * j;
            if (i >= ((nv + 63) & ~63u)) break;  // wave-uniform
            const uint64_t v = v0 + i;
            const unsigned long long fr = x[j] & inj & ~sv[j];
            const unsigned long long b = __ballot(fr != 0);
            if (b && i < nv) {  // new -> Message-List insert (peer.cpp:281-282)
                a.seen[v] = sv[j] | fr;
                a.nx[v] = fr;
            }
            if (fr) {
                acc.fresh += (unsigned long long)__popcll(fr);
                acc.activated++;
                acc.fresh_or[0] |= fr;
            }
            if (a.tnx && b && lane == 0) {  // the tile joins the next round's frontier tiles
                const uint64_t t = v >> 6;
                atomicOr(&tmark_s[(t >> 6) - ((uint64_t)v0 >> 12)], 1ull << (t & 63));  // (v0: a whole tile)
            }
        }
        __syncthreads();  // the accumulator is clear and the next segment table is in
        if (a.tnx && threadIdx.x < kMarkWords) {
            const unsigned long long m = tmark_s[threadIdx.x];
            if (m) {
                atomicOr(reinterpret_cast<unsigned long long*>(a.tnx) + ((uint64_t)v0 >> 12) + threadIdx.x, m);
                tmark_s[threadIdx.x] = 0ull;  // (read and cleared by this thread alone; the next bin marks after
            }                                  //  its record loop's barrier)
        }
    }
    flush<1024 / 64>(acc, a.st);
}

// ---- bootstrap: bins and segment capacities from the overlay's edges -------
// in-degree per 64-peer tile, and the row pointer at every tile boundary
__global__ void k_pb_tiles(const uint64_t* rp, const uint32_t* col, uint64_t n_local, uint64_t n_edges,
                           unsigned long long* tile_in, uint64_t* rp_tile) {
    const uint64_t n_tiles = (n_local + 63) / 64;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_edges; e += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&tile_in[(col[e] & ~kMaskedEdge) >> 6], 1ull);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n_tiles; i += (uint64_t)gridDim.x * blockDim.x)
        rp_tile[i] = rp[i * 64 < n_local ? i * 64 : n_local];
}

__device__ __forceinline__ void pb_count_edge(const PbArgs& p, const uint32_t* clo_s, uint32_t w, uint32_t v,
                                              uint32_t* cnt1, uint32_t* cnt2) {
    if (v < p.direct_end) return;  // delivered at once, never a record
    const uint32_t k = find_bin<kPbCoarse>(clo_s, v);
    uint32_t lo = p.c_fine[k], hi = p.c_fine[k + 1];  // the fine bin: binary search over the coarse bin's
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (p.f_lo[mid] <= v) lo = mid;
        else hi = mid;
    }
    atomicAdd(&cnt1[(uint64_t)w * p.n_coarse + k], 1u);
    atomicAdd(&cnt2[(uint64_t)(w / (kPbGrid / kPbSlices)) * p.n_fine + lo], 1u);
}

// every edge u -> v: cnt1[w][coarse(v)]++, cnt2[slice(w)][fine(v)]++ with w the level-1 workgroup that
// expands it (the worst case of a round: every source active).  Light rows: one thread each; heavy
// chunks: one wave each.
__global__ __launch_bounds__(256) void k_pb_count(const uint64_t* rp, const uint32_t* col, uint64_t n_local,
                                                  uint32_t heavy, const HeavyChunk* chunks, uint64_t n_chunks,
                                                  PbArgs p, uint32_t* cnt1, uint32_t* cnt2) {
    __shared__ uint32_t clo_s[kPbCoarse + 1];
    for (uint32_t i = threadIdx.x; i <= kPbCoarse; i += blockDim.x) clo_s[i] = i <= p.n_coarse ? p.c_lo[i] : 0xFFFFFFFFu;
    __syncthreads();
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n_local; u += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e0 = rp[u], e1 = rp[u + 1];
        if (e1 - e0 > heavy) continue;
        const uint32_t w = (uint32_t)((u >> 6) % kPbGrid);
        for (uint64_t e = e0; e < e1; ++e) pb_count_edge(p, clo_s, w, col[e] & ~kMaskedEdge, cnt1, cnt2);
    }
    const int lane = threadIdx.x & 63;
    for (uint64_t ci = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; ci < n_chunks;
         ci += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const HeavyChunk ch = chunks[ci];
        const uint32_t w = (uint32_t)(ci % kPbGrid);
        for (uint64_t e = ch.e0 + lane; e < ch.e1; e += 64) pb_count_edge(p, clo_s, w, col[e] & ~kMaskedEdge, cnt1, cnt2);
    }
}

}  // namespace

void free_pb(PbState* p) {
    hipFree(p->c_lo);
    hipFree(p->c_fine);
    hipFree(p->f_lo);
    hipFree(p->s1_base);
    hipFree(p->s2_base);
    hipFree(p->s1_cap);
    hipFree(p->s2_cap);
    hipFree(p->s1_len);
    hipFree(p->s2_len);
    hipFree(p->err);
    hipFree(p->r1_dst);
    hipFree(p->r1_w);
    hipFree(p->r2_dst);
    hipFree(p->r2_w);
    hipFree(p->rec_out);
    *p = PbState{};
}

PbArgs pb_args(const PbState& p) {
    PbArgs a{};
    a.n_coarse = p.n_coarse;
    a.n_fine = p.n_fine;
    a.c_lo = p.c_lo;
    a.c_fine = p.c_fine;
    a.f_lo = p.f_lo;
    a.s1_base = p.s1_base;
    a.s1_cap = p.s1_cap;
    a.s1_len = p.s1_len;
    a.s2_base = p.s2_base;
    a.s2_cap = p.s2_cap;
    a.s2_len = p.s2_len;
    a.r1_dst = p.r1_dst;
    a.r1_w = p.r1_w;
    a.r2_dst = p.r2_dst;
    a.r2_w = p.r2_w;
    a.err = p.err;
    a.direct_end = p.direct_end;
    a.map_shift = p.map_shift;
    if (p.rank_mode) {  // the own block [c_lo[own], c_lo[own + 1]) is delivered at once (set by the caller)
        a.keep_end = 0;
    } else {
        a.dir_lo = 0;
        a.dir_hi = p.direct_end;
        a.dir_base = 0;
        a.keep_end = p.direct_end;
    }
    return a;
}

#define PCHECK(x)                                                         \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            if (err) *err = std::string(#x ": ") + hipGetErrorString(e_); \
            hipGetLastError();                                            \
            hipFree(d_cnt1);                                              \
            hipFree(d_cnt2);                                              \
            hipFree(d_rpt);                                               \
            hipFree(d_tin);                                               \
            free_pb(&st);                                                 \
            return e_;                                                    \
        }                                                                 \
    } while (0)

hipError_t build_pb(const uint64_t* rp, const uint32_t* col, uint64_t n_local, uint64_t n_edges, uint32_t heavy,
                    const HeavyChunk* chunks, uint64_t n_chunks, uint64_t direct_in, hipStream_t s, PbState* out,
                    std::string* err) {
    PbState st;
    uint32_t *d_cnt1 = nullptr, *d_cnt2 = nullptr;
    uint64_t* d_rpt = nullptr;
    unsigned long long* d_tin = nullptr;
    if (!n_edges || n_local >= (1ull << 31)) return hipErrorInvalidValue;
    const uint64_t n_tiles = (n_local + 63) / 64;
    // in-degree per tile, row pointer per tile boundary
    std::vector<unsigned long long> tin(n_tiles);
    std::vector<uint64_t> rpt(n_tiles + 1);
    PCHECK(hipMalloc((void**)&d_tin, n_tiles * sizeof(unsigned long long)));
    PCHECK(hipMalloc((void**)&d_rpt, (n_tiles + 1) * sizeof(uint64_t)));
    PCHECK(hipMemsetAsync(d_tin, 0, n_tiles * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_pb_tiles, dim3(8192), dim3(256), 0, s, rp, col, n_local, n_edges, d_tin, d_rpt);
    PCHECK(hipGetLastError());
    PCHECK(hipMemcpyAsync(tin.data(), d_tin, n_tiles * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    PCHECK(hipMemcpyAsync(rpt.data(), d_rpt, (n_tiles + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    PCHECK(hipStreamSynchronize(s));
    hipFree(d_tin);
    hipFree(d_rpt);
    d_tin = nullptr;
    d_rpt = nullptr;
    // fine bins: runs of whole tiles, <= kBinWords peers and <= kPbFineIn in-degree (at least one tile)
    std::vector<uint32_t> f_lo;
    std::vector<uint64_t> f_in;
    for (uint64_t t = 0; t < n_tiles;) {
        f_lo.push_back((uint32_t)(t * 64));
        uint64_t in = 0, peers = 0;
        while (t < n_tiles && (peers == 0 || (peers + 64 <= kBinWords && in + tin[t] <= kPbFineIn))) {
            in += tin[t];
            peers += 64;
            ++t;
        }
        f_in.push_back(in);
    }
    const uint64_t n_fine = f_lo.size();
    f_lo.push_back((uint32_t)n_local);
    // the hubs: the leading tiles of over direct_in in-degree each (a Chung-Lu overlay's lowest ids)
    {
        uint64_t t = 0;
        while (t < n_tiles && tin[t] > direct_in) ++t;
        st.direct_end = (uint32_t)std::min<uint64_t>(t * 64, n_local);
    }
    // coarse bins: runs of whole fine bins of about equal in-degree, <= kPbFineMax fine bins each, at most
    // kPbCoarseMax of them (an overlay with more fine bins than fit gets no blocked rounds)
    if (n_fine > (uint64_t)kPbCoarseMax * kPbFineMax) {
        if (err) *err = "blocked rounds: more fine bins than the level-2 staging can hold";
        free_pb(&st);
        return hipErrorInvalidValue;
    }
    std::vector<uint32_t> c_fine;
    for (uint64_t target = (n_edges + kPbCoarseMax - 1) / kPbCoarseMax;; target += target / 8 + 1) {
        c_fine.assign(1, 0u);
        uint64_t sum = 0;
        for (uint64_t b = 0; b < n_fine; ++b) {
            if (b > c_fine.back() && (b - c_fine.back() >= kPbFineMax || sum + f_in[b] > target)) {
                c_fine.push_back((uint32_t)b);
                sum = 0;
            }
            sum += f_in[b];
        }
        c_fine.push_back((uint32_t)n_fine);
        if (c_fine.size() - 1 <= kPbCoarseMax) break;
    }
    st.n_coarse = (uint32_t)(c_fine.size() - 1);
    st.n_fine = n_fine;
    while (((uint64_t)kPbMap << st.map_shift) < n_local) ++st.map_shift;
    std::vector<uint32_t> c_lo(st.n_coarse + 1);
    for (uint32_t k = 0; k <= st.n_coarse; ++k) c_lo[k] = f_lo[c_fine[k]];
    PCHECK(hipMalloc((void**)&st.f_lo, f_lo.size() * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.c_lo, c_lo.size() * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.c_fine, c_fine.size() * sizeof(uint32_t)));
    PCHECK(hipMemcpyAsync(st.f_lo, f_lo.data(), f_lo.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    PCHECK(hipMemcpyAsync(st.c_lo, c_lo.data(), c_lo.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    PCHECK(hipMemcpyAsync(st.c_fine, c_fine.data(), c_fine.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    // edge counts per (producer, bin): the segments' capacities
    const uint64_t n1s = (uint64_t)kPbGrid * st.n_coarse, n2s = (uint64_t)kPbSlices * n_fine;
    PCHECK(hipMalloc((void**)&d_cnt1, n1s * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&d_cnt2, n2s * sizeof(uint32_t)));
    PCHECK(hipMemsetAsync(d_cnt1, 0, n1s * sizeof(uint32_t), s));
    PCHECK(hipMemsetAsync(d_cnt2, 0, n2s * sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_pb_count, dim3(8192), dim3(256), 0, s, rp, col, n_local, heavy, chunks, n_chunks,
                       pb_args(st), d_cnt1, d_cnt2);
    PCHECK(hipGetLastError());
    std::vector<uint32_t> cnt1(n1s), cnt2(n2s), cap1(n1s), cap2(n2s);
    std::vector<uint64_t> base1(n1s), base2(n2s);
    PCHECK(hipMemcpyAsync(cnt1.data(), d_cnt1, n1s * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PCHECK(hipMemcpyAsync(cnt2.data(), d_cnt2, n2s * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PCHECK(hipStreamSynchronize(s));
    hipFree(d_cnt1);
    hipFree(d_cnt2);
    d_cnt1 = d_cnt2 = nullptr;
    uint64_t n1 = 0, n2 = 0;
    for (uint64_t i = 0; i < n1s; ++i) {  // whole flushes (the last one padded)
        cap1[i] = (cnt1[i] + kPbB1 - 1) / kPbB1 * kPbB1;
        base1[i] = n1;
        n1 += cap1[i];
    }
    for (uint64_t i = 0; i < n2s; ++i) {
        cap2[i] = (cnt2[i] + kPbB2 - 1) / kPbB2 * kPbB2;
        base2[i] = n2;
        n2 += cap2[i];
    }
    st.n1 = n1;
    st.n2 = n2;
    size_t free_b = 0, total_b = 0;
    PCHECK(hipMemGetInfo(&free_b, &total_b));
    if (n1 * 12 + n2 * 10 + (1ull << 30) > free_b) {
        free_pb(&st);
        if (err) *err = "blocked-push records do not fit in free device memory";
        return hipErrorOutOfMemory;
    }
    PCHECK(hipMalloc((void**)&st.s1_base, n1s * sizeof(uint64_t)));
    PCHECK(hipMalloc((void**)&st.s2_base, n2s * sizeof(uint64_t)));
    PCHECK(hipMalloc((void**)&st.s1_cap, n1s * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.s2_cap, n2s * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.s1_len, n1s * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.s2_len, n2s * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.err, sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.r1_dst, (n1 + 1) * sizeof(uint32_t)));
    PCHECK(hipMalloc((void**)&st.r1_w, (n1 + 1) * sizeof(unsigned long long)));
    PCHECK(hipMalloc((void**)&st.r2_dst, (n2 + 1) * sizeof(uint16_t)));
    PCHECK(hipMalloc((void**)&st.r2_w, (n2 + 1) * sizeof(unsigned long long)));
    PCHECK(hipMemcpyAsync(st.s1_base, base1.data(), n1s * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    PCHECK(hipMemcpyAsync(st.s2_base, base2.data(), n2s * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    PCHECK(hipMemcpyAsync(st.s1_cap, cap1.data(), n1s * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    PCHECK(hipMemcpyAsync(st.s2_cap, cap2.data(), n2s * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    PCHECK(hipMemsetAsync(st.s1_len, 0, n1s * sizeof(uint32_t), s));
    PCHECK(hipMemsetAsync(st.s2_len, 0, n2s * sizeof(uint32_t), s));
    PCHECK(hipMemsetAsync(st.err, 0, sizeof(uint32_t), s));
    PCHECK(hipStreamSynchronize(s));  // the host vectors go out of scope
    *out = st;
    return hipSuccess;
}
#undef PCHECK

// ---- a vertex block's sparse push as records (P > 1) ----
namespace {
// every edge u -> v of the block into another block q: cnt[w][q]++ with w the level-1 workgroup that expands it
__global__ __launch_bounds__(256) void k_px_count(const uint64_t* rp, const uint32_t* col, uint64_t n_local,
                                                  uint32_t heavy, const HeavyChunk* chunks, uint64_t n_chunks,
                                                  const uint32_t* lo, uint32_t world, uint32_t own, uint32_t* cnt) {
    __shared__ uint32_t lo_s[kPbCoarse + 1];
    for (uint32_t i = threadIdx.x; i <= kPbCoarse; i += blockDim.x) lo_s[i] = i <= world ? lo[i] : 0xFFFFFFFFu;
    __syncthreads();
    auto edge = [&](uint32_t w, uint32_t v) {
        const uint32_t q = find_bin<kPbCoarse>(lo_s, v);
        if (q != own) atomicAdd(&cnt[(uint64_t)w * world + q], 1u);
    };
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n_local; u += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e0 = rp[u], e1 = rp[u + 1];
        if (e1 - e0 > heavy) continue;
        const uint32_t w = (uint32_t)((u >> 6) % kPbGrid);
        for (uint64_t e = e0; e < e1; ++e) edge(w, col[e] & ~kMaskedEdge);
    }
    const int lane = threadIdx.x & 63;
    for (uint64_t ci = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; ci < n_chunks;
         ci += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const HeavyChunk ch = chunks[ci];
        const uint32_t w = (uint32_t)(ci % kPbGrid);
        for (uint64_t e = ch.e0 + lane; e < ch.e1; e += 64) edge(w, col[e] & ~kMaskedEdge);
    }
}

// block (w, q): segment (w, q)'s records to seg + (q * stride + sum of the lengths of segments (w' < w, q)) * 2
__global__ __launch_bounds__(256) void k_px_pack(PbArgs p, uint32_t world, uint32_t own, const uint64_t* part,
                                                 uint64_t stride, uint64_t* seg, unsigned long long* counts,
                                                 const HeavyChunk* chunks, uint64_t n_chunks, uint64_t* nw) {
    const uint32_t w = blockIdx.x, q = blockIdx.y;
    __shared__ unsigned long long off_s;
    if (threadIdx.x < 64) {  // one wave: the lengths of the segments before this one (and the total, block 0)
        const uint32_t n = w == 0 ? kPbGrid : w;
        unsigned long long x = 0;
        for (uint32_t i = threadIdx.x; i < n; i += 64) x += i < w || w == 0 ? p.s1_len[(uint64_t)i * world + q] : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        if (threadIdx.x == 0) {
            off_s = w == 0 ? 0ull : x;
            if (w == 0) counts[q] = q == own ? 0ull : x;
        }
    }
    __syncthreads();
    if (q != own) {
        const uint64_t len = p.s1_len[(uint64_t)w * world + q], base = p.s1_base[(uint64_t)w * world + q];
        uint64_t* out = seg + (q * stride + off_s) * 2;
        const uint64_t first = part[q];
        for (uint64_t i = threadIdx.x; i < len; i += blockDim.x) {
            const uint32_t d = p.r1_dst[base + i];
            const bool pad = d == kPbPad;
            out[2 * i] = pad ? first : (uint64_t)d;
            out[2 * i + 1] = pad ? 0ull : p.r1_w[base + i];
        }
    }
    if (q == 0)  // the heavy rows' words, read by every workgroup's chunks during level 1
        for (uint64_t ci = (uint64_t)w * blockDim.x + threadIdx.x; ci < n_chunks; ci += (uint64_t)kPbGrid * blockDim.x)
            nw[chunks[ci].v] = 0ull;
}
}  // namespace

hipError_t build_px(const uint64_t* rp, const uint32_t* col, uint64_t n_local, uint64_t n_global, uint32_t heavy,
                    const HeavyChunk* chunks, uint64_t n_chunks, const uint64_t* part, uint32_t world, uint32_t own,
                    hipStream_t s, PbState* out, std::string* err) {
    PbState st;
    uint32_t* d_cnt = nullptr;
    auto bail = [&](hipError_t e, const char* what) {
        if (err) *err = std::string(what) + ": " + hipGetErrorString(e);
        hipGetLastError();
        hipFree(d_cnt);
        free_pb(&st);
        return e;
    };
    if (world < 2 || world > kPbCoarseMax || n_global >= (1ull << 32)) return hipErrorInvalidValue;
    st.rank_mode = 1;
    st.n_coarse = world;
    while (((uint64_t)kPbMap << st.map_shift) < n_global) ++st.map_shift;
    std::vector<uint32_t> lo(world + 1);
    for (uint32_t q = 0; q <= world; ++q) lo[q] = (uint32_t)part[q];
    hipError_t e = hipMalloc((void**)&st.c_lo, (world + 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpyAsync(st.c_lo, lo.data(), (world + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, s);
    const uint64_t n1s = (uint64_t)kPbGrid * world;
    if (e == hipSuccess) e = hipMalloc((void**)&d_cnt, n1s * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(d_cnt, 0, n1s * sizeof(uint32_t), s);
    if (e != hipSuccess) return bail(e, "record push tables");
    hipLaunchKernelGGL(k_px_count, dim3(8192), dim3(256), 0, s, rp, col, n_local, heavy, chunks, n_chunks, st.c_lo,
                       world, own, d_cnt);
    if ((e = hipGetLastError()) != hipSuccess) return bail(e, "k_px_count");
    std::vector<uint32_t> cnt(n1s), cap(n1s);
    std::vector<uint64_t> base(n1s), per_q(world, 0);
    if ((e = hipMemcpyAsync(cnt.data(), d_cnt, n1s * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return bail(e, "record push counts");
    uint64_t n1 = 0;
    for (uint64_t i = 0; i < n1s; ++i) {  // whole flushes (the last one padded)
        cap[i] = (cnt[i] + kPbB1 - 1) / kPbB1 * kPbB1;
        base[i] = n1;
        n1 += cap[i];
        per_q[i % world] += cap[i];
    }
    // the packed records of destination q at rec_out + q * stride (the receivers grow their buffers to a round's
    // records, gossip_dist.hip)
    uint64_t stride = 0;
    for (uint32_t q = 0; q < world; ++q) stride = std::max(stride, per_q[q]);
    st.rec_stride = std::max<uint64_t>(stride, 1);
    st.n1 = n1;
    size_t free_b = 0, total_b = 0;
    if ((e = hipMemGetInfo(&free_b, &total_b)) != hipSuccess) return bail(e, "hipMemGetInfo");
    if (n1 * 12 + (uint64_t)world * st.rec_stride * 16 + (1ull << 30) > free_b) {
        hipFree(d_cnt);
        free_pb(&st);
        if (err) *err = "record-push segments do not fit in free device memory";
        return hipErrorOutOfMemory;
    }
    if ((e = hipMalloc((void**)&st.s1_base, n1s * sizeof(uint64_t))) != hipSuccess ||
        (e = hipMalloc((void**)&st.s1_cap, n1s * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void**)&st.s1_len, n1s * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void**)&st.err, sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void**)&st.r1_dst, (n1 + 1) * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void**)&st.r1_w, (n1 + 1) * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipMalloc((void**)&st.rec_out, (uint64_t)world * st.rec_stride * 16)) != hipSuccess ||
        (e = hipMemcpyAsync(st.s1_base, base.data(), n1s * sizeof(uint64_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(st.s1_cap, cap.data(), n1s * sizeof(uint32_t), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemsetAsync(st.s1_len, 0, n1s * sizeof(uint32_t), s)) != hipSuccess ||
        (e = hipMemsetAsync(st.err, 0, sizeof(uint32_t), s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return bail(e, "record push segments");
    hipFree(d_cnt);
    *out = st;
    return hipSuccess;
}

hipError_t launch_px_pack(const PbArgs& p, uint32_t world, uint32_t own, const uint64_t* d_part, uint64_t stride,
                          uint64_t* seg, unsigned long long* counts, const HeavyChunk* chunks, uint64_t n_chunks,
                          uint64_t* nw, hipStream_t s) {
    hipLaunchKernelGGL(k_px_pack, dim3(kPbGrid, world), dim3(256), 0, s, p, world, own, d_part, stride, seg, counts,
                       chunks, n_chunks, nw);
    return hipGetLastError();
}

hipError_t launch_pb_scatter(const RoundArgs& a, const PbArgs& p, bool check_alive, uint32_t wd, hipStream_t s) {
    const bool cov = a.cov != nullptr;
#define GOSSIP_PB(CA, COV) hipLaunchKernelGGL((k_pb_scatter<CA, COV>), dim3(kPbGrid), dim3(kPbBlock), 0, s, a, p, wd)
    if (cov) {
        if (check_alive) GOSSIP_PB(true, true);
        else GOSSIP_PB(false, true);
    } else {
        if (check_alive) GOSSIP_PB(true, false);
        else GOSSIP_PB(false, false);
    }
#undef GOSSIP_PB
    return hipGetLastError();
}

hipError_t launch_pb_split(const PbArgs& p, hipStream_t s) {
    if (p.pipe) hipLaunchKernelGGL(k_pb_split<true>, dim3(p.n_coarse * kPbSlices), dim3(kPbBlock), 0, s, p);
    else hipLaunchKernelGGL(k_pb_split<false>, dim3(p.n_coarse * kPbSlices), dim3(kPbBlock), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_pb_apply(const RoundArgs& a, const PbArgs& p, hipStream_t s) {
    if (!p.n_fine) return hipSuccess;
    const unsigned g = (unsigned)std::min<uint64_t>(p.n_fine, kPbApplyGrid);
    if (p.pipe) hipLaunchKernelGGL(k_pb_apply<true>, dim3(g), dim3(1024), 0, s, a, p);
    else hipLaunchKernelGGL(k_pb_apply<false>, dim3(g), dim3(1024), 0, s, a, p);
    return hipGetLastError();
}

}  // namespace gossip
