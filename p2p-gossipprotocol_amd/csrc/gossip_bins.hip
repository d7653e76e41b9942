// gossip_bins.hip -- bootstrap-time bin layout for binned dense rounds.
//
// A dense round of the round contract is, per owned peer v,
//   next[v] = (OR over u in N(v) of new[u]) & ~seen[v]
// -- handleClient's dedup (peer.cpp:277-285) applied to every copy that
// broadcastMessage (peer.cpp:310-316) sends.  Gathering new[u] per edge costs
// one random HBM line per edge.  The overlay is static, so instead every edge
// into a light owned peer v gets a fixed "slot" in a destination-bin-major
// array.  On a symmetric overlay the in-edges of v are v's own row, so the
// layout is built from the owned rows alone: destination = the row (local),
// source = the column (global).  That holds for one partition (P = 1) and for
// a vertex block of a partitioned run, where the sources' words come from the
// all-gathered buffer.  A binned round then
//   (1) scatter (k_bin_scatter_lds): per source chunk (kBinChunkWords words,
//       staged in LDS), walk the chunk's edges in bin order (the cb lists) and
//       store new[src] into their slots.  Within a (chunk, bin) pair the slots
//       are consecutive, so the stores form short runs; the runs of the chunks
//       an XCD works on together are adjacent and merge in its L2;
//   (2) apply (k_bin_apply): fold each bin's slots into an LDS accumulator.
// Rows longer than the heavy threshold are not binned: k_pull_heavy gathers
// them (they are satisfied after a few edges).
//
// Layout (built here, once per overlay):
//   bins    : whole 64-peer tiles, <= kBinWords/Wp peers and <= kBinSlotCap slots
//   bdst    : u16 per slot -> destination - bin.v0 (padding slots: 0, val 0)
//   val     : Wp u64 per slot (the source's words of the last binned round)
//   cb_src  : u16 chunk-local source per binned edge, (source chunk, bin) order;
//             bit 15 marks the first entry of a run of consecutive slots
//   cb_run  : u32 per run: slot - position (the slot of entry p is p + cb_run[run])
//   cb_grp  : u32 per 64 entries: the run of the group's first entry, so a
//             wave finds each lane's run with one ballot of the bit-15 flags
//   chunk_begin     : offsets of each (global) source chunk's cb entries
//   units, xcd_units: scatter work units and their split over the 8 XCDs
// Construction: (a) 64-bit key (bin << 32 | source) per edge of a light row,
// radix sort -> slot of an edge = b.s0 + (position - b.u0), so a bin's slots are
// in source order; (b) key = chunk(source) * n_bins + bin per slot-order
// position, stable sort -> cb order.  The (chunk, bin) slots are contiguous
// because chunks are source ranges, and the cb entries of a pair are in slot
// order, so a run of consecutive entries stores to consecutive slots; (c) the
// slots are stored once per run (about 7 entries at config 4), not per entry.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "gossip_internal.hpp"

namespace gossip {

namespace {

unsigned gridn(uint64_t items) {
    uint64_t g = (items + 255) / 256;
    if (g < 1) g = 1;
    if (g > 65536) g = 65536;
    return (unsigned)g;
}

// Per 64-peer tile: number of binned slots (sum of light row lengths; on a
// symmetric overlay a row's length is also its in-degree) + light bitmap.
__global__ void k_tile_slots(const uint64_t* rp, uint64_t n, uint32_t heavy, uint32_t* tile_slots,
                             unsigned long long* light_bits) {
    const uint64_t n_tiles = (n + 63) / 64;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n_tiles * 64;
         v += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t d = 0;
        bool light = false;
        if (v < n) {
            d = rp[v + 1] - rp[v];
            light = d <= heavy;
        }
        const unsigned long long bits = __ballot(light);
        uint64_t sl = light ? d : 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sl += __shfl_xor(sl, off);
        if ((threadIdx.x & 63) == 0) {  // blockDim is a multiple of 64: a wave is one tile
            tile_slots[v >> 6] = (uint32_t)sl;
            light_bits[v >> 6] = bits;
        }
    }
}

__global__ void k_degree(const uint64_t* rp, uint64_t n, uint32_t* deg) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x)
        deg[v] = (uint32_t)(rp[v + 1] - rp[v]);
}

__global__ void k_edge_rows(const uint64_t* rp, uint64_t n, uint32_t* row) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x)
        for (uint64_t e = rp[v]; e < rp[v + 1]; ++e) row[e] = (uint32_t)v;
}

// (a) key = bin of the (light) destination row << 32 | source; heavy rows last.
__global__ void k_bin_keys(const uint32_t* row, const uint32_t* col, uint64_t m, const unsigned long long* light_bits,
                           const uint32_t* bin_of_tile, unsigned long long* keys, uint32_t* vals) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = row[e];
        const bool light = (light_bits[v >> 6] >> (v & 63)) & 1ull;
        keys[e] = light ? ((unsigned long long)bin_of_tile[v >> 6] << 32) | (col[e] & ~kMaskedEdge) : ~0ull;
        vals[e] = (uint32_t)e;
    }
}

__global__ void k_bin_assign(const unsigned long long* skeys, const uint32_t* svals, uint64_t m, const Bin* bins,
                             uint32_t n_bins, const uint32_t* row, uint16_t* bdst) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = skeys[i] >> 32;
        if (b >= n_bins) continue;
        const Bin bn = bins[b];
        bdst[bn.s0 + (i - bn.u0)] = (uint16_t)(row[svals[i]] - bn.v0);
    }
}

// (b) per position i of the slot order (sorted keys of (a)): key = chunk(source)
// * n_bins + bin, chunk(u) = (u / seg) * cps + u % seg / chunk.  Sorted stably, so
// the entries of a (chunk, bin) pair stay in slot order: consecutive cb entries
// of a pair have consecutive slots.
__global__ void k_cb_keys(const unsigned long long* skeys, uint64_t n_binned, uint32_t n_bins, uint32_t chunk,
                          uint32_t seg, uint32_t cps, uint32_t* keys, uint32_t* vals) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_binned;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = skeys[i];
        const uint32_t u = (uint32_t)(k & 0xFFFFFFFFu);
        keys[i] = (u / seg * cps + u % seg / chunk) * n_bins + (uint32_t)(k >> 32);
        vals[i] = (uint32_t)i;
    }
}

__global__ void k_cb_fill(const uint32_t* svals, uint64_t n_binned, const unsigned long long* skeys, const Bin* bins,
                          uint32_t chunk, uint32_t seg, uint32_t* cb_slot, uint16_t* cb_src) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_binned;
         p += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t i = svals[p];
        const uint64_t k = skeys[i];
        const Bin bn = bins[k >> 32];
        cb_slot[p] = (uint32_t)(bn.s0 + (i - bn.u0));
        cb_src[p] = (uint16_t)((uint32_t)(k & 0xFFFFFFFFu) % seg % chunk);  // source, local to its chunk
    }
}

// (c) run encoding: an entry starts a run unless its slot follows the previous
// entry's; the slot of entry p of run r is p + cb_run[r] (mod 2^32).
__global__ void k_run_flags(const uint32_t* cb_slot, uint64_t n_binned, uint16_t* cb_src, uint32_t* flag) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_binned;
         p += (uint64_t)gridDim.x * blockDim.x) {
        const bool st = p == 0 || cb_slot[p] != cb_slot[p - 1] + 1;
        flag[p] = st;
        if (st) cb_src[p] |= kRunStart;
    }
}

// ids: inclusive prefix sum of the flags (run of entry p = ids[p] - 1)
__global__ void k_run_fill(const uint32_t* cb_slot, const uint32_t* flag, const uint32_t* ids, uint64_t n_binned,
                           uint32_t* cb_run, uint32_t* cb_grp, uint32_t* run_start) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_binned;
         p += (uint64_t)gridDim.x * blockDim.x) {
        if (flag[p]) {
            cb_run[ids[p] - 1] = cb_slot[p] - (uint32_t)p;
            run_start[ids[p] - 1] = cb_slot[p];
        }
        if ((p & 63) == 0) cb_grp[p >> 6] = ids[p] - 1;
    }
}

// (d) the apply side of the streamed layout (val in cb order): the runs in
// slot order (ap_start sorted, ap_run = slot - position as cb_run), the first
// slot of each run flagged in bdst, and per 64-slot group the number of runs
// that start before it.  The value of slot q of run r sits at q - ap_run[r].
__global__ void k_ap_flags(const uint32_t* ap_start, uint64_t n_runs, uint16_t* bdst) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_runs; r += (uint64_t)gridDim.x * blockDim.x)
        bdst[ap_start[r]] |= kRunStart;
}

__global__ void k_ap_grp(const uint32_t* ap_start, uint64_t n_runs, uint64_t n_groups, uint32_t* ap_grp) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t want = g * 64;
        uint64_t lo = 0, hi = n_runs;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (ap_start[mid] < want) lo = mid + 1;
            else hi = mid;
        }
        ap_grp[g] = (uint32_t)lo;
    }
}

// chunk_begin[c] = first cb position whose key >= c * n_bins (keys sorted).
__global__ void k_chunk_bounds(const uint32_t* skeys, uint64_t n_binned, uint32_t n_bins, uint64_t n_chunks,
                               uint64_t* chunk_begin) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > n_chunks) return;
    if (c == n_chunks) {
        chunk_begin[c] = n_binned;
        return;
    }
    const uint64_t want = c * n_bins;
    uint64_t lo = 0, hi = n_binned;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (skeys[mid] < want) lo = mid + 1;
        else hi = mid;
    }
    chunk_begin[c] = lo;
}

#define BCHECK(x)                                                         \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            if (err) *err = std::string(#x ": ") + hipGetErrorString(e_); \
            rc = e_;                                                      \
            goto done;                                                    \
        }                                                                 \
    } while (0)

}  // namespace

void free_bins(BinState* b) {
    hipFree(b->bins);
    hipFree(b->cb_src);
    hipFree(b->cb_run);
    hipFree(b->cb_grp);
    hipFree(b->ap_run);
    hipFree(b->ap_grp);
    hipFree(b->chunk_begin);
    hipFree(b->units);
    hipFree(b->stage_units);
    hipFree(b->xcd_units);
    hipFree(b->bdst);
    hipFree(b->val);
    hipFree(b->dummy);
    hipFree(b->deg);
    *b = BinState{};
}

hipError_t build_bins(const uint64_t* rp, const uint32_t* col, uint64_t n_local, uint64_t n_global, uint64_t m,
                      uint32_t heavy, uint32_t Wp, bool stream, uint32_t bin_words_req, uint32_t chunk_words_req,
                      uint64_t seg, uint64_t min_units, hipStream_t s, BinState* out, std::string* err) {
    hipError_t rc = hipSuccess;
    const uint64_t n_tiles = (n_local + 63) / 64;
    // bigger bins -> longer slot runs per (source chunk, bin) in the scatter
    // (measured: 16 K-word bins 86 ms/step at config 4, 8 K-word bins 101 ms)
    // ... and several bins per CU on small overlays (config 2, 2^20 peers: 57 bins of 18 K left most CUs
    // idle in the apply; 256 bins of 4 K: kernels 9.2-9.3 -> 7.9 ms per step; round 5: 512 bins of 2 K with
    // the small-bin apply, eight workgroups per CU, 5.06 -> 4.68 ms per step, profiles/r05/ab/r05b/sweep_c2.txt;
    // config 3 keeps whole bins: 4 K bins cost it 0.5 ms)
    uint32_t bin_words = (uint32_t)std::min<uint64_t>(kBinWords, std::max<uint64_t>(2048, n_local * Wp / 512 / 512 * 512));
    if (bin_words_req) bin_words = std::max<uint32_t>(512, std::min<uint32_t>(kBinWords, bin_words_req / 512 * 512));
    const uint32_t max_peers = bin_words / Wp;  // a multiple of 64 for Wp <= 8
    const uint64_t slot_cap = kBinSlotCap * bin_words / kBinWords;
    uint32_t* tile_slots = nullptr;
    unsigned long long* light_bits = nullptr;
    uint32_t* bin_of_tile = nullptr;
    unsigned long long *keys64_in = nullptr, *keys64_out = nullptr;
    uint32_t *keys_in = nullptr, *vals_in = nullptr, *keys_out = nullptr, *vals_out = nullptr;
    uint32_t* row = nullptr;
    uint32_t* cb_slot = nullptr;  // per cb entry, until the run encoding is built
    // source chunk (chosen once the bins are known, below)
    uint64_t chunk_words = kBinChunkWords, chunk = 0, n_chunks = 0;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    BinState st;
    std::vector<uint32_t> h_tile(n_tiles), h_bot(n_tiles);
    std::vector<Bin> h_bins;
    uint64_t slots = 0, upos = 0;
    int end_bit = 33, end_bit2 = 1;
    size_t free_b = 0, total_b = 0;

    if (m >= kNoSlot || n_global >= (1ull << 32)) {
        if (err) *err = "too many edges for 32-bit slots";
        return hipErrorInvalidValue;
    }
    BCHECK(hipMalloc((void**)&tile_slots, n_tiles * sizeof(uint32_t)));
    BCHECK(hipMalloc((void**)&light_bits, n_tiles * sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_tile_slots, dim3(gridn(n_tiles * 64)), dim3(256), 0, s, rp, n_local, heavy, tile_slots,
                       light_bits);
    BCHECK(hipGetLastError());
    BCHECK(hipMemcpyAsync(h_tile.data(), tile_slots, n_tiles * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    BCHECK(hipStreamSynchronize(s));

    // bins: greedy runs of whole tiles
    for (uint64_t t = 0; t < n_tiles;) {
        Bin b{};
        b.v0 = (uint32_t)(t * 64);
        b.s0 = slots;
        b.u0 = upos;
        uint64_t cnt = 0, peers = 0;
        while (t < n_tiles && (peers == 0 || (peers + 64 <= max_peers && cnt + h_tile[t] <= slot_cap))) {
            h_bot[t] = (uint32_t)h_bins.size();
            cnt += h_tile[t];
            peers += 64;
            ++t;
        }
        b.v1 = (uint32_t)std::min<uint64_t>(b.v0 + peers, n_local);
        upos += cnt;
        slots += (cnt + kBinSlotPad - 1) / kBinSlotPad * kBinSlotPad;
        b.s1 = b.s0 + cnt;
        h_bins.push_back(b);
    }
    while ((1ull << (end_bit - 32)) <= h_bins.size()) ++end_bit;
    // Source chunk: the whole LDS slice, unless a quarter of it or less still gives runs of about 32
    // entries (run ≈ binned edges · |chunk| · |bin| / (n_local · n_global)); then that (a multiple of
    // 512 words, at least 1024), so the scatter has several units per CU.  Config 2 (2^20): 57 whole
    // chunks left 199 of the 256 CUs idle (scatter 10.6 -> 3.5-3.7 ms per step with 1024-word chunks);
    // config 3 (2^24): 2.95-2.99 -> 2.54-2.57 ms with 4096; config 5 (2^26, runs of ≈ 35 at the whole
    // slice) measured 12.5 against 14.4 ms with 16896-word chunks, so near-full chunks stay whole.
    if (upos) {
        const double want = 32.0 * (double)n_global * (double)n_local / ((double)upos * (double)(bin_words / Wp)) * Wp;
        if (want * 4 <= (double)kBinChunkWords) chunk_words = std::max<uint64_t>(1024, ((uint64_t)want + 511) / 512 * 512);
    }
    if (chunk_words_req)
        chunk_words = std::max<uint64_t>(512, std::min<uint64_t>(kBinChunkWords, chunk_words_req / 512 * 512));
    chunk = std::max<uint64_t>(64, chunk_words / Wp);
    // source segments: one (seg = n_global rounded to whole chunks) unless the caller cuts the ids (a vertex
    // block: bin_segment), chunks never straddle a segment
    if (!seg) seg = (n_global + chunk - 1) / chunk * chunk;
    chunk = std::min<uint64_t>(chunk, seg);
    st.seg = seg;
    st.cps = (seg + chunk - 1) / chunk;
    n_chunks = (n_global + seg - 1) / seg * st.cps;
    if (seg >= (1ull << 32) || seg % 64) {
        if (err) *err = "source segments must be whole 64-peer tiles below 2^32 peers";
        rc = hipErrorInvalidValue;
        goto done;
    }
    if (n_chunks * h_bins.size() >= kNoSlot) {
        if (err) *err = "too many (chunk, bin) pairs for 32-bit keys";
        rc = hipErrorInvalidValue;
        goto done;
    }
    // (the kNoSlot sentinel's low end_bit2 bits are all ones: it sorts last)
    while ((1ull << end_bit2) <= n_chunks * h_bins.size()) ++end_bit2;

    // memory peak: row + 64-bit keys in/out + vals in/out (+ temp) next to bdst/val
    BCHECK(hipMemGetInfo(&free_b, &total_b));
    {
        const uint64_t persist = slots * 2 + slots * Wp * 8 + upos * 8 + h_bins.size() * sizeof(Bin);
        const uint64_t peak = m * 36 + persist + (1ull << 30);
        if (peak > free_b) {
            if (err) *err = "bin layout does not fit in free device memory";
            rc = hipErrorOutOfMemory;
            goto done;
        }
    }
    BCHECK(hipMalloc((void**)&st.bins, h_bins.size() * sizeof(Bin)));
    BCHECK(hipMemcpyAsync(st.bins, h_bins.data(), h_bins.size() * sizeof(Bin), hipMemcpyHostToDevice, s));
    BCHECK(hipMalloc((void**)&bin_of_tile, n_tiles * sizeof(uint32_t)));
    BCHECK(hipMemcpyAsync(bin_of_tile, h_bot.data(), n_tiles * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    BCHECK(hipMalloc((void**)&row, (m + 1) * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_edge_rows, dim3(gridn(n_local)), dim3(256), 0, s, rp, n_local, row);
    BCHECK(hipGetLastError());

    // (a) slots
    BCHECK(hipMalloc((void**)&keys64_in, (m + 1) * sizeof(unsigned long long)));
    BCHECK(hipMalloc((void**)&keys64_out, (m + 1) * sizeof(unsigned long long)));
    BCHECK(hipMalloc((void**)&vals_in, (m + 1) * sizeof(uint32_t)));
    BCHECK(hipMalloc((void**)&vals_out, (m + 1) * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_bin_keys, dim3(gridn(m)), dim3(256), 0, s, row, col, m, light_bits, bin_of_tile, keys64_in,
                       vals_in);
    BCHECK(hipGetLastError());
    BCHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys64_in, keys64_out, vals_in, vals_out, (size_t)m,
                                              0, end_bit, s));
    BCHECK(hipMalloc(&temp, temp_bytes + 16));
    BCHECK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys64_in, keys64_out, vals_in, vals_out, (size_t)m, 0,
                                              end_bit, s));
    BCHECK(hipStreamSynchronize(s));
    hipFree(keys64_in);
    hipFree(temp);
    keys64_in = nullptr;
    temp = nullptr;

    st.n_bins = h_bins.size();
    st.bin_words = bin_words;
    st.n_slots = slots;
    st.n_binned = upos;
    st.n_chunks = n_chunks;
    st.chunk = chunk;
    // (+64: the apply reads whole 64-slot groups; val is indexed by slot or, streamed, by cb position)
    BCHECK(hipMalloc((void**)&st.bdst, (slots + 64) * sizeof(uint16_t)));
    BCHECK(hipMalloc((void**)&st.val, (slots + 64) * Wp * sizeof(uint64_t)));
    BCHECK(hipMemsetAsync(st.bdst, 0, (slots + 64) * sizeof(uint16_t), s));
    BCHECK(hipMemsetAsync(st.val, 0, (slots + 64) * Wp * sizeof(uint64_t), s));
    BCHECK(hipMalloc((void**)&st.dummy, (uint64_t)kScatterGrid * kScatterBlock * Wp * sizeof(uint64_t)));
    BCHECK(hipMalloc((void**)&st.deg, (n_local + 1) * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_degree, dim3(gridn(n_local)), dim3(256), 0, s, rp, n_local, st.deg);
    BCHECK(hipGetLastError());
    hipLaunchKernelGGL(k_bin_assign, dim3(gridn(m)), dim3(256), 0, s, keys64_out, vals_out, m, st.bins,
                       (uint32_t)st.n_bins, row, st.bdst);
    BCHECK(hipGetLastError());
    BCHECK(hipStreamSynchronize(s));
    hipFree(row);
    row = nullptr;

    // (b) cb order: (source chunk, bin), slot order inside a pair
    BCHECK(hipMalloc((void**)&keys_in, (upos + 1) * sizeof(uint32_t)));
    BCHECK(hipMalloc((void**)&keys_out, (upos + 1) * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_cb_keys, dim3(gridn(upos)), dim3(256), 0, s, keys64_out, upos, (uint32_t)st.n_bins,
                       (uint32_t)chunk, (uint32_t)st.seg, (uint32_t)st.cps, keys_in, vals_in);
    BCHECK(hipGetLastError());
    temp_bytes = 0;
    BCHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys_in, keys_out, vals_in, vals_out, (size_t)upos,
                                              0, end_bit2, s));
    BCHECK(hipMalloc(&temp, temp_bytes + 16));
    BCHECK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (size_t)upos, 0,
                                              end_bit2, s));
    BCHECK(hipStreamSynchronize(s));
    hipFree(keys_in);
    hipFree(vals_in);
    hipFree(temp);
    keys_in = vals_in = nullptr;
    temp = nullptr;
    BCHECK(hipMalloc((void**)&cb_slot, (upos + 1) * sizeof(uint32_t)));
    BCHECK(hipMalloc((void**)&st.cb_src, (upos + 16) * sizeof(uint16_t)));  // k_bin_stream reads aligned 8-entry blocks
    BCHECK(hipMalloc((void**)&st.chunk_begin, (n_chunks + 1) * sizeof(uint64_t)));
    hipLaunchKernelGGL(k_cb_fill, dim3(gridn(upos)), dim3(256), 0, s, vals_out, upos, keys64_out, st.bins,
                       (uint32_t)chunk, (uint32_t)st.seg, cb_slot, st.cb_src);
    BCHECK(hipGetLastError());
    hipLaunchKernelGGL(k_chunk_bounds, dim3(gridn(n_chunks + 1)), dim3(256), 0, s, keys_out, upos,
                       (uint32_t)st.n_bins, n_chunks, st.chunk_begin);
    BCHECK(hipGetLastError());
    BCHECK(hipStreamSynchronize(s));
    hipFree(keys64_out);
    keys64_out = nullptr;

    // (c) runs: flags into keys_out, their inclusive sum into vals_out (both >= upos + 1 words)
    {
        uint32_t n_runs = 0;
        if (upos) {
            hipLaunchKernelGGL(k_run_flags, dim3(gridn(upos)), dim3(256), 0, s, cb_slot, upos, st.cb_src, keys_out);
            BCHECK(hipGetLastError());
            temp_bytes = 0;
            BCHECK(hipcub::DeviceScan::InclusiveSum(nullptr, temp_bytes, keys_out, vals_out, upos, s));
            BCHECK(hipMalloc(&temp, temp_bytes + 16));
            BCHECK(hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, keys_out, vals_out, upos, s));
            BCHECK(hipMemcpyAsync(&n_runs, vals_out + upos - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            BCHECK(hipStreamSynchronize(s));
            hipFree(temp);
            temp = nullptr;
        }
        st.n_runs = n_runs;
        BCHECK(hipMalloc((void**)&st.cb_run, ((uint64_t)n_runs + 1) * sizeof(uint32_t)));
        BCHECK(hipMalloc((void**)&st.cb_grp, ((upos + 63) / 64 + 1) * sizeof(uint32_t)));
        // run starts (slot of each run's first entry) in cb_slot's place once it is consumed: keys_in
        BCHECK(hipMalloc((void**)&keys_in, ((uint64_t)n_runs + 1) * sizeof(uint32_t)));
        if (upos) {
            hipLaunchKernelGGL(k_run_fill, dim3(gridn(upos)), dim3(256), 0, s, cb_slot, keys_out, vals_out, upos,
                               st.cb_run, st.cb_grp, keys_in);
            BCHECK(hipGetLastError());
        }
        BCHECK(hipStreamSynchronize(s));
        hipFree(cb_slot);
        cb_slot = nullptr;
        // (d) apply side of the streamed layout: runs sorted by first slot (keys_out / vals_out are free again)
        const uint64_t n_groups = (slots + 63) / 64 + 1;
        if (!stream) goto no_stream;
        BCHECK(hipMalloc((void**)&st.ap_run, ((uint64_t)n_runs + 1) * sizeof(uint32_t)));
        BCHECK(hipMalloc((void**)&st.ap_grp, n_groups * sizeof(uint32_t)));
        if (n_runs) {
            int end_bit3 = 1;
            while (end_bit3 < 32 && (1ull << end_bit3) <= slots) ++end_bit3;
            temp_bytes = 0;
            BCHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys_in, keys_out, st.cb_run, st.ap_run,
                                                      (size_t)n_runs, 0, end_bit3, s));
            BCHECK(hipMalloc(&temp, temp_bytes + 16));
            BCHECK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, st.cb_run, st.ap_run,
                                                      (size_t)n_runs, 0, end_bit3, s));
            hipLaunchKernelGGL(k_ap_flags, dim3(gridn(n_runs)), dim3(256), 0, s, keys_out, (uint64_t)n_runs, st.bdst);
            BCHECK(hipGetLastError());
        }
        hipLaunchKernelGGL(k_ap_grp, dim3(gridn(n_groups)), dim3(256), 0, s, keys_out, (uint64_t)n_runs, n_groups,
                           st.ap_grp);
        BCHECK(hipGetLastError());
        BCHECK(hipStreamSynchronize(s));
        hipFree(temp);
        temp = nullptr;
    no_stream:
        hipFree(keys_in);
        keys_in = nullptr;
    }

    // scatter work units (every chunk has at least one: its first unit books
    // the chunk's source-side stats).  Row mode: a unit is a whole chunk, except
    // hub chunks (more than kHubFactor times the mean), which are cut into units
    // of about the mean; the units, in chunk order, form rows of kScatterGrid / 8,
    // row r goes to XCD r % 8, and member j of the XCD takes unit j of each of
    // its rows, so the workgroups of a row stage consecutive chunks and write
    // adjacent slot runs in every bin at about the same time (adjacent runs can
    // merge in the XCD's L2; with the single-role scatter 36.0 against 39.2 ms
    // per step for capped units dealt round-robin; global
    // rows over all XCDs measured no better).  Rows are dealt round-robin over
    // the XCDs (round 4): cut into 8 contiguous ranges of equal entry counts,
    // the XCD of the high-id chunks (more, shorter chunks: more staging per
    // entry) took 4.8 ms and the first 3.6 (config 4, k_bin_stream).
    // xcd_units[8] holds the unit count (a multiple of the row length).
    {
        std::vector<uint64_t> cbeg(n_chunks + 1);
        BCHECK(hipMemcpy(cbeg.data(), st.chunk_begin, (n_chunks + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
        std::vector<BinUnit> units;
        std::vector<uint64_t> xu(9, 0);
        const uint64_t members = kScatterGrid / 8;
        {
            const uint64_t mean = std::max<uint64_t>(1024, upos / std::max<uint64_t>(1, n_chunks));
            // min_units ("scatter_units"): chunks split into units of at most upos / min_units entries, so a
            // small overlay's few chunks still spread over the grid (config 2: 410 chunks of about 18 K entries
            // for 256 workgroups, each unit a chain of dependent round trips)
            const uint64_t cap = min_units ? std::max<uint64_t>(256, (upos + min_units - 1) / min_units) : ~0ull;
            for (uint64_t c = 0; c < n_chunks; ++c) {
                const uint64_t len = cbeg[c + 1] - cbeg[c];
                // a chunk of the last segment that starts past the ids has no sources (n = 100000 in segments
                // of 1600 and chunks of 1024: chunk 125 starts at 100224; its staging read past the gather buffer)
                if (chunk_vb(c, st.seg, st.cps, chunk) >= n_global) continue;
                uint64_t k = len > kHubFactor * mean ? (len + mean - 1) / mean : 1;
                if (len > cap) k = std::max<uint64_t>(k, (len + cap - 1) / cap);
                for (uint64_t j = 0; j < k; ++j)
                    units.push_back(
                        BinUnit{(uint32_t)c, j == 0 ? 1u : 0u, cbeg[c] + len * j / k, cbeg[c] + len * (j + 1) / k});
            }
            while (units.size() % members) units.push_back(BinUnit{0u, 0u, 0, 0});  // empty: skipped
            xu[8] = units.size();
        }
        st.n_units = units.size();
        st.h_units = units;
        BCHECK(hipMalloc((void**)&st.units, units.size() * sizeof(BinUnit)));
        BCHECK(hipMemcpy(st.units, units.data(), units.size() * sizeof(BinUnit), hipMemcpyHostToDevice));
        BCHECK(hipMalloc((void**)&st.xcd_units, 9 * sizeof(uint64_t)));
        BCHECK(hipMemcpy(st.xcd_units, xu.data(), 9 * sizeof(uint64_t), hipMemcpyHostToDevice));
    }

done:
    hipFree(tile_slots);
    hipFree(light_bits);
    hipFree(bin_of_tile);
    hipFree(keys64_in);
    hipFree(keys64_out);
    hipFree(keys_in);
    hipFree(vals_in);
    hipFree(keys_out);
    hipFree(vals_out);
    hipFree(temp);
    hipFree(row);
    hipFree(cb_slot);
    if (rc != hipSuccess) {
        hipGetLastError();  // clear a sticky allocation error
        free_bins(&st);
        return rc;
    }
    *out = st;
    return hipSuccess;
}

// The staged order of the units (a pipelined dense exchange, gossip_dist.hip): group 0 = the units whose
// chunk lies inside the own block [begin, end) (their words are local when the exchange starts), group 1 + j
// = the others of segments s = j (mod S) (stage j of the exchange delivers those segments' words from every
// block); each group in chunk order, padded to whole rows of kScatterGrid / 8 units.  A chunk that straddles
// the own block's edge waits for its segment's stage.
hipError_t build_stage_units(BinState* b, uint32_t S, uint64_t begin, uint64_t end, uint64_t n_global) {
    if (S < 1 || S > kMaxStages) return hipErrorInvalidValue;
    if (b->stages == S) return hipSuccess;
    const uint64_t members = kScatterGrid / 8;
    std::vector<std::vector<BinUnit>> grp(S + 1);
    for (const BinUnit& u : b->h_units) {
        if (u.p0 >= u.p1 && !u.first) continue;  // row padding
        const uint64_t vb = chunk_vb(u.c, b->seg, b->cps, b->chunk), ve = chunk_ve(u.c, b->seg, b->cps, b->chunk, n_global);
        const bool own = vb >= begin && ve <= end;
        grp[own ? 0 : 1 + (u.c / b->cps) % S].push_back(u);
    }
    std::vector<BinUnit> all;
    for (uint32_t g = 0; g <= S; ++g) {
        b->stage_lo[g] = all.size();
        all.insert(all.end(), grp[g].begin(), grp[g].end());
        while (all.size() % members) all.push_back(BinUnit{0u, 0u, 0, 0});
    }
    b->stage_lo[S + 1] = all.size();
    hipFree(b->stage_units);
    b->stage_units = nullptr;
    b->stages = 0;
    hipError_t e = hipMalloc((void**)&b->stage_units, std::max<size_t>(all.size(), 1) * sizeof(BinUnit));
    if (e == hipSuccess && !all.empty())
        e = hipMemcpy(b->stage_units, all.data(), all.size() * sizeof(BinUnit), hipMemcpyHostToDevice);
    if (e == hipSuccess) b->stages = S;
    return e;
}

}  // namespace gossip
