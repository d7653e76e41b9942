// gossip_internal.hpp -- internal (non-ABI) declarations of libgossip_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/gossip/gossip.h"

namespace gossip {

// roctx range around a round or one of its phases (rocprofv3 --marker-trace shows them per round;
// without a profiler attached a push/pop is a call into an empty dispatch table)
struct TraceRange {
    template <class... A>
    explicit TraceRange(const char* fmt, A... args) {
        char buf[64];
        std::snprintf(buf, sizeof(buf), fmt, args...);
        roctxRangePushA(buf);
    }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

constexpr uint32_t kMaskedEdge = 0x80000000u;  // col[e] bit 31: edge dropped by liveness (peer.cpp:388)
constexpr uint32_t kHeavyDegree = 256;         // default: rows longer than this go to the edge-chunked kernels
constexpr uint32_t kHeavyDegreeLarge = 512;    // ... on overlays of kHeavyLargePeers peers or more (round 6, config 4:
constexpr uint64_t kHeavyLargePeers = 1ull << 27;  // 44.05 -> 43.47 ms per step in one process; config 5 at 2^26
                                               // measured 21.80 -> 22.02 and keeps 256)
constexpr uint32_t kHeavyChunk = 1024;         // edges per heavy chunk (one wave); 256 below 2^22 owned peers
constexpr int kBlock = 256;                    // 4 waves of 64
constexpr int kMaxWords = 8;                   // M <= 512 concurrent messages
constexpr int kStatLines = 64;                 // striped DevStats lines per round (summed at read)
constexpr uint32_t kHeavyExitEvery = 4;        // k_pull_heavy checks its early exit every 4 batches of 64 edges

// Per-round device counters (all integer; order-independent sums).
struct DevStats {
    unsigned long long frontier, traversals, deliveries, undelivered, new_receipts, injected, died, reports,
        seed_removals, digest, covered, heavy_traversals, live_checked, activated, pull_edges, pull_gathers,
        reconnects, rejoined, atomics,  // atomics: device-scope atomics issued on peer state (seen, nx, marks)
        diag,                           // measurement counters (GOSSIP_PULL_DIAG)
        dead_covered;                   // (peer, message) pairs held by the peers that died this round
    unsigned long long fresh_or[8];     // OR of the round's receipts (the next round's new words), word w
};
constexpr int kStatSums = 21;                 // fields summed; the kMaxWords after them are OR-ed
constexpr int kStatFields = kStatSums + 8;
static_assert(sizeof(DevStats) == kStatFields * 8, "DevStats layout");

struct HeavyChunk {
    uint32_t v;      // local row
    uint32_t first;  // index of the row's first chunk (the row's word in RoundArgs.hacc)
    uint64_t e0, e1;
};

// Binned dense rounds (layout in gossip_bins.hip).
constexpr uint32_t kBinWords = 18432;       // LDS accumulator words per bin (144 KB; "bin_words": fewer)
constexpr uint32_t kBinSlotPad = 8;         // bin slot ranges padded to 8 slots (16-B loads)
constexpr uint64_t kBinSlotCap = 1u << 18;  // slots per bin (load balance between bins)
constexpr uint32_t kBinChunkWords = 18432;     // source chunk: its new words (144 KB) are staged in LDS
constexpr uint64_t kHubFactor = 4;             // chunks with more than 4x the mean cb entries are split into units
constexpr int kScatterBlock = 1024;            // k_bin_scatter_lds: one 16-wave workgroup per CU
constexpr int kScatterGrid = 256;              // one workgroup per CU
constexpr uint32_t kSmallChunkWords = 4096;    // streamed scatter of chunks this small: 256-thread blocks ...
constexpr int kSmallGrid = 1024;               // ... four per CU
constexpr uint32_t kSmallBinWords = 2048;      // streamed apply of bins this small: 256-thread blocks, eight per CU
constexpr uint32_t kApplyRow = 32;            // streamed apply: consecutive bins one XCD group applies together
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr uint16_t kRunStart = 0x8000u;        // cb_src flag; chunk-local sources are < kBinChunkWords < 2^15
static_assert(kBinChunkWords < kRunStart, "chunk-local sources fit 15 bits");

constexpr uint32_t kMaxStages = 16;   // pipelined dense exchange: source segments delivered in at most this many stages
constexpr uint32_t kMaxWorld = 64;    // blocks of a partitioned run (their bounds are staged in LDS by the exchange kernels)

struct Bin {
    uint32_t v0, v1;  // destination peers [v0, v1) (local ids, whole 64-peer tiles)
    uint64_t s0, s1;  // padded slot range
    uint64_t u0;      // first position of this bin in the unpadded (sorted) order
};

struct BinUnit {        // one scatter work unit: cb entries [p0, p1) of source chunk c
    uint32_t c, first;  // first: this unit books the chunk's source-side stats
    uint64_t p0, p1;
};

struct BinArgs {
    const Bin* bins;
    uint64_t n_bins;
    const uint16_t* cb_src;       // per binned edge, chunk-major order: its source peer, local to the chunk;
                                  // bit 15 (kRunStart): the entry starts a run of consecutive slots
    const uint32_t* cb_run;       // per run: slot - position of its entries (mod 2^32)
    const uint32_t* cb_grp;       // per 64-entry group: the run of its first entry
    uint64_t n_binned;            // cb entries
    const uint64_t* chunk_begin;  // n_chunks + 1 offsets into cb_*
    uint64_t n_chunks, chunk;     // source chunks of `chunk` peers ...
    uint64_t seg, cps;            // ... cut out of segments of `seg` peers, cps chunks each: chunk c covers
                                  // [chunk_vb(c), chunk_ve(c)) (one segment at P = 1: c * chunk; a vertex block
                                  // cuts the global ids into segments so a pipelined exchange can deliver the
                                  // sources of whole chunks stage by stage, gossip_dist.hip)
    const BinUnit* units;         // scatter work units, in chunk order (or a stage's units, staged exchange)
    uint64_t n_units;             // units of this launch (a multiple of kScatterGrid / 8)
    const uint64_t* xcd_units;    // 9 words, only xcd_units[8] is meaningful: the unit count, a multiple of
                                  // kScatterGrid / 8 (scatter_rows deals rows of units round-robin over the XCDs)
    const uint16_t* bdst;         // per slot: destination - bin.v0
    uint64_t* val;                // per slot: Wp words, the source's new words of this round
    uint32_t bin_words;           // LDS accumulator words of a bin (kBinWords or kBinWords / 2)
    uint64_t* dummy;              // kScatterGrid * kScatterBlock * Wp words: stores of lanes with no slot
    uint32_t noskip;              // every slot is rewritten: the first binned round after a reset
    uint64_t n_runs_m1;           // cb_run entries - 1 (clamp for the run index of past-the-end lanes)
    // streamed layout (the default): val is in cb order, written front to back by k_bin_stream; the
    // apply walks its bin's slots and finds each value through the run of the slot
    const uint32_t* ap_run;       // per run, in slot order: slot - cb position (as cb_run)
    const uint32_t* ap_grp;       // per 64-slot group: runs that start before the group
    uint32_t stream;              // 1: streamed layout, 0: val in slot order (k_bin_scatter_*)
    const uint32_t* deg;          // per owned peer: its row length (source-side stats booked by the apply)
    uint32_t apply_pipe;          // streamed apply's pipeline shape (k_bin_apply_runs, "apply_pipe"; 0 default)
    uint32_t small;               // streamed scatter: the small-chunk instance (4096-word slices, 256 threads, four
                                  // workgroups per CU) when the chunks fit it ("scatter_small")
    uint32_t direct;              // streamed scatter of a vertex block: chunks without owned sources read their
                                  // words from the gather buffer instead of staging them ("scatter_direct")
    uint32_t split_direct;        // streamed scatter: the units of a split chunk after its first read their words
                                  // from nw_src instead of staging the chunk again ("scatter_split_direct")
    uint32_t wide;                // streamed apply of small bins: 16-wave workgroups ("apply_wide")
    uint32_t needy_check;         // 1: the apply first tests whether any peer of the bin can still learn
                                  // something (a pass over the bin's seen words) and skips its slots if not;
                                  // 0 on rounds with more than one missing pair per peer, where every bin is
                                  // needy and the pass only costs a read of seen (2 GB at config 4) and a
                                  // round trip per bin
    uint32_t src_stats;           // 1: the scatter books the source side of the round's pushes (its first
                                  // unit of each chunk, row bounds loaded after the slice); 0: the apply
                                  // does, for its bin's peers (bin_src_stats), and the scatter's staging is
                                  // one round trip
    uint32_t* work;               // persistent streamed apply ("apply_persist"): one bin counter per XCD group
                                  // of workgroups, zero at the launch; null: one workgroup per bin
    unsigned long long* probe;    // "apply_probe" (diagnostics): the streamed apply's per-phase wall-clock
                                  // ticks summed over bins (kProbe* slots); null otherwise
};
// apply_probe slots: wall-clock (100 MHz) ticks of the streamed apply's phases, summed over bins
enum { kProbeSrc = 0, kProbeInit, kProbeSlots, kProbeFinish, kProbeBins, kProbeSlotsN, kProbeBlock, kProbeBlocks,
       kProbeXcd, kProbeN = kProbeXcd + 8 };  // (kProbeXcd + x: lifetimes of the blocks of XCD group x)

struct BinState {
    Bin* bins = nullptr;
    uint64_t seg = 0, cps = 0;    // BinArgs.seg, .cps
    uint64_t n_bins = 0;
    uint16_t* cb_src = nullptr;
    uint32_t* cb_run = nullptr;
    uint32_t* cb_grp = nullptr;
    uint64_t n_runs = 0;
    uint32_t* ap_run = nullptr;
    uint32_t* ap_grp = nullptr;
    uint64_t* chunk_begin = nullptr;
    uint64_t n_chunks = 0, chunk = 0;
    BinUnit* units = nullptr;
    uint64_t* xcd_units = nullptr;
    uint64_t n_units = 0;
    // staged exchange (P > 1, gossip_dist.hip): the units reordered -- the chunks of the own block first,
    // then stage j = the chunks of segments s = j (mod S) -- each group padded to whole rows
    BinUnit* stage_units = nullptr;
    uint64_t stage_lo[kMaxStages + 2] = {};  // group g (0: own block, 1 + j: stage j) = [stage_lo[g], stage_lo[g + 1])
    uint32_t stages = 0;                      // S the staged order was built for (0: none)
    std::vector<BinUnit> h_units;             // the units (host copy)
    uint16_t* bdst = nullptr;
    uint64_t* val = nullptr;
    uint64_t* dummy = nullptr;
    uint32_t* deg = nullptr;      // n_local row lengths (BinArgs.deg)
    uint32_t bin_words = kBinWords;
    uint64_t n_slots = 0;   // padded
    uint64_t n_binned = 0;  // edges with a slot (light destinations)
};

// Propagation-blocked push rounds (gossip_blocked.hip; P = 1, one word per peer).  A push round
// whose frontier is too wide for per-delivery atomics and too narrow for a binned round (which streams
// every edge) writes one record {destination, new word} per delivery instead, in two binning passes:
// level 1 into kPbCoarse coarse bins, level 2 into the fine bins of the slot layout; the apply folds
// each fine bin's records into an LDS accumulator and test-and-sets its peers with plain stores.
// Every (producer, bin) pair owns a segment of the record arrays sized at bootstrap by the overlay's
// edge counts (its worst case: every source active), so records are written without global atomics:
// a level-1 workgroup owns every kPbGrid-th tile and heavy chunk, a level-2 slice the segments of
// kPbGrid / kPbSlices of them.
constexpr uint32_t kPbCoarse = 256;    // level-1 search table (a power of two: the LDS search is branch-free)
constexpr uint32_t kPbCoarseMax = 160; // level-1 bins: two 32-record buffers each fit the LDS (round 4; 256 bins
                                       // with one buffer each in round 3)
constexpr uint32_t kPbFineMax = 100;   // fine bins per coarse bin (level-2 LDS staging)
constexpr uint32_t kPbFineIn = 1u << 18;  // a fine bin: whole tiles, <= kBinWords peers and <= this in-degree
                                          // (unless one tile has more): no hot bin in level 2
constexpr uint32_t kPbB1 = 32;         // level-1 records per flush: 128 B of destinations, 256 B of words
constexpr uint32_t kPbH1 = 2;          // ... two buffers per coarse bin (gossip_stage.hpp)
constexpr uint32_t kPbB2 = 64;         // level-2 records per flush: 128 B of destinations, 512 B of words
constexpr uint32_t kPbH2 = 2;          // ... two buffers per fine bin
constexpr uint32_t kPbSlices = 4;      // level-2 workgroups per coarse bin
constexpr int kPbBlock = 1024;         // 16 waves per workgroup, one workgroup per CU (level 1)
constexpr int kPbGrid = 256;           // level-1 workgroups (row ranges)
constexpr uint32_t kPbPad = 0xFFFFFFFFu;  // level-1 padding record (level 2: 0xFFFF)
constexpr uint32_t kPbMap = 4096;         // level 1's id buckets (coarse bin lookup)
constexpr uint32_t kPbLoPermille = 10;    // push rounds from this frontier run blocked ...
constexpr uint64_t kPbPushPeers = 1ull << 26;  // ... on overlays of this many peers ...
constexpr uint64_t kPbBinSlots = 1ull << 28;  // ... and dense rounds where the slot array has this many slots ...
constexpr uint32_t kPbHiPermille = 300;   // ... and dense rounds below this one (gossip_config.blocked_permille)

struct PbArgs {
    uint32_t n_coarse;
    uint64_t n_fine;
    const uint32_t* c_lo;     // n_coarse + 1: first owned peer of each coarse bin (whole fine bins)
    const uint32_t* c_fine;   // n_coarse + 1: first fine bin of each coarse bin
    const uint32_t* f_lo;     // n_fine + 1: first owned peer of each fine bin
                              // level-1 workgroup w: tiles and heavy chunks w (mod kPbGrid)
    const uint64_t* s1_base;  // [w][k] (kPbGrid x n_coarse): level-1 segment of workgroup w, coarse bin k
    const uint32_t* s1_cap;   //   its capacity (records; a multiple of kPbB1)
    uint32_t* s1_len;         //   records written this round (whole flushes)
    const uint64_t* s2_base;  // [s][f] (kPbSlices x n_fine): level-2 segment of slice s, fine bin f
    const uint32_t* s2_cap;
    uint32_t* s2_len;
    uint32_t* r1_dst;         // level-1 records: destination (global id; kPbPad: padding) ...
    unsigned long long* r1_w;  // ... and the source's new word
    uint16_t* r2_dst;         // level-2 records: destination - fine bin's first peer (0xFFFF: padding) ...
    unsigned long long* r2_w;
    uint32_t* err;            // set if a segment would overflow (cannot happen: capacities are edge counts)
    uint32_t map_shift;       // level 1's LDS map of the coarse bins: id >> map_shift -> a kPbMap-entry table
    uint32_t direct_end;      // destinations below this (the hubs' tiles, each over kPbFineIn in-degree: one
                              // fine bin each, every record of a round into one LDS buffer) are delivered
                              // at once, as the push does (a read of seen, then an atomic if bits are new)
    uint32_t dir_lo, dir_hi;  // level 1 delivers destinations in [dir_lo, dir_hi) at once (P = 1: [0, direct_end);
    uint32_t dir_base;        //   a vertex block's record push: its own block), at local index c - dir_base
    uint32_t keep_end;        // level 1 leaves the new words of sources below this (P = 1: the hubs, direct_end)
    const HeavyChunk* chunks; // the heavy rows' chunks (row order) ...
    uint64_t n_chunks;
    unsigned long long* nw;   // ... whose new words the split clears (set per round: the buffers rotate)
    uint32_t clear_all;       // a wide frontier: the split clears every new word in whole pieces, and level 1
                              // clears none (scattered 8-B clears of a dense frontier cost a read-modify-write
                              // per touched sector)
    const unsigned long long* marks;  // narrow rounds with valid tile marks (RoundArgs.tcur: every tile with new
                              // words marked): level 1 reads the new words of marked tiles only; null: every tile
    uint64_t n_local;
    uint32_t pipe;            // "blocked_pipe": the split's and the apply's record loops pipelined (k_pb_split<true>,
                              // k_pb_apply<true>)
};

struct PbState {
    uint32_t rank_mode = 0;   // a vertex block's record push (build_px): the coarse bins are the destination blocks
    uint32_t n_coarse = 0;
    uint64_t n_fine = 0;
    uint32_t *c_lo = nullptr, *c_fine = nullptr, *f_lo = nullptr;
    uint32_t direct_end = 0, map_shift = 0;
    uint64_t *s1_base = nullptr, *s2_base = nullptr;
    uint32_t *s1_cap = nullptr, *s2_cap = nullptr, *s1_len = nullptr, *s2_len = nullptr, *err = nullptr;
    uint32_t* r1_dst = nullptr;
    unsigned long long* r1_w = nullptr;
    uint16_t* r2_dst = nullptr;
    unsigned long long* r2_w = nullptr;
    uint64_t n1 = 0, n2 = 0;  // record capacities of the two levels
    uint64_t* rec_out = nullptr;  // rank mode: the packed {peer, word} records, rec_stride per destination block
    uint64_t rec_stride = 0;
};

struct DeadReport {
    uint32_t round, reporter, dead;
};

// Everything a round kernel needs; passed by value.
struct RoundArgs {
    const uint64_t* rp;     // n_local + 1 local offsets
    uint32_t* col;          // global ids, bit 31 = masked
    uint32_t* alive;        // global bitset (n_global bits)
    uint32_t* registered;   // global bitset (seed registry view)
    uint64_t* seen;         // n_local * W
    uint64_t* nw;           // this round's new words (sources); cleared by push_light
    uint64_t* nx;           // next round's new words (fresh)
    uint64_t* send;         // dense remote staging (n_global * W) or null
    // near-empty sparse push rounds of a vertex block (one word per peer): a remote delivery appends a record
    // {peer, word} to its destination block's slice of rec_out (rec_stride records each: the record push's
    // buffer, sized by the block's edges into each block), its place from rec_cnt[q] (one atomic per wave and
    // destination); no staging, no compaction
    uint64_t* rec_out;
    unsigned long long* rec_cnt;
    uint64_t rec_stride;
    const uint64_t* part;          // the blocks' bounds (world + 1)
    uint32_t world;
    unsigned long long* smark;  // sparse push rounds: 1 bit per 64 global peers whose staging words this round
                                // wrote (the compaction reads only those tiles); null otherwise
    uint8_t* miss;          // per-edge miss counters
    DevStats* st;           // this round's kStatLines striped lines
    unsigned long long* cov;  // per-message coverage increments of this round (history) or null
    const HeavyChunk* chunks;
    uint64_t n_chunks;
    uint64_t n_local, begin, end, n_global;
    DeadReport* reports;
    unsigned long long* n_reports;
    uint64_t report_cap;
    uint32_t round;
    uint32_t max_missed;
    uint32_t heavy;                // light/heavy row threshold (rows > heavy are chunked)
    uint32_t dead_mode;            // some peers are dead: dense rounds skip dead destinations and the
                                   // traversal stats come from k_src_count (per-edge alive test)
    uint64_t inj_mask[kMaxWords];  // messages scheduled so far (pull: bits a peer can still learn)
    uint64_t in_flight[kMaxWords]; // P = 1, use_flight: a superset of the bits in this round's new words (the
                                   // previous round's receipts OR this round's injections); a bit outside it
                                   // cannot be learned this round
    uint32_t use_flight;
    uint64_t* inj_live;            // P = 1: messages actually injected so far (an origin dead at its round
                                   // never injects; nobody can learn those bits); k_inject sets them.  A
                                   // partition injects only its own origins, so P > 1 passes nullptr
    uint64_t* tcur;                // push rounds (P = 1): 1 bit per 64-peer tile, a superset of the tiles with
                                   // nonzero new words; cleared as consumed (nullptr: not kept)
    uint64_t* tnx;                 // the same bits for the next round's words, set at activation
    uint32_t tsparse;              // tcur is valid: push_light visits only its tiles
    uint32_t defer;                // push round with a deferred seen update: deliveries test against the
                                   // round-start seen and OR the unseen bits into nx only (one atomic per
                                   // delivery); the next round's sweep (fold), or k_commit_nx, folds nx
                                   // into seen
    uint32_t fold;                 // round after a deferred round: seen lacks this round's new words (nw);
                                   // k_bin_apply, k_pull_rows's or k_pb_scatter's sweep folds them in
                                   // (seen | nw) for every owned peer before anything else of the round
                                   // reads seen (k_pb_scatter's hub deliveries test against seen | nw)
    const uint64_t* first2;        // pull rounds with many needy rows (nullptr otherwise): per owned peer the
                                   // first two entries of its row (col[rp[v]] | col[rp[v] + 1] << 32; no
                                   // masked edges), read with the sweep so a row's first step needs no
                                   // random col line
    uint64_t* front;               // pull rounds: 1 bit per source peer, set iff its new words are nonzero
    const uint64_t* nw_src;        // pull rounds: new words of every source, indexed by (global) peer id
    uint64_t n_src;                // peers covered by nw_src / front
    // re-bootstrap overflow rows (extra_cap > 0): extra out-edges of the owned peers
    uint32_t* ex_col;              // n_local * ex_cap, global ids, bit 31 = masked by liveness
    uint32_t* ex_cnt;              // n_local
    uint8_t* ex_miss;              // n_local * ex_cap
    uint32_t ex_cap;
    uint32_t heavy_exit;           // k_pull_heavy stops a chunk once it holds every needed bit
    // single-partition symmetric overlays without rejoin (DESIGN.md section 6,
    // "closed-form liveness"): per-peer death round and per-source edge counters
    uint16_t* death_r;             // n_local: round of death, 0xFFFF = alive (null: not kept)
    uint32_t* dgone;               // n_local: out-edges whose target has died (masked or not)
    uint32_t* dmask;               // n_local: out-edges masked by liveness
    uint32_t* rev;                 // n_edges: rev[e] for e = (v -> u) is the position of v in u's row
    // k_pull_heavy: per heavy row (at its first chunk) the bits its chunks have found so far this
    // round, n_chunks * Wp words cleared per launch; a chunk stops once they cover the row's need
    uint64_t* hacc;
    // late pull rounds (DESIGN.md section 6.5, P = 1, one word per peer, no deaths): a round may book the
    // next round's source side at activation (st_pre: frontier, traversals, deliveries, digest, covered
    // of the peers it activates) and list the light rows that still lack a bit (lst_out); the next round
    // then pulls only those rows (k_pull_list) with its source side already booked (src_booked)
    DevStats* st_pre;              // nullptr: no booking
    uint32_t* lst_out;             // nullptr: no list
    uint32_t* lst_n;               // entries appended (may pass lst_cap: the list overflowed)
    uint32_t lst_cap;
    uint32_t src_booked;           // k_pull_rows: the sweep books no source side
    uint32_t row_step;             // k_pull_rows: neighbour words gathered per row per step (1 or 2)
    uint32_t row_q;                // k_pull_rows: queue entries per wave (128; 256: "row_queue", A/B)
    uint32_t row_grid;             // k_pull_rows: workgroups (0: kMaxGrid; "row_grid", A/B)
    unsigned long long* chk;       // checked-index build (GOSSIP_CHECKED): {trips, site, index, bound} of the
                                   // first index past its bound (gossip_device.hpp GOSSIP_IDX); unused otherwise
};

// GOSSIP_IDX sites (the checked-index build reports the first one that trips)
enum : uint32_t {
    kChkStreamDirect = 1,  // k_bin_stream, scatter_direct: a chunk's source word read from the gather buffer
    kChkStreamSlice,       // k_bin_stream: a chunk-local source in the LDS slice
    kChkStageSrc,          // scatter_stage: a source word staged from nw_src
    kChkStreamVal,         // k_bin_stream: a value slot
    kChkApplyRecord,       // k_apply_records: a record's peer in the block
    kChkPullGather,        // k_pull_rows / k_pull_heavy: a neighbour's word in nw_src
    kChkApplyRemote,       // k_apply_remote: a received word of the block
    kChkPushSeen,          // push: a local delivery's seen word
    kChkRecordOut,         // push at P > 1: an appended record's place in its destination block's slice
    kChkListRow,           // k_pull_list: a listed row
    kChkApplyVal,          // k_bin_apply_runs: a slot's value (its cb position)
};

// Re-bootstrap draw (handleDeadPeer peer.cpp:398-404 -> selectAndConnectPeers
// :214-253): one seed response of L candidates, keyed by (round, dead peer).
struct RebootArgs {
    uint32_t thr[64];  // power-law thresholds t[j], 1 <= j < L
    uint32_t L;
    uint32_t seed;
};

// A whole run of a small overlay in one launch (gossip_tiny.hip): everything one workgroup needs.
struct TinyArgs {
    const uint32_t* erow;                  // per edge: its row (source)
    uint32_t* col;                         // bit 31 = masked
    uint32_t *alive, *registered;          // global bitsets
    uint64_t *seen, *nw, *nx;              // n * Wp words
    uint8_t* miss;                         // per edge (null: no liveness)
    DeadReport* reports;
    unsigned long long* n_reports;
    uint64_t report_cap;
    uint64_t* inj_live;                    // kMaxWords: messages injected since the reset
    const uint32_t *inj_origin, *inj_msg, *inj_round;  // the schedule, sorted by round
    const uint32_t *kill_peer, *kill_round;
    uint32_t n_inj, n_kill;
    uint32_t n, n_edges, wd;               // peers, edges, words per peer (unpadded)
    uint32_t seed, churn, ping_every, max_missed;
    uint32_t start, min_rounds, max_rounds, last_inject_round, has_schedule;
    gossip_round_stats* out;               // one entry per round run
    uint32_t out_cap;
    uint32_t* result;                      // [rounds run, new words in the nx buffer]
};

// ---- launchers (gossip_kernels.hip) ----
hipError_t launch_churn(const RoundArgs& a, uint32_t W, uint32_t seed, uint32_t threshold, hipStream_t s);
hipError_t launch_kills(const RoundArgs& a, uint32_t W, const uint32_t* kill_peers, uint32_t n, hipStream_t s);
hipError_t launch_liveness(const RoundArgs& a, hipStream_t s, int heavy);
hipError_t launch_inject(const RoundArgs& a, uint32_t W, const uint32_t* origin, const uint32_t* msg_id, uint32_t n,
                         hipStream_t s);
hipError_t launch_push_heavy(const RoundArgs& a, uint32_t W, bool check_alive, bool remote, hipStream_t s);
hipError_t launch_push_light(const RoundArgs& a, uint32_t W, bool check_alive, bool remote, hipStream_t s);
hipError_t launch_frontier_bits(const RoundArgs& a, uint32_t W, hipStream_t s);
hipError_t launch_pull_rows(const RoundArgs& a, uint32_t W, hipStream_t s);
// defer: the rows' finds only ORed into hacc (binned rounds, run beside the scatter); launch_heavy_commit applies
// them after the apply
hipError_t launch_pull_heavy(const RoundArgs& a, uint32_t W, hipStream_t s, bool hacc_zeroed = false, bool defer = false);
hipError_t launch_heavy_commit(const RoundArgs& a, uint32_t W, hipStream_t s);
// late pull rounds over a needy list (one word per peer): the stale new words of the round before last
// cleared (by its list, or n_local words), then the list's rows pulled
hipError_t launch_list_zero(const RoundArgs& a, const uint32_t* lst, uint32_t n, hipStream_t s);
hipError_t launch_pull_list(const RoundArgs& a, const uint32_t* lst, uint32_t n, hipStream_t s);
hipError_t launch_apply_remote(const RoundArgs& a, uint32_t W, const uint64_t* recv, uint32_t world,
                               uint64_t part_stride, hipStream_t s);
// sparse push exchange: send -> per-destination {peer, words} records at seg + q * stride, counts[q] of them
// (part / toff: the blocks' bounds and tile offsets on the device, tiles = toff[world]; bits: tiles + 1 words,
// the last kept zero; pos: as many; scan_tmp: compact_send_scratch)
hipError_t compact_send_scratch(uint64_t tiles, size_t* scan_bytes);
// a sparse round's staging marks: 1 bit per 64 global peers (+ a word of slack)
inline uint64_t smark_bytes(uint64_t n_global) { return ((n_global + 4095) / 4096 + 1) * 8; }
// (smark: the round's staging marks, cleared here for the next sparse round)
hipError_t launch_compact_send(const RoundArgs& a, uint32_t W, const uint64_t* part, const uint64_t* toff,
                               uint64_t tiles, uint32_t world, uint64_t stride, unsigned long long* counts,
                               uint64_t* seg, uint64_t* bits, uint64_t* pos, void* scan_tmp, size_t scan_bytes,
                               hipStream_t s);
hipError_t launch_apply_records(const RoundArgs& a, uint32_t W, const uint64_t* rec, uint64_t n_rec, hipStream_t s);
hipError_t launch_bin_scatter(const RoundArgs& a, const BinArgs& b, uint32_t W, hipStream_t s);
hipError_t launch_bin_apply(const RoundArgs& a, const BinArgs& b, uint32_t W, hipStream_t s);
hipError_t launch_liveness_extra(const RoundArgs& a, hipStream_t s);
hipError_t launch_push_extra(const RoundArgs& a, uint32_t W, bool check_alive, bool remote, hipStream_t s);
// this round's reports [first, first + n) -> keys (local reporter << 32 | dead), unsorted
hipError_t launch_reboot_keys(const RoundArgs& a, uint64_t first, uint64_t n, unsigned long long* keys, hipStream_t s);
// keys sorted: every reporter re-selects once per report, in dead order
hipError_t launch_rebootstrap(const RoundArgs& a, const RebootArgs& r, const unsigned long long* keys, uint64_t n,
                              hipStream_t s);
hipError_t launch_src_count(const RoundArgs& a, uint32_t W, hipStream_t s);
// after the round's deaths: dgone[u]++ for every in-neighbour u of a peer
// that died this round (its own row, the overlay being symmetric)
hipError_t launch_dead_edges(const RoundArgs& a, uint32_t lo, uint32_t hi, hipStream_t s);  // deaths of rounds [lo, hi]
// closed-form liveness of a ping round: the in-edges of peers that died in
// death rounds [lo, hi] reach max_missed misses now; alive reporters mask them,
// report and (dmask) count them
hipError_t launch_liveness_window(const RoundArgs& a, uint32_t lo, uint32_t hi, hipStream_t s);
// measurement (timing on): a ping round's pings (unmasked out-edges of alive owned peers) and those peers,
// added to out[0], out[1]
hipError_t launch_live_count(const RoundArgs& a, unsigned long long* out, hipStream_t s);
// rev[] of the symmetric overlay (once per overlay)
hipError_t launch_reverse_edges(const RoundArgs& a, hipStream_t s);
// join churn, before the round's kills and deaths: peers dead at round start
// restart (alive, registered, seen cleared, row dropped, overflow row emptied);
// owned ones are appended to list (count in *n_list)
hipError_t launch_rejoin(const RoundArgs& a, uint32_t W, uint32_t seed, uint32_t thr, uint64_t n_boot, uint32_t* list,
                         unsigned long long* n_list, hipStream_t s);
// after the round's deaths: the restarted peers' fresh out-edges (extra_cap > 0)
hipError_t launch_rejoin_select(const RoundArgs& a, const RebootArgs& r, const uint32_t* list,
                                const unsigned long long* n_list, uint64_t max_list, hipStream_t s);
hipError_t launch_commit_nx(uint64_t* seen, const uint64_t* nx, uint64_t n_words, hipStream_t s);
hipError_t launch_first2(const uint64_t* rp, const uint32_t* col, uint64_t n, uint64_t* out, hipStream_t s);
hipError_t launch_zero_words(uint64_t* words, uint64_t n_words, hipStream_t s, bool fill);
// up to kZeroRanges small device ranges (whole 32-bit words) cleared by one launch: a round's stat lines,
// tile marks, heavy-row accumulators and list counters, instead of one fill each (config 2: 55 rounds a
// step, ~7 us of GPU time and launch gap per fill)
constexpr int kZeroRanges = 8;
struct ZeroBatch {
    uint32_t* p[kZeroRanges];
    uint32_t n[kZeroRanges];     // words
    uint32_t* save[kZeroRanges];  // non-null: the range is copied here before it is cleared (a replayed run's
                                  // stat lines into the history, without a copy launch per round)
    uint32_t count;
};
hipError_t launch_zero_batch(const ZeroBatch& z, hipStream_t s);
hipError_t launch_coverage(const uint64_t* words, uint64_t n_local, uint32_t W, unsigned long long* counts,
                           hipStream_t s);
hipError_t launch_heavy_count(const uint64_t* rp, uint64_t n_local, uint32_t heavy, uint32_t clen,
                              unsigned long long* n_chunks, hipStream_t s);
hipError_t launch_heavy_fill(const uint64_t* rp, uint64_t n_local, uint32_t heavy, uint32_t clen, HeavyChunk* chunks,
                             unsigned long long* cursor, hipStream_t s);

// ---- propagation-blocked push rounds (gossip_blocked.hip) ----
// Bins and segments of both levels (P = 1; rows longer than heavy are the chunks', in row order); the
// leading tiles of over direct_in in-degree each are delivered directly (kPbFineIn by default).
// hipErrorOutOfMemory: skipped (state untouched).
hipError_t build_pb(const uint64_t* rp, const uint32_t* col, uint64_t n_local, uint64_t n_edges, uint32_t heavy,
                    const HeavyChunk* chunks, uint64_t n_chunks, uint64_t direct_in, hipStream_t s, PbState* out,
                    std::string* err);
void free_pb(PbState* p);
PbArgs pb_args(const PbState& p);
// one blocked push round: level 1 (each workgroup's heavy rows, then its light rows), level 2, apply
hipError_t launch_pb_scatter(const RoundArgs& a, const PbArgs& p, bool check_alive, uint32_t wd, hipStream_t s);
// A vertex block's sparse push rounds as records (P > 1, one word per peer): level 1 with the destination
// blocks as its coarse bins and the own block delivered at once; its segments' capacities from the block's
// edge counts.  The records for one destination can outnumber its block: the receivers grow their record
// buffers to a round's records (exchange_records, gossip_dist.hip).  hipErrorInvalidValue: world outside
// [2, kPbCoarseMax] or n_global >= 2^32 (the staging push stays).
hipError_t build_px(const uint64_t* rp, const uint32_t* col, uint64_t n_local, uint64_t n_global, uint32_t heavy,
                    const HeavyChunk* chunks, uint64_t n_chunks, const uint64_t* part, uint32_t world, uint32_t own,
                    hipStream_t s, PbState* out, std::string* err);
// the record buffer of the sparse push round in flight ({peer, words} per record, stride records per destination
// block): the staging push's compaction (the exchange's seg buffer) or the record push's own (gossip_dist.hip)
void ctx_send_records(gossip_ctx* c, const uint64_t** base, uint64_t* stride);
// after level 1: every destination block's records packed at seg + q * stride * 2 as {peer, word} (level 1's
// padding as {first peer of q, 0}), counts[q] records; the heavy rows' new words cleared
hipError_t launch_px_pack(const PbArgs& p, uint32_t world, uint32_t own, const uint64_t* d_part, uint64_t stride,
                          uint64_t* seg, unsigned long long* counts, const HeavyChunk* chunks, uint64_t n_chunks,
                          uint64_t* nw, hipStream_t s);
hipError_t launch_pb_split(const PbArgs& p, hipStream_t s);
hipError_t launch_pb_apply(const RoundArgs& a, const PbArgs& p, hipStream_t s);

// ---- small overlays (gossip_tiny.hip) ----
hipError_t launch_tiny_erow(const uint64_t* rp, uint32_t n, uint32_t* erow, hipStream_t s);
hipError_t launch_tiny_reset(const TinyArgs& t, uint64_t words, uint32_t n_started, bool unmask, uint64_t tact_words,
                             uint64_t* tact0, uint64_t* tact1, DevStats* st, hipStream_t s);
hipError_t launch_tiny_run(const TinyArgs& t, uint32_t Wp, hipStream_t s);
constexpr uint32_t kTinyPeers = 65536;  // overlays up to this many peers and edges run whole in one launch
constexpr uint32_t kTinyEdges = 65536;
// a round pulls (gathers or runs binned) once the frontier reaches this per-mille of the owned peers:
// a push touches deg x frontier edges with atomics, a binned round streams all of them; measured
// crossover 6-9 % (config 2: 5.05 %-frontier rounds cost 0.03 ms pushed, 0.13 ms binned)
constexpr uint32_t kPullPermille = 60;
// partitioned dense rounds exchange every block's {64-peer tile bitmap, packed non-zero new words} instead of
// its whole slice of new words while the round's frontier is below this per-mille of the peers
// (gossip_dist.hip; "gather_permille": 0 never, 1000 always)
constexpr uint32_t kGatherPermille = 600;

// ---- overlay generator (gossip_graph.hip) ----
// Builds the owned rows of the powerlaw overlay on the device.  On success
// *rp (n_local+1) and *col (n_edges) are device allocations owned by the caller.
hipError_t build_powerlaw_device(uint64_t n_global, uint64_t begin, uint64_t end, uint32_t list_len, uint32_t seed,
                                 uint64_t** rp, uint32_t** col, uint64_t* n_edges, hipStream_t s, std::string* err);

// ---- bin layout (gossip_bins.hip) ----
// Lays out the edges into the light owned rows of a symmetric overlay
// bin-major (P = 1, or one vertex block of a partitioned run).  Returns
// hipErrorOutOfMemory (state untouched) when the layout does not fit next to
// what is already resident.
// bin_words / chunk_words: LDS words of a bin / a source chunk (0: chosen from the overlay's size)
// seg: source segment size (0: one segment; a vertex block of a partitioned run passes bin_segment(n_global))
hipError_t build_bins(const uint64_t* rp, const uint32_t* col, uint64_t n_local, uint64_t n_global, uint64_t n_edges,
                      uint32_t heavy, uint32_t Wp, bool stream, uint32_t bin_words, uint32_t chunk_words, uint64_t seg,
                      uint64_t min_units, hipStream_t s, BinState* out, std::string* err);
void free_bins(BinState* b);
// a vertex block's source segments: 64 of them over the global ids (whole 64-peer tiles)
inline uint64_t bin_segment(uint64_t n_global) { return ((n_global + 63) / 64 + 63) / 64 * 64; }
// host side of BinArgs' chunk geometry
inline uint64_t chunk_vb(uint64_t c, uint64_t seg, uint64_t cps, uint64_t chunk) { return (c / cps) * seg + (c % cps) * chunk; }
inline uint64_t chunk_ve(uint64_t c, uint64_t seg, uint64_t cps, uint64_t chunk, uint64_t n) {
    const uint64_t vb = chunk_vb(c, seg, cps, chunk);
    return std::max(vb, std::min(std::min(vb + chunk, (c / cps + 1) * seg), n));  // (empty past n)
}
// the staged unit order for S stages of a vertex block [begin, end) (host side; BinState.stage_*)
hipError_t build_stage_units(BinState* b, uint32_t S, uint64_t begin, uint64_t end, uint64_t n_global);

// ---- library-driven multi-GPU rounds (gossip_dist.hip) ----
struct DistDriver;
gossip_status set_error(gossip_status s, const std::string& msg);
hipStream_t ctx_stream(gossip_ctx* c);
int ctx_device(gossip_ctx* c);
const gossip_config& ctx_config(gossip_ctx* c);
void ctx_range(gossip_ctx* c, uint64_t* begin, uint64_t* end);
void ctx_attach_dist(gossip_ctx* c, DistDriver* d, bool owned);
DistDriver* ctx_dist(gossip_ctx* c);
bool ctx_timing(gossip_ctx* c);
uint64_t ctx_frontier_est(gossip_ctx* c);  // peers the last round activated (this round's frontier)
uint32_t ctx_gather_pm(gossip_ctx* c);     // "gather_permille"
// staged dense exchange: the stages this ctx's binned rounds can take (1: none), its source segment size, and
// the events the next binned round's scatter waits on before the chunks of each stage
uint32_t ctx_stages(gossip_ctx* c);
uint64_t ctx_bin_seg(gossip_ctx* c);
gossip_status ctx_arm_stages(gossip_ctx* c, uint32_t S, const hipEvent_t* ev);
void ctx_timer_start_on(gossip_ctx* c, hipStream_t s, void** token);
void ctx_timer_stop_on(gossip_ctx* c, const char* name, hipStream_t s, void* token);
// forget the exchange buffers registered by gossip_set_exchange / _gather / _sparse (they are being freed)
void ctx_clear_exchange(gossip_ctx* c);
// time device work issued on the ctx's stream under `name` (gossip_kernel_time) while timing is on
void ctx_timer_start(gossip_ctx* c, const char* name, void** token);
void ctx_timer_stop(gossip_ctx* c, const char* name, void* token);
void ctx_add_bytes(gossip_ctx* c, const char* name, double bytes);  // gossip_kernel_bytes
gossip_status dist_step_ctx(gossip_ctx* c, gossip_round_stats* out);
void dist_reset(DistDriver* d);
void dist_free(DistDriver* d);

// Exact integer threshold ceil(2^32 (j/L)^2.5) (host only).
uint64_t pick_threshold(uint32_t j, uint32_t L);

}  // namespace gossip
