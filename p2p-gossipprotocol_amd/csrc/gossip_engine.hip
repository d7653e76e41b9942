// gossip_engine.hip -- C-ABI of libgossip_hip (include/gossip/gossip.h).
//
// Host orchestration of the round kernels.  One gossip_ctx owns one vertex
// partition of the overlay in HBM; each round is a short chain of kernels on
// the ctx stream (kills -> churn -> liveness -> inject -> push heavy -> push
// light) followed by one 128-byte stats read-back that decides termination.
// No exception crosses the ABI; all errors become gossip_status codes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "../../include/gossip/gossip.h"
#include "gossip_internal.hpp"
#include "philox.hpp"

using namespace gossip;

namespace {

thread_local std::string g_last_error;

gossip_status fail(gossip_status s, const std::string& msg) {
    g_last_error = msg;
    return s;
}

}  // namespace

namespace gossip {
gossip_status set_error(gossip_status s, const std::string& msg) { return fail(s, msg); }
}  // namespace gossip

namespace {

#define HIPCHK(call)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(GOSSIP_EHIP, std::string(#call) + " failed: " + hipGetErrorString(e_));   \
    } while (0)

// clears the liveness masks of the last run: a read of col, and a store only for the 16-B pieces holding
// a masked entry (config 5: 0.86 ms when every piece was rewritten)
__global__ void k_unmask(uint32_t* col, uint64_t m) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint4* c4 = reinterpret_cast<uint4*>(col);
    const uint32_t mk = kMaskedEdge;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m / 4; i += stride) {
        const uint4 x = c4[i];
        if ((x.x | x.y | x.z | x.w) & mk) c4[i] = make_uint4(x.x & ~mk, x.y & ~mk, x.z & ~mk, x.w & ~mk);
    }
    for (uint64_t e = m / 4 * 4 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += stride)
        col[e] &= ~mk;
}

struct TimerRec {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    double ms = 0.0;
    uint64_t launches = 0;
};

}  // namespace

constexpr uint32_t kDeferAuto = 0xFFFFFFFFu;  // defer_pm: chosen per round (round_begin)

struct gossip_ctx {
    gossip_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // binned rounds at P = 1: the heavy rows' pull on a second stream beside the scatter (round 6)
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    uint64_t n = 0, begin = 0, end = 0, n_local = 0;
    uint32_t M = 0, W = 0, Wp = 0;

    // overlay
    uint64_t* rp = nullptr;
    uint32_t* col = nullptr;
    uint64_t n_edges = 0;
    HeavyChunk* chunks = nullptr;
    uint64_t n_chunks = 0;
    uint64_t* hacc = nullptr;  // k_pull_heavy's per-row found bits (n_chunks * Wp words)
    uint64_t* inj_live = nullptr;  // kMaxWords: messages actually injected since the reset (k_inject)
    uint64_t* first2 = nullptr;    // per owned peer: its row's first two entries (k_pull_rows, RoundArgs.first2)
    bool graph_ready = false;

    // dynamic state
    uint64_t *seen = nullptr, *nw = nullptr, *nx = nullptr;
    uint64_t* front = nullptr;  // pull-round frontier bitmap
    uint64_t* tact[2] = {nullptr, nullptr};  // push-round frontier tiles (1 bit per 64 peers), this / next round
    int tcur = 0;                            // tact[tcur]: this round's
    uint64_t prev_frontier_est = 0;          // frontier_est of the round before
    bool tact_ok = true;                     // tact[tcur] covers every tile with nonzero new words
    bool tact_marked = false;                // this round's activations mark tact[tcur ^ 1]
    uint32_t* alive = nullptr;
    uint32_t* registered = nullptr;
    uint8_t* miss = nullptr;
    DevStats* st = nullptr;    // kStatLines striped lines of the current round (zeroed after each read)
    DevStats* h_st = nullptr;  // pinned, kStatLines lines
    DevStats last_st{};        // decoded sums of round last_st_round
    uint32_t last_st_round = ~0u;
    unsigned long long* cov_hist = nullptr;
    DeadReport* reports = nullptr;
    unsigned long long* n_reports = nullptr;
    uint64_t report_cap = 0;
    bool any_masked = false;

    // schedule
    std::vector<uint32_t> origin, inject_round;
    std::vector<uint32_t> inj_round_sorted;  // per sorted entry
    uint32_t* d_inj_origin = nullptr;
    uint32_t* d_inj_msg = nullptr;
    std::vector<uint32_t> kill_round_sorted;
    uint32_t* d_kill_peer = nullptr;
    uint32_t last_inject_round = 0;
    bool has_schedule = false;

    // run state
    uint32_t round = 0;
    bool finished = false;
    bool any_dead = false;
    bool symmetric = false;      // overlay is symmetric (pull rounds allowed)
    uint64_t n_started = 0;      // peers 0..n_started-1 start; the rest failed registration (list_cap, F10)
    bool nx_dirty = false;       // nx holds stale words (after a pull round)
    bool bufs_zero = false;      // nw and nx are all zero: the last round was a single-partition push round
                                 // that activated nobody (push_light clears the words it consumes)
    bool last_pull = false;      // mode of the round in flight
    bool last_front = false;     // pull round used the frontier bitmap
    bool in_round = false;       // between round_begin and round_compute
    bool cur_remote = false;
    RoundArgs cur{};
    uint64_t* gather = nullptr;  // partitioned pull: every rank's new words, indexed by global peer
    // re-bootstrap overflow rows (cfg.extra_cap > 0)
    uint32_t* ex_col = nullptr;
    uint32_t* ex_cnt = nullptr;
    uint8_t* ex_miss = nullptr;
    uint64_t n_rep_seen = 0;                  // reports already re-bootstrapped
    unsigned long long* rb_keys = nullptr;    // this round's report keys (sorted in place via rb_keys2)
    unsigned long long* rb_keys2 = nullptr;
    uint64_t rb_cap = 0;
    void* rb_temp = nullptr;
    size_t rb_temp_bytes = 0;
    RebootArgs reboot{};
    // closed-form liveness + per-source dead-edge counters (single partition, symmetric, no rejoin)
    bool closed_live = false;
    uint16_t* death_r = nullptr;
    uint32_t* dgone = nullptr;
    uint32_t* dmask = nullptr;
    uint32_t* rev = nullptr;              // reverse-edge positions (closed-form liveness); per overlay
    uint32_t* rj_list = nullptr;          // join churn: this round's restarted owned peers (local ids)
    unsigned long long* rj_n = nullptr;   // their count
    BinState bins;               // binned dense rounds: slot layout (gossip_bins.hip)
    bool bins_ready = false;
    PbState pb;                  // propagation-blocked push rounds: record regions (gossip_blocked.hip)
    bool pb_ready = false;
    bool cur_pb = false;         // the round in flight runs propagation-blocked
    // a vertex block's sparse push rounds as records (build_px; P > 1, one word per peer)
    PbState px;
    int px_state = 0;            // 0: not built yet, 1: ready, -1: not eligible (staging push)
    uint64_t* d_part = nullptr;  // the partition's block bounds (device copy: the record pack's, the compaction's)
    uint64_t* d_toff = nullptr;  // the 64-peer tiles of the blocks before each block (device; the compaction's)
    uint64_t n_tiles_all = 0;    // ... all of them
    uint64_t blk_stride = 0;     // the largest block: a destination's staged records in the compaction's output
    // "px_per100k" ("px_permille": x 100): record push from this frontier, per 100 000 peers of the block (-1:
    // never).  5: config 4 as 8 parts pushes round 2 (6.7 K frontier peers per block, 3.4 M traversals, most
    // from hubs) as records, 1.3 against 3.7 ms of kernels summed with appended records, whose counters every
    // wave of the block hits; rounds 0, 1, 10 and 11 (tens of frontier peers) append (0.4 against 0.7 ms)
    int32_t px_pm = 5;
    bool cur_px = false;         // the round in flight pushes records (level 1)
    bool cur_arec = false;       // ... or appends them from the push (a near-empty frontier)
    // late pull rounds over needy lists (k_pull_list)
    bool list_req = true;          // "list_rounds": 0 never
    uint32_t list_cap_req = 0;     // "list_cap": entries per list (0: n_local / 16, at least 2^16)
    uint32_t* lst[3] = {};         // needy lists (light rows that still lack a bit), three in rotation
    uint32_t* d_lst_n = nullptr;   // their lengths (device counters)
    uint32_t lst_cap = 0;
    DevStats* st_pre = nullptr;    // the next round's source side (kStatLines lines)
    bool pre_booked = false;       // the previous round booked the next one's source side into st_pre
    int lst_in = -1;               // the list the previous round wrote (without overflow) and its length
    uint32_t lst_in_n = 0;
    bool cur_list = false;         // the round in flight pulls list lst_in ...
    bool cur_pre = false;          // ... books the next round's source side ...
    int cur_lst_out = -1;          // ... and writes list cur_lst_out
    uint32_t lst_out_n = 0;        // (read with the round's stats)
    int lin_idx[2] = {-1, -1};     // input lists of the last two rounds (-1: not a list round), lengths
    uint32_t lin_n[2] = {0, 0};
    bool last_bin = false;       // the pull round in flight runs binned
    uint64_t last_fresh = 0;     // new receipts of the previous round
    bool bins_first = false;             // no binned round since the last reset: rewrite every slot
    // engineering options (gossip_set_tuning; A/B variants that are parity-tested, and layout sizes)
    uint32_t bin_front_pm = 0;    // "bin_front_permille": binned rounds need a frontier of >= this per-mille
                                  // (0: 20 -- see round_begin)
    bool heavy_exit = true;       // "heavy_exit": k_pull_heavy's early exit
    uint32_t heavy_chunk = 0;     // "heavy_chunk": edges per heavy chunk (0: by overlay size)
    uint32_t bin_words_req = 0;   // "bin_words" / "bin_chunk": LDS words of a bin / a source chunk (0: by size)
    uint32_t bin_chunk_req = 0;
    int val_tune = -1;            // "val_tune": pick the slot array's allocation by trial scatters (-1: by size,
                                  // 0: never, 1: always, 2: and print the trials)
    int src_stats_req = -1;       // "src_stats": who books a binned round's source side (-1 auto = 1: the scatter)
    uint64_t pb_bin_slots = kPbBinSlots;  // "blocked_bin_slots": slot arrays from this size run their
                                          // sparser dense rounds blocked
    uint64_t pb_direct_in = kPbFineIn;    // "blocked_direct_in": leading tiles of more in-degree are hubs
    uint32_t pb_lo_pm = kPbLoPermille;    // "blocked_push_permille": push rounds from this frontier run blocked
    uint32_t stages_req = 4;     // "exchange_stages": a partitioned binned round's all-gather in this many stages,
                                 // the scatter of each stage's chunks overlapping the next stage (1: one piece)
    uint32_t stage_n = 0;        // armed by the driver for this round: the scatter waits stage_ev[j] ...
    hipEvent_t stage_ev[gossip::kMaxStages] = {};  // ... before the chunks of stage j (gossip_dist.hip)
    uint32_t gather_pm = kGatherPermille; // "gather_permille": partitioned dense rounds below this frontier per-mille
                                          // exchange {tile bitmap, packed non-zero words} (gossip_dist.hip)
    uint32_t row_step = 1;                // "pull_step": k_pull_rows's neighbour words per row per step
    uint32_t row_q = 128, row_grid = 0;   // "row_queue" / "row_grid": k_pull_rows's queue and grid (A/B)
                                          // (config 4 round 7: 2 -> 1, 180 -> 101 M gathers, 6.6-6.8 ->
                                          // 5.4-5.7 ms; most rows stop at their first neighbour)
    bool bin_stream = false;      // streamed binned layout (chosen in prepare_bins)
    int bin_stream_req = -1;      // "bin_stream": 0/1 forces the layout; -1: by slot-array size
    uint32_t defer_pm = kDeferAuto;  // "defer_permille": push rounds with a frontier of >= this per-mille defer
                                     // the seen update (0: never; auto: 10 where the fold can be fused)
    bool fold_pending = false;    // a deferred round's receipts (now nw) are not yet in seen: the next
                                  // binned round's apply or row-pull sweep folds them in, anything else
                                  // commits first
    bool first_ok = true;         // "pull_first2": k_pull_rows carries a row's first two entries
    bool flight_ok = true;        // "in_flight": needy tests wait only for bits that are in flight
    uint64_t flight[kMaxWords] = {};  // receipts of round flight_round (from its stats)
    uint32_t flight_round = ~0u;
    uint32_t dgone_next = 0;      // first round whose deaths dgone does not count yet
    bool cur_defer = false;       // this round defers: advance() folds nx into seen
    bool full_liveness = false;  // "full_liveness": ping every edge each ping round (A/B against closed form)
    uint64_t cur_missing = 0;    // (peer, message) pairs still missing at the round's push start (round_begin)
    uint32_t apply_pipe = 5;     // "apply_pipe": the streamed apply's pipeline shape (0-10; round 6: 5, the
                                 // contiguous-group shape with every load two iterations ahead, measured best)
    bool pb_clear_all = true;    // "blocked_clear_all": wide blocked rounds clear new words whole in level 2
    bool pb_marks = true;        // "blocked_marks": narrow blocked rounds' level 1 sweeps the marked tiles only
    bool pb_pipe = true;         // "blocked_pipe": the split's and the blocked apply's record loops pipelined
    bool zero_fill = true;       // "zero_fill": the reset clears its word arrays with hipMemsetAsync (0: k_zero2;
                                 // round 6, arms alternated: config 4 42.34 -> 42.10 ms, config 2 4.36 -> 4.30)
    bool heavy_side = true;      // "heavy_side": a binned round's heavy-row pull beside its scatter (P = 1)
    bool cur_clear_all = false;  // (the round in flight does)
    bool scatter_direct = false; // "scatter_direct": a vertex block's scatter reads other blocks' words directly
    bool scatter_small = false;  // "scatter_small": the streamed scatter's small-chunk instance where chunks fit it
    uint32_t scatter_units = 0;  // "scatter_units": at least this many scatter units (chunks split; 0: hubs only)
    bool split_direct = false;   // "scatter_split_direct": a split chunk's later units read words from nw_src
    bool apply_wide = false;     // "apply_wide": small bins applied by 16-wave workgroups
    unsigned long long* d_probe = nullptr;  // "apply_probe": the streamed apply's phase clocks (kProbeN slots)
    bool apply_persist = true;   // "apply_persist": the streamed apply as 256 workgroups taking bins from
                                 // per-XCD counters (d_work), not one workgroup per bin
    uint32_t* d_work = nullptr;  // (8 counters, zeroed by each launch)
    bool needy_skip = true;      // "bin_needy_skip": binned rounds with over one missing pair per peer skip the
                                 // apply's needy test
    uint64_t* seg = nullptr;     // sparse push: per-destination record segments (world x chunk records)
    unsigned long long* d_counts = nullptr;  // records per destination rank
    uint64_t* h_counts = nullptr;            // pinned copy
    unsigned long long* smark = nullptr;     // sparse push rounds' staging marks (RoundArgs.smark)
    uint64_t *sx_bits = nullptr, *sx_pos = nullptr;  // the compaction's tile bitmap and popcount prefix
    void* sx_tmp = nullptr;
    size_t sx_bytes = 0;
    bool cur_sparse = false;
    bool send_dirty = false;     // the dense staging buffer holds a dense push round's masks
    uint32_t heavy = kHeavyDegree;      // light/heavy row threshold of the resident overlay (its chunks, bins and
                                        // blocked segments were laid out with it)
    uint32_t heavy_req = 0;             // "heavy_degree": the threshold of the next build (0: kHeavyDegree, or
                                        // kHeavyDegreeLarge on overlays of >= kHeavyLargePeers peers)
    uint64_t frontier_est = 0;   // activated peers of the previous round
    std::vector<uint64_t> inj_prefix;  // per sorted injection: cumulative mask words
    uint64_t cum_digest = 0, cum_covered = 0;
    uint64_t cum_dead_cov = 0, cum_died = 0, cum_injected = 0;  // P = 1: for the binned-round test

    // partitioned exchange
    uint64_t* send = nullptr;
    const uint64_t* recv = nullptr;
    uint32_t world = 1;
    std::vector<uint64_t> part_begins;

    // small clears queued for the round's next kernel launch (one k_zero_batch instead of a fill each)
    gossip::ZeroBatch zq{};

    // timing
    bool timing = false;
    unsigned long long* d_live = nullptr;  // ping rounds while timing: 8(d)'s pings and alive peers (k_live_count)
    bool live_counted = false;             // this round's d_live holds a count
    std::map<std::string, TimerRec> timers;
    std::map<std::string, double> kbytes;
    std::vector<hipEvent_t> event_pool;

    // small overlays: a whole run in one launch (gossip_tiny.hip)
    bool tiny_off = false;                 // "tiny" = 0: round by round (A/B, tests)
    uint32_t* tiny_erow = nullptr;         // per edge: its row
    gossip_round_stats* tiny_out = nullptr;  // device, tiny_cap rounds
    uint32_t tiny_cap = 0;
    uint32_t* tiny_result = nullptr;       // device [rounds, buffers swapped]
    uint32_t* d_inj_round = nullptr;       // the sorted schedule rounds on the device
    uint32_t* d_kill_round = nullptr;

    // recorded schedule (gossip_run on one partition): the host decisions of a run depend only on the
    // round's stats, and a rerun from reset of the same inputs produces the same stats, so the first run
    // records each round's stat sums and the next ones issue every round without waiting for its stats
    // (replay_run); the device still computes and stores every round's stats, and they are checked
    // against the recording at the end.  Anything that could change a run drops the recording.
    bool replay_req = true;                // "replay": 0 never
    bool recording = false, replaying = false, rec_valid = false;
    std::vector<DevStats> rec_st;          // per round: the decoded stat sums
    std::vector<uint32_t> rec_lst;         // per round: entries its needy list received
    DevStats* d_hist = nullptr;            // replay: every round's kStatLines stat lines (and one more row)
    uint32_t hist_cap = 0, rep_round = 0;
    // replay: per-round copies of the state a round otherwise clears for the next (tile marks, heavy-row
    // accumulators, the apply's counters, needy-list counters), zeroed once per replayed run with the history,
    // so a replayed round queues no clears (config 2: one 5 us launch per round of 55)
    uint64_t* rep_aux = nullptr;
    uint64_t rep_aux_words = 0, rep_tw = 0, rep_hw = 0;

    // library-driven multi-GPU rounds (gossip_dist.hip): the driver that issues
    // this ctx's collectives; owned here for gossip_comm_init, by the group otherwise
    gossip::DistDriver* dist = nullptr;
    bool dist_owned = false;
};

namespace gossip {
hipStream_t ctx_stream(gossip_ctx* c) { return c->stream; }

int ctx_device(gossip_ctx* c) { return c->device; }
const gossip_config& ctx_config(gossip_ctx* c) { return c->cfg; }
void ctx_range(gossip_ctx* c, uint64_t* begin, uint64_t* end) {
    *begin = c->begin;
    *end = c->end;
}
void ctx_attach_dist(gossip_ctx* c, DistDriver* d, bool owned) {
    c->dist = d;
    c->dist_owned = owned;
}
DistDriver* ctx_dist(gossip_ctx* c) { return c->dist; }
bool ctx_timing(gossip_ctx* c) { return c->timing; }
uint64_t ctx_frontier_est(gossip_ctx* c) { return c->frontier_est; }
uint32_t ctx_gather_pm(gossip_ctx* c) { return c->gather_pm; }
uint32_t ctx_stages(gossip_ctx* c) {
    return c->bins_ready && c->bin_stream && c->n_local != c->n ? std::min<uint32_t>(c->stages_req, kMaxStages) : 1u;
}
uint64_t ctx_bin_seg(gossip_ctx* c) { return c->bins.seg; }
void ctx_send_records(gossip_ctx* c, const uint64_t** base, uint64_t* stride) {
    *base = c->cur_px || c->cur_arec ? c->px.rec_out : c->seg;
    *stride = c->cur_px || c->cur_arec ? c->px.rec_stride : c->blk_stride;
}
gossip_status ctx_arm_stages(gossip_ctx* c, uint32_t S, const hipEvent_t* ev) {  // (the caller set the device)
    if (const hipError_t e = build_stage_units(&c->bins, S, c->begin, c->end, c->n))
        return fail(GOSSIP_EHIP, std::string("staged scatter units: ") + hipGetErrorString(e));
    std::copy(ev, ev + S, c->stage_ev);
    c->stage_n = S;
    return GOSSIP_OK;
}
void ctx_clear_exchange(gossip_ctx* c) {
    c->send = nullptr;
    c->recv = nullptr;
    c->gather = nullptr;
    c->seg = nullptr;
    c->world = 1;
    c->part_begins.clear();
}
}  // namespace gossip

namespace {

uint32_t pad_words(uint32_t w) {
    if (w <= 1) return 1;
    if (w <= 2) return 2;
    if (w <= 4) return 4;
    return 8;
}

uint32_t pack_w(const gossip_ctx* c) { return (c->W << 16) | c->Wp; }

gossip_status set_dev(gossip_ctx* c) {
    HIPCHK(hipSetDevice(c->device));
    return GOSSIP_OK;
}

// Events come from a per-ctx pool (creating two events per launch inside a
// timed loop cost more than recording them).
hipEvent_t take_event(gossip_ctx* c) {
    hipEvent_t e = nullptr;
    if (!c->event_pool.empty()) {
        e = c->event_pool.back();
        c->event_pool.pop_back();
    } else {
        hipEventCreate(&e);
    }
    return e;
}

// queued clears go out before the next kernel (every kernel that writes stats, tile marks or heavy-row
// accumulators is launched through timed())
hipError_t flush_zero(gossip_ctx* c) {
    gossip::ZeroBatch& z = c->zq;
    if (!z.count) return hipSuccess;
    hipError_t e = z.count == 1 && !z.save[0] ? hipMemsetAsync(z.p[0], 0, (size_t)z.n[0] * 4, c->stream)
                                              : gossip::launch_zero_batch(z, c->stream);
    z.count = 0;
    return e;
}

hipError_t queue_zero(gossip_ctx* c, void* p, uint64_t bytes, void* save = nullptr) {
    if (c->zq.count == gossip::kZeroRanges)
        if (hipError_t e = flush_zero(c)) return e;
    c->zq.p[c->zq.count] = static_cast<uint32_t*>(p);
    c->zq.n[c->zq.count] = (uint32_t)(bytes / 4);
    c->zq.save[c->zq.count] = static_cast<uint32_t*>(save);
    c->zq.count++;
    return hipSuccess;
}

// GOSSIP_SYNC_DEBUG (diagnostics): every launch waited for, a device fault named by its kernel on stderr
const bool kSyncDebug = std::getenv("GOSSIP_SYNC_DEBUG") != nullptr;

hipError_t sync_debug(gossip_ctx* c, const char* name) {
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess)
        std::fprintf(stderr, "[gossip] %s (round %u, block at %llu): %s\n", name, c->round,
                     (unsigned long long)c->begin, hipGetErrorString(e));
    return e;
}

template <class F>
hipError_t timed(gossip_ctx* c, const char* name, F&& launch) {
    if (hipError_t e = flush_zero(c)) return e;
    if (!c->timing) {
        const hipError_t e = launch();
        return e == hipSuccess && kSyncDebug ? sync_debug(c, name) : e;
    }
    hipEvent_t a = take_event(c), b = take_event(c);
    hipEventRecord(a, c->stream);
    hipError_t e = launch();
    hipEventRecord(b, c->stream);
    c->timers[name].pending.emplace_back(a, b);
    return e == hipSuccess && kSyncDebug ? sync_debug(c, name) : e;
}

}  // namespace

namespace gossip {
// Device work the dist driver issues on the ctx's stream (collectives, device
// copies) timed like a kernel: events recorded on the stream around it.
void ctx_timer_start(gossip_ctx* c, const char* name, void** token) {
    *token = nullptr;
    if (!c->timing) return;
    hipEvent_t a = take_event(c);
    hipEventRecord(a, c->stream);
    *token = a;
    (void)name;
}
void ctx_timer_stop(gossip_ctx* c, const char* name, void* token) {
    if (!c->timing || !token) return;
    hipEvent_t b = take_event(c);
    hipEventRecord(b, c->stream);
    c->timers[name].pending.emplace_back(static_cast<hipEvent_t>(token), b);
}
// the same on another stream of the ctx's device (the staged exchange's copy / collective stream)
void ctx_timer_start_on(gossip_ctx* c, hipStream_t s, void** token) {
    *token = nullptr;
    if (!c->timing) return;
    hipEvent_t a = take_event(c);
    hipEventRecord(a, s);
    *token = a;
}
void ctx_timer_stop_on(gossip_ctx* c, const char* name, hipStream_t s, void* token) {
    if (!c->timing || !token) return;
    hipEvent_t b = take_event(c);
    hipEventRecord(b, s);
    c->timers[name].pending.emplace_back(static_cast<hipEvent_t>(token), b);
}
void ctx_add_bytes(gossip_ctx* c, const char* name, double bytes) {
    if (c->timing) c->kbytes[name] += bytes;
}
}  // namespace gossip

namespace {

void drain_timers(gossip_ctx* c) {
    for (auto& kv : c->timers) {
        for (auto& ev : kv.second.pending) {
            float ms = 0.f;
            hipEventSynchronize(ev.second);
            hipEventElapsedTime(&ms, ev.first, ev.second);
            kv.second.ms += ms;
            kv.second.launches++;
            c->event_pool.push_back(ev.first);
            c->event_pool.push_back(ev.second);
        }
        kv.second.pending.clear();
    }
}

void free_state(gossip_ctx* c) {
    c->zq.count = 0;
    hipFree(c->seen);
    hipFree(c->nw);
    hipFree(c->nx);
    hipFree(c->front);
    hipFree(c->tact[0]);
    hipFree(c->tact[1]);
    c->tact[0] = c->tact[1] = nullptr;
    hipFree(c->alive);
    hipFree(c->registered);
    hipFree(c->miss);
    hipFree(c->death_r);
    hipFree(c->dgone);
    hipFree(c->dmask);
    hipFree(c->rev);
    c->death_r = nullptr;
    c->dgone = c->dmask = c->rev = nullptr;
    hipFree(c->st);
    hipFree(c->st_pre);
    c->st_pre = nullptr;
    for (auto& l : c->lst) {
        hipFree(l);
        l = nullptr;
    }
    hipFree(c->d_lst_n);
    c->d_lst_n = nullptr;
    c->lst_cap = 0;
    if (c->h_st) hipHostFree(c->h_st);
    hipFree(c->cov_hist);
    hipFree(c->reports);
    hipFree(c->n_reports);
    hipFree(c->inj_live);
    hipFree(c->ex_col);
    hipFree(c->ex_cnt);
    hipFree(c->ex_miss);
    hipFree(c->rb_keys);
    hipFree(c->rb_keys2);
    hipFree(c->rb_temp);
    hipFree(c->rj_list);
    hipFree(c->rj_n);
    c->rj_list = nullptr;
    c->rj_n = nullptr;
    c->ex_col = c->ex_cnt = nullptr;
    c->ex_miss = nullptr;
    c->rb_keys = c->rb_keys2 = nullptr;
    c->rb_temp = nullptr;
    c->rb_cap = 0;
    c->rb_temp_bytes = 0;
    c->seen = c->nw = c->nx = nullptr;
    c->alive = c->registered = nullptr;
    c->miss = nullptr;
    c->st = c->h_st = nullptr;
    c->cov_hist = nullptr;
    c->reports = nullptr;
    c->n_reports = nullptr;
    c->inj_live = nullptr;
}

void free_graph(gossip_ctx* c) {
    hipFree(c->tiny_erow);
    c->tiny_erow = nullptr;
    free_bins(&c->bins);
    c->bins_ready = false;
    free_pb(&c->pb);
    c->pb_ready = false;
    free_pb(&c->px);
    c->px_state = 0;
    hipFree(c->rp);
    hipFree(c->col);
    hipFree(c->chunks);
    hipFree(c->hacc);
    hipFree(c->first2);
    c->first2 = nullptr;
    // closed-form liveness state belongs to the overlay: round_begin rebuilds
    // all of it (rev included) for the next one
    hipFree(c->rev);
    hipFree(c->death_r);
    hipFree(c->dgone);
    hipFree(c->dmask);
    c->death_r = nullptr;
    c->dgone = c->dmask = nullptr;
    c->rp = nullptr;
    c->col = nullptr;
    c->chunks = nullptr;
    c->hacc = nullptr;
    c->rev = nullptr;
    c->n_edges = c->n_chunks = 0;
    c->graph_ready = false;
}

void rec_drop(gossip_ctx* c);  // forget a recorded schedule (gossip_run)

uint64_t tact_bytes(const gossip_ctx* c) { return (((c->n_local + 63) / 64 + 63) / 64 + 1) * 8; }

// replay: round r's rows of the per-round state (gossip_ctx.rep_aux, laid out for hist_cap rounds)
uint64_t* rep_tact(gossip_ctx* c, uint32_t r) { return c->rep_aux + c->rep_tw * r; }
uint32_t* rep_work(gossip_ctx* c, uint32_t r) {
    return reinterpret_cast<uint32_t*>(c->rep_aux + c->rep_tw * (c->hist_cap + 1) + c->rep_hw * c->hist_cap) + 16ull * r;
}
uint32_t* rep_lstn(gossip_ctx* c, uint32_t r) {
    return reinterpret_cast<uint32_t*>(c->rep_aux + c->rep_tw * (c->hist_cap + 1) + c->rep_hw * c->hist_cap +
                                       8ull * c->hist_cap) + 4ull * r;
}

RoundArgs make_args(gossip_ctx* c) {
    RoundArgs a{};
    a.rp = c->rp;
    a.col = c->col;
    a.alive = c->alive;
    a.registered = c->registered;
    a.seen = c->seen;
    a.nw = c->nw;
    a.nw_src = c->nw;
    a.n_src = c->n_local;
    a.nx = c->nx;
    a.front = c->front;
    // (a vertex block keeps marks of its own tiles: local deliveries, and the remote applies -- k_apply_records,
    // k_apply_remote -- mark the tiles of the peers they activate; round 5, before which a block swept every
    // tile in every push round: config 4 as 8 parts, ≈ 1.2 ms of kernels per near-empty round)
    if (c->tact[0]) {
        a.tcur = c->replaying ? rep_tact(c, c->rep_round) : c->tact[c->tcur];
        // the marked-tile sweep only for a nearly empty frontier (it walks 64 tiles per wave in turn;
        // at a 1.3 % frontier, 57 % of the tiles, the full sweep was faster: 3.1 against 4.4 ms)
        a.tsparse = c->tact_ok && c->frontier_est * 500 < c->n_local ? 1u : 0u;
        // marks cost a check per activation (push_heavy +2 ms per step at config 4 when kept in every
        // round): kept only where the next frontier is likely small -- a tiny frontier, or a shrinking one
        const bool small = c->frontier_est * 500 < c->n_local ||
                           (c->frontier_est < c->prev_frontier_est && c->frontier_est * 100 < c->n_local);
        a.tnx = small ? (c->replaying ? rep_tact(c, c->rep_round + 1) : c->tact[c->tcur ^ 1]) : nullptr;
        c->tact_marked = small;
    }
    a.send = c->send;
    a.miss = c->miss;
    a.st = c->replaying ? c->d_hist + (uint64_t)c->rep_round * kStatLines : c->st;
    a.cov = c->cov_hist ? c->cov_hist + (uint64_t)c->round * 64 * c->Wp : nullptr;
    a.chunks = c->chunks;
    a.n_chunks = c->n_chunks;
    a.hacc = c->replaying && c->hacc ? c->rep_aux + c->rep_tw * (c->hist_cap + 1) + c->rep_hw * c->rep_round : c->hacc;
    a.row_step = c->row_step;
    a.row_q = c->row_q;
    a.row_grid = c->row_grid;
    a.chk = reinterpret_cast<unsigned long long*>(c->inj_live + kMaxWords);
    a.inj_live = c->world <= 1 && c->n_local == c->n ? c->inj_live : nullptr;  // a partition injects its own only
    a.n_local = c->n_local;
    a.begin = c->begin;
    a.end = c->end;
    a.n_global = c->n;
    a.reports = c->reports;
    a.n_reports = c->n_reports;
    a.report_cap = c->report_cap;
    a.round = c->round;
    a.max_missed = c->cfg.max_missed;
    a.heavy = c->heavy;
    a.ex_col = c->ex_col;
    a.ex_cnt = c->ex_cnt;
    a.ex_miss = c->ex_miss;
    a.ex_cap = c->cfg.extra_cap;
    a.heavy_exit = c->heavy_exit ? 1u : 0u;
    a.defer = c->cur_defer ? 1u : 0u;
    a.death_r = c->death_r;
    a.dgone = c->dgone;
    a.dmask = c->dmask;
    a.rev = c->rev;
    return a;
}

// Upload a host-built CSR and derive the heavy-row chunk list.
gossip_status install_graph(gossip_ctx* c, uint64_t* d_rp, uint32_t* d_col, uint64_t m) {
    free_graph(c);
    // the next reset clears nw / nx whole (the last run's list rows and heavy rows were the old overlay's)
    c->lin_idx[0] = c->lin_idx[1] = -1;
    c->bufs_zero = false;
    // layout key: the chunk list, bins and blocked segments below all use it
    c->heavy = c->heavy_req ? c->heavy_req : c->n >= kHeavyLargePeers ? kHeavyDegreeLarge : kHeavyDegree;
    c->rp = d_rp;
    c->col = d_col;
    c->n_edges = m;
    c->n_started = c->n;
    unsigned long long* d_cnt = nullptr;
    HIPCHK(hipMalloc((void**)&d_cnt, 2 * sizeof(unsigned long long)));
    HIPCHK(hipMemsetAsync(d_cnt, 0, 2 * sizeof(unsigned long long), c->stream));
    // heavy chunks: a wave each; on small overlays (cache-resident) a chunk's chain of 64-edge batches, not the
    // number of chunks, sets k_pull_heavy's time -- shorter chunks there ("heavy_chunk" overrides)
    uint32_t clen = c->n_local < (1ull << 22) ? 256u : kHeavyChunk;
    if (c->heavy_chunk) clen = std::max<uint32_t>(64, c->heavy_chunk) / 64 * 64;
    HIPCHK(launch_heavy_count(c->rp, c->n_local, c->heavy, clen, d_cnt, c->stream));
    unsigned long long nch = 0;
    HIPCHK(hipMemcpyAsync(&nch, d_cnt, sizeof(nch), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->n_chunks = nch;
    if (nch) {
        HIPCHK(hipMalloc((void**)&c->chunks, nch * sizeof(HeavyChunk)));
        HIPCHK(hipMalloc((void**)&c->hacc, nch * c->Wp * sizeof(uint64_t)));
        HIPCHK(launch_heavy_fill(c->rp, c->n_local, c->heavy, clen, c->chunks, d_cnt + 1, c->stream));
        // in row order (the fill appends rows in any order): a vertex range's chunks are then contiguous
        // (blocked push rounds give each workgroup the chunks of its rows); first = the row's first chunk
        std::vector<HeavyChunk> h(nch);
        HIPCHK(hipMemcpyAsync(h.data(), c->chunks, nch * sizeof(HeavyChunk), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        std::sort(h.begin(), h.end(), [](const HeavyChunk& x, const HeavyChunk& y) {
            return x.v != y.v ? x.v < y.v : x.e0 < y.e0;
        });
        for (uint64_t i = 0; i < nch; ++i) h[i].first = i && h[i - 1].v == h[i].v ? h[i - 1].first : (uint32_t)i;
        HIPCHK(hipMemcpyAsync(c->chunks, h.data(), nch * sizeof(HeavyChunk), hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    hipFree(d_cnt);
    if (c->cfg.ping_every && !c->reports) {
        uint64_t cap = c->cfg.report_capacity ? c->cfg.report_capacity : std::min<uint64_t>(m + (1u << 20), 1ull << 28);
        c->report_cap = cap;
        HIPCHK(hipMalloc((void**)&c->reports, cap * sizeof(DeadReport)));
    }
    if (c->cfg.ping_every) {
        hipFree(c->miss);
        HIPCHK(hipMalloc((void**)&c->miss, m + 1));
        HIPCHK(hipMemsetAsync(c->miss, 0, m + 1, c->stream));
    }
    HIPCHK(hipMalloc((void**)&c->first2, (c->n_local + 1) * sizeof(uint64_t)));
    HIPCHK(launch_first2(c->rp, c->col, c->n_local, c->first2, c->stream));
    c->graph_ready = true;
    rec_drop(c);  // a new overlay
    return GOSSIP_OK;
}

// Literal bootstrap (peer.cpp:63-72,214-253; seed.cpp:117-125): peer i
// registers with seeds 0..q-1 in file order; each returns the registry
// {0..i}; power-law k, Fisher-Yates shuffle, first k, skip self; union.
void host_ref_bootstrap(uint32_t n, uint32_t n_seeds, uint32_t seed, std::vector<uint64_t>& rp,
                        std::vector<uint32_t>& col) {
    const uint32_t q = n_seeds / 2 + 1;
    rp.assign(n + 1, 0);
    col.clear();
    std::vector<uint32_t> perm(n);
    std::vector<uint8_t> chosen(n);
    std::vector<uint64_t> thr(n + 1);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t L = i + 1;
        for (uint32_t j = 0; j < L; ++j) thr[j] = pick_threshold(j, L);
        std::fill(chosen.begin(), chosen.begin() + L, 0);
        for (uint32_t s = 0; s < q; ++s) {
            const uint32_t x = philox4x32_10(P_DEGREE, s, 0, 0, seed, i).x;
            uint32_t k = 0;
            for (uint32_t j = 1; j < L; ++j) k += (uint64_t)x >= thr[j];
            for (uint32_t j = 0; j < L; ++j) perm[j] = j;
            uint32_t d = 0;
            for (uint32_t idx = L - 1; idx >= 1; --idx, ++d) {
                const uint32_t r = lane_of(philox4x32_10(P_SHUFFLE, s, d >> 2, 0, seed, i), d & 3);
                const uint32_t jj = (uint32_t)(((uint64_t)r * (idx + 1)) >> 32);
                std::swap(perm[idx], perm[jj]);
            }
            for (uint32_t t = 0; t < k; ++t)
                if (perm[t] != i) chosen[perm[t]] = 1;
        }
        rp[i] = col.size();
        for (uint32_t c = 0; c < L; ++c)
            if (chosen[c]) col.push_back(c);
    }
    rp[n] = col.size();
}

// Bytes of one peer_list entry (surface/formats.cpp peer_list_json with
// peer_address(id, n) and a 10-digit lastSeen):
// {"ip":"<ip>","lastSeen":<10 digits>,"port":<port>}
uint64_t peer_entry_bytes(uint64_t id, uint64_t n) {
    uint64_t ip = 9, port = 5000 + id;  // "127.0.0.1":5000+id up to 60000 peers
    if (n > 60000) {                     // "10.a.b.c":5000+(id>>24)
        ip = 3;
        for (int sh = 16; sh >= 0; sh -= 8) ip += std::to_string((id >> sh) & 255).size();
        port = 5000 + (id >> 24);
    }
    return 39 + ip + std::to_string(port).size();
}

// Peers that start under the 4 KB peer-list read (peer.cpp:186-210,62-78; F10):
// peer i registers with seeds 0, 1, ... in file order; seeds 0..q-1 all hold
// the registry {0..i} (every peer, started or not, registers there first), so
// either all q answers fit in list_cap bytes or none does, and the seeds
// q..S-1 alone cannot reach the quorum.  The first peer whose list
// {"peers":[...],"type":"peer_list"} does not fit, and every later one (the
// lists only grow), never starts.
uint64_t started_under_cap(uint64_t n, uint32_t list_cap) {
    if (!list_cap) return n;
    uint64_t bytes = 31;  // {"peers":[ + ],"type":"peer_list"}
    for (uint64_t i = 0; i < n; ++i) {
        bytes += (i ? 1 : 0) + peer_entry_bytes(i, n);
        if (bytes > list_cap) return i;
    }
    return n;
}

gossip_status upload_csr(gossip_ctx* c, const uint64_t* rp, const uint32_t* col, uint64_t m) {
    uint64_t* d_rp = nullptr;
    uint32_t* d_col = nullptr;
    HIPCHK(hipMalloc((void**)&d_rp, (c->n_local + 1) * sizeof(uint64_t)));
    HIPCHK(hipMalloc((void**)&d_col, (m + 1) * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(d_rp, rp, (c->n_local + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
    if (m) HIPCHK(hipMemcpy(d_col, col, m * sizeof(uint32_t), hipMemcpyHostToDevice));
    return install_graph(c, d_rp, d_col, m);
}

// The scatter's store rate depends on where the slot array's pages landed: the same library ran its
// binned rounds' scatter at 9.2-9.4 ms in some processes and 10.7-11.8 in others, the apply (a
// sequential read of the same array) at 5.0-5.8 in all, and a physically contiguous array at 14 ms.
// Allocations in one process differ too (trial scatters of 9.3 / 10.3 / 8.8 ms), though some processes
// get only slow ones.  On big layouts, time one full scatter (every slot rewritten) into each of eight
// allocations (four in round 2) and keep the fastest ("val_tune" 0: keep the first; 2: print the trials); config 4,
// five processes each: scatter 9.3-11.3 (mean 9.9) against 9.7-11.7 (mean 10.4) ms.  The trial words
// are garbage: the first binned round rewrites every slot.
BinArgs bin_args(const gossip_ctx* c, bool noskip, uint32_t src_side) {
    // (field by field: a positional initializer put src_side into apply_pipe and the tuning keys one field
    // off, unnoticed because every path it selected computes the same results)
    const BinState& s = c->bins;
    BinArgs b{};
    b.bins = s.bins;
    b.n_bins = s.n_bins;
    b.cb_src = s.cb_src;
    b.cb_run = s.cb_run;
    b.cb_grp = s.cb_grp;
    b.n_binned = s.n_binned;
    b.chunk_begin = s.chunk_begin;
    b.n_chunks = s.n_chunks;
    b.chunk = s.chunk;
    b.seg = s.seg;
    b.cps = s.cps;
    b.n_units = s.n_units;
    b.units = s.units;
    b.xcd_units = s.xcd_units;
    b.bdst = s.bdst;
    b.val = s.val;
    b.bin_words = s.bin_words;
    b.dummy = s.dummy;
    b.noskip = noskip ? 1u : 0u;
    b.n_runs_m1 = s.n_runs ? s.n_runs - 1 : 0;
    b.ap_run = s.ap_run;
    b.ap_grp = s.ap_grp;
    b.stream = c->bin_stream ? 1u : 0u;
    b.deg = s.deg;
    b.apply_pipe = c->apply_pipe;
    b.direct = c->scatter_direct && c->gather ? 1u : 0u;
    b.small = c->scatter_small ? 1u : 0u;
    b.split_direct = c->split_direct ? 1u : 0u;
    b.wide = c->apply_wide ? 1u : 0u;
    b.needy_check = 1u;
    b.src_stats = src_side;
    b.work = c->apply_persist && c->bin_stream ? c->d_work : nullptr;
    b.probe = c->d_probe;
    return b;
}

gossip_status tune_val(gossip_ctx* c) {
    // single partition only: a vertex block's scatter stages global source chunks from the all-gathered
    // words, which do not exist at bootstrap (the trial launch read past the block's own words)
    if (c->val_tune == 0 || c->bin_stream || c->n_local != c->n || (c->val_tune < 0 && c->bins.n_slots < (1ull << 26)))
        return GOSSIP_OK;
    const uint64_t bytes = (c->bins.n_slots + 64) * c->Wp * sizeof(uint64_t);
    constexpr int kCand = 8;  // (8 x 16 GB at config 4, freed before the blocked regions are laid out)
    uint64_t* cand[kCand] = {c->bins.val};
    for (int k = 1; k < kCand; ++k)
        if (hipMalloc((void**)&cand[k], bytes) != hipSuccess) {
            hipGetLastError();
            cand[k] = nullptr;
        }
    RoundArgs a = make_args(c);
    a.dead_mode = 0;
    a.cov = nullptr;
    a.defer = 0;
    a.fold = 0;
    a.tcur = a.tnx = nullptr;
    BinArgs b = bin_args(c, true, 1u);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float best = 0.f;
    int bi = 0;
    // every exit frees the candidates not kept (only the first one, the layout's own, on an error)
    auto finish = [&](hipError_t err) {
        if (e0) hipEventDestroy(e0);
        if (e1) hipEventDestroy(e1);
        if (err != hipSuccess) bi = 0;
        for (int k = 0; k < kCand; ++k)
            if (cand[k] && k != bi) hipFree(cand[k]);
        c->bins.val = cand[bi];
        return err;
    };
    hipError_t err = hipEventCreate(&e0);
    if (err == hipSuccess) err = hipEventCreate(&e1);
    for (int k = 0; k < kCand && err == hipSuccess; ++k) {
        if (!cand[k]) continue;
        b.val = cand[k];
        float ms = 0.f;
        for (int rep = 0; rep < 2 && err == hipSuccess; ++rep) {  // the second launch is timed
            err = hipEventRecord(e0, c->stream);
            if (err == hipSuccess) err = launch_bin_scatter(a, b, pack_w(c), c->stream);
            if (err == hipSuccess) err = hipEventRecord(e1, c->stream);
            if (err == hipSuccess) err = hipEventSynchronize(e1);
            if (err == hipSuccess) err = hipEventElapsedTime(&ms, e0, e1);
        }
        if (err != hipSuccess) break;
        if (c->val_tune == 2) fprintf(stderr, "tune_val: candidate %d %.3f ms\n", k, ms);
        if (k == 0 || ms < best) {
            best = ms;
            bi = k;
        }
    }
    c->bins_first = true;  // the trials left words in every slot
    HIPCHK(finish(err));
    HIPCHK(hipMemsetAsync(c->st, 0, kStatLines * sizeof(DevStats), c->stream));  // the trials' stats
    return GOSSIP_OK;
}

// Record segments of propagation-blocked push rounds: one partition, one word per peer, no overflow rows
// (re-bootstrap and rejoin edges are not in the CSR the segments are counted from); skipped, not failed,
// when they do not fit.
gossip_status prepare_pb(gossip_ctx* c) {
    if (c->Wp != 1 || c->n_local != c->n || (c->cfg.flags & GOSSIP_FLAG_NO_BLOCKED) || c->cfg.extra_cap ||
        c->cfg.rejoin_threshold || !c->n_edges)
        return GOSSIP_OK;
    std::string err;
    const hipError_t e = build_pb(c->rp, c->col, c->n_local, c->n_edges, c->heavy, c->chunks, c->n_chunks,
                                  c->pb_direct_in, c->stream, &c->pb, &err);
    if (e == hipErrorOutOfMemory || e == hipErrorInvalidValue) return GOSSIP_OK;  // push rounds stay atomic
    if (e != hipSuccess) return fail(GOSSIP_EHIP, "blocked-push regions: " + err);
    c->pb_ready = true;
    return GOSSIP_OK;
}

// Slot layout for binned dense rounds: only for a full, symmetric overlay
// (pull-eligible); skipped, not failed, when it does not fit in HBM.
gossip_status prepare_bins(gossip_ctx* c) {
    c->bins_first = false;  // a fresh layout holds zeros
    free_bins(&c->bins);
    c->bins_ready = false;
    free_pb(&c->pb);
    c->pb_ready = false;
    if (c->symmetric && !(c->cfg.flags & GOSSIP_FLAG_NO_BIN) && c->n_edges) {
        // the streamed layout (values in cb order: the scatter writes front to back, the apply reads runs) at
        // every size since round 4.  Round 2 kept it for slot arrays under 128 MB (config 4: 62.6 vs 64.5 ms
        // per step for the slot layout); since its scatter's whole-line pieces and its apply's pipelined run
        // loads it wins everywhere (round 4, alternated on one box: config 4 49.5 vs 51.8 ms per step, config 5
        // 25.5-25.9 vs 26.3-27.2, config 3 4.87-5.09 vs 5.24-5.34; config 4's dense rounds: scatter 4.4 ms,
        // no partial-sector stores, no allocation trials).  "bin_stream" 0 keeps the slot layout (A/B, tests).
        c->bin_stream = c->bin_stream_req != 0;
        std::string err;
        // a vertex block cuts the source ids into segments (the staged dense exchange delivers whole ones)
        const uint64_t seg = c->n_local != c->n ? bin_segment(c->n) : 0;
        const hipError_t e = build_bins(c->rp, c->col, c->n_local, c->n, c->n_edges, c->heavy, c->Wp, c->bin_stream,
                                        c->bin_words_req, c->bin_chunk_req, seg, c->scatter_units, c->stream, &c->bins,
                                        &err);
        if (e == hipSuccess) {
            c->bins_ready = true;
            if (gossip_status ts = tune_val(c)) return ts;
        } else if (e != hipErrorOutOfMemory && e != hipErrorInvalidValue) {  // else dense rounds gather instead
            return fail(GOSSIP_EHIP, "bin layout: " + err);
        }
    }
    return prepare_pb(c);
}

// the needy lists and the booking lines of late pull rounds, on first use
gossip_status ensure_lists(gossip_ctx* c) {
    const uint32_t cap = c->list_cap_req ? c->list_cap_req
                                         : (uint32_t)std::min<uint64_t>(std::max<uint64_t>(c->n_local / 16, 1u << 16),
                                                                        0xFFFFFFFFull);
    // a new capacity takes effect only between chains: a list in flight (this round's input, or the input of
    // one of the last two rounds, which k_list_zero clears by) must stay where it is
    const bool live = c->lst_in >= 0 || c->lin_idx[0] >= 0 || c->lin_idx[1] >= 0;
    if (c->st_pre && (c->lst_cap == cap || live)) return GOSSIP_OK;
    for (auto& l : c->lst) {
        hipFree(l);
        l = nullptr;
    }
    if (!c->st_pre) {
        HIPCHK(hipMalloc((void**)&c->st_pre, kStatLines * sizeof(DevStats)));
        HIPCHK(hipMemsetAsync(c->st_pre, 0, kStatLines * sizeof(DevStats), c->stream));
    }
    if (!c->d_lst_n) HIPCHK(hipMalloc((void**)&c->d_lst_n, 4 * sizeof(uint32_t)));
    for (auto& l : c->lst) HIPCHK(hipMalloc((void**)&l, (uint64_t)cap * sizeof(uint32_t)));
    c->lst_cap = cap;
    return GOSSIP_OK;
}

// seen |= nw for a deferred round whose fold was left to the next binned round
gossip_status settle_fold(gossip_ctx* c) {
    if (!c->fold_pending) return GOSSIP_OK;
    c->fold_pending = false;
    HIPCHK(timed(c, "commit", [&] { return launch_commit_nx(c->seen, c->nw, c->n_local * c->Wp, c->stream); }));
    return GOSSIP_OK;
}

uint32_t kills_in_round(const gossip_ctx* c, uint32_t r, uint32_t* first) {
    auto lo = std::lower_bound(c->kill_round_sorted.begin(), c->kill_round_sorted.end(), r);
    auto hi = std::upper_bound(c->kill_round_sorted.begin(), c->kill_round_sorted.end(), r);
    *first = (uint32_t)(lo - c->kill_round_sorted.begin());
    return (uint32_t)(hi - lo);
}

uint32_t injections_in_round(const gossip_ctx* c, uint32_t r, uint32_t* first) {
    auto lo = std::lower_bound(c->inj_round_sorted.begin(), c->inj_round_sorted.end(), r);
    auto hi = std::upper_bound(c->inj_round_sorted.begin(), c->inj_round_sorted.end(), r);
    *first = (uint32_t)(lo - c->inj_round_sorted.begin());
    return (uint32_t)(hi - lo);
}

// Re-bootstrap (handleDeadPeer peer.cpp:398-404): this round's reports, sorted
// by (reporter, dead), each make the reporter re-select from a seed response.
gossip_status rebootstrap_round(gossip_ctx* c, const RoundArgs& a) {
    unsigned long long total = 0;
    HIPCHK(hipMemcpyAsync(&total, c->n_reports, sizeof(total), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint64_t upto = std::min<uint64_t>(total, c->report_cap);
    const uint64_t n = upto > c->n_rep_seen ? upto - c->n_rep_seen : 0;
    if (!n) return GOSSIP_OK;
    if (n > c->rb_cap) {
        hipFree(c->rb_keys);
        hipFree(c->rb_keys2);
        hipFree(c->rb_temp);
        c->rb_keys = c->rb_keys2 = nullptr;
        c->rb_temp = nullptr;
        c->rb_cap = std::max<uint64_t>(n, 1u << 16);
        HIPCHK(hipMalloc((void**)&c->rb_keys, c->rb_cap * sizeof(unsigned long long)));
        HIPCHK(hipMalloc((void**)&c->rb_keys2, c->rb_cap * sizeof(unsigned long long)));
        c->rb_temp_bytes = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, c->rb_temp_bytes, c->rb_keys, c->rb_keys2, (size_t)c->rb_cap,
                                                 0, 64, c->stream));
        HIPCHK(hipMalloc(&c->rb_temp, c->rb_temp_bytes + 16));
    }
    HIPCHK(timed(c, "rebootstrap", [&] {
        hipError_t e = launch_reboot_keys(a, c->n_rep_seen, n, c->rb_keys, c->stream);
        size_t tb = c->rb_temp_bytes;
        if (e == hipSuccess)
            e = hipcub::DeviceRadixSort::SortKeys(c->rb_temp, tb, c->rb_keys, c->rb_keys2, (size_t)n, 0, 64, c->stream);
        return e != hipSuccess ? e : launch_rebootstrap(a, c->reboot, c->rb_keys2, n, c->stream);
    }));
    c->n_rep_seen = upto;
    return GOSSIP_OK;
}

// Round phase 1: churn, kills, liveness, injection; choose push or pull.
// requested: GOSSIP_MODE_AUTO (P = 1: the engine's frontier estimate decides),
// GOSSIP_MODE_PUSH or GOSSIP_MODE_PULL (partitioned runs: the driver decides
// from global stats so every rank agrees; an ineligible pull falls back to
// push, and eligibility is itself global state, so ranks still agree).
gossip_status round_begin(gossip_ctx* c, bool remote, int requested, int* mode) {
    c->bufs_zero = false;  // any round may write nw / nx
    if (!c->graph_ready) return fail(GOSSIP_ESTATE, "no overlay: call gossip_build_graph or gossip_load_csr");
    if (!c->has_schedule) return fail(GOSSIP_ESTATE, "no schedule: call gossip_inject");
    if (c->finished) return fail(GOSSIP_ESTATE, "run finished: call gossip_reset");
    if (c->round >= c->cfg.max_rounds) return fail(GOSSIP_ESTATE, "max_rounds reached");
    if (c->closed_live && !c->death_r && (c->cfg.churn_threshold || !c->kill_round_sorted.empty())) {
        HIPCHK(hipMalloc((void**)&c->death_r, c->n_local * 2 + 2));
        HIPCHK(hipMalloc((void**)&c->dgone, c->n_local * 4 + 4));
        HIPCHK(hipMalloc((void**)&c->dmask, c->n_local * 4 + 4));
        HIPCHK(hipMemsetAsync(c->death_r, 0xFF, c->n_local * 2 + 2, c->stream));
        HIPCHK(hipMemsetAsync(c->dgone, 0, c->n_local * 4 + 4, c->stream));
        HIPCHK(hipMemsetAsync(c->dmask, 0, c->n_local * 4 + 4, c->stream));
        if (c->cfg.ping_every && !c->rev) {  // the ping rounds find u -> v from v's row through rev
            HIPCHK(hipMalloc((void**)&c->rev, c->n_edges * 4 + 4));
            RoundArgs r0 = make_args(c);
            HIPCHK(launch_reverse_edges(r0, c->stream));
        }
    }
    if (c->fold_pending) {  // kills and churn book a dying peer's words: seen must hold them first
        uint32_t kf = 0;
        if (c->cfg.rejoin_threshold || c->cfg.churn_threshold || kills_in_round(c, c->round, &kf))
            if (gossip_status fs = settle_fold(c)) return fs;
    }
    // the previous round booked this round's source side (late pull rounds): those lines are this round's
    const bool booked = c->pre_booked;
    c->pre_booked = false;
    if (booked && !c->replaying) std::swap(c->st, c->st_pre);  // (replayed: the booking went to this round's row)
    RoundArgs a = make_args(c);
    const uint32_t pw = pack_w(c);
    if (c->cfg.rejoin_threshold) {  // restarts first: a peer dying this round cannot restart in it
        HIPCHK(hipMemsetAsync(c->rj_n, 0, sizeof(unsigned long long), c->stream));
        HIPCHK(timed(c, "rejoin", [&] {
            return launch_rejoin(a, pw, c->cfg.rng_seed, c->cfg.rejoin_threshold, c->n_started, c->rj_list, c->rj_n,
                                 c->stream);
        }));
        c->any_masked = true;
    }
    uint32_t first = 0, cnt = kills_in_round(c, c->round, &first);
    if (cnt) {
        c->any_dead = true;
        HIPCHK(timed(c, "kills", [&] { return launch_kills(a, pw, c->d_kill_peer + first, cnt, c->stream); }));
    }
    if (c->cfg.churn_threshold) {
        c->any_dead = true;
        HIPCHK(timed(c, "churn", [&] { return launch_churn(a, pw, c->cfg.rng_seed, c->cfg.churn_threshold, c->stream); }));
    }
    if (c->cfg.rejoin_threshold && c->cfg.extra_cap)  // the restarted peers' new out-edges, after the deaths
        HIPCHK(timed(c, "rejoin", [&] {
            return launch_rejoin_select(a, c->reboot, c->rj_list, c->rj_n, c->n_local, c->stream);
        }));
    c->live_counted = false;
    if (c->cfg.ping_every && c->round % c->cfg.ping_every == 0) {
        if (c->timing) {  // the pings this round sends (before its masking), for 8(d)'s liveness bytes
            if (!c->d_live) HIPCHK(hipMalloc((void**)&c->d_live, 2 * sizeof(unsigned long long)));
            HIPCHK(hipMemsetAsync(c->d_live, 0, 2 * sizeof(unsigned long long), c->stream));
            HIPCHK(launch_live_count(a, c->d_live, c->stream));
            c->live_counted = true;
        }
        HIPCHK(timed(c, "liveness", [&] {
            hipError_t e = hipSuccess;
            if (c->closed_live) {
                // the in-edges of peers whose max_missed-th ping round since death is this one
                const int64_t pe = c->cfg.ping_every, mm = std::max<uint32_t>(c->cfg.max_missed, 1u);
                const int64_t hi = (int64_t)c->round - (mm - 1) * pe;
                if (c->rev && hi >= 0)
                    e = launch_liveness_window(a, (uint32_t)std::max<int64_t>(0, hi - pe + 1), (uint32_t)hi, c->stream);
            } else {
                e = launch_liveness(a, c->stream, 1);
                if (e == hipSuccess) e = launch_liveness(a, c->stream, 0);
            }
            if (e == hipSuccess && c->cfg.extra_cap) e = launch_liveness_extra(a, c->stream);
            return e;
        }));
        c->any_masked = true;
        if (c->cfg.extra_cap) {
            gossip_status rs = rebootstrap_round(c, a);
            if (rs) return rs;
        }
    }
    cnt = injections_in_round(c, c->round, &first);
    if (cnt)
        HIPCHK(timed(c, "inject", [&] {
            return launch_inject(a, pw, c->d_inj_origin + first, c->d_inj_msg + first, cnt, c->stream);
        }));
    // messages injected up to and including this round (what a peer can still learn)
    {
        uint32_t hi = (uint32_t)(std::upper_bound(c->inj_round_sorted.begin(), c->inj_round_sorted.end(), c->round) -
                                 c->inj_round_sorted.begin());
        for (int w = 0; w < kMaxWords; ++w) a.inj_mask[w] = hi ? c->inj_prefix[(uint64_t)(hi - 1) * kMaxWords + w] : 0;
        // bits in flight this round (P = 1): the previous round's receipts (read with its stats) and this
        // round's injections; nothing else is in a new word
        const uint32_t lo = c->round ? (uint32_t)(std::upper_bound(c->inj_round_sorted.begin(), c->inj_round_sorted.end(),
                                                                   c->round - 1) - c->inj_round_sorted.begin())
                                     : 0u;
        const bool known = c->round == 0 || c->flight_round == c->round - 1;
        if (c->flight_ok && known && c->world <= 1 && c->n_local == c->n && !c->cfg.rejoin_threshold) {
            a.use_flight = 1;
            for (int w = 0; w < kMaxWords; ++w) {
                const uint64_t before = lo ? c->inj_prefix[(uint64_t)(lo - 1) * kMaxWords + w] : 0;
                a.in_flight[w] = (c->round ? c->flight[w] : 0) | (a.inj_mask[w] & ~before);
            }
        }
    }
    // dead peers are fine for pull / binned rounds (a live peer's in-edges from
    // live peers are never masked: only edges to dead peers are); re-bootstrap
    // edges are not (they break the symmetry the pull relies on)
    // (nor are restarted peers: their dropped rows break it too)
    const bool pull_ok = c->symmetric && (!c->any_dead || (!c->cfg.extra_cap && !c->cfg.rejoin_threshold)) &&
                         !(c->cfg.flags & GOSSIP_FLAG_FORCE_PUSH) && (!remote || c->gather != nullptr);
    a.dead_mode = c->any_dead ? 1u : 0u;
    bool pull;
    if (requested == GOSSIP_MODE_AUTO) {
        const uint32_t permille = c->cfg.pull_permille ? c->cfg.pull_permille : kPullPermille;
        pull = !remote && pull_ok &&
               ((c->cfg.flags & GOSSIP_FLAG_FORCE_PULL) || (c->frontier_est + cnt) * 1000 >= c->n_local * (uint64_t)permille);
    } else {
        pull = (requested == GOSSIP_MODE_PULL || requested == GOSSIP_MODE_BIN) && pull_ok;
    }
    // binned (single partition): every pull-eligible round when forced; in auto
    // mode while many (peer, message) pairs are still missing -- then nearly
    // every edge has to be looked at and streaming beats gathering.
    bool bin = pull && c->bins_ready && requested == GOSSIP_MODE_BIN;  // driver-chosen (partitioned runs)
    // (peer, message) pairs still missing at push start (P = 1: the own counters are global)
    uint64_t missing = 0;
    {
        uint64_t injected = 0;
        for (int w = 0; w < kMaxWords; ++w) injected += (uint64_t)__builtin_popcountll(a.inj_mask[w]);
        uint64_t have = c->cum_covered + c->last_fresh + cnt, peers = c->n_local;
        // P = 1 with every round's stats read: only the live peers can still learn, only messages that were
        // injected exist, and the pairs the dead held leave the count (config 5 at round 7: ≈ 4 of the
        // "missing" pairs per peer were dead peers' and never-injected messages', which kept it binned)
        if (c->world <= 1 && c->n_local == c->n && !c->cfg.rejoin_threshold && c->flight_round + 1 == c->round &&
            c->round > 0) {
            const uint64_t sched = injected;
            injected = std::min<uint64_t>(sched, c->cum_injected + cnt);
            peers = c->n_started > c->cum_died ? c->n_started - c->cum_died : 0;
            have = have > c->cum_dead_cov ? have - c->cum_dead_cov : 0;
        }
        const uint64_t total = injected * peers;
        missing = total > have ? total - have : 0;
    }
    c->cur_missing = missing;
    if (!remote && pull_ok && c->bins_ready && requested == GOSSIP_MODE_AUTO) {
        if (c->cfg.flags & GOSSIP_FLAG_FORCE_BIN) {
            pull = bin = true;
        } else if (pull && !(c->cfg.flags & GOSSIP_FLAG_FORCE_PULL)) {
            const uint32_t bpm = c->cfg.bin_permille ? c->cfg.bin_permille : 4000;
            // binned from a 2 % frontier: config 5 (2^26, round 3 at an 8 % frontier) pull 8.6 ms against
            // 4.0 binned; config 2 (2^20, 5 % rounds) kernels 7.5-7.6 against 6.9-7.1 ms per step once its
            // bins and chunks were sized for small overlays (with whole-slice bins pull had won, 0.18
            // against 0.33 ms per round)
            const uint32_t front_pm = c->bin_front_pm ? c->bin_front_pm : 20u;
            // and only on a wide frontier: a narrow one is cheaper to gather from (frontier bitmap)
            bin = missing * 1000 >= c->n_local * (uint64_t)bpm &&
                  (c->frontier_est + cnt) * 1000 >= c->n_local * (uint64_t)front_pm;
        }
    }
    // propagation-blocked push (gossip_blocked.hip; one partition, one word per peer): a push round from a
    // 1 % frontier estimate on overlays of >= kPbPushPeers peers (config 4 round 3, 1.25 %, 53.5 M
    // traversals: push 4.4 ms, blocked 3.4-3.5 ms; smaller overlays lose to the blocked round's fixed
    // passes: config 3 round 2, 2.1 %: push 0.25 ms, blocked 0.79 ms; config 2 at 5.05 %: blocked 0.097 ms
    // per round, 9 rounds a step) -- and, where the slot array
    // outgrows the MALL many times over (>= kPbBinSlots slots: its scattered stores go to HBM as partial
    // lines), a binned round below blocked_permille (every edge streamed for a minority of active
    // sources) write one record per delivery instead (config 4 round 4, 17 %: binned 15.6 ms, blocked
    // 11.5 ms; config 3 round 3, 16 %, 1 GiB of slots: binned 1.17 ms, blocked 2.05 ms)
    c->cur_pb = false;
    if (c->pb_ready && !remote && c->world <= 1 && requested == GOSSIP_MODE_AUTO &&
        !(c->cfg.flags & (GOSSIP_FLAG_FORCE_PUSH | GOSSIP_FLAG_FORCE_PULL | GOSSIP_FLAG_FORCE_BIN))) {
        const uint64_t front = c->frontier_est + cnt;
        const uint32_t hi = c->cfg.blocked_permille ? c->cfg.blocked_permille : kPbHiPermille;
        if (c->cfg.flags & GOSSIP_FLAG_FORCE_BLOCKED)
            c->cur_pb = !pull || bin;
        else
            c->cur_pb = (!pull && c->n_local >= kPbPushPeers && front * 1000 >= c->n_local * (uint64_t)c->pb_lo_pm) ||
                        (bin && (!c->bins_ready || c->bins.n_slots >= c->pb_bin_slots) &&
                         front * 1000 < c->n_local * (uint64_t)hi);
        if (c->cur_pb) pull = bin = false;
    }
    // late pull rounds over needy lists (k_pull_list): a round whose source side the previous one booked
    // pulls that round's list -- or, when the list overflowed, sweeps as a row pull that books no source
    // side.  A row pull on a shrinking frontier (the rounds after the dense ones: config 4 round 7), and
    // every list round, books the next round's source side and lists its still-needy rows.  One word per
    // peer, one partition, no deaths, no coverage history, nothing injected or killed later.
    c->cur_list = c->cur_pre = false;
    c->cur_lst_out = -1;
    if (booked) {
        pull = true;
        bin = c->cur_pb = false;
        c->cur_list = c->lst_in >= 0;
    }
    {
        const bool later_inj = c->has_schedule && c->last_inject_round > c->round;
        const bool later_kill = !c->kill_round_sorted.empty() && c->kill_round_sorted.back() > c->round;
        const bool list_ok = c->list_req && c->world <= 1 && !remote && c->Wp == 1 && c->n_local == c->n &&
                             c->symmetric && !c->any_dead && !later_kill && !later_inj && !c->cfg.churn_threshold &&
                             !c->cfg.rejoin_threshold && !c->cfg.extra_cap && !c->cov_hist && !c->gather &&
                             requested == GOSSIP_MODE_AUTO && !(c->cfg.flags & GOSSIP_FLAG_FORCE_BIN);
        const bool rows = pull && !bin && !c->cur_pb;
        if (list_ok && (c->cur_list || (rows && c->frontier_est < c->prev_frontier_est))) {
            if (gossip_status ls = ensure_lists(c)) return ls;
            // not this round's input, nor the previous round's (the next round clears by it)
            int out = 0;
            while (out == (c->cur_list ? c->lst_in : -1) || out == c->lin_idx[0]) ++out;
            c->cur_lst_out = out;
            c->cur_pre = true;
            HIPCHK(queue_zero(c, c->d_lst_n + out, sizeof(uint32_t)));
        }
    }
    c->cur_sparse = !pull && remote && requested == GOSSIP_MODE_PUSH_SPARSE && c->seg != nullptr;
    // a sparse push from a frontier the marked-tile sweep would not take (0.2 % of the block) writes records
    // per destination block (gossip_blocked.hip build_px) instead of OR-ing into the staging buffer and
    // compacting it: config 4 round 3 as 8 parts staged 47 M deliveries and then swept every part's whole
    // 2 GB staging buffer for them (every 64-peer tile of it marked)
    // Below that frontier the push appends its remote deliveries as records to the same buffer (one counter
    // atomic per wave and destination block): the staging buffer's compaction swept every tile of every
    // destination block whatever the round's size (config 4 at P = 8: ≈ 90 us per part in near-empty rounds)
    // (only under the library's own driver, which reads the records where ctx_send_records says: a caller of
    // the phase API takes them from its gossip_set_sparse buffer)
    c->cur_px = c->cur_arec = false;
    if (c->dist && c->cur_sparse && c->Wp == 1 && c->px_pm >= 0 && !c->cfg.extra_cap && c->symmetric && c->world <= kPbCoarseMax) {
        if (c->px_state == 0) {
            std::string err;
            const hipError_t e =
                build_px(c->rp, c->col, c->n_local, c->n, c->heavy, c->chunks, c->n_chunks, c->part_begins.data(),
                         c->world, (uint32_t)(std::find(c->part_begins.begin(), c->part_begins.end(), c->begin) -
                                              c->part_begins.begin()),
                         c->stream, &c->px, &err);
            if (e == hipSuccess) {
                c->px_state = 1;  // (d_part: set with the sparse exchange, gossip_set_sparse)
            } else if (e == hipErrorOutOfMemory || e == hipErrorInvalidValue) {
                c->px_state = -1;  // the staging push stays
            } else {
                return fail(GOSSIP_EHIP, "record push: " + err);
            }
        }
        const bool wide = (c->frontier_est + cnt) * 100000 >= c->n_local * (uint64_t)c->px_pm;
        c->cur_px = c->px_state == 1 && wide;
        c->cur_arec = c->px_state == 1 && !wide;
    }
    // a wide push round (the explosion before the dense rounds) is bound by memory-side atomics, two per
    // fresh delivery (seen, then nx); deferring the seen update halves them for one streamed pass
    // (k_commit_nx).  A per-rank choice: results do not depend on it.
    // Auto: only where the fold can ride on the next dense round's sweep (one partition, the slot layout
    // or the blocked regions, no churn); config 4 round 3: push 5.6 -> 4.1 ms, the 1.3 ms fold pass removed.
    const bool fusable = c->world <= 1 && !remote && (c->bins_ready || c->pb_ready) && !c->cfg.churn_threshold &&
                         !c->cfg.rejoin_threshold && requested == GOSSIP_MODE_AUTO;
    const uint32_t dpm = c->defer_pm == kDeferAuto ? (fusable ? 10u : 0u) : c->defer_pm;
    c->cur_defer = !pull && !c->cur_pb && dpm && (c->frontier_est + cnt) * 1000 >= c->n_local * (uint64_t)dpm;
    // no-return atomics (the receipts counted from nx after the round) unless tile marks need the old words
    a.defer = c->cur_defer ? 1u : 0u;
    const bool rows_pull = pull && !bin;  // k_pull_rows
    if (c->fold_pending) {  // the previous round deferred: its receipts are this round's nw
        if ((bin || rows_pull || c->cur_pb) && c->world <= 1 && !remote) {
            a.fold = 1;  // k_bin_apply / k_pull_rows's / k_pb_scatter's sweep folds them (before k_pull_heavy
                         // or k_pb_apply read seen)
            c->fold_pending = false;
        } else if (gossip_status fs = settle_fold(c)) {
            return fs;
        }
    }
    // a row's first step from its queue entry: worth the extra 8 B per swept peer while many rows are
    // needy (config 4 round 7: 90 M rows, one random col line each); rows are unmasked (no liveness yet)
    a.first2 = rows_pull && c->first_ok && !c->any_masked && missing * 4 >= c->n_local ? c->first2 : nullptr;
    // the deaths since the last dense round -> their in-neighbours' dgone, which only the source side of
    // dense rounds reads (one walk over their rows instead of one per round; the deaths of the push rounds
    // after the last dense round are never walked: config 5, rounds 9-11)
    if (pull && c->death_r && c->dgone_next <= c->round) {
        const uint32_t lo = c->dgone_next, hi = c->round;
        HIPCHK(timed(c, "churn", [&] { return launch_dead_edges(a, lo, hi, c->stream); }));
        c->dgone_next = c->round + 1;
    }
    a.src_booked = booked ? 1u : 0u;
    a.st = c->replaying ? c->d_hist + (uint64_t)c->rep_round * kStatLines : c->st;
    a.st_pre = !c->cur_pre ? nullptr : c->replaying ? c->d_hist + (uint64_t)(c->rep_round + 1) * kStatLines : c->st_pre;
    a.lst_out = c->cur_lst_out >= 0 ? c->lst[c->cur_lst_out] : nullptr;
    a.lst_n = c->cur_lst_out < 0 ? nullptr : c->replaying ? rep_lstn(c, c->rep_round) : c->d_lst_n + c->cur_lst_out;
    a.lst_cap = c->lst_cap;
    c->last_pull = pull;
    c->last_bin = bin;
    c->last_front = false;
    if (pull) {
        if (a.tcur) {  // pull / binned rounds set no tile marks: this round's go, the next push round scans
            if (!c->replaying) HIPCHK(queue_zero(c, a.tcur, tact_bytes(c)));
            a.tcur = a.tnx = nullptr;
            a.tsparse = 0;
        }
        a.nw_src = c->nw;
        a.n_src = c->n_local;
        if (remote) {  // publish this block's new words; the caller all-gathers c->gather
            HIPCHK(hipMemcpyAsync(c->gather + c->begin * c->Wp, c->nw, c->n_local * c->Wp * sizeof(uint64_t),
                                  hipMemcpyDeviceToDevice, c->stream));
            a.nw_src = c->gather;
            a.n_src = c->n;
        }
        // frontier bitmap only when enough neighbours are outside the frontier to pay for the probe, and
        // enough pairs are still missing to pay for building it (a pass over every new word): config 4
        // round 8 (under 0.1 missing pairs per peer) built it (0.45 ms) to save 2.7 K of 1.78 M gathers --
        // its few needy rows stop after a gather or two, at hubs that are in the frontier anyway
        const uint32_t fpm = c->cfg.front_permille ? c->cfg.front_permille : 400;
        if (!bin && requested == GOSSIP_MODE_AUTO && (c->frontier_est + cnt) * 1000 < c->n_local * (uint64_t)fpm &&
            (remote || c->cfg.front_permille || missing * 4 >= c->n_local) && !c->cur_list) {  // (list: no bitmap)
            a.front = c->front;
            c->last_front = true;
        } else {
            a.front = nullptr;
        }
    } else {
        if (c->nx_dirty) {
            HIPCHK(hipMemsetAsync(c->nx, 0, c->n_local * c->Wp * sizeof(uint64_t), c->stream));
            c->nx_dirty = false;
        }
        // dense exchange: clear the staging buffer; sparse: it is kept clear by the compaction pass
        // (a sparse round after a dense one first clears what the dense round left)
        if (remote && (!c->cur_sparse || c->send_dirty)) {
            HIPCHK(hipMemsetAsync(c->send, 0, c->n * c->Wp * sizeof(uint64_t), c->stream));
            c->send_dirty = false;
        }
        if (remote && !c->cur_sparse) c->send_dirty = true;
    }
    a.smark = remote && c->cur_sparse && !c->cur_arec ? c->smark : nullptr;
    if (c->cur_arec) {
        a.rec_out = c->px.rec_out;
        a.rec_cnt = c->d_counts;
        a.rec_stride = c->px.rec_stride;
        a.part = c->d_part;
        a.world = c->world;
    }
    if (c->cur_pb) a.tsparse = 0;  // the blocked round sweeps every tile (round_compute clears the marks)
    c->cur = a;
    c->cur_remote = remote;
    c->in_round = true;
    if (mode)
        *mode = bin ? GOSSIP_MODE_BIN
                : pull ? GOSSIP_MODE_PULL
                : c->cur_pb ? GOSSIP_MODE_BLOCKED
                : c->cur_sparse ? GOSSIP_MODE_PUSH_SPARSE
                : GOSSIP_MODE_PUSH;
    return GOSSIP_OK;
}

// Small overlays run whole in one launch (gossip_tiny.hip) unless they use a feature only the round-by-round
// engine has (re-bootstrap, join churn, coverage history) or are partitioned.
// (the one-launch run writes every round's stats into one pinned buffer of max_rounds entries: a caller's
// "no limit" max_rounds runs round by round instead of allocating it)
constexpr uint32_t kTinyMaxRounds = 1u << 16;

bool tiny_ok(const gossip_ctx* c) {
    return !c->tiny_off && c->graph_ready && c->n_local == c->n && c->world <= 1 && !c->dist && !c->gather &&
           c->n <= kTinyPeers && c->n_edges <= kTinyEdges && !c->cfg.extra_cap && !c->cfg.rejoin_threshold &&
           !c->cov_hist && !c->in_round && c->cfg.max_rounds <= kTinyMaxRounds;
}

TinyArgs tiny_args(gossip_ctx* c) {
    TinyArgs t{};
    t.erow = c->tiny_erow;
    t.col = c->col;
    t.alive = c->alive;
    t.registered = c->registered;
    t.seen = c->seen;
    t.nw = c->nw;
    t.nx = c->nx;
    t.miss = c->miss;
    t.reports = c->reports;
    t.n_reports = c->n_reports;
    t.report_cap = c->report_cap;
    t.inj_live = c->inj_live;
    t.inj_origin = c->d_inj_origin;
    t.inj_msg = c->d_inj_msg;
    t.inj_round = c->d_inj_round;
    t.n_inj = c->has_schedule ? (uint32_t)c->inj_round_sorted.size() : 0u;
    t.kill_peer = c->d_kill_peer;
    t.kill_round = c->d_kill_round;
    t.n_kill = (uint32_t)c->kill_round_sorted.size();
    t.n = (uint32_t)c->n;
    t.n_edges = (uint32_t)c->n_edges;
    t.wd = c->W;
    t.seed = c->cfg.rng_seed;
    t.churn = c->cfg.churn_threshold;
    t.ping_every = c->cfg.ping_every;
    t.max_missed = c->cfg.max_missed;
    t.start = c->round;
    t.min_rounds = c->cfg.min_rounds;
    t.max_rounds = c->cfg.max_rounds;
    t.last_inject_round = c->last_inject_round;
    t.has_schedule = c->has_schedule ? 1u : 0u;
    t.out = c->tiny_out;
    t.out_cap = c->tiny_cap;
    t.result = c->tiny_result;
    return t;
}

// A whole run (from round 0) in one launch; the host reads every round's stats once.
gossip_status tiny_run(gossip_ctx* c, gossip_round_stats* per_round, uint32_t cap, uint32_t* rounds) {
    if (!c->tiny_erow) {
        HIPCHK(hipMalloc((void**)&c->tiny_erow, (c->n_edges + 1) * sizeof(uint32_t)));
        HIPCHK(launch_tiny_erow(c->rp, (uint32_t)c->n, c->tiny_erow, c->stream));
    }
    // the kernel writes the stats straight into pinned host memory: after it, one stream sync and no copies
    if (!c->tiny_out || c->tiny_cap < c->cfg.max_rounds) {
        if (c->tiny_out) hipHostFree(c->tiny_out);
        c->tiny_out = nullptr;
        HIPCHK(hipHostMalloc((void**)&c->tiny_out, (uint64_t)c->cfg.max_rounds * sizeof(gossip_round_stats)));
        c->tiny_cap = c->cfg.max_rounds;
    }
    if (!c->tiny_result) HIPCHK(hipHostMalloc((void**)&c->tiny_result, 4 * sizeof(uint32_t)));
    if (!c->d_kill_round) {  // no kills scheduled: an empty list
        const uint32_t none = 0xFFFFFFFFu;
        HIPCHK(hipMalloc((void**)&c->d_kill_round, sizeof(uint32_t)));
        HIPCHK(hipMemcpy(c->d_kill_round, &none, sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    const TinyArgs t = tiny_args(c);
    HIPCHK(timed(c, "tiny", [&] { return launch_tiny_run(t, c->Wp, c->stream); }));
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint32_t k = std::min(c->tiny_result[0], c->tiny_cap);
    const std::vector<gossip_round_stats> st(c->tiny_out, c->tiny_out + k);
    if (c->tiny_result[1]) std::swap(c->nw, c->nx);
    uint64_t died = 0, reps = 0;
    for (const auto& x : st) {
        died += x.died;
        reps += x.reports;
        if (c->timing) c->kbytes["tiny"] += 32.0 * (double)x.frontier + 20.0 * (double)x.traversals;
    }
    c->round += k;
    c->finished = true;
    c->any_dead |= died > 0;
    c->any_masked |= reps > 0;
    if (k) {
        c->last_fresh = st.back().new_receipts;
        c->cum_digest = st.back().digest;
        c->cum_covered = st.back().covered;
    }
    c->bufs_zero = c->last_fresh == 0;  // the last round consumed every new word and produced none
    c->nx_dirty = !c->bufs_zero;
    c->last_pull = c->last_bin = false;
    c->last_st_round = ~0u;
    c->flight_round = ~0u;
    if (per_round) std::copy(st.begin(), st.begin() + std::min<size_t>(cap, st.size()), per_round);
    if (rounds) *rounds = k;
    return GOSSIP_OK;
}

// Who books the source side of a binned round: the scatter's staging (auto, both layouts) or the apply
// ("src_stats" 0)
uint32_t src_stats(const gossip_ctx* c) {
    return c->src_stats_req >= 0 ? (uint32_t)(c->src_stats_req != 0) : 1u;
}

// Round phase 2: the push or pull kernels (after the caller's all-gather in a
// partitioned pull round).
gossip_status round_compute(gossip_ctx* c) {
    if (!c->in_round) return fail(GOSSIP_ESTATE, "gossip_round_begin first");
    RoundArgs a = c->cur;
    const uint32_t pw = pack_w(c);
    c->in_round = false;
    TraceRange tr("%s", c->last_bin ? "binned" : c->last_pull ? "pull" : c->cur_pb ? "push (blocked)" : c->cur_sparse ? "push (sparse exchange)" : "push");
    if (c->cur_pb) {
        PbArgs p = pb_args(c->pb);
        p.pipe = c->pb_pipe ? 1u : 0u;
        p.chunks = c->chunks;
        p.n_chunks = c->n_chunks;
        p.nw = reinterpret_cast<unsigned long long*>(c->nw);
        p.n_local = c->n_local;
        // whole-array clear from a 5 % frontier (config 4 round 4: 17 %; round 3, 1.25 %, clears per peer)
        p.clear_all = c->pb_clear_all && c->frontier_est * 20 >= c->n_local ? 1u : 0u;
        c->cur_clear_all = p.clear_all != 0;
        // narrow rounds with valid marks: level 1 reads the marked tiles' new words only (config 4 round 3)
        p.marks = c->pb_marks && c->tact_ok && a.tcur && c->frontier_est * 20 < c->n_local
                      ? reinterpret_cast<const unsigned long long*>(a.tcur) : nullptr;
        HIPCHK(timed(c, "pb_scatter", [&] { return launch_pb_scatter(a, p, c->any_dead, c->W, c->stream); }));
        if (a.tcur && !c->replaying) HIPCHK(queue_zero(c, a.tcur, tact_bytes(c)));  // read: cleared before the split
        HIPCHK(timed(c, "pb_split", [&] { return launch_pb_split(p, c->stream); }));
        HIPCHK(timed(c, "pb_apply", [&] { return launch_pb_apply(a, p, c->stream); }));
        return GOSSIP_OK;
    }
    // k_pull_heavy's per-row accumulators, cleared with the round's first kernel
    const bool hz = c->hacc && c->n_chunks && (c->cur_list || c->last_bin || c->last_pull);
    if (hz && !c->replaying) HIPCHK(queue_zero(c, c->hacc, c->n_chunks * c->Wp * sizeof(uint64_t)));
    if (c->cur_list) {
        // nx holds the new words of the round before last: its list's rows (and the heavy rows) if that was
        // a list round, anything otherwise
        HIPCHK(timed(c, "list_zero", [&] {
            if (c->lin_idx[1] >= 0) return launch_list_zero(a, c->lst[c->lin_idx[1]], c->lin_n[1], c->stream);
            return hipMemsetAsync(c->nx, 0, c->n_local * sizeof(uint64_t), c->stream);
        }));
        HIPCHK(timed(c, "pull_list", [&] { return launch_pull_list(a, c->lst[c->lst_in], c->lst_in_n, c->stream); }));
        HIPCHK(timed(c, "pull_heavy", [&] { return launch_pull_heavy(a, pw, c->stream, hz); }));
        return GOSSIP_OK;
    }
    if (c->last_pull && a.dead_mode && !a.dgone)  // else the per-source counters give the source side
        HIPCHK(timed(c, "src_count", [&] { return launch_src_count(a, pw, c->stream); }));
    if (c->last_bin) {
        if (c->apply_persist && c->bin_stream && !c->d_work)
            HIPCHK(hipMalloc((void**)&c->d_work, 8 * sizeof(uint32_t)));
        if (c->apply_persist && c->bin_stream && !c->replaying)  // the apply's bin counters, zeroed with the round's first launch
            HIPCHK(queue_zero(c, c->d_work, 8 * sizeof(uint32_t)));
        BinArgs b = bin_args(c, c->bins_first, src_stats(c));
        if (b.work && c->replaying) b.work = rep_work(c, c->rep_round);
        // the heavy rows' pull on the second stream, beside the scatter (it reads seen and the new words, which
        // the scatter leaves alone, and ORs its finds into hacc); k_heavy_commit applies them after the apply,
        // whose whole-tile stores rewrite the heavy rows' seen and nx words
        const bool side = c->heavy_side && c->n_chunks && c->hacc && !a.st_pre && c->world <= 1 && hz;
        if (side) {
            if (!c->aux) HIPCHK(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
            if (!c->ev_fork) HIPCHK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
            if (!c->ev_join) HIPCHK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
            HIPCHK(flush_zero(c));  // (the round's clears -- hacc among them -- before the fork)
            HIPCHK(hipEventRecord(c->ev_fork, c->stream));
            HIPCHK(hipStreamWaitEvent(c->aux, c->ev_fork, 0));
            void* tok = nullptr;
            ctx_timer_start_on(c, c->aux, &tok);
            HIPCHK(launch_pull_heavy(a, pw, c->aux, true, true));
            ctx_timer_stop_on(c, "pull_heavy", c->aux, tok);
            HIPCHK(hipEventRecord(c->ev_join, c->aux));
        }
        // every bin is needy while more than one (peer, message) pair per peer is missing: no check pass
        b.needy_check = c->cur_missing > c->n_local && c->needy_skip ? 0u : 1u;
        if (c->stage_n && c->bins.stages == c->stage_n) {
            // staged exchange (gossip_dist.hip): the own block's chunks first, then each stage's chunks once
            // the driver's event says their words have landed in the gather buffer
            const uint32_t S = c->stage_n;
            c->stage_n = 0;
            for (uint32_t g = 0; g <= S; ++g) {
                if (g) HIPCHK(hipStreamWaitEvent(c->stream, c->stage_ev[g - 1], 0));
                BinArgs bg = b;
                bg.units = c->bins.stage_units + c->bins.stage_lo[g];
                bg.n_units = c->bins.stage_lo[g + 1] - c->bins.stage_lo[g];
                if (bg.n_units) HIPCHK(timed(c, "bin_scatter", [&] { return launch_bin_scatter(a, bg, pw, c->stream); }));
            }
        } else {
            HIPCHK(timed(c, "bin_scatter", [&] { return launch_bin_scatter(a, b, pw, c->stream); }));
        }
        HIPCHK(timed(c, "bin_apply", [&] { return launch_bin_apply(a, b, pw, c->stream); }));
        c->bins_first = false;
        if (side) {
            // (timed from before the join: a wait for the side stream counts in the round's critical path)
            HIPCHK(timed(c, "heavy_commit", [&] {
                const hipError_t e = hipStreamWaitEvent(c->stream, c->ev_join, 0);
                return e != hipSuccess ? e : launch_heavy_commit(a, pw, c->stream);
            }));
        } else {
            HIPCHK(timed(c, "pull_heavy", [&] { return launch_pull_heavy(a, pw, c->stream, hz); }));
        }
        return GOSSIP_OK;
    }
    if (c->last_pull) {
        if (a.front) HIPCHK(timed(c, "frontier_bits", [&] { return launch_frontier_bits(a, pw, c->stream); }));
        // nx is written whole by the light rows' pull; heavy rows are OR-ed in afterwards
        HIPCHK(timed(c, "pull_light", [&] { return launch_pull_rows(a, pw, c->stream); }));
        HIPCHK(timed(c, "pull_heavy", [&] { return launch_pull_heavy(a, pw, c->stream, hz); }));
        return GOSSIP_OK;
    }
    const bool remote = c->cur_remote;
    if (c->cur_arec) HIPCHK(queue_zero(c, c->d_counts, c->world * sizeof(unsigned long long)));  // append counters
    if (c->cur_px) {  // records per destination block (level 1 of a blocked round, the own block delivered at once)
        PbArgs p = pb_args(c->px);
        const uint32_t own =
            (uint32_t)(std::find(c->part_begins.begin(), c->part_begins.end(), c->begin) - c->part_begins.begin());
        p.dir_lo = (uint32_t)c->begin;
        p.dir_hi = (uint32_t)c->end;
        p.dir_base = (uint32_t)c->begin;
        p.chunks = c->chunks;
        p.n_chunks = c->n_chunks;
        p.nw = reinterpret_cast<unsigned long long*>(c->nw);
        p.n_local = c->n_local;
        p.clear_all = 0;
        if (a.tcur) HIPCHK(queue_zero(c, a.tcur, tact_bytes(c)));  // unread marks go
        HIPCHK(timed(c, "px_scatter", [&] { return launch_pb_scatter(a, p, c->any_dead, c->W, c->stream); }));
        HIPCHK(timed(c, "compact_send", [&] {
            return launch_px_pack(p, c->world, own, c->d_part, c->px.rec_stride, c->px.rec_out, c->d_counts, c->chunks,
                                  c->n_chunks, c->nw, c->stream);
        }));
        HIPCHK(hipMemcpyAsync(c->h_counts, c->d_counts, c->world * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        return GOSSIP_OK;
    }
    if (c->cfg.extra_cap)
        HIPCHK(timed(c, "push_extra", [&] { return launch_push_extra(a, pw, c->any_dead, remote, c->stream); }));
    HIPCHK(timed(c, "push_heavy", [&] { return launch_push_heavy(a, pw, c->any_dead, remote, c->stream); }));
    if (a.tcur && !a.tsparse && !c->replaying) HIPCHK(queue_zero(c, a.tcur, tact_bytes(c)));  // unread marks go
    HIPCHK(timed(c, "push_light", [&] { return launch_push_light(a, pw, c->any_dead, remote, c->stream); }));
    if (c->cur_arec) {
        HIPCHK(hipMemcpyAsync(c->h_counts, c->d_counts, c->world * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    } else if (c->cur_sparse) {
        HIPCHK(timed(c, "compact_send", [&] {
            return launch_compact_send(a, pw, c->d_part, c->d_toff, c->n_tiles_all, c->world, c->blk_stride, c->d_counts,
                                       c->seg, c->sx_bits, c->sx_pos, c->sx_tmp, c->sx_bytes, c->stream);
        }));
        HIPCHK(hipMemcpyAsync(c->h_counts, c->d_counts, c->world * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    }
    return GOSSIP_OK;
}

// Checked-index build (GOSSIP_CHECKED): the first index a kernel found past its bound since the last check
// (gossip_device.hpp GOSSIP_IDX), reported once and cleared.  The product build reads nothing.
gossip_status check_bounds(gossip_ctx* c) {
#ifdef GOSSIP_CHECKED
    unsigned long long h[4] = {};
    unsigned long long* d = reinterpret_cast<unsigned long long*>(c->inj_live + kMaxWords);
    HIPCHK(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (!h[0]) return GOSSIP_OK;
    HIPCHK(hipMemsetAsync(d, 0, sizeof(h), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    char msg[192];
    std::snprintf(msg, sizeof(msg), "round %u: %llu indices past their bounds; first: site %llu, index %llu, bound %llu",
                  c->round, h[0], h[1], h[2], h[3]);
    return fail(GOSSIP_EBOUNDS, msg);
#else
    (void)c;
    return GOSSIP_OK;
#endif
}

gossip_status read_slot(gossip_ctx* c, gossip_round_stats* out, bool cumulative) {
    if (c->replaying && c->last_st_round != c->round) {  // the recorded sums; the lines go to the history
        // copied to the history and cleared by the next round's first launch (the zero batch); whatever is
        // queued before goes out first (a queued clear of these lines would run before their copy)
        // (the round's kernels wrote its lines straight into its row of the history)
        c->last_st = c->rec_st[c->rep_round];
        c->lst_out_n = c->rec_lst[c->rep_round];
        c->last_st_round = c->round;
        for (int w = 0; w < kMaxWords; ++w) c->flight[w] = c->last_st.fresh_or[w];
        c->flight_round = c->round;
    }
    if (c->last_st_round != c->round) {  // read once per round, then the lines are re-zeroed for the next
        HIPCHK(flush_zero(c));
        HIPCHK(hipMemcpyAsync(c->h_st, c->st, kStatLines * sizeof(DevStats), hipMemcpyDeviceToHost, c->stream));
        if (c->cur_lst_out >= 0)
            HIPCHK(hipMemcpyAsync(&c->lst_out_n, c->d_lst_n + c->cur_lst_out, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(queue_zero(c, c->st, kStatLines * sizeof(DevStats)));  // cleared with the next round's first launch
        if (gossip_status cs = check_bounds(c)) return cs;
        if (c->cur_pb || c->cur_px) {
            // bit 4: a wave gave up waiting for its staging generation (gossip_stage.hpp, kStageSpin: the
            // protocol always progresses, so this means a bug, not load); bits 1/2: a record region that
            // would have overflowed (cannot happen: capacities are in-degrees).  The round's results are
            // incomplete either way; the flags stay set until the next reset.
            uint32_t e = 0;
            HIPCHK(hipMemcpy(&e, c->cur_px ? c->px.err : c->pb.err, sizeof(e), hipMemcpyDeviceToHost));
            if (e & 4u) return fail(GOSSIP_ESTALL, "blocked round: a record-staging wave stalled past its bound");
            if (e) return fail(GOSSIP_EOVERFLOW, "blocked round: a record region overflowed");
        }
        DevStats sum{};
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(c->h_st);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(&sum);
        for (int l = 0; l < kStatLines; ++l)
            for (int f = 0; f < kStatFields; ++f)
                dst[f] = f < kStatSums ? dst[f] + src[l * kStatFields + f] : dst[f] | src[l * kStatFields + f];
        c->last_st = sum;
        c->last_st_round = c->round;
        if (c->recording) {
            c->rec_st.push_back(sum);
            c->rec_lst.push_back(c->cur_lst_out >= 0 ? c->lst_out_n : 0u);
        }
        // the bits of the round's receipts: the next round's new words (with its injections)
        for (int w = 0; w < kMaxWords; ++w) c->flight[w] = sum.fresh_or[w];
        c->flight_round = c->round;
    }
    const DevStats d = c->last_st;
    c->prev_frontier_est = c->frontier_est;
    c->frontier_est = d.activated;
    c->last_fresh = d.new_receipts;
    if (c->timing) {
        if (c->last_bin) {
            const double wb = 8.0 * c->Wp;
            // slices of every source chunk + row bounds of the frontier + the run-encoded cb list (2 B per
            // binned edge, 4 B per run, 4 B per 64 entries) + slot writes
            const double n_src = c->gather ? (double)c->n : (double)c->n_local;
            // the run tables (4 B per run + 4 B per 64 entries or slots): the scatter's in slot order,
            // the apply's when streamed
            const double runs = 4.0 * c->bins.n_runs + 4.0 * ((c->bins.n_binned + 63) / 64);
            const double cb = 2.0 * c->bins.n_binned + (c->bin_stream ? 0.0 : runs);
            const bool ss = src_stats(c) != 0;  // source side: row bounds in the scatter, or nw + deg in the apply
            c->kbytes["bin_scatter"] += wb * n_src + (ss ? 16.0 * d.frontier : 0.0) + cb + wb * (double)d.pull_gathers;
            c->kbytes["bin_apply"] += (2.0 + wb) * (double)d.pull_edges + 2.0 * wb * c->n_local +
                                      (c->bin_stream && d.pull_edges ? runs : 0.0) + (ss ? 0.0 : (wb + 4.0) * c->n_local);
            c->kbytes["pull_heavy"] += 12.0 * (double)d.heavy_traversals;
        }
        if (c->last_pull && c->cur.dead_mode) c->kbytes["src_count"] += 32.0 * d.frontier + 4.125 * (double)d.traversals;
        if (c->cur_pb) {
            // level 1: the new words swept, the frontier's rows and cleared words, 4 B of col and a 12-B record
            // per traversal (an upper bound with dead targets); level 2: 12 B read + 10 B written per record;
            // apply: 10 B per record + the seen read and seen / nx writes of the activated peers
            const double t = (double)d.traversals;
            c->kbytes["pb_scatter"] += 8.0 * c->n_local + 24.0 * d.frontier + 16.0 * t;
            c->kbytes["pb_split"] += 22.0 * t + (c->cur_clear_all ? 8.0 * c->n_local : 0.0);
            c->kbytes["pb_apply"] += 10.0 * t + 24.0 * (double)d.activated;
        }
        if (c->last_bin) {
            // booked above
        } else if (c->cur_list) {
            // list, seen, row bounds per entry, 4 B per edge scanned, 8 B per gather, seen + nx per
            // activated row, 4 B per entry listed; the clear: 12 B per entry of its list, or every nx word
            c->kbytes["pull_list"] += 28.0 * c->lst_in_n + 4.0 * (double)d.pull_edges + 8.0 * (double)d.pull_gathers +
                                      16.0 * (double)d.activated + 4.0 * std::min(c->lst_out_n, c->lst_cap);
            c->kbytes["list_zero"] += c->lin_idx[1] >= 0 ? 12.0 * c->lin_n[1] : 8.0 * c->n_local;
            c->kbytes["pull_heavy"] += 12.0 * (double)d.heavy_traversals;
        } else if (c->last_pull) {
            if (c->last_front) c->kbytes["frontier_bits"] += 8.125 * (c->gather ? c->n : c->n_local);
            c->kbytes["pull_light"] += 40.0 * c->n_local + 4.0 * (double)d.pull_edges + 8.0 * (double)d.pull_gathers;
            c->kbytes["pull_heavy"] += 12.0 * (double)d.heavy_traversals;
        } else if (c->cur_px) {  // as blocked level 1; the pack reads a 12-B record and writes 16 B per remote one
            const double t = (double)d.traversals;
            c->kbytes["px_scatter"] += 8.0 * c->n_local + 24.0 * d.frontier + 16.0 * t;
            c->kbytes["compact_send"] += 28.0 * t;
        } else if (!c->cur_pb) {
            c->kbytes["push_light"] += 32.0 * d.frontier + 20.0 * (double)(d.traversals - d.heavy_traversals);
            c->kbytes["push_heavy"] += 20.0 * (double)d.heavy_traversals;
        }
        c->kbytes["liveness"] += 6.125 * (double)d.live_checked;
        if (c->live_counted) {  // 8(d): 6.125 B per ping + 16 B per alive peer of a ping round
            unsigned long long lv[2] = {0, 0};
            HIPCHK(hipMemcpy(lv, c->d_live, sizeof(lv), hipMemcpyDeviceToHost));
            c->kbytes["#pings"] += (double)lv[0];
            c->kbytes["#pinging_peers"] += (double)lv[1];
            c->live_counted = false;
        }
        // counters (not bytes): device-scope atomics on peer state, traversals by row class
        c->kbytes["#atomics"] += (double)d.atomics;
        c->kbytes["#heavy_trav"] += (double)d.heavy_traversals;
        c->kbytes["#trav"] += (double)d.traversals;
        if (c->last_pull && !c->last_bin) {  // pull rounds: edges whose row still wanted something, gathers issued
            c->kbytes["#pulled"] += (double)d.pull_edges;
            c->kbytes["#gathers"] += (double)d.pull_gathers;
            c->kbytes["#needy_rows"] += (double)(d.diag & 0xFFFFFFFFull);
            c->kbytes["#exit_gathers"] += (double)(d.diag >> 32);
        }
    }
    gossip_round_stats s{};
    s.round = c->round;
    s.flags = (c->cfg.ping_every && c->round % c->cfg.ping_every == 0) ? 1u : 0u;
    s.frontier = d.frontier;
    s.traversals = d.traversals;
    s.deliveries = d.deliveries;
    s.undelivered = d.undelivered;
    s.new_receipts = d.new_receipts;
    s.duplicates = d.deliveries - d.new_receipts;
    s.injected = d.injected;
    s.died = d.died;
    s.reports = d.reports;
    s.seed_removals = d.seed_removals;
    s.reconnects = d.reconnects;
    s.rejoined = d.rejoined;
    if (cumulative) {
        c->cum_digest += d.digest;
        c->cum_covered += d.covered;
        c->cum_dead_cov += d.dead_covered;
        c->cum_died += d.died;
        c->cum_injected += d.injected;
        s.digest = c->cum_digest;
        s.covered = c->cum_covered;
    } else {
        s.digest = d.digest;
        s.covered = d.covered;
    }
    if (out) *out = s;
    return GOSSIP_OK;
}

gossip_status advance(gossip_ctx* c, uint64_t fresh_global) {
    bool pend = false;
    if (c->cur_defer) {  // every delivery of the round is in nx (remote applies included): fold it into seen
        if (c->world <= 1 && (c->bins_ready || c->pb_ready))
            pend = true;  // after the swap, in nw: the next round folds it (k_bin_apply, k_pb_scatter's or
                          // k_pull_rows's sweep) or commits it first (settle_fold)
        else
            HIPCHK(timed(c, "commit", [&] { return launch_commit_nx(c->seen, c->nx, c->n_local * c->Wp, c->stream); }));
        c->cur_defer = false;
    }
    std::swap(c->nw, c->nx);
    // late pull rounds: the next round's source side is booked; its list, unless it overflowed; this
    // round's input list is kept two rounds (the round after next clears nx by it)
    c->pre_booked = c->cur_pre;
    c->lin_idx[1] = c->lin_idx[0];
    c->lin_n[1] = c->lin_n[0];
    c->lin_idx[0] = c->cur_list ? c->lst_in : -1;
    c->lin_n[0] = c->cur_list ? c->lst_in_n : 0u;
    c->lst_in = c->cur_lst_out >= 0 && c->lst_out_n <= c->lst_cap && c->last_st_round == c->round ? c->cur_lst_out : -1;
    c->lst_in_n = c->lst_in >= 0 ? c->lst_out_n : 0u;
    c->cur_list = c->cur_pre = false;
    c->cur_lst_out = -1;
    c->fold_pending = pend;  // push: nw was cleared by push_light; pull: the old nw is stale
    // a push round clears every word it consumes; if nobody was activated nx stayed zero too
    // (only when this round's stats were read: frontier_est / last_fresh are then this round's)
    c->bufs_zero = c->world <= 1 && !c->last_pull && c->last_st_round == c->round && c->frontier_est == 0 &&
                   c->last_fresh == 0;
    c->tcur ^= 1;             // push with marks: every activation marked its tile; otherwise no marks
    c->tact_ok = !c->last_pull && c->tact_marked;
    c->nx_dirty = c->last_pull;
    const uint32_t r = c->round;
    c->round++;
    const bool pending = c->has_schedule && c->last_inject_round > r;
    if ((fresh_global == 0 && !pending && c->round >= c->cfg.min_rounds) || c->round >= c->cfg.max_rounds)
        c->finished = true;
    return GOSSIP_OK;
}

// the host decisions of a run may be replayed from its recording: one partition, nothing that reads device
// state mid-round (re-bootstrap reads the report count, join churn its restarts), no timing
bool replay_eligible(const gossip_ctx* c) {
    return c->replay_req && !c->timing && c->world <= 1 && !c->dist && !c->gather && c->n_local == c->n &&
           !c->cfg.extra_cap && !c->cfg.rejoin_threshold && c->graph_ready && c->has_schedule;
}

void rec_drop(gossip_ctx* c) {
    c->rec_valid = c->recording = false;
    c->rec_st.clear();
    c->rec_lst.clear();
}

gossip_status step_round(gossip_ctx* c, gossip_round_stats* out);

// Every round of the recorded run issued back to back (no host wait between rounds), each round's stat lines
// copied to d_hist; then one read of them, checked field by field against the recording.
gossip_status replay_run(gossip_ctx* c, gossip_round_stats* per_round, uint32_t cap, uint32_t* rounds) {
    const uint32_t R = (uint32_t)c->rec_st.size();
    const uint64_t tw = c->tact[0] ? tact_bytes(c) / 8 : 0, hw = c->hacc ? c->n_chunks * c->Wp : 0;
    if (c->hist_cap != R || c->rep_tw != tw || c->rep_hw != hw) {  // (the rows below are laid out for R rounds)
        hipFree(c->d_hist);
        c->d_hist = nullptr;
        c->hist_cap = 0;
        hipFree(c->rep_aux);
        c->rep_aux = nullptr;
        // rows 0..R (a round may book the next one's source side into row R)
        HIPCHK(hipMalloc((void**)&c->d_hist, (uint64_t)(R + 1) * kStatLines * sizeof(DevStats)));
        c->rep_tw = tw;
        c->rep_hw = hw;
        // tile marks (R + 1 rows), heavy accumulators, 16 apply counters and 4 list counters (u32) per round
        c->rep_aux_words = c->rep_tw * (R + 1) + c->rep_hw * R + 8ull * R + 2ull * R + 1;
        HIPCHK(hipMalloc((void**)&c->rep_aux, c->rep_aux_words * sizeof(uint64_t)));
        c->hist_cap = R;
    }
    HIPCHK(flush_zero(c));
    HIPCHK(hipMemsetAsync(c->d_hist, 0, (uint64_t)(R + 1) * kStatLines * sizeof(DevStats), c->stream));
    HIPCHK(hipMemsetAsync(c->rep_aux, 0, c->rep_aux_words * sizeof(uint64_t), c->stream));
    c->replaying = true;
    uint32_t k = 0;
    gossip_status s = GOSSIP_OK;
    bool any_pb = false;
    for (c->rep_round = 0; c->rep_round < R && !c->finished; ++c->rep_round) {
        gossip_round_stats st;
        s = step_round(c, &st);
        if (s < 0) break;
        any_pb |= c->cur_pb;
        if (per_round && k < cap) per_round[k] = st;
        ++k;
    }
    c->replaying = false;
    if (s < 0) {
        rec_drop(c);
        return s;
    }
    std::vector<DevStats> h((uint64_t)R * kStatLines);
    HIPCHK(flush_zero(c));
    HIPCHK(hipMemcpyAsync(h.data(), c->d_hist, h.size() * sizeof(DevStats), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    bool same = k == R && c->finished;
    for (uint32_t r = 0; same && r < R; ++r) {
        DevStats sum{};
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&h[(uint64_t)r * kStatLines]);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(&sum);
        for (int l = 0; l < kStatLines; ++l)
            for (int f = 0; f < kStatFields; ++f)
                dst[f] = f < kStatSums ? dst[f] + src[l * kStatFields + f] : dst[f] | src[l * kStatFields + f];
        // every result field (the measurement counters -- heavy-row edges scanned, pull edges scanned and
        // gathers, atomics issued, diag -- depend on timing: an early exit racing another chunk's find, a
        // plain read racing another thread's atomic)
        const unsigned long long* x = reinterpret_cast<const unsigned long long*>(&sum);
        const unsigned long long* y = reinterpret_cast<const unsigned long long*>(&c->rec_st[r]);
        for (int f = 0; same && f < kStatFields; ++f)
            same = f == 11 || f == 14 || f == 15 || f == 18 || f == 19 || x[f] == y[f];
    }
    if (gossip_status cs = check_bounds(c)) {
        rec_drop(c);
        return cs;
    }
    if (same && any_pb) {
        uint32_t e = 0;
        HIPCHK(hipMemcpy(&e, c->pb.err, sizeof(e), hipMemcpyDeviceToHost));
        if (e & 4u) return fail(GOSSIP_ESTALL, "blocked round: a record-staging wave stalled past its bound");
        if (e) return fail(GOSSIP_EOVERFLOW, "blocked round: a record region overflowed");
    }
    if (!same) {
        rec_drop(c);
        return fail(GOSSIP_ESTATE, "a replayed run's device stats differ from its recording");
    }
    c->kbytes["#replayed_runs"] += 1.0;  // (gossip_kernel_bytes: how many runs issued from their recording)
    if (rounds) *rounds = k;
    return GOSSIP_OK;
}

}  // namespace

extern "C" {

const char* gossip_strerror(gossip_status s) {
    switch (s) {
        case GOSSIP_OK: return "ok";
        case GOSSIP_EINVAL: return "invalid argument";
        case GOSSIP_ENOMEM: return "out of memory";
        case GOSSIP_EHIP: return "HIP runtime error";
        case GOSSIP_ESTATE: return "call out of order";
        case GOSSIP_ENODEV: return "no gfx950 device";
        case GOSSIP_EOVERFLOW: return "report buffer overflow";
        case GOSSIP_ECOMM: return "RCCL error";
        case GOSSIP_ESTALL: return "device work stalled";
        case GOSSIP_EBOUNDS: return "index past its bound (checked build)";
        default: return "unknown status";
    }
}

const char* gossip_last_error(void) { return g_last_error.c_str(); }

gossip_status gossip_create(const gossip_config* cfg, gossip_ctx** out) {
    if (!cfg || !out) return fail(GOSSIP_EINVAL, "null argument");
    *out = nullptr;
    if (cfg->n_peers < 1 || cfg->n_peers > 0x7FFFFFFFull) return fail(GOSSIP_EINVAL, "n_peers out of range");
    if (cfg->n_msgs < 1 || cfg->n_msgs > 64u * kMaxWords) return fail(GOSSIP_EINVAL, "n_msgs must be 1..512");
    uint64_t b = cfg->part_begin, e = cfg->part_end;
    if (b == 0 && e == 0) e = cfg->n_peers;
    if (b >= e || e > cfg->n_peers) return fail(GOSSIP_EINVAL, "bad partition range");
    if (cfg->rejoin_threshold && !(b == 0 && e == cfg->n_peers))
        return fail(GOSSIP_EINVAL, "rejoin_threshold needs a single partition");
    if (cfg->graph_model == GOSSIP_GRAPH_REF_BOOTSTRAP && cfg->n_peers > 4096)
        return fail(GOSSIP_EINVAL, "ref_bootstrap supports n_peers <= 4096");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(GOSSIP_ENODEV, "no HIP device visible");
    int dev = cfg->device;
    if (dev < 0) hipGetDevice(&dev);
    if (dev >= ndev) return fail(GOSSIP_ENODEV, "device ordinal out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(GOSSIP_ENODEV, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(GOSSIP_ENODEV, std::string("libgossip_hip is built for gfx950, device is ") + prop.gcnArchName);

    gossip_ctx* c = new (std::nothrow) gossip_ctx();
    if (!c) return fail(GOSSIP_ENOMEM, "ctx allocation");
    c->cfg = *cfg;
    if (!c->cfg.max_missed) c->cfg.max_missed = 3;
    if (!c->cfg.max_rounds) c->cfg.max_rounds = 4096;
    if (!c->cfg.list_len) c->cfg.list_len = 6;
    if (!c->cfg.n_seeds) c->cfg.n_seeds = 20;
    if (!c->cfg.graph_model) c->cfg.graph_model = GOSSIP_GRAPH_POWERLAW;
    c->device = dev;
    c->n = cfg->n_peers;
    c->begin = b;
    c->end = e;
    c->n_local = e - b;
    c->M = cfg->n_msgs;
    c->W = (cfg->n_msgs + 63) / 64;
    c->Wp = pad_words(c->W);
    auto bail = [&](const char* what, hipError_t err) {
        std::string m = std::string(what) + ": " + hipGetErrorString(err);
        free_state(c);
        if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
        delete c;
        return fail(err == hipErrorOutOfMemory ? GOSSIP_ENOMEM : GOSSIP_EHIP, m);
    };
    hipError_t err;
    if ((err = hipSetDevice(dev)) != hipSuccess) return bail("hipSetDevice", err);
    if ((err = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bail("stream", err);
    c->own_stream = true;
    const uint64_t words = c->n_local * c->Wp;
    const uint64_t words2 = (words + 1) & ~1ull;  // k_commit_nx streams 16-B pairs
    const uint64_t bitwords = (c->n + 31) / 32;
    if ((err = hipMalloc((void**)&c->seen, words2 * 8)) != hipSuccess) return bail("seen", err);
    if ((err = hipMalloc((void**)&c->nw, words2 * 8)) != hipSuccess) return bail("new", err);
    if ((err = hipMalloc((void**)&c->nx, words2 * 8)) != hipSuccess) return bail("next", err);
    if ((err = hipMalloc((void**)&c->front, ((c->n_local + 63) / 64 + 1) * 8)) != hipSuccess) return bail("front", err);
    for (int k = 0; k < 2; ++k)
        if ((err = hipMalloc((void**)&c->tact[k], tact_bytes(c))) != hipSuccess) return bail("frontier tiles", err);
    if ((err = hipMalloc((void**)&c->alive, bitwords * 4)) != hipSuccess) return bail("alive", err);
    if ((err = hipMalloc((void**)&c->registered, bitwords * 4)) != hipSuccess) return bail("registry", err);
    if ((err = hipMalloc((void**)&c->st, kStatLines * sizeof(DevStats))) != hipSuccess)
        return bail("stats", err);
    if ((err = hipHostMalloc((void**)&c->h_st, kStatLines * sizeof(DevStats))) != hipSuccess) return bail("pinned stats", err);
    if ((err = hipMalloc((void**)&c->n_reports, sizeof(unsigned long long))) != hipSuccess) return bail("nrep", err);
    // (+4 words: the checked-index build's record, RoundArgs.chk, behind the injected messages)
    if ((err = hipMalloc((void**)&c->inj_live, (kMaxWords + 4) * sizeof(uint64_t))) != hipSuccess) return bail("inj", err);
    if ((err = hipMemset(c->inj_live + kMaxWords, 0, 4 * sizeof(uint64_t))) != hipSuccess) return bail("chk", err);
    if (c->cfg.extra_cap) {
        if (c->cfg.extra_cap > 64) {
            free_state(c);
            if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
            delete c;
            return fail(GOSSIP_EINVAL, "extra_cap must be <= 64");
        }
        const uint64_t slots = c->n_local * c->cfg.extra_cap;
        if ((err = hipMalloc((void**)&c->ex_col, slots * 4 + 4)) != hipSuccess) return bail("extra edges", err);
        if ((err = hipMalloc((void**)&c->ex_cnt, c->n_local * 4 + 4)) != hipSuccess) return bail("extra counts", err);
        if ((err = hipMalloc((void**)&c->ex_miss, slots + 1)) != hipSuccess) return bail("extra misses", err);
        c->reboot.L = c->cfg.list_len;
        c->reboot.seed = c->cfg.rng_seed;
        for (uint32_t j = 1; j < c->cfg.list_len && j < 64; ++j) c->reboot.thr[j] = (uint32_t)pick_threshold(j, c->cfg.list_len);
    }
    if (c->cfg.rejoin_threshold) {
        if ((err = hipMalloc((void**)&c->rj_list, c->n_local * 4 + 4)) != hipSuccess) return bail("rejoin list", err);
        if ((err = hipMalloc((void**)&c->rj_n, sizeof(unsigned long long))) != hipSuccess) return bail("rejoin count", err);
    }
    if (c->cfg.flags & GOSSIP_FLAG_COVERAGE_HISTORY) {
        if ((err = hipMalloc((void**)&c->cov_hist, (uint64_t)c->cfg.max_rounds * 64 * c->Wp * 8)) != hipSuccess)
            return bail("coverage history", err);
    }
    c->n_started = c->n;  // every peer starts until an overlay with a list_cap says otherwise
    if (gossip_status rs = gossip_reset(c)) {
        const std::string m = g_last_error;
        free_state(c);
        if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
        delete c;
        return fail(rs, m);
    }
    *out = c;
    return GOSSIP_OK;
}

// Engineering options (parity-tested A/B variants and layout sizes): explicit per ctx, never read from
// the environment.  Layout options take effect at the next gossip_build_graph / gossip_load_csr.
gossip_status gossip_set_tuning(gossip_ctx* c, const char* key, int64_t value) {
    if (!c || !key) return fail(GOSSIP_EINVAL, "null argument");
    const std::string k(key);
    const uint32_t u = value < 0 ? 0u : (uint32_t)std::min<int64_t>(value, 0xFFFFFFFFll);
    rec_drop(c);  // (any option may change the schedule the recording holds)
    if (k == "tiny") c->tiny_off = value == 0;
    else if (k == "full_liveness") c->full_liveness = value != 0;
    else if (k == "defer_permille") c->defer_pm = value < 0 ? kDeferAuto : u;
    else if (k == "bin_stream") c->bin_stream_req = value < 0 ? -1 : (value != 0);
    else if (k == "pull_first2") c->first_ok = value != 0;
    else if (k == "in_flight") c->flight_ok = value != 0;
    else if (k == "heavy_exit") c->heavy_exit = value != 0;
    else if (k == "heavy_degree") c->heavy_req = value < 0 ? 0u : std::max<uint32_t>(1u, u);
    else if (k == "heavy_chunk") c->heavy_chunk = u;
    else if (k == "bin_front_permille") c->bin_front_pm = u;
    else if (k == "bin_words") c->bin_words_req = u;
    else if (k == "bin_chunk") c->bin_chunk_req = u;
    else if (k == "val_tune") c->val_tune = value < 0 ? -1 : (int)std::min<int64_t>(value, 2);
    else if (k == "src_stats") c->src_stats_req = value < 0 ? -1 : (value != 0);
    else if (k == "blocked_bin_slots") c->pb_bin_slots = value < 0 ? kPbBinSlots : (uint64_t)value;
    else if (k == "blocked_direct_in") c->pb_direct_in = value < 0 ? kPbFineIn : (uint64_t)value;
    else if (k == "list_rounds") c->list_req = value != 0;
    else if (k == "pull_step") {
        if (value != 1 && value != 2) return fail(GOSSIP_EINVAL, "pull_step must be 1 or 2");
        c->row_step = (uint32_t)value;
    }
    else if (k == "blocked_push_permille") c->pb_lo_pm = value < 0 ? kPbLoPermille : u;
    else if (k == "list_cap") c->list_cap_req = u;
    else if (k == "bin_needy_skip") c->needy_skip = value != 0;
    else if (k == "replay") c->replay_req = value != 0;
    else if (k == "scatter_direct") c->scatter_direct = value != 0;
    else if (k == "row_queue") c->row_q = value == 256 ? 256u : 128u;
    else if (k == "row_grid") c->row_grid = u;
    else if (k == "scatter_units") c->scatter_units = u;
    else if (k == "scatter_split_direct") c->split_direct = value != 0;
    else if (k == "apply_wide") c->apply_wide = value != 0;
    else if (k == "scatter_small") c->scatter_small = value != 0;
    else if (k == "blocked_clear_all") c->pb_clear_all = value != 0;
    else if (k == "blocked_marks") c->pb_marks = value != 0;
    else if (k == "blocked_pipe") c->pb_pipe = value != 0;
    else if (k == "zero_fill") c->zero_fill = value != 0;
    else if (k == "heavy_side") c->heavy_side = value != 0;
    else if (k == "apply_pipe") {
        if (value < 0 || value > 10) return fail(GOSSIP_EINVAL, "apply_pipe must be 0..10");
        c->apply_pipe = (uint32_t)value;
    }
    else if (k == "apply_persist") c->apply_persist = value != 0;
    else if (k == "apply_probe") {  // diagnostics: the streamed apply's phase clocks, read back as #probe_*
        if (value && !c->d_probe) {
            if (hipMalloc((void**)&c->d_probe, kProbeN * sizeof(unsigned long long)) != hipSuccess)
                return fail(GOSSIP_ENOMEM, "apply_probe buffer");
            if (hipMemset(c->d_probe, 0, kProbeN * sizeof(unsigned long long)) != hipSuccess)
                return fail(GOSSIP_EHIP, "apply_probe buffer");
        } else if (!value && c->d_probe) {
            hipFree(c->d_probe);
            c->d_probe = nullptr;
        }
    }
    else if (k == "gather_permille") c->gather_pm = value < 0 ? kGatherPermille : u;
    else if (k == "px_permille") c->px_pm = value < 0 ? -1 : (int32_t)std::min<int64_t>(value * 100, 1 << 30);
    else if (k == "px_per100k") c->px_pm = value < 0 ? -1 : (int32_t)std::min<int64_t>(value, 1 << 30);
    else if (k == "exchange_stages") {
        if (value < 1 || value > (int64_t)kMaxStages) return fail(GOSSIP_EINVAL, "exchange_stages must be 1..16");
        c->stages_req = (uint32_t)value;
    }
    else return fail(GOSSIP_EINVAL, "unknown tuning option: " + k);
    return GOSSIP_OK;
}

void gossip_destroy(gossip_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    drain_timers(c);
    for (hipEvent_t e : c->event_pool) hipEventDestroy(e);
    free_state(c);
    free_graph(c);
    hipFree(c->d_inj_origin);
    hipFree(c->d_inj_msg);
    hipFree(c->d_kill_peer);
    hipFree(c->d_inj_round);
    hipFree(c->d_kill_round);
    if (c->tiny_out) hipHostFree(c->tiny_out);
    if (c->tiny_result) hipHostFree(c->tiny_result);
    hipFree(c->d_counts);
    if (c->h_counts) hipHostFree(c->h_counts);
    hipFree(c->d_live);
    hipFree(c->sx_bits);
    hipFree(c->smark);
    hipFree(c->d_probe);
    hipFree(c->d_work);
    hipFree(c->d_hist);
    hipFree(c->rep_aux);
    hipFree(c->d_part);
    hipFree(c->d_toff);
    hipFree(c->sx_pos);
    hipFree(c->sx_tmp);
    if (c->aux) {
        hipStreamSynchronize(c->aux);
        hipStreamDestroy(c->aux);
    }
    if (c->ev_fork) hipEventDestroy(c->ev_fork);
    if (c->ev_join) hipEventDestroy(c->ev_join);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    if (c->dist && c->dist_owned) gossip::dist_free(c->dist);
    delete c;
}

gossip_status gossip_set_stream(gossip_ctx* c, void* s) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (set_dev(c)) return GOSSIP_EHIP;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->own_stream) hipStreamDestroy(c->stream);
    c->stream = (hipStream_t)s;
    c->own_stream = false;
    return GOSSIP_OK;
}

gossip_status gossip_get_shape(gossip_ctx* c, uint32_t* words, uint32_t* exchange_words, uint64_t* n_local,
                               uint64_t* n_edges) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (words) *words = c->W;
    if (exchange_words) *exchange_words = c->Wp;
    if (n_local) *n_local = c->n_local;
    if (n_edges) *n_edges = c->n_edges;
    return GOSSIP_OK;
}

gossip_status gossip_build_graph(gossip_ctx* c) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (set_dev(c)) return GOSSIP_EHIP;
    if (c->cfg.graph_model == GOSSIP_GRAPH_REF_BOOTSTRAP) {
        if (c->n_local != c->n) return fail(GOSSIP_EINVAL, "ref_bootstrap is single-partition");
        std::vector<uint64_t> rp;
        std::vector<uint32_t> col;
        host_ref_bootstrap((uint32_t)c->n, c->cfg.n_seeds, c->cfg.rng_seed, rp, col);
        gossip_status st = upload_csr(c, rp.data(), col.data(), col.size());
        c->symmetric = false;  // the literal bootstrap overlay is a DAG (F8)
        c->n_started = started_under_cap(c->n, c->cfg.list_cap);
        return st ? st : gossip_reset(c);  // round 0 state of the new overlay
    }
    if (c->cfg.graph_model != GOSSIP_GRAPH_POWERLAW) return fail(GOSSIP_EINVAL, "unknown graph_model");
    if (c->cfg.list_len < 2 || c->cfg.list_len > 64) return fail(GOSSIP_EINVAL, "list_len must be 2..64");
    if (c->n < 2) return fail(GOSSIP_EINVAL, "powerlaw needs n_peers >= 2");
    uint64_t* rp = nullptr;
    uint32_t* col = nullptr;
    uint64_t m = 0;
    std::string err;
    if (build_powerlaw_device(c->n, c->begin, c->end, c->cfg.list_len, c->cfg.rng_seed, &rp, &col, &m, c->stream,
                              &err) != hipSuccess)
        return fail(GOSSIP_EHIP, "overlay generator: " + err);
    gossip_status st = install_graph(c, rp, col, m);
    c->symmetric = true;  // powerlaw overlay is symmetrised by construction
    if (!st) st = prepare_bins(c);
    return st ? st : gossip_reset(c);  // round 0 state of the new overlay
}

gossip_status gossip_load_csr(gossip_ctx* c, const uint64_t* rp, const uint32_t* col, uint64_t n_rows,
                              uint64_t n_edges) {
    if (!c || !rp || (n_edges && !col)) return fail(GOSSIP_EINVAL, "null argument");
    if (n_rows != c->n_local) return fail(GOSSIP_EINVAL, "n_rows must equal the owned peer count");
    if (rp[0] != 0 || rp[n_rows] != n_edges) return fail(GOSSIP_EINVAL, "row_ptr must start at 0 and end at n_edges");
    for (uint64_t v = 0; v < n_rows; ++v) {
        if (rp[v + 1] < rp[v]) return fail(GOSSIP_EINVAL, "row_ptr not monotone");
        for (uint64_t e = rp[v]; e < rp[v + 1]; ++e) {
            if (col[e] >= c->n) return fail(GOSSIP_EINVAL, "col entry out of range");
            if (col[e] == c->begin + v) return fail(GOSSIP_EINVAL, "self loop");
            if (e > rp[v] && col[e] <= col[e - 1]) return fail(GOSSIP_EINVAL, "row not sorted/unique");
        }
    }
    // symmetric iff every edge v->c has its reverse (rows are sorted): enables pull rounds
    bool sym = c->n_local == c->n;
    for (uint64_t v = 0; sym && v < n_rows; ++v)
        for (uint64_t e = rp[v]; sym && e < rp[v + 1]; ++e) {
            const uint32_t* b = col + rp[col[e]];
            const uint32_t* x = col + rp[col[e] + 1];
            sym = std::binary_search(b, x, (uint32_t)v);
        }
    if (set_dev(c)) return GOSSIP_EHIP;
    gossip_status st = upload_csr(c, rp, col, n_edges);
    c->symmetric = sym;
    if (!st) st = prepare_bins(c);
    return st ? st : gossip_reset(c);  // round 0 state of the new overlay
}

gossip_status gossip_read_csr(gossip_ctx* c, uint64_t* rp, uint32_t* col) {
    if (!c || !rp || !col) return fail(GOSSIP_EINVAL, "null argument");
    if (!c->graph_ready) return fail(GOSSIP_ESTATE, "no overlay");
    if (set_dev(c)) return GOSSIP_EHIP;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(rp, c->rp, (c->n_local + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (c->n_edges) HIPCHK(hipMemcpy(col, c->col, c->n_edges * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return GOSSIP_OK;
}

gossip_status gossip_read_extra(gossip_ctx* c, uint32_t* counts, uint32_t* cols) {
    if (!c || !counts || !cols) return fail(GOSSIP_EINVAL, "null argument");
    if (set_dev(c)) return GOSSIP_EHIP;
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint32_t K = c->cfg.extra_cap;
    if (!K) {
        std::memset(counts, 0, c->n_local * 4);
        return GOSSIP_OK;
    }
    HIPCHK(hipMemcpy(counts, c->ex_cnt, c->n_local * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cols, c->ex_col, c->n_local * K * 4, hipMemcpyDeviceToHost));
    for (uint64_t u = 0; u < c->n_local; ++u)  // entries past the count are stale: report zeros
        for (uint32_t k = counts[u]; k < K; ++k) cols[u * K + k] = 0;
    return GOSSIP_OK;
}

gossip_status gossip_inject(gossip_ctx* c, const uint32_t* origin, const uint32_t* inject_round, uint32_t n_msgs) {
    if (!c || !origin || !inject_round) return fail(GOSSIP_EINVAL, "null argument");
    if (n_msgs != c->M) return fail(GOSSIP_EINVAL, "n_msgs must equal cfg.n_msgs");
    std::vector<uint32_t> idx(n_msgs);
    for (uint32_t m = 0; m < n_msgs; ++m) {
        if (origin[m] >= c->n) return fail(GOSSIP_EINVAL, "origin out of range");
        idx[m] = m;
    }
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return inject_round[a] < inject_round[b]; });
    std::vector<uint32_t> o(n_msgs), mid(n_msgs);
    c->inj_round_sorted.resize(n_msgs);
    c->last_inject_round = 0;
    for (uint32_t i = 0; i < n_msgs; ++i) {
        o[i] = origin[idx[i]];
        mid[i] = idx[i];
        c->inj_round_sorted[i] = inject_round[idx[i]];
        c->last_inject_round = std::max(c->last_inject_round, inject_round[idx[i]]);
    }
    c->inj_prefix.assign((uint64_t)n_msgs * kMaxWords, 0);
    for (uint32_t i = 0; i < n_msgs; ++i) {
        for (int w = 0; w < kMaxWords; ++w) c->inj_prefix[(uint64_t)i * kMaxWords + w] = i ? c->inj_prefix[(uint64_t)(i - 1) * kMaxWords + w] : 0;
        c->inj_prefix[(uint64_t)i * kMaxWords + (mid[i] >> 6)] |= 1ull << (mid[i] & 63);
    }
    c->origin.assign(origin, origin + n_msgs);
    c->inject_round.assign(inject_round, inject_round + n_msgs);
    if (set_dev(c)) return GOSSIP_EHIP;
    hipFree(c->d_inj_origin);
    hipFree(c->d_inj_msg);
    c->d_inj_origin = c->d_inj_msg = nullptr;
    HIPCHK(hipMalloc((void**)&c->d_inj_origin, n_msgs * sizeof(uint32_t)));
    HIPCHK(hipMalloc((void**)&c->d_inj_msg, n_msgs * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(c->d_inj_origin, o.data(), n_msgs * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_inj_msg, mid.data(), n_msgs * sizeof(uint32_t), hipMemcpyHostToDevice));
    hipFree(c->d_inj_round);
    c->d_inj_round = nullptr;
    HIPCHK(hipMalloc((void**)&c->d_inj_round, n_msgs * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(c->d_inj_round, c->inj_round_sorted.data(), n_msgs * sizeof(uint32_t), hipMemcpyHostToDevice));
    c->has_schedule = true;
    rec_drop(c);
    return GOSSIP_OK;
}

gossip_status gossip_schedule_kills(gossip_ctx* c, const uint32_t* peer, const uint32_t* round, uint32_t n) {
    if (!c || (n && (!peer || !round))) return fail(GOSSIP_EINVAL, "null argument");
    std::vector<std::pair<uint32_t, uint32_t>> k(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (peer[i] >= c->n) return fail(GOSSIP_EINVAL, "kill peer out of range");
        k[i] = {round[i], peer[i]};
    }
    std::sort(k.begin(), k.end());
    rec_drop(c);
    c->kill_round_sorted.resize(n);
    std::vector<uint32_t> p(n + 1);
    for (uint32_t i = 0; i < n; ++i) {
        c->kill_round_sorted[i] = k[i].first;
        p[i] = k[i].second;
    }
    if (set_dev(c)) return GOSSIP_EHIP;
    hipFree(c->d_kill_peer);
    c->d_kill_peer = nullptr;
    HIPCHK(hipMalloc((void**)&c->d_kill_peer, (n + 1) * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(c->d_kill_peer, p.data(), (n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice));
    hipFree(c->d_kill_round);
    c->d_kill_round = nullptr;
    std::vector<uint32_t> kr(c->kill_round_sorted);
    kr.push_back(0xFFFFFFFFu);
    HIPCHK(hipMalloc((void**)&c->d_kill_round, kr.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(c->d_kill_round, kr.data(), kr.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    return GOSSIP_OK;
}

gossip_status gossip_device_count(int32_t* count) {
    if (!count) return fail(GOSSIP_EINVAL, "null argument");
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) n = 0;
    else if (e != hipSuccess) return fail(GOSSIP_EHIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    *count = n;
    return GOSSIP_OK;
}

gossip_status gossip_pick_origins(uint64_t n, uint32_t seed, uint32_t count, uint32_t* out) {
    if (!out || n == 0) return fail(GOSSIP_EINVAL, "bad argument");
    for (uint32_t k = 0; k < count; ++k) {
        for (uint32_t attempt = 0;; ++attempt) {
            const uint32_t x = philox4x32_10(P_ORIGIN, k, attempt, 0, seed, 0xFFFFFFFFu).x;
            const uint32_t o = (uint32_t)(((uint64_t)x * n) >> 32);
            bool dup = false;
            for (uint32_t i = 0; i < k; ++i) dup |= out[i] == o;
            if (!dup || (uint64_t)k >= n) {
                out[k] = o;
                break;
            }
        }
    }
    return GOSSIP_OK;
}

gossip_status gossip_reset(gossip_ctx* c) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (set_dev(c)) return GOSSIP_EHIP;
    hipStream_t s = c->stream;
    const uint64_t words = c->n_local * c->Wp;
    const uint64_t bitwords = (c->n + 31) / 32;
    c->fold_pending = false;  // seen is cleared
    c->tact_ok = true;        // no new words anywhere
    c->tact_marked = false;
    c->last_st_round = ~0u;
    const bool tiny = tiny_ok(c);
    if (tiny) {  // small overlays: every clear below in one launch
        HIPCHK(launch_tiny_reset(tiny_args(c), words, (uint32_t)c->n_started, c->any_masked, tact_bytes(c) / 8,
                                 c->tact[0], c->tact[1], c->st, s));
        c->bufs_zero = true;
    } else {
        HIPCHK(launch_zero_words(c->seen, words, s, c->zero_fill));
        if (!c->bufs_zero && !c->in_round && c->lin_idx[0] >= 0 && c->lin_idx[1] >= 0) {
            // the last two rounds pulled needy lists: each wrote only its list's rows and the heavy rows into a
            // buffer cleared before it (the list rounds' contract: one word per peer, nothing injected or
            // killed later), so those rows are all that is left -- nw holds the last round's, nx the one's
            // before (config 4: two 2 GB fills, 0.94 ms of a step, became two list clears)
            RoundArgs a = make_args(c);
            HIPCHK(launch_list_zero(a, c->lst[c->lin_idx[1]], c->lin_n[1], s));
            a.nx = c->nw;
            HIPCHK(launch_list_zero(a, c->lst[c->lin_idx[0]], c->lin_n[0], s));
            c->bufs_zero = true;
        }
        if (!c->bufs_zero) {  // (a run that ended normally left both zero)
            HIPCHK(launch_zero_words(c->nw, words, s, c->zero_fill));
            HIPCHK(launch_zero_words(c->nx, words, s, c->zero_fill));
            c->bufs_zero = true;
        }
        for (int k = 0; k < 2; ++k) HIPCHK(hipMemsetAsync(c->tact[k], 0, tact_bytes(c), s));
        HIPCHK(hipMemsetAsync(c->alive, 0xFF, bitwords * 4, s));
        HIPCHK(hipMemsetAsync(c->registered, 0xFF, bitwords * 4, s));
        if (c->n % 32) {
            static thread_local uint32_t tail;
            tail = (1u << (c->n % 32)) - 1u;
            HIPCHK(hipMemcpyAsync(c->alive + bitwords - 1, &tail, 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(c->registered + bitwords - 1, &tail, 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        if (c->n_started < c->n) {  // failed registration (list_cap): registered, never alive
            std::vector<uint32_t> bits(bitwords, 0u);
            for (uint64_t v = 0; v < c->n_started; ++v) bits[v >> 5] |= 1u << (v & 31);
            HIPCHK(hipMemcpyAsync(c->alive, bits.data(), bitwords * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        HIPCHK(hipMemsetAsync(c->st, 0, kStatLines * sizeof(DevStats), s));
        HIPCHK(hipMemsetAsync(c->n_reports, 0, sizeof(unsigned long long), s));
        HIPCHK(hipMemsetAsync(c->inj_live, 0, kMaxWords * sizeof(uint64_t), s));
        // per-edge miss counters: only the per-edge liveness scan uses them (the closed form, below, never
        // does; config 5: a 0.5 GB clear per step saved).  An overlay small enough for the one-launch run
        // clears them anyway: that run scans every edge's counter, and it may run after this reset even
        // though the reset itself did not take the tiny path ("tiny" turned on in between)
        const bool closed = c->n_local == c->n && c->symmetric && !c->cfg.rejoin_threshold &&
                            c->cfg.max_rounds < 0xFFFF && !c->full_liveness;
        const bool small = c->n <= kTinyPeers && c->n_edges <= kTinyEdges;
        if (c->miss && (!closed || small)) HIPCHK(hipMemsetAsync(c->miss, 0, c->n_edges + 1, s));
        if (c->any_masked && c->col && c->n_edges) {
            hipLaunchKernelGGL(k_unmask, dim3(2048), dim3(256), 0, s, c->col, c->n_edges);
            HIPCHK(hipGetLastError());
        }
    }
    if (c->cov_hist) HIPCHK(hipMemsetAsync(c->cov_hist, 0, (uint64_t)c->cfg.max_rounds * 64 * c->Wp * 8, s));
    // slots still hold words of the last run: the first binned round of the next rewrites every slot
    c->bins_first = true;
    if (c->cfg.extra_cap) {
        HIPCHK(hipMemsetAsync(c->ex_cnt, 0, c->n_local * 4 + 4, s));
        HIPCHK(hipMemsetAsync(c->ex_miss, 0, c->n_local * c->cfg.extra_cap + 1, s));
    }
    // closed-form liveness: deaths are permanent and every in-edge of a peer is in its own row
    c->closed_live = c->n_local == c->n && c->symmetric && !c->cfg.rejoin_threshold && c->cfg.max_rounds < 0xFFFF &&
                     !c->full_liveness;
    if (c->death_r) {
        HIPCHK(hipMemsetAsync(c->death_r, 0xFF, c->n_local * 2 + 2, s));
        HIPCHK(hipMemsetAsync(c->dgone, 0, c->n_local * 4 + 4, s));
        HIPCHK(hipMemsetAsync(c->dmask, 0, c->n_local * 4 + 4, s));
    }
    if (c->pb_ready) HIPCHK(hipMemsetAsync(c->pb.err, 0, sizeof(uint32_t), s));  // error flags of the last run
    if (c->px_state == 1) HIPCHK(hipMemsetAsync(c->px.err, 0, sizeof(uint32_t), s));
    c->n_rep_seen = 0;
    c->pre_booked = c->cur_list = c->cur_pre = false;
    c->lst_in = c->cur_lst_out = -1;
    c->lin_idx[0] = c->lin_idx[1] = -1;
    if (c->st_pre) HIPCHK(hipMemsetAsync(c->st_pre, 0, kStatLines * sizeof(DevStats), s));
    c->any_masked = false;
    c->nx_dirty = false;
    c->last_pull = false;
    c->last_bin = false;
    c->cur_defer = false;
    c->flight_round = ~0u;
    c->dgone_next = 0;
    c->last_fresh = 0;
    c->frontier_est = c->prev_frontier_est = 0;
    c->round = 0;
    c->finished = false;
    c->any_dead = c->n_started < c->n;
    c->cum_digest = c->cum_covered = 0;
    c->cum_dead_cov = c->cum_died = c->cum_injected = 0;
    if (c->dist) gossip::dist_reset(c->dist);
    // no host wait: the clears above are ordered before the run's kernels on the stream, and every host read of
    // device state synchronises the stream first (a wait here left the GPU idle while the host issued the run's
    // first round)
    return GOSSIP_OK;
}

gossip_status gossip_step(gossip_ctx* c, gossip_round_stats* out) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (set_dev(c)) return GOSSIP_EHIP;
    if (c->dist) return gossip::dist_step_ctx(c, out);  // the library's own collectives (gossip_comm_init)
    if (c->world > 1) return fail(GOSSIP_ESTATE, "partitioned ctx: use gossip_comm_init or gossip_round_*");
    c->recording = false;  // (a run driven round by round records nothing)
    return step_round(c, out);
}

}  // extern "C"

namespace {
gossip_status step_round(gossip_ctx* c, gossip_round_stats* out) {
    TraceRange tr("gossip round %u", c->round);
    gossip_status s = round_begin(c, false, GOSSIP_MODE_AUTO, nullptr);
    if (!s) s = round_compute(c);
    if (s) return s;
    gossip_round_stats st;
    if ((s = read_slot(c, &st, true))) return s;
    if (out) *out = st;
    if ((s = advance(c, st.new_receipts))) return s;
    return c->finished ? 1 : 0;
}
}  // namespace

extern "C" {

gossip_status gossip_run(gossip_ctx* c, gossip_round_stats* per_round, uint32_t cap, uint32_t* rounds) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (c->round == 0 && !c->finished && tiny_ok(c)) {
        if (set_dev(c)) return GOSSIP_EHIP;
        return tiny_run(c, per_round, cap, rounds);
    }
    if (c->dist || c->world > 1) {
        uint32_t k = 0;
        while (!c->finished) {
            gossip_round_stats st;
            gossip_status s = gossip_step(c, &st);
            if (s < 0) return s;
            if (per_round && k < cap) per_round[k] = st;
            ++k;
        }
        if (rounds) *rounds = k;
        return GOSSIP_OK;
    }
    if (set_dev(c)) return GOSSIP_EHIP;
    const bool fresh = c->round == 0 && !c->finished && replay_eligible(c);
    if (fresh && c->rec_valid) return replay_run(c, per_round, cap, rounds);
    if (fresh) {
        rec_drop(c);
        c->recording = true;
    }
    uint32_t k = 0;
    while (!c->finished) {
        gossip_round_stats st;
        gossip_status s = step_round(c, &st);
        if (s < 0) {
            rec_drop(c);
            return s;
        }
        if (per_round && k < cap) per_round[k] = st;
        ++k;
    }
    c->rec_valid = c->recording;
    c->recording = false;
    if (rounds) *rounds = k;
    return GOSSIP_OK;
}

gossip_status gossip_set_exchange(gossip_ctx* c, void* send, void* recv, uint32_t world, const uint64_t* pb) {
    if (!c || !send || !recv || !pb || world < 1) return fail(GOSSIP_EINVAL, "null argument");
    bool found = false;
    for (uint32_t p = 0; p < world; ++p) {
        if (pb[p + 1] < pb[p]) return fail(GOSSIP_EINVAL, "part_begins not monotone");
        found |= (pb[p] == c->begin && pb[p + 1] == c->end);
    }
    if (pb[0] != 0 || pb[world] != c->n || !found) return fail(GOSSIP_EINVAL, "partition table does not match ctx");
    if (world > gossip::kMaxWorld) return fail(GOSSIP_EINVAL, "at most 64 blocks");
    c->send = (uint64_t*)send;
    c->recv = (const uint64_t*)recv;
    c->world = world;
    c->part_begins.assign(pb, pb + world + 1);
    return GOSSIP_OK;
}

gossip_status gossip_set_gather(gossip_ctx* c, void* gather) {
    if (!c || !gather) return fail(GOSSIP_EINVAL, "null argument");
    if (c->part_begins.size() < 2) return fail(GOSSIP_ESTATE, "call gossip_set_exchange first");
    if (set_dev(c)) return GOSSIP_EHIP;
    hipFree(c->front);
    c->front = nullptr;
    HIPCHK(hipMalloc((void**)&c->front, ((c->n + 63) / 64 + 1) * 8));  // bitmap over all peers
    c->gather = (uint64_t*)gather;
    return GOSSIP_OK;
}

gossip_status gossip_set_sparse(gossip_ctx* c, void* seg) {
    if (!c || !seg) return fail(GOSSIP_EINVAL, "null argument");
    if (c->part_begins.size() < 2) return fail(GOSSIP_ESTATE, "call gossip_set_exchange first");
    if (set_dev(c)) return GOSSIP_EHIP;
    if (!c->d_counts) {
        HIPCHK(hipMalloc((void**)&c->d_counts, (c->world + 1) * sizeof(unsigned long long)));
        HIPCHK(hipHostMalloc((void**)&c->h_counts, (c->world + 1) * sizeof(uint64_t)));
        // the blocks (any contiguous partition): bounds and tile offsets on the device, the largest block
        std::vector<uint64_t> toff(c->world + 1, 0);
        c->blk_stride = 0;
        for (uint32_t q = 0; q < c->world; ++q) {
            toff[q + 1] = toff[q] + (c->part_begins[q + 1] - c->part_begins[q] + 63) / 64;
            c->blk_stride = std::max(c->blk_stride, c->part_begins[q + 1] - c->part_begins[q]);
        }
        c->n_tiles_all = toff[c->world];
        hipFree(c->d_part);
        hipFree(c->d_toff);
        c->d_part = c->d_toff = nullptr;
        HIPCHK(hipMalloc((void**)&c->d_part, (c->world + 1) * sizeof(uint64_t)));
        HIPCHK(hipMalloc((void**)&c->d_toff, (c->world + 1) * sizeof(uint64_t)));
        HIPCHK(hipMemcpy(c->d_part, c->part_begins.data(), (c->world + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(c->d_toff, toff.data(), (c->world + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
        const uint64_t tiles = c->n_tiles_all;
        HIPCHK(hipMalloc((void**)&c->sx_bits, (tiles + 1) * sizeof(uint64_t)));
        HIPCHK(hipMemset(c->sx_bits, 0, (tiles + 1) * sizeof(uint64_t)));
        HIPCHK(hipMalloc((void**)&c->sx_pos, (tiles + 1) * sizeof(uint64_t)));
        HIPCHK(compact_send_scratch(tiles, &c->sx_bytes));
        HIPCHK(hipMalloc(&c->sx_tmp, c->sx_bytes + 16));
        HIPCHK(hipMalloc((void**)&c->smark, smark_bytes(c->n)));
        HIPCHK(hipMemset(c->smark, 0, smark_bytes(c->n)));
    }
    c->seg = (uint64_t*)seg;
    return GOSSIP_OK;
}

gossip_status gossip_sparse_counts(gossip_ctx* c, uint64_t* counts) {
    if (!c || !counts) return fail(GOSSIP_EINVAL, "null argument");
    if (!c->cur_sparse) return fail(GOSSIP_ESTATE, "not a sparse push round");
    if (set_dev(c)) return GOSSIP_EHIP;
    HIPCHK(hipStreamSynchronize(c->stream));
    std::memcpy(counts, c->h_counts, c->world * sizeof(uint64_t));
    return GOSSIP_OK;
}

gossip_status gossip_round_finish_sparse(gossip_ctx* c, const void* records, uint64_t n_records,
                                         gossip_round_stats* out) {
    if (!c || (n_records && !records)) return fail(GOSSIP_EINVAL, "null argument");
    if (!c->cur_sparse) return fail(GOSSIP_ESTATE, "not a sparse push round");
    if (set_dev(c)) return GOSSIP_EHIP;
    RoundArgs a = make_args(c);
    HIPCHK(timed(c, "apply_remote", [&] {
        return launch_apply_records(a, pack_w(c), (const uint64_t*)records, n_records, c->stream);
    }));
    return read_slot(c, out, false);
}

gossip_status gossip_round_begin(gossip_ctx* c, int requested_mode, int* mode) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (c->world > 1 && !c->send) return fail(GOSSIP_ESTATE, "call gossip_set_exchange first");
    if (c->world > 1 && requested_mode == GOSSIP_MODE_AUTO)
        return fail(GOSSIP_EINVAL, "partitioned rounds need an explicit mode (chosen from global stats)");
    if (set_dev(c)) return GOSSIP_EHIP;
    return round_begin(c, c->world > 1, requested_mode, mode);
}

gossip_status gossip_round_compute(gossip_ctx* c) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (set_dev(c)) return GOSSIP_EHIP;
    return round_compute(c);
}

gossip_status gossip_round_push(gossip_ctx* c) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (!c->send) return fail(GOSSIP_ESTATE, "call gossip_set_exchange first");
    if (set_dev(c)) return GOSSIP_EHIP;
    gossip_status s = round_begin(c, true, GOSSIP_MODE_PUSH, nullptr);
    return s ? s : round_compute(c);
}

gossip_status gossip_round_finish(gossip_ctx* c, gossip_round_stats* out) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (!c->recv) return fail(GOSSIP_ESTATE, "call gossip_set_exchange first");
    if (c->in_round) return fail(GOSSIP_ESTATE, "gossip_round_compute first");
    if (c->cur_sparse) return fail(GOSSIP_ESTATE, "sparse push round: use gossip_round_finish_sparse");
    if (set_dev(c)) return GOSSIP_EHIP;
    RoundArgs a = make_args(c);
    if (!c->last_pull)  // push round: OR in what the other blocks sent; pull rounds pulled it already
        HIPCHK(timed(c, "apply_remote",
                     [&] { return launch_apply_remote(a, pack_w(c), c->recv, c->world, c->n_local, c->stream); }));
    return read_slot(c, out, false);
}

gossip_status gossip_round_commit(gossip_ctx* c, uint64_t global_new_receipts, int* finished) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (gossip_status s = advance(c, global_new_receipts)) return s;
    if (finished) *finished = c->finished ? 1 : 0;
    return GOSSIP_OK;
}

gossip_status gossip_read_seen(gossip_ctx* c, uint64_t* out) {
    if (!c || !out) return fail(GOSSIP_EINVAL, "null argument");
    if (set_dev(c)) return GOSSIP_EHIP;
    if (gossip_status fs = settle_fold(c)) return fs;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->W == c->Wp) {
        HIPCHK(hipMemcpy(out, c->seen, c->n_local * c->W * 8, hipMemcpyDeviceToHost));
        return GOSSIP_OK;
    }
    std::vector<uint64_t> tmp(c->n_local * c->Wp);
    HIPCHK(hipMemcpy(tmp.data(), c->seen, tmp.size() * 8, hipMemcpyDeviceToHost));
    for (uint64_t v = 0; v < c->n_local; ++v)
        for (uint32_t w = 0; w < c->W; ++w) out[v * c->W + w] = tmp[v * c->Wp + w];
    return GOSSIP_OK;
}

gossip_status gossip_read_coverage(gossip_ctx* c, uint64_t* counts) {
    if (!c || !counts) return fail(GOSSIP_EINVAL, "null argument");
    if (set_dev(c)) return GOSSIP_EHIP;
    if (gossip_status fs = settle_fold(c)) return fs;
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc((void**)&d, 64 * c->Wp * 8));
    HIPCHK(hipMemsetAsync(d, 0, 64 * c->Wp * 8, c->stream));
    HIPCHK(launch_coverage(c->seen, c->n_local, pack_w(c), d, c->stream));
    std::vector<uint64_t> h(64 * c->Wp);
    HIPCHK(hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    hipFree(d);
    std::memcpy(counts, h.data(), c->M * 8);
    return GOSSIP_OK;
}

gossip_status gossip_read_coverage_history(gossip_ctx* c, uint64_t* buf, uint32_t max_rounds, uint32_t* rounds) {
    if (!c || !buf) return fail(GOSSIP_EINVAL, "null argument");
    if (!c->cov_hist) return fail(GOSSIP_ESTATE, "ctx created without GOSSIP_FLAG_COVERAGE_HISTORY");
    if (set_dev(c)) return GOSSIP_EHIP;
    const uint32_t R = std::min(c->round, max_rounds);
    std::vector<uint64_t> h((uint64_t)R * 64 * c->Wp);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (R) HIPCHK(hipMemcpy(h.data(), c->cov_hist, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<uint64_t> acc(c->M, 0);
    for (uint32_t r = 0; r < R; ++r)
        for (uint32_t m = 0; m < c->M; ++m) {
            acc[m] += h[(uint64_t)r * 64 * c->Wp + m];
            buf[(uint64_t)r * c->M + m] = acc[m];
        }
    if (rounds) *rounds = R;
    return GOSSIP_OK;
}

gossip_status gossip_read_reports(gossip_ctx* c, gossip_dead_report* buf, uint64_t cap, uint64_t* count) {
    if (!c || !count) return fail(GOSSIP_EINVAL, "null argument");
    if (set_dev(c)) return GOSSIP_EHIP;
    HIPCHK(hipStreamSynchronize(c->stream));
    unsigned long long n = 0;
    HIPCHK(hipMemcpy(&n, c->n_reports, sizeof(n), hipMemcpyDeviceToHost));
    *count = n;
    if (n > c->report_cap) return fail(GOSSIP_EOVERFLOW, "report buffer overflowed");
    if (!buf || !n) return GOSSIP_OK;
    std::vector<DeadReport> h(n);
    HIPCHK(hipMemcpy(h.data(), c->reports, n * sizeof(DeadReport), hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end(), [](const DeadReport& x, const DeadReport& y) {
        if (x.round != y.round) return x.round < y.round;
        if (x.reporter != y.reporter) return x.reporter < y.reporter;
        return x.dead < y.dead;
    });
    const uint64_t k = std::min<uint64_t>(n, cap);
    for (uint64_t i = 0; i < k; ++i) buf[i] = gossip_dead_report{h[i].round, h[i].reporter, h[i].dead};
    return GOSSIP_OK;
}

static gossip_status read_bits(gossip_ctx* c, const uint32_t* d, uint8_t* out) {
    if (!c || !out) return fail(GOSSIP_EINVAL, "null argument");
    if (set_dev(c)) return GOSSIP_EHIP;
    HIPCHK(hipStreamSynchronize(c->stream));
    std::vector<uint32_t> h((c->n + 31) / 32);
    HIPCHK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    for (uint64_t v = 0; v < c->n; ++v) out[v] = (h[v >> 5] >> (v & 31)) & 1u;
    return GOSSIP_OK;
}

gossip_status gossip_read_alive(gossip_ctx* c, uint8_t* out) { return read_bits(c, c ? c->alive : nullptr, out); }
gossip_status gossip_read_registered(gossip_ctx* c, uint8_t* out) {
    return read_bits(c, c ? c->registered : nullptr, out);
}

gossip_status gossip_enable_timing(gossip_ctx* c, int enable) {
    if (!c) return fail(GOSSIP_EINVAL, "null ctx");
    if (set_dev(c)) return GOSSIP_EHIP;
    drain_timers(c);
    c->timers.clear();
    c->kbytes.clear();
    c->timing = enable != 0;
    return GOSSIP_OK;
}

gossip_status gossip_kernel_time(gossip_ctx* c, const char* kernel, double* ms, uint64_t* launches) {
    if (!c || !kernel) return fail(GOSSIP_EINVAL, "null argument");
    if (set_dev(c)) return GOSSIP_EHIP;
    drain_timers(c);
    auto it = c->timers.find(kernel);
    if (ms) *ms = it == c->timers.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == c->timers.end() ? 0 : it->second.launches;
    return GOSSIP_OK;
}

gossip_status gossip_kernel_bytes(gossip_ctx* c, const char* kernel, double* bytes) {
    if (!c || !kernel || !bytes) return fail(GOSSIP_EINVAL, "null argument");
    if (c->d_probe && !strncmp(kernel, "#probe_", 7)) {  // apply_probe's clocks (a device read: syncs)
        static const char* const names[] = {"src",    "init",   "slots",  "finish", "bins",   "slots_n", "block", "blocks",
                                            "xcd0",   "xcd1",   "xcd2",   "xcd3",   "xcd4",   "xcd5",    "xcd6",  "xcd7"};
        unsigned long long h[kProbeN];
        if (hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(h, c->d_probe, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
            return fail(GOSSIP_EHIP, "apply_probe read");
        *bytes = 0.0;
        for (int i = 0; i < kProbeN; ++i)
            if (!strcmp(kernel + 7, names[i])) *bytes = (double)h[i];
        return GOSSIP_OK;
    }
    auto it = c->kbytes.find(kernel);
    *bytes = it == c->kbytes.end() ? 0.0 : it->second;
    return GOSSIP_OK;
}

}  // extern "C"
