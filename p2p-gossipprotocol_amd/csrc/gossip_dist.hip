// gossip_dist.hip -- multi-GPU rounds driven by libgossip_hip itself (RCCL over xGMI).
//
// The reference sends every gossip message to another PeerNode process over
// TCP (broadcastMessage peer.cpp:310-316 -> handleClient peer.cpp:255-295).
// Here peers are 1D vertex-partitioned into contiguous blocks (SURVEY.md
// 8(e); gossip_partition: ceil(n/P) peers each, gossip_partition_edges: about
// equal edge counts, round 5) and one round's cross-block traffic is ONE
// exchange, issued by this driver on the block's HIP stream:
//   dense rounds (PULL / BIN): an all-gather (send / recv pairs of the blocks'
//     slices) of every block's new words into a buffer indexed by global peer; each block then pulls or
//     streams its in-edges from it (no second exchange, no atomics).  Below
//     gather_permille of frontier the blocks exchange a bitmap of their
//     64-peer tiles' non-zero words and those words packed instead (an
//     all-gather of the bitmaps, then of the packed words as send / recv
//     pairs), expanded into the same buffer;
//   push rounds: the block's pushes to remote peers are OR-ed into a dense
//     staging buffer indexed by global peer, and an all-to-all of ncclSend /
//     ncclRecv pairs (all ranks' sends and receives in one group, every link
//     of the xGMI mesh at once) hands rank q its slice; narrow rounds
//     (PUSH_SPARSE) first compact the staging buffer into {peer, words}
//     records and exchange only those (counts first, then the records);
//   then one ncclAllReduce (uint64 sum, so the digest wraps mod 2^64 exactly
//   as on one GPU) of the round's stats drives the common termination.
// The mode is chosen from the previous round's GLOBAL stats, so every rank
// picks the same one.  Results equal the single-partition run bit for bit
// (set semantics; tests/test_gpu_group.py).
//
// Two deployments share this code:
//   gossip_comm_init: one process per GPU (the bench's torchrun launch), one
//     local rank per driver, communicator from ncclCommInitRank;
//   gossip_group_*:   one process driving several GPUs,
//     communicators from ncclCommInitAll, every collective of the local ranks
//     inside one ncclGroupStart/End; when all parts sit on ONE device the
//     exchange is done by device copies on one shared stream (a single-GPU
//     rehearsal of the partitioned path: the remote staging, record
//     compaction and remote-apply kernels and this driver's schedule).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gossip/gossip.h"
#include "gossip_internal.hpp"

namespace gossip {

namespace {

constexpr int kStatSlots = 15;  // all-reduced stat fields (see pack_stats)

struct DistRank {
    gossip_ctx* ctx = nullptr;
    uint32_t rank = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    uint64_t begin = 0, n_local = 0;
    uint64_t *send = nullptr, *recv = nullptr, *gather = nullptr, *seg = nullptr, *rec_in = nullptr;
    uint64_t rec_cap = 0;  // records rec_in holds (grown when a round's records do not fit: a record push
                           // sends one per remote delivery, a small block of hubs receives many)
    uint64_t* d_io = nullptr;  // device scratch: stats all-reduce, record counts
    uint64_t* h_io = nullptr;  // pinned mirror
    // compact dense exchange: every block's tile bitmap (block q's tiles from toff[q], block order), the
    // exclusive prefix of their popcounts (a tile's first packed word), the packed words of all blocks
    uint64_t *bits = nullptr, *pos = nullptr, *pk = nullptr;
    uint64_t *d_part = nullptr, *d_toff = nullptr;  // the partition's block bounds and tile offsets (device)
    void* scan_tmp = nullptr;
    size_t scan_bytes = 0;
    std::vector<uint64_t> counts_out, counts_in;
    gossip_round_stats local{};
    // staged dense exchange: its stream (an emulated group shares one), the event after the own block's
    // words are published, and one event per stage
    hipStream_t xs = nullptr;
    hipEvent_t ev_pub = nullptr;
    hipEvent_t ev_stage[kMaxStages] = {};
};

}  // namespace

struct DistDriver {
    std::vector<DistRank> ranks;  // the ranks this process drives
    uint32_t world = 1;
    bool emulate = false;         // every rank local on one device: device copies, one stream
    std::vector<uint64_t> part;  // begins[world + 1]: any contiguous partition (every block non-empty)
    std::vector<uint64_t> toff;  // toff[q]: the 64-peer tiles of the blocks before q (compact exchange)
    uint64_t n = 0;
    uint64_t maxb = 0;           // the largest block (a staging push's records per destination stay below it)
    uint32_t X = 1, R = 2;
    uint32_t pull_pm = kPullPermille, sparse_pm = 250, bin_pm = 4000, bin_front_pm = 100;
    // schedule state, from global stats (identical on every rank)
    uint64_t prev_new = 0, injected = 0, cum_digest = 0, cum_covered = 0;
    uint64_t front = 0;  // this round's frontier (the peers the last round activated, all ranks)
    // stages of a binned round's staged all-gather: the count every rank asked for at the last stats all-reduce
    // when they all asked for the same, else 1 (one process per GPU: a rank whose bin layout failed, or tuned
    // differently, would post other send/recv sizes than its peers -- a hang or a corrupt gather buffer)
    uint32_t stages = 1;
    bool finished = false;
    std::vector<int32_t> modes;
};

namespace {

#define DHIP(call)                                                                                  \
    do {                                                                                            \
        hipError_t e_ = (call);                                                                     \
        if (e_ != hipSuccess) return set_error(GOSSIP_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define DNCCL(call)                                                                                 \
    do {                                                                                            \
        ncclResult_t r_ = (call);                                                                   \
        if (r_ != ncclSuccess) return set_error(GOSSIP_ECOMM, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

std::vector<uint64_t> blocks(uint64_t n, uint32_t world) {
    const uint64_t chunk = (n + world - 1) / world;
    std::vector<uint64_t> b(world + 1);
    for (uint32_t p = 0; p <= world; ++p) b[p] = std::min<uint64_t>((uint64_t)p * chunk, n);
    return b;
}

// ---- compact dense exchange ----
struct PopOp {
    __host__ __device__ uint64_t operator()(uint64_t x) const { return (uint64_t)__builtin_popcountll(x); }
};
using TilePop = hipcub::TransformInputIterator<uint64_t, PopOp, const uint64_t*>;

// bit i of bits[t] <=> peer 64 t + i of the block has a non-zero new word (one wave per tile)
__global__ __launch_bounds__(256) void k_tile_bits(const uint64_t* words, uint64_t n, uint32_t X, uint64_t* bits) {
    const int lane = threadIdx.x & 63;
    const uint64_t tiles = (n + 63) / 64;
    for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < tiles;
         t += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const uint64_t v = t * 64 + lane;
        uint64_t any = 0;
        if (v < n)
            for (uint32_t x = 0; x < X; ++x) any |= words[v * X + x];
        const unsigned long long b = __ballot(any != 0);
        if (lane == 0) bits[t] = b;
    }
}

// block q of tile T (toff: the tile offsets of the world + 1 block bounds; world is small)
__device__ __forceinline__ uint32_t tile_block(const uint64_t* toff, uint32_t world, uint64_t T) {
    uint32_t q = 0;
    while (q + 1 < world && toff[q + 1] <= T) ++q;
    return q;
}

// the block's non-zero words, packed in peer order at out[pos[t] + rank of the peer in its tile]
__global__ __launch_bounds__(256) void k_tile_pack(const uint64_t* words, uint64_t n, uint32_t X, const uint64_t* bits,
                                                   const uint64_t* pos, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t tiles = (n + 63) / 64;
    for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < tiles;
         t += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const uint64_t b = bits[t];
        if (!((b >> lane) & 1)) continue;
        const uint64_t at = pos[t] + (uint64_t)__builtin_popcountll(b & ((1ull << lane) - 1));
        const uint64_t v = t * 64 + lane;
        for (uint32_t x = 0; x < X; ++x) out[at * X + x] = words[v * X + x];
    }
}

// every other block's words back into the gather buffer (zeros where the bitmap has none)
__global__ __launch_bounds__(256) void k_tile_expand(uint64_t* gather, const uint64_t* bits, const uint64_t* pos,
                                                     const uint64_t* pk, uint32_t X, uint32_t world, uint32_t own,
                                                     const uint64_t* part_g, const uint64_t* toff_g) {
    __shared__ uint64_t part[kMaxWorld + 1], toff[kMaxWorld + 1];  // (a dependent global load per lookup step)
    for (uint32_t i = threadIdx.x; i <= world; i += blockDim.x) {
        part[i] = part_g[i];
        toff[i] = toff_g[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t tiles = toff[world];
    for (uint64_t T = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; T < tiles;
         T += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const uint32_t q = tile_block(toff, world, T);
        const uint64_t t = T - toff[q];
        const uint64_t v = part[q] + t * 64 + lane;
        const uint64_t end = part[q + 1];
        if (q == own) continue;  // wave-uniform
        const uint64_t b = bits[T];
        const bool set = (b >> lane) & 1;
        const uint64_t at = pos[T] + (uint64_t)__builtin_popcountll(b & ((1ull << lane) - 1));
        if (v < end)
            for (uint32_t x = 0; x < X; ++x) gather[v * X + x] = set ? pk[at * X + x] : 0ull;
    }
}

__global__ void k_pick_offsets(const uint64_t* pos, uint32_t world, const uint64_t* toff, uint64_t* out) {
    const uint32_t q = threadIdx.x;
    if (q <= world) out[q] = pos[toff[q]];
}

// Buffers and communicator of one rank (its stream is released by dist_free).
void free_rank(DistRank& r) {
    hipSetDevice(r.device);
    if (r.stream) hipStreamSynchronize(r.stream);
    if (r.comm) ncclCommDestroy(r.comm);
    hipFree(r.send);
    hipFree(r.recv);
    hipFree(r.gather);
    hipFree(r.seg);
    hipFree(r.rec_in);
    hipFree(r.d_io);
    hipFree(r.bits);
    hipFree(r.pos);
    hipFree(r.pk);
    hipFree(r.scan_tmp);
    hipFree(r.d_part);
    hipFree(r.d_toff);
    r.d_part = r.d_toff = nullptr;
    if (r.ev_pub) hipEventDestroy(r.ev_pub);
    for (hipEvent_t& e : r.ev_stage)
        if (e) hipEventDestroy(e);
    r.ev_pub = nullptr;
    std::fill(std::begin(r.ev_stage), std::end(r.ev_stage), nullptr);
    if (r.h_io) hipHostFree(r.h_io);
    r.send = r.recv = r.gather = r.seg = r.rec_in = r.d_io = r.h_io = nullptr;
    r.bits = r.pos = r.pk = nullptr;
    r.scan_tmp = nullptr;
    r.comm = nullptr;
}

// Exchange buffers of one rank (device memory of its GPU) and their
// registration with its ctx; the ctx then issues its work on r.stream.
gossip_status setup_rank(DistDriver* d, DistRank& r) {
    DHIP(hipSetDevice(r.device));
    const uint64_t X = d->X, R = d->R, W = d->world;
    auto alloc = [&](uint64_t** p, uint64_t words) -> hipError_t {
        hipError_t e = hipMalloc((void**)p, std::max<uint64_t>(words, 1) * 8);
        return e == hipSuccess ? hipMemsetAsync(*p, 0, std::max<uint64_t>(words, 1) * 8, r.stream) : e;
    };
    DHIP(alloc(&r.send, d->n * X));
    DHIP(alloc(&r.recv, W * r.n_local * X));
    DHIP(alloc(&r.gather, d->n * X));  // indexed by global peer: block q's words at part[q]
    DHIP(alloc(&r.seg, W * d->maxb * R));
    DHIP(alloc(&r.rec_in, W * r.n_local * R));
    r.rec_cap = W * r.n_local;
    DHIP(alloc(&r.d_io, 2 * std::max<uint64_t>(W + 1, kStatSlots)));
    DHIP(hipHostMalloc((void**)&r.h_io, 2 * std::max<uint64_t>(W + 1, kStatSlots) * 8));
    DHIP(alloc(&r.d_part, W + 1));
    DHIP(alloc(&r.d_toff, W + 1));
    DHIP(hipMemcpyAsync(r.d_part, d->part.data(), (W + 1) * 8, hipMemcpyHostToDevice, r.stream));
    DHIP(hipMemcpyAsync(r.d_toff, d->toff.data(), (W + 1) * 8, hipMemcpyHostToDevice, r.stream));
    if (W > 1) {  // compact dense exchange
        const uint64_t tiles = d->toff[W];
        DHIP(alloc(&r.bits, tiles + 1));  // (+1: a zero past the last tile, so the scan yields the total)
        DHIP(alloc(&r.pos, tiles + 1));
        DHIP(alloc(&r.pk, d->n * X));
        DHIP(hipcub::DeviceScan::ExclusiveSum(nullptr, r.scan_bytes, TilePop(r.bits, PopOp()), r.pos, (int)(tiles + 1),
                                              r.stream));
        DHIP(hipMalloc(&r.scan_tmp, r.scan_bytes + 16));
    }
    r.counts_out.assign(W, 0);
    r.counts_in.assign(W, 0);
    DHIP(hipStreamSynchronize(r.stream));
    gossip_status s = gossip_set_stream(r.ctx, r.stream);
    if (!s) s = gossip_set_exchange(r.ctx, r.send, r.recv, d->world, d->part.data());
    if (!s) s = gossip_set_gather(r.ctx, r.gather);
    if (!s) s = gossip_set_sparse(r.ctx, r.seg);
    return s;
}

// Checks the ctx's block against the partition and fills the rank's shape.
gossip_status bind_rank(DistDriver* d, DistRank& r) {
    uint64_t b = 0, e = 0;
    ctx_range(r.ctx, &b, &e);
    if (b != d->part[r.rank] || e != d->part[r.rank + 1])
        return set_error(GOSSIP_EINVAL, "ctx part range is not rank " + std::to_string(r.rank) +
                                            "'s block of gossip_partition(n_peers, world)");
    r.begin = b;
    r.n_local = e - b;
    r.device = ctx_device(r.ctx);
    uint32_t words = 0, x = 0;
    gossip_status s = gossip_get_shape(r.ctx, &words, &x, nullptr, nullptr);
    if (s) return s;
    d->X = x;
    d->R = 1 + x;
    return GOSSIP_OK;
}

// part: the blocks' bounds (world + 1, from 0 to n, every block non-empty)
void init_schedule(DistDriver* d, const gossip_config& cfg, const std::vector<uint64_t>& part) {
    d->n = cfg.n_peers;
    d->part = part;
    d->toff.assign(d->world + 1, 0);
    d->maxb = 0;
    for (uint32_t q = 0; q < d->world; ++q) {
        d->toff[q + 1] = d->toff[q] + (part[q + 1] - part[q] + 63) / 64;
        d->maxb = std::max(d->maxb, part[q + 1] - part[q]);
    }
    if (cfg.pull_permille) d->pull_pm = cfg.pull_permille;
    if (cfg.bin_permille) d->bin_pm = cfg.bin_permille;
}

// The round's exchange mode from the previous round's GLOBAL stats (the
// single-partition engine's switch points).
int choose_mode(const DistDriver* d) {
    const uint64_t n = d->n;
    if (d->prev_new * 1000 >= (uint64_t)d->pull_pm * n) {
        const uint64_t have = d->cum_covered + d->prev_new, total = d->injected * n;
        const uint64_t missing = total > have ? total - have : 0;
        const bool wide = d->prev_new * 1000 >= (uint64_t)d->bin_front_pm * n;
        return wide && missing * 1000 >= (uint64_t)d->bin_pm * n ? GOSSIP_MODE_BIN : GOSSIP_MODE_PULL;
    }
    return d->prev_new * 1000 < (uint64_t)d->sparse_pm * n ? GOSSIP_MODE_PUSH_SPARSE : GOSSIP_MODE_PUSH;
}

// ---- collectives (RCCL, or device copies when emulating on one GPU) ----

// Times one exchange on every local rank's stream (gossip_kernel_time(name)
// of each part while timing is on) and books its bytes received per rank.
// With one GPU per rank every rank's interval brackets the whole exchange on its
// own stream.  An emulated group shares ONE stream: an interval opened on every
// part before any copy would cover all parts' copies, so each part is timed only
// around its own work (part(i, f): the copies into part i, or a kernel of part
// i), and the intervals of the parts partition the exchange's time.
struct ExchTimer {
    DistDriver* d;
    const char* name;
    std::vector<void*> tok;
    TraceRange tr;
    ExchTimer(DistDriver* d_, const char* n) : d(d_), name(n), tok(d_->ranks.size(), nullptr), tr("%s", n) {
        if (d->emulate) return;
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            hipSetDevice(d->ranks[i].device);
            ctx_timer_start(d->ranks[i].ctx, name, &tok[i]);
        }
    }
    void bytes(size_t i, double b) { ctx_add_bytes(d->ranks[i].ctx, name, b); }
    template <class F>
    gossip_status part(size_t i, F&& f) {
        if (!d->emulate) return f();
        void* t = nullptr;
        ctx_timer_start(d->ranks[i].ctx, name, &t);
        const gossip_status s = f();
        ctx_timer_stop(d->ranks[i].ctx, name, t);
        return s;
    }
    ~ExchTimer() {
        if (d->emulate) return;
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            hipSetDevice(d->ranks[i].device);
            ctx_timer_stop(d->ranks[i].ctx, name, tok[i]);
        }
    }
};

// every block's new words (published at gather + part[rank] * X) to every rank: send / recv pairs of the
// blocks' slices (the blocks may differ in size), every link at once
gossip_status all_gather(DistDriver* d) {
    const uint64_t X = d->X;
    auto size = [&](uint32_t q) { return (d->part[q + 1] - d->part[q]) * X; };
    ExchTimer t(d, "all_gather");
    for (size_t i = 0; i < d->ranks.size(); ++i) t.bytes(i, 8.0 * X * (double)(d->n - d->ranks[i].n_local));
    if (d->emulate) {
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            DistRank& q = d->ranks[i];
            gossip_status s = t.part(i, [&]() -> gossip_status {
                for (auto& p : d->ranks)
                    if (p.rank != q.rank)
                        DHIP(hipMemcpyAsync(q.gather + d->part[p.rank] * X, p.gather + d->part[p.rank] * X,
                                            size(p.rank) * 8, hipMemcpyDeviceToDevice, q.stream));
                return GOSSIP_OK;
            });
            if (s) return s;
        }
        return GOSSIP_OK;
    }
    DNCCL(ncclGroupStart());
    for (auto& r : d->ranks) {
        hipSetDevice(r.device);
        for (uint32_t q = 0; q < d->world; ++q) {
            if (q == r.rank) continue;
            DNCCL(ncclSend(r.gather + d->part[r.rank] * X, size(r.rank), ncclUint64, (int)q, r.comm, r.stream));
            DNCCL(ncclRecv(r.gather + d->part[q] * X, size(q), ncclUint64, (int)q, r.comm, r.stream));
        }
    }
    DNCCL(ncclGroupEnd());
    return GOSSIP_OK;
}

// The same exchange for a sparse frontier: each block's tile bitmap, all-gathered; the prefix of the
// tiles' popcounts (on every rank: where each block's packed words sit in the concatenation); the own
// block's words packed there and exchanged as send / recv pairs (sizes from the prefix); every other
// block expanded into the gather buffer.  Bytes received per rank: (P - 1) tpb 8 B of bitmap + 8 X B per
// non-zero peer of the other blocks, against 8 X B per peer of them.
gossip_status compact_gather(DistDriver* d) {
    const uint32_t W = d->world;
    const uint64_t X = d->X, tiles = d->toff[W];
    auto ntl = [&](uint32_t q) { return d->toff[q + 1] - d->toff[q]; };
    ExchTimer t(d, "all_gather");
    gossip_status s = GOSSIP_OK;
    for (size_t i = 0; i < d->ranks.size(); ++i) {  // own tile bitmap
        DistRank& r = d->ranks[i];
        DHIP(hipSetDevice(r.device));
        s = t.part(i, [&]() -> gossip_status {
            hipLaunchKernelGGL(k_tile_bits, dim3((unsigned)std::min<uint64_t>((ntl(r.rank) + 3) / 4, 8192)), dim3(256),
                               0, r.stream, r.gather + d->part[r.rank] * X, r.n_local, (uint32_t)X,
                               r.bits + d->toff[r.rank]);
            DHIP(hipGetLastError());
            return GOSSIP_OK;
        });
        if (s) return s;
    }
    if (d->emulate) {
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            DistRank& q = d->ranks[i];
            s = t.part(i, [&]() -> gossip_status {
                for (auto& p : d->ranks)
                    if (p.rank != q.rank)
                        DHIP(hipMemcpyAsync(q.bits + d->toff[p.rank], p.bits + d->toff[p.rank], ntl(p.rank) * 8,
                                            hipMemcpyDeviceToDevice, q.stream));
                return GOSSIP_OK;
            });
            if (s) return s;
        }
    } else {
        DNCCL(ncclGroupStart());
        for (auto& r : d->ranks) {
            hipSetDevice(r.device);
            for (uint32_t q = 0; q < W; ++q) {
                if (q == r.rank) continue;
                DNCCL(ncclSend(r.bits + d->toff[r.rank], ntl(r.rank), ncclUint64, (int)q, r.comm, r.stream));
                DNCCL(ncclRecv(r.bits + d->toff[q], ntl(q), ncclUint64, (int)q, r.comm, r.stream));
            }
        }
        DNCCL(ncclGroupEnd());
    }
    std::vector<uint64_t> off(W + 1);
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        DistRank& r = d->ranks[i];
        DHIP(hipSetDevice(r.device));
        s = t.part(i, [&]() -> gossip_status {
            size_t tb = r.scan_bytes;
            DHIP(hipcub::DeviceScan::ExclusiveSum(r.scan_tmp, tb, TilePop(r.bits, PopOp()), r.pos, (int)(tiles + 1),
                                                  r.stream));
            hipLaunchKernelGGL(k_pick_offsets, dim3(1), dim3(64 * ((W + 64) / 64)), 0, r.stream, r.pos, W, r.d_toff,
                               r.d_io);
            DHIP(hipGetLastError());
            DHIP(hipMemcpyAsync(r.h_io, r.d_io, (W + 1) * 8, hipMemcpyDeviceToHost, r.stream));
            return GOSSIP_OK;
        });
        if (s) return s;
        DHIP(hipStreamSynchronize(r.stream));
        std::memcpy(off.data(), r.h_io, (W + 1) * 8);  // (identical on every rank)
        s = t.part(i, [&]() -> gossip_status {
            hipLaunchKernelGGL(k_tile_pack, dim3((unsigned)std::min<uint64_t>((ntl(r.rank) + 3) / 4, 8192)), dim3(256),
                               0, r.stream, r.gather + d->part[r.rank] * X, r.n_local, (uint32_t)X,
                               r.bits + d->toff[r.rank], r.pos + d->toff[r.rank], r.pk);
            DHIP(hipGetLastError());
            return GOSSIP_OK;
        });
        if (s) return s;
    }
    for (size_t i = 0; i < d->ranks.size(); ++i)
        t.bytes(i, 8.0 * (double)(tiles - ntl(d->ranks[i].rank)) +
                       8.0 * X * (double)(off[W] - (off[d->ranks[i].rank + 1] - off[d->ranks[i].rank])));
    if (d->emulate) {
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            DistRank& q = d->ranks[i];
            s = t.part(i, [&]() -> gossip_status {
                for (auto& p : d->ranks) {
                    const uint64_t c = off[p.rank + 1] - off[p.rank];
                    if (p.rank != q.rank && c)
                        DHIP(hipMemcpyAsync(q.pk + off[p.rank] * X, p.pk + off[p.rank] * X, c * X * 8,
                                            hipMemcpyDeviceToDevice, q.stream));
                }
                return GOSSIP_OK;
            });
            if (s) return s;
        }
    } else {
        DNCCL(ncclGroupStart());
        for (auto& r : d->ranks) {
            hipSetDevice(r.device);
            const uint64_t mine = off[r.rank + 1] - off[r.rank];
            for (uint32_t q = 0; q < W; ++q) {  // every rank knows every block's count: empty pairs skipped
                if (q == r.rank) continue;
                if (mine) DNCCL(ncclSend(r.pk + off[r.rank] * X, mine * X, ncclUint64, (int)q, r.comm, r.stream));
                const uint64_t theirs = off[q + 1] - off[q];
                if (theirs) DNCCL(ncclRecv(r.pk + off[q] * X, theirs * X, ncclUint64, (int)q, r.comm, r.stream));
            }
        }
        DNCCL(ncclGroupEnd());
    }
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        DistRank& r = d->ranks[i];
        DHIP(hipSetDevice(r.device));
        s = t.part(i, [&]() -> gossip_status {
            hipLaunchKernelGGL(k_tile_expand, dim3((unsigned)std::min<uint64_t>((tiles + 3) / 4, 16384)), dim3(256), 0,
                               r.stream, r.gather, r.bits, r.pos, r.pk, (uint32_t)X, W, r.rank, r.d_part, r.d_toff);
            DHIP(hipGetLastError());
            return GOSSIP_OK;
        });
        if (s) return s;
    }
    return GOSSIP_OK;
}

// The all-gather of a binned round in S stages: the global ids are cut into segments of
// G peers (the bin layout's, bin_segment), stage j delivers every block's part of the segments s = j (mod S),
// so every block sends in every stage, over every link at once.  The stages go out on the rank's exchange
// stream after the own block's words are published; each ends with an event, and the rank's scatter stages
// the own block's chunks first, then waits for each stage's event before the chunks of its segments
// (ctx_arm_stages, round_compute).  The exchange of stage j + 1 runs under the scatter of stage j.
// The ranges of block q in stage j, in the order both sides of a send / recv pair walk them
void stage_ranges(const DistDriver* d, uint32_t q, uint32_t j, uint32_t S, uint64_t G,
                  std::vector<std::pair<uint64_t, uint64_t>>& out) {
    out.clear();
    const uint64_t b = d->part[q], e = d->part[q + 1];
    if (b >= e) return;
    for (uint64_t sg = b / G; sg * G < e; ++sg)
        if (sg % S == j) out.emplace_back(std::max(sg * G, b), std::min((sg + 1) * G, e));
}

gossip_status staged_gather(DistDriver* d, uint32_t S) {
    const uint64_t X = d->X;
    const uint64_t G = ctx_bin_seg(d->ranks[0].ctx);
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        DistRank& r = d->ranks[i];
        DHIP(hipSetDevice(r.device));
        if (!r.xs) {
            if (d->emulate && i) r.xs = d->ranks[0].xs;  // one exchange stream for the whole emulated group
            else DHIP(hipStreamCreateWithFlags(&r.xs, hipStreamNonBlocking));
        }
        if (!r.ev_pub) DHIP(hipEventCreateWithFlags(&r.ev_pub, hipEventDisableTiming));
        for (uint32_t j = 0; j < S; ++j)
            if (!r.ev_stage[j]) DHIP(hipEventCreateWithFlags(&r.ev_stage[j], hipEventDisableTiming));
        DHIP(hipEventRecord(r.ev_pub, r.stream));  // after round_begin's publish of the own words
        DHIP(hipStreamWaitEvent(r.xs, r.ev_pub, 0));
    }
    // bytes received per rank: every other block's words, as in all_gather
    std::vector<void*> tok(d->ranks.size(), nullptr);
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        ctx_add_bytes(d->ranks[i].ctx, "all_gather", 8.0 * X * (double)(d->n - d->ranks[i].n_local));
        if (!d->emulate) ctx_timer_start_on(d->ranks[i].ctx, d->ranks[i].xs, &tok[i]);
    }
    std::vector<std::pair<uint64_t, uint64_t>> rg, rg2;
    for (uint32_t j = 0; j < S; ++j) {
        if (d->emulate) {
            for (size_t i = 0; i < d->ranks.size(); ++i) {
                DistRank& q = d->ranks[i];
                void* t = nullptr;
                ctx_timer_start_on(q.ctx, q.xs, &t);
                for (auto& p : d->ranks) {
                    if (p.rank == q.rank) continue;
                    stage_ranges(d, p.rank, j, S, G, rg);
                    for (auto& x : rg)
                        DHIP(hipMemcpyAsync(q.gather + x.first * X, p.gather + x.first * X, (x.second - x.first) * X * 8,
                                            hipMemcpyDeviceToDevice, q.xs));
                }
                ctx_timer_stop_on(q.ctx, "all_gather", q.xs, t);
            }
        } else {
            DNCCL(ncclGroupStart());
            for (auto& r : d->ranks) {
                hipSetDevice(r.device);
                stage_ranges(d, r.rank, j, S, G, rg);
                for (uint32_t q = 0; q < d->world; ++q) {
                    if (q == r.rank) continue;
                    for (auto& x : rg)
                        DNCCL(ncclSend(r.gather + x.first * X, (x.second - x.first) * X, ncclUint64, (int)q, r.comm, r.xs));
                    stage_ranges(d, q, j, S, G, rg2);
                    for (auto& x : rg2)
                        DNCCL(ncclRecv(r.gather + x.first * X, (x.second - x.first) * X, ncclUint64, (int)q, r.comm, r.xs));
                }
            }
            DNCCL(ncclGroupEnd());
        }
        for (auto& r : d->ranks) {
            DHIP(hipSetDevice(r.device));
            DHIP(hipEventRecord(r.ev_stage[j], r.xs));
        }
    }
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        DistRank& r = d->ranks[i];
        DHIP(hipSetDevice(r.device));
        if (!d->emulate) ctx_timer_stop_on(r.ctx, "all_gather", r.xs, tok[i]);
        if (gossip_status s = ctx_arm_stages(r.ctx, S, r.ev_stage)) return s;
    }
    return GOSSIP_OK;
}

// dense push: rank p's staged masks for block q (send + begins[q] * X) to q,
// received at recv + p * n_local(q) * X
gossip_status all_to_all(DistDriver* d) {
    const uint64_t X = d->X;
    ExchTimer t(d, "all_to_all");
    for (size_t i = 0; i < d->ranks.size(); ++i) t.bytes(i, 8.0 * X * d->ranks[i].n_local * (d->world - 1));
    if (d->emulate) {
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            DistRank& q = d->ranks[i];
            gossip_status s = t.part(i, [&]() -> gossip_status {
                for (auto& p : d->ranks)
                    if (p.rank != q.rank)  // own pushes went straight to seen; the own slice of recv stays zero
                        DHIP(hipMemcpyAsync(q.recv + p.rank * q.n_local * X, p.send + d->part[q.rank] * X,
                                            q.n_local * X * 8, hipMemcpyDeviceToDevice, q.stream));
                return GOSSIP_OK;
            });
            if (s) return s;
        }
        return GOSSIP_OK;
    }
    DNCCL(ncclGroupStart());
    for (auto& r : d->ranks) {
        hipSetDevice(r.device);
        for (uint32_t q = 0; q < d->world; ++q) {
            if (q == r.rank && d->world > 1) continue;  // own pushes went straight to seen (world 1 still exchanges)
            DNCCL(ncclSend(r.send + d->part[q] * X, (d->part[q + 1] - d->part[q]) * X, ncclUint64, (int)q, r.comm,
                           r.stream));
            DNCCL(ncclRecv(r.recv + (uint64_t)q * r.n_local * X, r.n_local * X, ncclUint64, (int)q, r.comm, r.stream));
        }
    }
    DNCCL(ncclGroupEnd());
    return GOSSIP_OK;
}

// sparse push: record counts (per destination) then the records themselves;
// rank q receives sender p's records after those of senders < p
gossip_status exchange_records(DistDriver* d, std::vector<uint64_t>& total_in) {
    const uint32_t W = d->world;
    const uint64_t R = d->R;
    for (auto& r : d->ranks) {
        gossip_status s = gossip_sparse_counts(r.ctx, r.counts_out.data());
        if (s) return s;
    }
    if (d->emulate) {
        for (auto& q : d->ranks)
            for (auto& p : d->ranks) q.counts_in[p.rank] = p.counts_out[q.rank];
    } else {
        for (auto& r : d->ranks) {
            hipSetDevice(r.device);
            std::memcpy(r.h_io, r.counts_out.data(), W * 8);
            DHIP(hipMemcpyAsync(r.d_io, r.h_io, W * 8, hipMemcpyHostToDevice, r.stream));
        }
        DNCCL(ncclGroupStart());
        for (auto& r : d->ranks) {
            hipSetDevice(r.device);
            for (uint32_t q = 0; q < W; ++q) {
                DNCCL(ncclSend(r.d_io + q, 1, ncclUint64, (int)q, r.comm, r.stream));
                DNCCL(ncclRecv(r.d_io + W + q, 1, ncclUint64, (int)q, r.comm, r.stream));
            }
        }
        DNCCL(ncclGroupEnd());
        for (auto& r : d->ranks) {
            hipSetDevice(r.device);
            DHIP(hipMemcpyAsync(r.h_io + W, r.d_io + W, W * 8, hipMemcpyDeviceToHost, r.stream));
            DHIP(hipStreamSynchronize(r.stream));
            std::memcpy(r.counts_in.data(), r.h_io + W, W * 8);
        }
    }
    total_in.assign(d->ranks.size(), 0);
    ExchTimer t(d, "records");
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        uint64_t c = 0;
        for (uint32_t q = 0; q < W; ++q) c += q == d->ranks[i].rank ? 0 : d->ranks[i].counts_in[q];
        t.bytes(i, 8.0 * R * c);
    }
    // where each rank's records for destination q sit (the staging push's compaction, or the record push's own
    // buffer), and how many each receiver can take
    std::vector<const uint64_t*> src(d->ranks.size());
    std::vector<uint64_t> stride(d->ranks.size());
    for (size_t i = 0; i < d->ranks.size(); ++i) ctx_send_records(d->ranks[i].ctx, &src[i], &stride[i]);
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        DistRank& r = d->ranks[i];
        uint64_t c = 0;
        for (uint32_t q = 0; q < W; ++q) c += r.counts_in[q];
        if (c > r.rec_cap) {  // (once, on the first round with that many records; hipFree waits for the device)
            DHIP(hipSetDevice(r.device));
            DHIP(hipStreamSynchronize(r.stream));
            hipFree(r.rec_in);
            r.rec_in = nullptr;
            r.rec_cap = 0;
            DHIP(hipMalloc((void**)&r.rec_in, c * R * 8));
            r.rec_cap = c;
        }
    }
    if (d->emulate) {
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            DistRank& q = d->ranks[i];
            uint64_t off = 0;
            gossip_status s = t.part(i, [&]() -> gossip_status {
                for (size_t k = 0; k < d->ranks.size(); ++k) {
                    const DistRank& p = d->ranks[k];
                    const uint64_t c = p.counts_out[q.rank];
                    if (c)
                        DHIP(hipMemcpyAsync(q.rec_in + off * R, src[k] + (uint64_t)q.rank * stride[k] * R, c * R * 8,
                                            hipMemcpyDeviceToDevice, q.stream));
                    off += c;
                }
                return GOSSIP_OK;
            });
            if (s) return s;
            total_in[i] = off;
        }
        return GOSSIP_OK;
    }
    DNCCL(ncclGroupStart());
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        DistRank& r = d->ranks[i];
        hipSetDevice(r.device);
        uint64_t off = 0;
        for (uint32_t q = 0; q < W; ++q) {  // both sides know every count: zero-length pairs are skipped on both
            if (r.counts_out[q])
                DNCCL(ncclSend(src[i] + (uint64_t)q * stride[i] * R, r.counts_out[q] * R, ncclUint64, (int)q, r.comm,
                               r.stream));
            if (r.counts_in[q])
                DNCCL(ncclRecv(r.rec_in + off * R, r.counts_in[q] * R, ncclUint64, (int)q, r.comm, r.stream));
            off += r.counts_in[q];
        }
        total_in[i] = off;
    }
    DNCCL(ncclGroupEnd());
    return GOSSIP_OK;
}

// the rank's round stats, and the peers it activated (the next round's frontier)
void pack_stats(DistRank& r, uint64_t* v) {
    const gossip_round_stats& s = r.local;
    const uint64_t f[kStatSlots] = {s.frontier, s.traversals, s.deliveries, s.undelivered, s.new_receipts,
                                    s.injected, s.died,       s.reports,    s.reconnects,  s.rejoined,
                                    s.digest,   s.covered,    ctx_frontier_est(r.ctx),
                                    ctx_stages(r.ctx), (uint64_t)ctx_stages(r.ctx) * ctx_stages(r.ctx)};
    std::memcpy(v, f, sizeof(f));
}

gossip_status all_reduce_stats(DistDriver* d, uint64_t* g) {
    if (d->emulate) {
        std::fill(g, g + kStatSlots, 0ull);
        for (auto& r : d->ranks) {
            uint64_t v[kStatSlots];
            pack_stats(r, v);
            for (int i = 0; i < kStatSlots; ++i) g[i] += v[i];  // mod 2^64, like ncclSum on uint64
        }
        return GOSSIP_OK;
    }
    for (auto& r : d->ranks) {
        hipSetDevice(r.device);
        pack_stats(r, r.h_io);
        DHIP(hipMemcpyAsync(r.d_io, r.h_io, kStatSlots * 8, hipMemcpyHostToDevice, r.stream));
    }
    DNCCL(ncclGroupStart());
    for (auto& r : d->ranks) {
        hipSetDevice(r.device);
        DNCCL(ncclAllReduce(r.d_io, r.d_io, kStatSlots, ncclUint64, ncclSum, r.comm, r.stream));
    }
    DNCCL(ncclGroupEnd());
    for (auto& r : d->ranks) {
        hipSetDevice(r.device);
        DHIP(hipMemcpyAsync(r.h_io, r.d_io, kStatSlots * 8, hipMemcpyDeviceToHost, r.stream));
        DHIP(hipStreamSynchronize(r.stream));
    }
    std::memcpy(g, d->ranks[0].h_io, kStatSlots * 8);
    return GOSSIP_OK;
}

// GOSSIP_SYNC_DEBUG (diagnostics): each exchange waited for, a device fault named on stderr
const bool kDistSyncDebug = std::getenv("GOSSIP_SYNC_DEBUG") != nullptr;

gossip_status dbg_sync(DistDriver* d, const char* what, gossip_status s) {
    if (s || !kDistSyncDebug) return s;
    for (auto& r : d->ranks) {
        hipSetDevice(r.device);
        hipError_t e = hipStreamSynchronize(r.stream);
        if (e == hipSuccess && r.xs) e = hipStreamSynchronize(r.xs);
        if (e != hipSuccess) {
            std::fprintf(stderr, "[gossip] exchange %s (round %zu, rank %u): %s\n", what, d->modes.size(), r.rank,
                         hipGetErrorString(e));
            return set_error(GOSSIP_EHIP, std::string("exchange ") + what + ": " + hipGetErrorString(e));
        }
    }
    return GOSSIP_OK;
}

// One round on every local rank, lockstep phases.
gossip_status dist_step(DistDriver* d, gossip_round_stats* out) {
    if (d->finished) return set_error(GOSSIP_ESTATE, "run finished: call gossip_reset");
    TraceRange tr("gossip round %zu (%u parts)", d->modes.size(), (unsigned)d->ranks.size());
    const int want = choose_mode(d);
    int mode = -1;
    for (auto& r : d->ranks) {
        int m = 0;
        gossip_status s = gossip_round_begin(r.ctx, want, &m);
        if (s) return s;
        if (mode >= 0 && m != mode) return set_error(GOSSIP_ESTATE, "ranks chose different round modes");
        mode = m;
    }
    d->modes.push_back(mode);
    gossip_status s = GOSSIP_OK;
    if (mode == GOSSIP_MODE_PULL || mode == GOSSIP_MODE_BIN) {
        // a narrow frontier exchanges its non-zero words only (the same gather buffer either way)
        const uint32_t gpm = ctx_gather_pm(d->ranks[0].ctx);
        const bool compact = d->world > 1 && d->front * 1000 < (uint64_t)gpm * d->n;
        // a binned round with a whole-slice exchange goes out in stages under its scatter (every rank has a
        // streamed bin layout and asks for the same number of stages)
        const uint32_t S = mode == GOSSIP_MODE_BIN && !compact && d->world > 1 ? d->stages : 1u;
        if ((s = dbg_sync(d, compact ? "compact_gather" : S > 1 ? "staged_gather" : "all_gather",
                          compact ? compact_gather(d) : S > 1 ? staged_gather(d, S) : all_gather(d))))
            return s;
        for (auto& r : d->ranks)
            if ((s = gossip_round_compute(r.ctx))) return s;
        for (auto& r : d->ranks)
            if ((s = gossip_round_finish(r.ctx, &r.local))) return s;
    } else if (mode == GOSSIP_MODE_PUSH_SPARSE) {
        for (auto& r : d->ranks)
            if ((s = gossip_round_compute(r.ctx))) return s;
        std::vector<uint64_t> total_in;
        if ((s = dbg_sync(d, "records", exchange_records(d, total_in)))) return s;
        for (size_t i = 0; i < d->ranks.size(); ++i)
            if ((s = gossip_round_finish_sparse(d->ranks[i].ctx, d->ranks[i].rec_in, total_in[i], &d->ranks[i].local)))
                return s;
    } else {
        for (auto& r : d->ranks)
            if ((s = gossip_round_compute(r.ctx))) return s;
        if ((s = dbg_sync(d, "all_to_all", all_to_all(d)))) return s;
        for (auto& r : d->ranks)
            if ((s = gossip_round_finish(r.ctx, &r.local))) return s;
    }
    uint64_t g[kStatSlots];
    if ((s = all_reduce_stats(d, g))) return s;
    gossip_round_stats o{};
    o.round = d->ranks[0].local.round;
    o.flags = d->ranks[0].local.flags;
    o.frontier = g[0];
    o.traversals = g[1];
    o.deliveries = g[2];
    o.undelivered = g[3];
    o.new_receipts = g[4];
    o.injected = g[5];
    o.died = g[6];
    o.reports = g[7];
    o.reconnects = g[8];
    o.rejoined = g[9];
    d->cum_digest += g[10];
    d->cum_covered += g[11];
    d->front = g[12];
    // every rank asked for the same stage count iff sum(S)^2 == world * sum(S^2) (equality in Cauchy-Schwarz);
    // every rank computes this from the same sums, so all take the same exchange in the next binned round
    d->stages = g[13] % d->world == 0 && g[13] * g[13] == (uint64_t)d->world * g[14]
                    ? (uint32_t)std::min<uint64_t>(g[13] / d->world, kMaxStages) : 1u;
    o.digest = d->cum_digest;
    o.covered = d->cum_covered;
    o.duplicates = o.deliveries - o.new_receipts;
    o.seed_removals = 0;  // from the gathered reports (gossip_comm_finalize)
    d->prev_new = o.new_receipts;
    d->injected += o.injected;
    int fin = -1;
    for (auto& r : d->ranks) {
        int f = 0;
        if ((s = gossip_round_commit(r.ctx, o.new_receipts, &f))) return s;
        if (fin >= 0 && f != fin) return set_error(GOSSIP_ESTATE, "ranks disagree on termination");
        fin = f;
    }
    d->finished = fin == 1;
    if (out) *out = o;
    return d->finished ? 1 : 0;
}

bool report_less(const gossip_dead_report& x, const gossip_dead_report& y) {
    if (x.round != y.round) return x.round < y.round;
    if (x.reporter != y.reporter) return x.reporter < y.reporter;
    return x.dead < y.dead;
}

gossip_status local_reports(DistRank& r, std::vector<gossip_dead_report>& out) {
    uint64_t n = 0;
    gossip_status s = gossip_read_reports(r.ctx, nullptr, 0, &n);
    if (s) return s;
    out.resize(n);
    return n ? gossip_read_reports(r.ctx, out.data(), n, &n) : GOSSIP_OK;
}

// Every rank's reports to every rank, merged and sorted; seed_removals of a
// round = peers whose first report falls in it (seed.cpp:158-167).
gossip_status dist_finalize(DistDriver* d, gossip_round_stats* per_round, uint32_t rounds,
                            std::vector<gossip_dead_report>& all) {
    all.clear();
    gossip_status s = GOSSIP_OK;
    if (d->world == (uint32_t)d->ranks.size()) {  // this process holds every rank: no collective needed
        for (auto& r : d->ranks) {
            std::vector<gossip_dead_report> mine;
            if ((s = local_reports(r, mine))) return s;
            all.insert(all.end(), mine.begin(), mine.end());
        }
    } else {
        // one local rank (gossip_comm_init): counts, then the padded lists, all-gathered
        DistRank& r = d->ranks[0];
        std::vector<gossip_dead_report> mine;
        if ((s = local_reports(r, mine))) return s;
        const uint32_t W = d->world;
        DHIP(hipSetDevice(r.device));
        r.h_io[0] = mine.size();
        DHIP(hipMemcpyAsync(r.d_io, r.h_io, 8, hipMemcpyHostToDevice, r.stream));
        DNCCL(ncclAllGather(r.d_io, r.d_io + W, 1, ncclUint64, r.comm, r.stream));
        DHIP(hipMemcpyAsync(r.h_io + W, r.d_io + W, W * 8, hipMemcpyDeviceToHost, r.stream));
        DHIP(hipStreamSynchronize(r.stream));
        std::vector<uint64_t> cnt(r.h_io + W, r.h_io + 2 * W);
        const uint64_t mx = std::max<uint64_t>(1, *std::max_element(cnt.begin(), cnt.end()));
        uint32_t *d_mine = nullptr, *d_all = nullptr;
        DHIP(hipMalloc((void**)&d_mine, mx * 12));
        if (hipMalloc((void**)&d_all, mx * 12 * W) != hipSuccess) {
            hipFree(d_mine);
            return set_error(GOSSIP_ENOMEM, "report gather buffer");
        }
        hipError_t he = mine.empty() ? hipSuccess
                                     : hipMemcpyAsync(d_mine, mine.data(), mine.size() * 12, hipMemcpyHostToDevice, r.stream);
        ncclResult_t nr = he == hipSuccess ? ncclAllGather(d_mine, d_all, mx * 3, ncclUint32, r.comm, r.stream)
                                           : ncclSuccess;
        std::vector<gossip_dead_report> buf(mx * W);
        if (he == hipSuccess && nr == ncclSuccess)
            he = hipMemcpyAsync(buf.data(), d_all, mx * 12 * W, hipMemcpyDeviceToHost, r.stream);
        if (he == hipSuccess) he = hipStreamSynchronize(r.stream);
        hipFree(d_mine);
        hipFree(d_all);
        if (he != hipSuccess) return set_error(GOSSIP_EHIP, std::string("report gather: ") + hipGetErrorString(he));
        if (nr != ncclSuccess) return set_error(GOSSIP_ECOMM, std::string("report gather: ") + ncclGetErrorString(nr));
        for (uint32_t p = 0; p < W; ++p) all.insert(all.end(), buf.begin() + p * mx, buf.begin() + p * mx + cnt[p]);
    }
    std::sort(all.begin(), all.end(), report_less);
    if (per_round) {
        std::vector<std::pair<uint32_t, uint32_t>> firsts;  // (dead, round) of its first report
        std::vector<gossip_dead_report> byv(all);
        std::stable_sort(byv.begin(), byv.end(),
                         [](const gossip_dead_report& x, const gossip_dead_report& y) { return x.dead < y.dead; });
        for (size_t i = 0; i < byv.size(); ++i)
            if (i == 0 || byv[i].dead != byv[i - 1].dead) firsts.emplace_back(byv[i].dead, byv[i].round);
        for (uint32_t i = 0; i < rounds; ++i) per_round[i].seed_removals = 0;
        for (const auto& f : firsts)
            for (uint32_t i = 0; i < rounds; ++i)
                if (per_round[i].round == f.second) {
                    per_round[i].seed_removals++;
                    break;
                }
    }
    return GOSSIP_OK;
}

}  // namespace

gossip_status dist_step_ctx(gossip_ctx* c, gossip_round_stats* out) {
    DistDriver* d = ctx_dist(c);
    if (d->ranks.size() != 1) return set_error(GOSSIP_ESTATE, "this ctx is a part of a group: use gossip_group_step");
    return dist_step(d, out);
}

void dist_reset(DistDriver* d) {
    d->prev_new = d->injected = d->cum_digest = d->cum_covered = d->front = 0;
    d->stages = 1;
    d->finished = false;
    d->modes.clear();
}

void dist_free(DistDriver* d) {
    if (!d) return;
    for (auto& r : d->ranks) free_rank(r);
    std::vector<hipStream_t> done;  // emulated groups share one stream (and one exchange stream)
    for (auto& r : d->ranks)
        for (hipStream_t st : {r.stream, r.xs}) {
            if (!st || std::find(done.begin(), done.end(), st) != done.end()) continue;
            hipSetDevice(r.device);
            hipStreamDestroy(st);
            done.push_back(st);
        }
    delete d;
}

}  // namespace gossip

using namespace gossip;

struct gossip_group {
    DistDriver* d = nullptr;
    std::vector<gossip_ctx*> parts;
    uint64_t n = 0;
    uint32_t W = 0;
};

extern "C" {

gossip_status gossip_partition(uint64_t n_peers, uint32_t world, uint64_t* begins) {
    if (!begins || world < 1 || n_peers < world) return set_error(GOSSIP_EINVAL, "need 1 <= world <= n_peers");
    const std::vector<uint64_t> b = blocks(n_peers, world);
    for (uint32_t p = 0; p < world; ++p)
        if (b[p + 1] <= b[p]) return set_error(GOSSIP_EINVAL, "peers do not split into non-empty ceil(n/world) blocks");
    std::copy(b.begin(), b.end(), begins);
    return GOSSIP_OK;
}

// Blocks of about equal work on the powerlaw overlay.  Its degree mass is skewed to the
// low ids: every peer draws k picks from one seed response of L candidates (E[k] = sum over j < L of
// 1 - (j/L)^2.5, 3.75 at L = 6) and candidate c = floor(n V^3), so P(c < x) = (x/n)^(1/3).  Symmetrised, the
// edges with an end in [0, x) are about E[k] (x + n (x/n)^(1/3)): at P = 8 the first eighth of the ids holds
// 3.2 times the edges of any other eighth (config 4 as 8 ceil(n/P) parts: part 0's kernels 18.9 ms per step,
// the others' 8.8-9.8).  A block's cost is its edges plus kPeerCost edge-equivalents per peer (its O(peers)
// sweeps and finishes); boundaries are whole 64-peer tiles.  A pure function of the config, so every rank
// computes the same blocks.
gossip_status gossip_partition_edges(const gossip_config* cfg, uint32_t world, uint64_t* begins) {
    if (!cfg || !begins || world < 1 || cfg->n_peers < (uint64_t)world * 64)
        return cfg ? gossip_partition(cfg->n_peers, world, begins) : set_error(GOSSIP_EINVAL, "null config");
    if (cfg->graph_model != GOSSIP_GRAPH_POWERLAW) return gossip_partition(cfg->n_peers, world, begins);
    constexpr double kPeerCost = 2.0;
    const uint64_t n = cfg->n_peers;
    const uint32_t L = cfg->list_len ? cfg->list_len : 6;
    double ek = 0.0;
    for (uint32_t j = 1; j < L; ++j) ek += 1.0 - std::pow((double)j / L, 2.5);
    auto cost = [&](double u) { return ek * (u + std::cbrt(u)) + kPeerCost * u; };
    const double total = cost(1.0);
    begins[0] = 0;
    for (uint32_t q = 1; q < world; ++q) {
        const double want = total * q / world;
        double lo = 0.0, hi = 1.0;
        for (int it = 0; it < 200; ++it) {
            const double mid = 0.5 * (lo + hi);
            (cost(mid) < want ? lo : hi) = mid;
        }
        uint64_t x = ((uint64_t)(hi * (double)n) + 63) / 64 * 64;
        x = std::max<uint64_t>(x, begins[q - 1] + 64);                  // non-empty, whole tiles
        x = std::min<uint64_t>(x, (n - (uint64_t)(world - q) * 64) / 64 * 64);  // room for the blocks after it
        begins[q] = x;
    }
    begins[world] = n;
    for (uint32_t q = 0; q < world; ++q)
        if (begins[q + 1] <= begins[q]) return gossip_partition(n, world, begins);
    return GOSSIP_OK;
}

gossip_status gossip_comm_unique_id(uint8_t* id) {
    if (!id) return set_error(GOSSIP_EINVAL, "null argument");
    ncclUniqueId u;
    DNCCL(ncclGetUniqueId(&u));
    static_assert(sizeof(u) == GOSSIP_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return GOSSIP_OK;
}

gossip_status gossip_comm_init(gossip_ctx* ctx, const uint8_t* id, uint32_t world, uint32_t rank) {
    if (!ctx || !id || world < 1 || rank >= world) return set_error(GOSSIP_EINVAL, "bad argument");
    if (ctx_dist(ctx)) return set_error(GOSSIP_ESTATE, "ctx already has a communicator");
    const gossip_config& cfg = ctx_config(ctx);
    if (cfg.rejoin_threshold) return set_error(GOSSIP_EINVAL, "rejoin_threshold needs a single partition");
    DistDriver* d = new DistDriver();
    d->world = world;
    d->ranks.resize(1);
    DistRank& r = d->ranks[0];
    r.ctx = ctx;
    r.rank = rank;
    r.device = ctx_device(ctx);
    gossip_status s = GOSSIP_OK;
    hipSetDevice(r.device);
    if (hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking) != hipSuccess) s = set_error(GOSSIP_EHIP, "stream");
    if (!s) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        const ncclResult_t nr = ncclCommInitRank(&r.comm, (int)world, u, (int)rank);
        if (nr != ncclSuccess) s = set_error(GOSSIP_ECOMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(nr));
    }
    if (!s) {  // every rank's block (any contiguous partition: gossip_partition or gossip_partition_edges)
        uint64_t b = 0, e = 0;
        ctx_range(ctx, &b, &e);
        uint64_t* dv = nullptr;
        std::vector<uint64_t> h(2 * (size_t)world + 2);
        hipError_t he = hipMalloc((void**)&dv, h.size() * 8);
        h[0] = b;
        h[1] = e;
        if (he == hipSuccess) he = hipMemcpyAsync(dv, h.data(), 16, hipMemcpyHostToDevice, r.stream);
        ncclResult_t nr = he == hipSuccess ? ncclAllGather(dv, dv + 2, 2, ncclUint64, r.comm, r.stream) : ncclSuccess;
        if (he == hipSuccess && nr == ncclSuccess)
            he = hipMemcpyAsync(h.data() + 2, dv + 2, 16 * (size_t)world, hipMemcpyDeviceToHost, r.stream);
        if (he == hipSuccess) he = hipStreamSynchronize(r.stream);
        hipFree(dv);
        if (he != hipSuccess) s = set_error(GOSSIP_EHIP, std::string("block table: ") + hipGetErrorString(he));
        else if (nr != ncclSuccess) s = set_error(GOSSIP_ECOMM, std::string("block table: ") + ncclGetErrorString(nr));
        std::vector<uint64_t> part(world + 1);
        for (uint32_t q = 0; !s && q < world; ++q) {
            part[q] = h[2 + 2 * q];
            part[q + 1] = h[3 + 2 * q];
            if (part[q + 1] <= part[q] || (q && h[1 + 2 * q] != part[q]))
                s = set_error(GOSSIP_EINVAL, "the ranks' part ranges are not contiguous non-empty blocks in rank order");
        }
        if (!s && (part[0] != 0 || part[world] != cfg.n_peers))
            s = set_error(GOSSIP_EINVAL, "the ranks' part ranges do not cover [0, n_peers)");
        if (!s) init_schedule(d, cfg, part);
    }
    if (!s) s = bind_rank(d, r);
    if (!s) s = setup_rank(d, r);
    if (s) {
        // the ctx must not keep pointers into the buffers dist_free releases: it stays a
        // single-partition ctx on the null stream, usable with gossip_step
        ctx_clear_exchange(ctx);
        gossip_set_stream(ctx, nullptr);
        dist_free(d);
        return s;
    }
    ctx_attach_dist(ctx, d, true);
    return GOSSIP_OK;
}

gossip_status gossip_comm_finalize(gossip_ctx* ctx, gossip_round_stats* per_round, uint32_t rounds,
                                   gossip_dead_report* reports, uint64_t cap, uint64_t* count) {
    if (!ctx) return set_error(GOSSIP_EINVAL, "null ctx");
    DistDriver* d = ctx_dist(ctx);
    if (!d) return set_error(GOSSIP_ESTATE, "no communicator: gossip_comm_init first");
    std::vector<gossip_dead_report> all;
    gossip_status s = dist_finalize(d, per_round, rounds, all);
    if (s) return s;
    if (count) *count = all.size();
    if (reports) std::copy(all.begin(), all.begin() + std::min<uint64_t>(cap, all.size()), reports);
    return GOSSIP_OK;
}

gossip_status gossip_comm_modes(gossip_ctx* ctx, int32_t* modes, uint32_t cap, uint32_t* n) {
    if (!ctx || !n) return set_error(GOSSIP_EINVAL, "null argument");
    DistDriver* d = ctx_dist(ctx);
    if (!d) return set_error(GOSSIP_ESTATE, "no communicator");
    *n = (uint32_t)d->modes.size();
    if (modes) std::copy(d->modes.begin(), d->modes.begin() + std::min<size_t>(cap, d->modes.size()), modes);
    return GOSSIP_OK;
}

gossip_status gossip_group_create(const gossip_config* cfg, uint32_t n_parts, const int32_t* devices,
                                  gossip_group** out) {
    if (!cfg || !devices || !out || n_parts < 1) return set_error(GOSSIP_EINVAL, "bad argument");
    *out = nullptr;
    std::vector<uint64_t> part(n_parts + 1);
    gossip_status s = cfg->flags & GOSSIP_FLAG_UNIFORM_PARTITION ? gossip_partition(cfg->n_peers, n_parts, part.data())
                                                                 : gossip_partition_edges(cfg, n_parts, part.data());
    if (s) return s;
    // gossip_group_create_parts takes blocks that start on whole 64-peer tiles; the uniform blocks (ref_bootstrap
    // overlays, GOSSIP_FLAG_UNIFORM_PARTITION, or fewer than 64 peers per block) are ceil(n/P) peers, so they
    // are rounded up to whole tiles here
    bool tiles = true;
    for (uint32_t q = 0; q < n_parts; ++q) tiles &= part[q] % 64 == 0;
    if (!tiles) {
        const uint64_t n = cfg->n_peers, chunk = ((n + n_parts - 1) / n_parts + 63) / 64 * 64;
        for (uint32_t q = 0; q <= n_parts; ++q) part[q] = std::min<uint64_t>((uint64_t)q * chunk, n);
        for (uint32_t q = 0; q < n_parts; ++q)
            if (part[q + 1] <= part[q])
                return set_error(GOSSIP_EINVAL, "n_peers too small: every part needs whole 64-peer tiles");
    }
    return gossip_group_create_parts(cfg, n_parts, devices, part.data(), out);
}

gossip_status gossip_group_create_parts(const gossip_config* cfg, uint32_t n_parts, const int32_t* devices,
                                        const uint64_t* begins, gossip_group** out) {
    if (!cfg || !devices || !out || !begins || n_parts < 1) return set_error(GOSSIP_EINVAL, "bad argument");
    *out = nullptr;
    if (begins[0] != 0 || begins[n_parts] != cfg->n_peers)
        return set_error(GOSSIP_EINVAL, "part begins must run from 0 to n_peers");
    for (uint32_t q = 0; q < n_parts; ++q)
        if (begins[q + 1] <= begins[q] || begins[q] % 64)
            return set_error(GOSSIP_EINVAL, "parts must be non-empty and start on whole 64-peer tiles");
    const std::vector<uint64_t> part(begins, begins + n_parts + 1);
    gossip_status s = GOSSIP_OK;
    if (cfg->rejoin_threshold && n_parts > 1) return set_error(GOSSIP_EINVAL, "rejoin_threshold needs a single partition");
    bool same = true, distinct = true;
    for (uint32_t p = 0; p < n_parts; ++p)
        for (uint32_t q = 0; q < p; ++q) {
            same &= devices[p] == devices[q];
            distinct &= devices[p] != devices[q];
        }
    same &= devices[0] == devices[n_parts - 1];
    if (!same && !distinct) return set_error(GOSSIP_EINVAL, "devices must be all distinct or all the same");
    gossip_group* g = new gossip_group();
    g->n = cfg->n_peers;
    g->W = (cfg->n_msgs + 63) / 64;
    DistDriver* d = new DistDriver();
    g->d = d;
    d->world = n_parts;
    d->emulate = same && n_parts > 1;
    init_schedule(d, *cfg, part);
    d->ranks.resize(n_parts);
    auto bail = [&](gossip_status st) {
        for (auto& r : d->ranks)
            if (r.ctx) ctx_attach_dist(r.ctx, nullptr, false);
        gossip_group_destroy(g);
        return st;
    };
    for (uint32_t p = 0; p < n_parts; ++p) {
        gossip_config c = *cfg;
        c.part_begin = part[p];
        c.part_end = part[p + 1];
        c.device = devices[p];
        if ((s = gossip_create(&c, &d->ranks[p].ctx))) return bail(s);
        g->parts.push_back(d->ranks[p].ctx);
        d->ranks[p].rank = p;
        if ((s = bind_rank(d, d->ranks[p]))) return bail(s);
        hipSetDevice(d->ranks[p].device);
        if (!d->emulate || p == 0) {
            if (hipStreamCreateWithFlags(&d->ranks[p].stream, hipStreamNonBlocking) != hipSuccess)
                return bail(set_error(GOSSIP_EHIP, "stream"));
        } else {
            d->ranks[p].stream = d->ranks[0].stream;  // one stream orders every part's work and copies
        }
    }
    for (auto& r : d->ranks)
        if ((s = setup_rank(d, r))) return bail(s);
    if (!d->emulate) {
        std::vector<ncclComm_t> comms(n_parts);
        std::vector<int> devs(devices, devices + n_parts);
        const ncclResult_t nr = ncclCommInitAll(comms.data(), (int)n_parts, devs.data());
        if (nr != ncclSuccess) return bail(set_error(GOSSIP_ECOMM, std::string("ncclCommInitAll: ") + ncclGetErrorString(nr)));
        for (uint32_t p = 0; p < n_parts; ++p) d->ranks[p].comm = comms[p];
    }
    for (auto& r : d->ranks) ctx_attach_dist(r.ctx, d, false);
    *out = g;
    return GOSSIP_OK;
}

void gossip_group_destroy(gossip_group* g) {
    if (!g) return;
    for (gossip_ctx* c : g->parts) {
        ctx_attach_dist(c, nullptr, false);
        gossip_set_stream(c, nullptr);  // the driver's streams go with it
    }
    if (g->d) {
        for (auto& r : g->d->ranks) r.ctx = nullptr;
        dist_free(g->d);
    }
    for (gossip_ctx* c : g->parts) gossip_destroy(c);
    delete g;
}

gossip_status gossip_group_part(gossip_group* g, uint32_t p, gossip_ctx** ctx) {
    if (!g || !ctx || p >= g->parts.size()) return set_error(GOSSIP_EINVAL, "bad argument");
    *ctx = g->parts[p];
    return GOSSIP_OK;
}

#define GROUP_EACH(g, call)                              \
    do {                                                 \
        if (!(g)) return set_error(GOSSIP_EINVAL, "null group"); \
        for (gossip_ctx* c_ : (g)->parts) {              \
            gossip_status s_ = call;                     \
            if (s_) return s_;                           \
        }                                                \
        return GOSSIP_OK;                                \
    } while (0)

gossip_status gossip_group_build_graph(gossip_group* g) { GROUP_EACH(g, gossip_build_graph(c_)); }
gossip_status gossip_group_inject(gossip_group* g, const uint32_t* origin, const uint32_t* inject_round, uint32_t n) {
    GROUP_EACH(g, gossip_inject(c_, origin, inject_round, n));
}
gossip_status gossip_group_schedule_kills(gossip_group* g, const uint32_t* peer, const uint32_t* round, uint32_t n) {
    GROUP_EACH(g, gossip_schedule_kills(c_, peer, round, n));
}
gossip_status gossip_group_reset(gossip_group* g) { GROUP_EACH(g, gossip_reset(c_)); }

gossip_status gossip_group_step(gossip_group* g, gossip_round_stats* out) {
    if (!g) return set_error(GOSSIP_EINVAL, "null group");
    return dist_step(g->d, out);
}

gossip_status gossip_group_run(gossip_group* g, gossip_round_stats* per_round, uint32_t cap, uint32_t* rounds) {
    if (!g) return set_error(GOSSIP_EINVAL, "null group");
    std::vector<gossip_round_stats> all;
    while (!g->d->finished) {
        gossip_round_stats st{};
        const gossip_status s = dist_step(g->d, &st);
        if (s < 0) return s;
        all.push_back(st);
    }
    std::vector<gossip_dead_report> reps;
    const gossip_status s = dist_finalize(g->d, all.data(), (uint32_t)all.size(), reps);
    if (s) return s;
    if (per_round) std::copy(all.begin(), all.begin() + std::min<size_t>(cap, all.size()), per_round);
    if (rounds) *rounds = (uint32_t)all.size();
    return GOSSIP_OK;
}

gossip_status gossip_group_read_seen(gossip_group* g, uint64_t* host_seen) {
    if (!g || !host_seen) return set_error(GOSSIP_EINVAL, "null argument");
    for (auto& r : g->d->ranks) {
        const gossip_status s = gossip_read_seen(r.ctx, host_seen + r.begin * g->W);
        if (s) return s;
    }
    return GOSSIP_OK;
}

gossip_status gossip_group_read_reports(gossip_group* g, gossip_dead_report* buf, uint64_t cap, uint64_t* count) {
    if (!g || !count) return set_error(GOSSIP_EINVAL, "null argument");
    std::vector<gossip_dead_report> all;
    const gossip_status s = dist_finalize(g->d, nullptr, 0, all);
    if (s) return s;
    *count = all.size();
    if (buf) std::copy(all.begin(), all.begin() + std::min<uint64_t>(cap, all.size()), buf);
    return GOSSIP_OK;
}

}  // extern "C"
