/*
 * gossip.h -- C-ABI of libgossip_hip, the MI355X (gfx950) gossip-propagation
 * engine.  This is the drop-in boundary for the reference's hot path:
 * plain C types, caller-owned host buffers, no C++ types, never throws.
 *
 * Each entry point replaces one piece of the reference's per-process,
 * thread-per-connection C++ (PareenShah27/P2P-GossipProtocol @ 2025-02-25;
 * file:line below).  One gossip_ctx simulates ALL peers of one vertex
 * partition: a reference PeerNode becomes a peer id inside the ctx.
 *
 * Threading: a ctx is single-caller-thread.  Device work is issued on the
 * ctx's HIP stream (its own, or the one given to gossip_set_stream).
 * Errors: every call returns gossip_status (0 = OK, < 0 = error);
 * gossip_last_error() gives the message of the last failure on this thread.
 */
#ifndef GOSSIP_GOSSIP_H
#define GOSSIP_GOSSIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gossip_ctx gossip_ctx;
typedef int gossip_status;

#define GOSSIP_OK 0
#define GOSSIP_EINVAL (-1)  /* bad argument */
#define GOSSIP_ENOMEM (-2)  /* host or device allocation failed */
#define GOSSIP_EHIP (-3)    /* HIP runtime error */
#define GOSSIP_ESTATE (-4)  /* call out of order (e.g. step before graph) */
#define GOSSIP_ENODEV (-5)  /* no gfx950 device visible */
#define GOSSIP_EOVERFLOW (-6) /* report buffer overflowed (reports dropped) */
#define GOSSIP_ESTALL (-8)    /* device work gave up waiting (a bounded spin tripped): results incomplete */
#define GOSSIP_EBOUNDS (-9)   /* checked-index build only (make checked): a kernel index passed its bound;
                                 gossip_last_error names the site, the index and the bound */

/* Overlay models. */
#define GOSSIP_GRAPH_POWERLAW 1      /* scale overlay: power-law pick (peer.cpp:219-222), skewed
                                        candidates, symmetrised */
#define GOSSIP_GRAPH_REF_BOOTSTRAP 2 /* literal bootstrap DAG (peer.cpp:63-72,214-253; seed.cpp:117), n <= 4096 */

/* gossip_config.flags */
#define GOSSIP_FLAG_COVERAGE_HISTORY 1u /* keep per-message coverage for every round */
#define GOSSIP_FLAG_FORCE_PUSH 2u       /* never use pull rounds */
#define GOSSIP_FLAG_FORCE_PULL 4u       /* pull every eligible round (symmetric overlay, nobody dead, P = 1) */
#define GOSSIP_FLAG_NO_BIN 8u           /* do not lay out the binned edge slots (saves ~(4 + 2 + 8W) B per edge) */
#define GOSSIP_FLAG_FORCE_BIN 16u       /* every pull-eligible round runs binned (needs the slot layout) */
#define GOSSIP_FLAG_NO_BLOCKED 32u      /* no propagation-blocked push rounds (saves ~22 B per edge of records) */
#define GOSSIP_FLAG_FORCE_BLOCKED 64u   /* every push or binned round runs propagation-blocked where it can
                                           (single partition, one word per peer, slot layout) */
#define GOSSIP_FLAG_UNIFORM_PARTITION 128u /* gossip_group_create: blocks of ceil(n/parts) peers, rounded up to
                                              whole 64-peer tiles, instead of gossip_partition_edges */

/*
 * Replaces: NetworkConfig's parsed values (config.cpp:31-42,93-96) plus the
 * constants PeerNode hard-codes (peer.cpp:219,330,337,353,358,377).
 */
typedef struct gossip_config {
    uint64_t n_peers;         /* global peer count (< 2^31) */
    uint64_t part_begin;      /* owned peer range [part_begin, part_end); both 0 = all */
    uint64_t part_end;
    uint32_t n_msgs;          /* M concurrent messages; W = ceil(M/64) 64-bit words per peer (M <= 512) */
    uint32_t rng_seed;        /* Philox key word 0 (overlay, churn, origins) */
    uint32_t graph_model;     /* GOSSIP_GRAPH_* */
    uint32_t list_len;        /* powerlaw: candidates per seed response (default 6) */
    uint32_t n_seeds;         /* ref_bootstrap: seeds in network.txt (quorum = n_seeds/2+1) */
    uint32_t churn_threshold; /* peer dies in round r iff philox.x < threshold; 0 = none */
    uint32_t ping_every;      /* liveness every k rounds (ping_interval gate, peer.cpp:329-330); 0 = none */
    uint32_t max_missed;      /* max_missed_pings (peer.cpp:337); default 3 */
    uint32_t max_rounds;      /* hard stop (default 4096) */
    uint32_t min_rounds;      /* run at least this many rounds (liveness demos) */
    int32_t device;           /* HIP device ordinal; -1 = current */
    uint32_t flags;           /* GOSSIP_FLAG_* */
    uint64_t report_capacity; /* dead-node report buffer entries (0 = default) */
    uint32_t pull_permille;   /* pull when the frontier estimate >= this per-mille of the owned peers (0 = 60) */
    uint32_t front_permille;  /* pull rounds probe a frontier bitmap below this per-mille (0 = 400; 1000 = always) */
    uint32_t bin_permille;    /* a dense round runs binned while the (peer, message) pairs still missing are
                                 >= this per-mille of the owned peers (0 = default) */
    uint32_t extra_cap;       /* re-bootstrap after a death (handleDeadPeer peer.cpp:398-404): a reporter
                                 re-selects from a seed response and keeps up to this many extra out-edges
                                 (0 = off, the reference's literal drop-only behaviour; <= 64) */
    uint32_t list_cap;        /* ref_bootstrap: bytes of a seed's peer_list a peer reads -- the reference's 4 KB
                                 recv (peer.cpp:188-190; 4095 = faithful).  A peer whose list is
                                 longer fails registration and never starts (registered, not alive).  0 = no cap */
    uint32_t rejoin_threshold; /* join churn (the reference has no rejoin path): a peer dead at the start of round
                                  r restarts in r iff philox({seed,v},{7,r,0,0}).x < threshold -- re-registered,
                                  empty Message-List, old connections gone, fresh out-edges from one seed response
                                  into its overflow row (extra_cap > 0).  0 = never.  Single partition only */
    uint32_t blocked_permille; /* propagation-blocked rounds (single partition, M <= 64):
                                  a binned round below this frontier per-mille runs blocked where the slot array
                                  has >= 2^28 slots (0 = 300); push rounds from a 1 % frontier on overlays of
                                  >= 2^26 peers ("blocked_push_permille" of gossip_set_tuning) */
} gossip_config;

/*
 * One round's statistics.  Replaces the observable side effects of one hop
 * of broadcastMessage (peer.cpp:310-316: a successful send adds to
 * MessageTracker.sentTo) and handleClient (peer.cpp:277-285: new message ->
 * "Received new message", duplicate -> dropped).
 */
typedef struct gossip_round_stats {
    uint32_t round;
    uint32_t flags;         /* bit0: liveness (ping) round */
    uint64_t frontier;      /* peers with new messages at push start */
    uint64_t traversals;    /* live out-edges scanned from the frontier */
    uint64_t deliveries;    /* sum popcount(new[u]) over traversed edges with alive target (= sentTo inserts) */
    uint64_t undelivered;   /* same for dead targets (send attempted, peer.cpp:312 fails) */
    uint64_t new_receipts;  /* (peer, message) pairs received for the first time */
    uint64_t duplicates;    /* deliveries - new_receipts (dropped by the Message-List check) */
    uint64_t injected;      /* messages generated this round (messageGenerationLoop) */
    uint64_t died;          /* peers that died this round */
    uint64_t reports;       /* dead-node reports emitted this round */
    uint64_t seed_removals; /* seed-registry entries removed (first report of a peer) */
    uint64_t digest;        /* sum_v,w g(v*W+w) * seen[v][w] mod 2^64 at push start */
    uint64_t covered;       /* sum popcount(seen) at push start */
    uint64_t reconnects;    /* out-edges added by re-bootstrap or a restart this round (extra_cap > 0) */
    uint64_t rejoined;      /* dead peers restarted this round (rejoin_threshold > 0) */
} gossip_round_stats;

/* A dead-node report: reporter u detected dead peer v in round r
 * (handleDeadPeer peer.cpp:381-397 -> the seed's dead_node handler seed.cpp:130-138). */
typedef struct gossip_dead_report {
    uint32_t round;
    uint32_t reporter;
    uint32_t dead;
} gossip_dead_report;

/* ---- lifecycle ---------------------------------------------------------- */
/* Replaces PeerNode::PeerNode (peer.cpp:19-22) for all peers of a partition. */
gossip_status gossip_create(const gossip_config* cfg, gossip_ctx** out);
/* Replaces PeerNode::~PeerNode / stop (peer.cpp:24-26,106-123). */
void gossip_destroy(gossip_ctx* ctx);
const char* gossip_strerror(gossip_status s);
const char* gossip_last_error(void);
/* Sets the HIP stream (hipStream_t passed as void*) the ctx issues work on. */
gossip_status gossip_set_stream(gossip_ctx* ctx, void* hip_stream);
/* Shape: W = ceil(M/64) words per peer in host buffers; exchange_words = the
 * (padded) words per peer of the device exchange buffers; owned peers; edges. */
gossip_status gossip_get_shape(gossip_ctx* ctx, uint32_t* words, uint32_t* exchange_words, uint64_t* n_local,
                               uint64_t* n_edges);

/* ---- overlay ------------------------------------------------------------ */
/* Replaces the seed bootstrap + selectAndConnectPeers (peer.cpp:63-72,161-253;
 * seed.cpp:109-129,153-178): builds the CSR overlay of the owned rows on the
 * device (Philox-keyed, deterministic). */
gossip_status gossip_build_graph(gossip_ctx* ctx);
/* Loads a caller-built CSR of the owned rows (row_ptr[n_local+1] local offsets,
 * col[n_edges] global ids, rows sorted, no self loops).  Copied; caller keeps ownership. */
gossip_status gossip_load_csr(gossip_ctx* ctx, const uint64_t* row_ptr, const uint32_t* col, uint64_t n_rows,
                              uint64_t n_edges);
/* Copies the owned CSR back (row_ptr: n_local+1, col: n_edges; masked edges have bit 31 set). */
gossip_status gossip_read_csr(gossip_ctx* ctx, uint64_t* row_ptr, uint32_t* col);
/* Re-bootstrap edges of the owned peers (connectedPeers entries added by
 * selectAndConnectPeers after a death, peer.cpp:398-404 -> :214-253):
 * counts[n_local], cols[n_local * extra_cap] (row u's first counts[u] entries,
 * global ids, bit 31 = dropped again by liveness). */
gossip_status gossip_read_extra(gossip_ctx* ctx, uint32_t* counts, uint32_t* cols);

/* ---- schedule ------------------------------------------------------------ */
/* Replaces messageGenerationLoop (peer.cpp:357-379): message m (msgNumber of
 * origin[m]) is generated by origin[m] in round inject_round[m]. n_msgs == cfg.n_msgs. */
gossip_status gossip_inject(gossip_ctx* ctx, const uint32_t* origin, const uint32_t* inject_round, uint32_t n_msgs);
/* Fault injection (README.md:6 "Ctrl+C to kill any peer"): peer kill_peer[i] dies in kill_round[i]. */
gossip_status gossip_schedule_kills(gossip_ctx* ctx, const uint32_t* kill_peer, const uint32_t* kill_round,
                                    uint32_t n_kills);
/* Philox-chosen distinct origins (host helper; same draw on every rank). */
gossip_status gossip_pick_origins(uint64_t n_peers, uint32_t rng_seed, uint32_t count, uint32_t* out);
/* HIP devices visible to this process (the GPUs a gossip_group can spread over). */
gossip_status gossip_device_count(int32_t* count);

/* ---- rounds (single partition) ------------------------------------------ */
/* Clears all dynamic state (seen/new, alive, edge masks, miss counters,
 * registry, reports) back to round 0; keeps overlay and schedule. */
gossip_status gossip_reset(gossip_ctx* ctx);
/* One round: churn -> liveness (if due) -> injection -> push (or, on dense
 * rounds of a symmetric overlay with nobody dead, the equivalent pull) -> advance.
 * Returns 1 when the run is finished after this round, 0 if not, < 0 on error. */
gossip_status gossip_step(gossip_ctx* ctx, gossip_round_stats* out);
/* Steps until finished or max_rounds; per_round (may be NULL) receives up to cap entries. */
gossip_status gossip_run(gossip_ctx* ctx, gossip_round_stats* per_round, uint32_t cap, uint32_t* rounds);

/* ---- rounds (vertex-partitioned, one process per GPU) --------------------- */
/* The caller owns the exchange buffers (device memory):
 *   send   n_peers*X u64, dense, indexed by global peer (X = exchange_words of gossip_get_shape)
 *   recv   world*n_local*X u64; rank p's slice for this block at offset p*n_local*X
 *   gather (optional, enables pull rounds) world*chunk*X u64, chunk = ceil(n_peers/world);
 *          needs blocks begins[p] = min(p*chunk, n_peers); rank p's new words at p*chunk*X
 * Per round:
 *   gossip_round_begin(mode)            churn, liveness, injection; returns the mode run
 *   PULL/BIN: all-gather(gather)        every rank's new words, before compute
 *   gossip_round_compute                push (writes send) or pull (reads gather)
 *   PUSH: all-to-all(send -> recv)
 *   PUSH_SPARSE: all-to-all(counts), all-to-all(records) -> gossip_round_finish_sparse
 *   gossip_round_finish                 applies recv (push); local stats, digest/covered as increments
 *   all-reduce of the stats; gossip_round_commit(global new_receipts)
 * The mode must be the same on every rank: choose it from global stats. */
#define GOSSIP_MODE_AUTO (-1) /* single partition only: the engine decides */
#define GOSSIP_MODE_PUSH 0
#define GOSSIP_MODE_PULL 1
#define GOSSIP_MODE_PUSH_SPARSE 2 /* push; only touched peers are exchanged (needs gossip_set_sparse) */
#define GOSSIP_MODE_BIN 3         /* pull semantics (same all-gather), run binned when the slot layout exists */
#define GOSSIP_MODE_BLOCKED 4     /* push semantics, propagation-blocked (single partition; chosen by the engine) */
gossip_status gossip_set_exchange(gossip_ctx* ctx, void* send_dev, void* recv_dev, uint32_t world,
                                  const uint64_t* part_begins /* world+1 */);
gossip_status gossip_set_gather(gossip_ctx* ctx, void* gather_dev);
/* Sparse push rounds: seg = device buffer of world*chunk*(1+X) u64; after
 * gossip_round_compute, destination q's records {peer, words[X]} sit at
 * seg + q*chunk*(1+X) and gossip_sparse_counts gives their numbers (the
 * staging buffer is left cleared).  The caller exchanges counts, then the
 * records, and finishes with gossip_round_finish_sparse(received records). */
gossip_status gossip_set_sparse(gossip_ctx* ctx, void* seg_dev);
gossip_status gossip_sparse_counts(gossip_ctx* ctx, uint64_t* counts /* world */);
gossip_status gossip_round_finish_sparse(gossip_ctx* ctx, const void* records_dev, uint64_t n_records,
                                         gossip_round_stats* local_out);
gossip_status gossip_round_begin(gossip_ctx* ctx, int requested_mode, int* mode);
gossip_status gossip_round_compute(gossip_ctx* ctx);
/* begin(PUSH) + compute: push-only partitioned rounds */
gossip_status gossip_round_push(gossip_ctx* ctx);
gossip_status gossip_round_finish(gossip_ctx* ctx, gossip_round_stats* local_out);
gossip_status gossip_round_commit(gossip_ctx* ctx, uint64_t global_new_receipts, int* finished);

/* ---- multi-GPU rounds driven by the library (RCCL over xGMI) --------------
 * Replaces the reference's cross-process send of a gossip message
 * (broadcastMessage peer.cpp:310-316 over TCP to another PeerNode process):
 * peers are 1D vertex-partitioned into the blocks of gossip_partition
 * (ceil(n/world) peers each) and every round exchanges the cross-block
 * frontier words with RCCL -- an all-gather of the new words in dense
 * (pull / binned) rounds, an all-to-all of staged masks (or of compacted
 * {peer, words} records) in push rounds, and one all-reduce of the stats.
 * The schedule is chosen from the previous round's GLOBAL stats, so every
 * rank runs the same one; results equal the single-partition run. */
#define GOSSIP_ECOMM (-7)           /* RCCL error */
#define GOSSIP_COMM_ID_BYTES 128    /* ncclUniqueId */
/* begins[world+1]: rank p owns peers [begins[p], begins[p+1]) -- blocks of ceil(n/world) peers */
gossip_status gossip_partition(uint64_t n_peers, uint32_t world, uint64_t* begins);
/* The same for cfg's overlay, blocks of about equal work (edges plus a per-peer share; whole 64-peer tiles):
 * the powerlaw overlay's degree mass sits at the low ids (config 4 as 8 blocks of ceil(n/8): the first holds
 * 3.2x the edges of any other).  Other overlays: gossip_partition.  gossip_group_create uses it (unless
 * GOSSIP_FLAG_UNIFORM_PARTITION); with gossip_comm_init any contiguous partition in rank order works. */
gossip_status gossip_partition_edges(const gossip_config* cfg, uint32_t world, uint64_t* begins);
/* One process per GPU: rank 0 creates the id, every rank receives it out of band. */
gossip_status gossip_comm_unique_id(uint8_t* id /* GOSSIP_COMM_ID_BYTES */);
/* Makes ctx (created with the rank's block of gossip_partition[_edges] as its part range)
 * rank `rank` of `world`: allocates the exchange buffers, joins the RCCL
 * communicator (collective: every rank calls it), after which gossip_step /
 * gossip_run issue the collectives themselves (call them in lockstep on every
 * rank).  Their stats are global; seed_removals are filled in by
 * gossip_comm_finalize.  Reads (gossip_read_*) stay per block. */
gossip_status gossip_comm_init(gossip_ctx* ctx, const uint8_t* id, uint32_t world, uint32_t rank);
/* Collective, after a run: gathers every rank's dead-node reports (sorted by
 * (round, reporter, dead); reports may be NULL) and sets per_round[i].seed_removals
 * (the registry drops a peer on its first report, SeedNode::handleDeadNode seed.cpp:158-167). */
gossip_status gossip_comm_finalize(gossip_ctx* ctx, gossip_round_stats* per_round, uint32_t rounds,
                                   gossip_dead_report* reports, uint64_t cap, uint64_t* count);
/* Exchange mode of every round run since the last reset (GOSSIP_MODE_*). */
gossip_status gossip_comm_modes(gossip_ctx* ctx, int32_t* modes, uint32_t cap, uint32_t* n);

/* One process, several GPUs (one ctx per part; RCCL communicators from
 * ncclCommInitAll).  devices[p] is part p's device; when every part names the
 * same device the parts exchange by device copies instead (a single-GPU
 * rehearsal of the partitioned path).  The group's calls drive all parts. */
typedef struct gossip_group gossip_group;
gossip_status gossip_group_create(const gossip_config* cfg, uint32_t n_parts, const int32_t* devices,
                                  gossip_group** out);
/* The same with the caller's partition: begins[0] = 0 < begins[1] < ... < begins[n_parts] = n_peers, every
 * block starting on a whole 64-peer tile (gossip_group_create: gossip_partition_edges; blocks of ceil(n/parts)
 * rounded up to whole tiles for other overlays, under GOSSIP_FLAG_UNIFORM_PARTITION, or when n_peers < 64 parts
 * -- GOSSIP_EINVAL if that leaves a part empty). */
gossip_status gossip_group_create_parts(const gossip_config* cfg, uint32_t n_parts, const int32_t* devices,
                                        const uint64_t* begins, gossip_group** out);
void gossip_group_destroy(gossip_group* g);
gossip_status gossip_group_part(gossip_group* g, uint32_t p, gossip_ctx** ctx);
gossip_status gossip_group_build_graph(gossip_group* g);
gossip_status gossip_group_inject(gossip_group* g, const uint32_t* origin, const uint32_t* inject_round,
                                  uint32_t n_msgs);
gossip_status gossip_group_schedule_kills(gossip_group* g, const uint32_t* kill_peer, const uint32_t* kill_round,
                                          uint32_t n_kills);
gossip_status gossip_group_reset(gossip_group* g);
/* one round on every part; 1 when finished, 0 if not, < 0 on error (seed_removals: 0 until the run ends) */
gossip_status gossip_group_step(gossip_group* g, gossip_round_stats* out);
/* steps until finished; per_round gets global stats with seed_removals */
gossip_status gossip_group_run(gossip_group* g, gossip_round_stats* per_round, uint32_t cap, uint32_t* rounds);
/* seen words of all n_peers peers (n_peers * W) */
gossip_status gossip_group_read_seen(gossip_group* g, uint64_t* host_seen);
/* every part's reports, merged and sorted by (round, reporter, dead) */
gossip_status gossip_group_read_reports(gossip_group* g, gossip_dead_report* buf, uint64_t cap, uint64_t* count);

/* ---- results ------------------------------------------------------------- */
/* Owned seen words (n_local * W): bit m of peer v = v's Message-List holds m (peer.hpp:52). */
gossip_status gossip_read_seen(gossip_ctx* ctx, uint64_t* host_seen);
/* Per-message coverage over owned peers (M counts). */
gossip_status gossip_read_coverage(gossip_ctx* ctx, uint64_t* counts);
/* Per-message coverage at push start of every executed round ([rounds][M]);
 * needs GOSSIP_FLAG_COVERAGE_HISTORY. */
gossip_status gossip_read_coverage_history(gossip_ctx* ctx, uint64_t* buf, uint32_t max_rounds, uint32_t* rounds);
/* Dead-node reports sorted by (round, reporter, dead). */
gossip_status gossip_read_reports(gossip_ctx* ctx, gossip_dead_report* buf, uint64_t cap, uint64_t* count);
/* Alive flags of all n_peers peers (1 byte each). */
gossip_status gossip_read_alive(gossip_ctx* ctx, uint8_t* out);
/* Seed-registry membership of all n_peers peers (seed.cpp peerList; 1 byte each). */
gossip_status gossip_read_registered(gossip_ctx* ctx, uint8_t* out);

/* ---- measurement ----------------------------------------------------------- */
/* Per-kernel device time (ms) accumulated since timing was last enabled, by kernel name
 * ("push_light", "push_heavy", "pull_light", "pull_heavy", "frontier_bits", "bin_scatter", "bin_apply",
 * "pb_scatter", "pb_split", "pb_apply", "liveness", "churn", "kills", "inject", "apply_remote"),
 * measured with HIP events on the ctx stream.  enable != 0 turns timing on. */
gossip_status gossip_enable_timing(gossip_ctx* ctx, int enable);
gossip_status gossip_kernel_time(gossip_ctx* ctx, const char* kernel, double* ms, uint64_t* launches);
/* Algorithmic HBM bytes of the same kernels over the same
 * interval: push = 32 B per frontier peer + 20 B per edge traversal (light
 * rows to "push_light", heavy rows to "push_heavy"); liveness = 6.125 B per
 * live edge checked; pull = 40 B per owned peer + 4 B per edge scanned + 8 B
 * per neighbour word gathered ("pull_light"), 12 B per heavy-row edge scanned
 * ("pull_heavy"), 8.125 B per owned peer ("frontier_bits"); binned rounds:
 * 8·Wp B per source word staged + 16 B per frontier peer + 6 B per binned edge
 * + 8·Wp B per slot written ("bin_scatter"), (2 + 8·Wp) B per slot scanned +
 * 16·Wp B per owned peer ("bin_apply"); propagation-blocked rounds: 8 B per owned
 * peer + 24 B per frontier peer + 16 B per traversal ("pb_scatter"), 22 B per
 * traversal ("pb_split"), 10 B per traversal + 24 B per activated peer
 * ("pb_apply"). */
gossip_status gossip_kernel_bytes(gossip_ctx* ctx, const char* kernel, double* bytes);

/* ---- engineering options ---------------------------------------------------- */
/* Parity-tested A/B variants and layout sizes of one ctx (never read from the
 * environment; results are identical under every setting).  Keys: "tiny" (0:
 * small overlays run round by round), "full_liveness" (ping every edge instead
 * of the closed form), "defer_permille" (-1 auto), "bin_stream" (the binned
 * layout: -1 / 1 streamed, the default; 0 the slot layout), "pull_first2", "in_flight", "heavy_exit", "heavy_degree"
 * (layout: rows longer than this are heavy; -1 auto, 256, or 512 on overlays of >= 2^27 peers)
 * (layout), "heavy_chunk", "bin_front_permille", "bin_words", "bin_chunk", "val_tune"
 * (-1 auto, 0, 1, 2 = print), "src_stats" (who books a binned round's source
 * side: -1 auto = 1 the scatter, 0 the apply), "blocked_bin_slots"
 * (slot-array size from which dense rounds below blocked_permille run
 * blocked; -1 default 2^28), "blocked_direct_in" (layout: leading 64-peer
 * tiles of more in-degree take direct deliveries; -1 default 2^18),
 * "blocked_push_permille" (push rounds from this frontier per-mille run
 * blocked on overlays of >= 2^26 peers; -1 default 10), "list_rounds" (0: no
 * needy-list rounds), "list_cap" (layout of the needy lists: rows per list;
 * 0 = max(n/16, 65536)), "pull_step" (neighbour words a row pull gathers
 * per row per step: 1 default, or 2; other values GOSSIP_EINVAL),
 * "gather_permille" (partitioned runs, read from each driver's first part:
 * dense rounds whose frontier is below this per-mille of the peers exchange
 * a tile bitmap and the packed non-zero new words instead of every word;
 * -1 default 600, 0 never, 1000 always), "bin_needy_skip" (binned rounds
 * with over one missing pair per peer skip the apply's per-bin needy test:
 * 1 default, 0 always test), "apply_pipe" (the streamed apply's load
 * pipeline shape, 0-10, A/B; default 5), "blocked_pipe" (1 default: the
 * blocked rounds' level-2 and apply record loops keep the next batch's loads
 * in flight; 0 the unpipelined loops), "zero_fill" (1 default: the reset
 * clears the seen and new-word arrays with the runtime's fill; 0 the
 * library's own 16-B store kernel), "apply_persist" (1 default: the
 * streamed apply runs as resident workgroups taking bins from per-XCD
 * counters; 0: one workgroup per bin), "replay" (0: gossip_run never replays a
 * recorded schedule), "scatter_direct" (partitioned runs: a block's binned
 * scatter reads other blocks' source words from the gather buffer instead of
 * staging them; 0 default), "apply_probe" (diagnostics: 1 clocks the
 * streamed apply's phases per bin; gossip_kernel_bytes "#probe_src",
 * "#probe_init", "#probe_slots", "#probe_finish" give 100 MHz ticks summed
 * over bins, "#probe_bins" and "#probe_slots_n" the bins and slots,
 * "#probe_block" and "#probe_blocks" the workgroups' lifetimes and count;
 * 0 off), "scatter_small" (the streamed scatter's 4096-word, 256-thread
 * instance where chunks fit it; 0 default), "scatter_units" (layout: split
 * chunks into at least this many scatter units; 0 default),
 * "scatter_split_direct" (a split chunk's later units read their words
 * instead of staging them; 0 default), "apply_wide" (small bins applied by
 * 16-wave workgroups; 0 default), "exchange_stages" (partitioned binned
 * rounds: the all-gather in this many stages under the scatter, 1-16; 4
 * default), "px_per100k" / "px_permille" (partitioned sparse push rounds
 * from this frontier per 100 000 / per 1000 of the block send records made
 * by the record push, below it records appended by the push; -1 never; 5
 * per 100 000 default), "row_queue" (128 default or 256: the row pull's
 * queue entries per wave), "row_grid" (the row pull's workgroups; 0 default:
 * those resident at once), "blocked_marks" (1 default: a narrow blocked
 * round -- under 5 % frontier, after a round that kept its tile marks -- reads
 * the new words of marked tiles only in level 1; 0: every tile),
 * "heavy_side" (1 default: at P = 1 a binned round's heavy-row pull runs on a
 * second stream beside the scatter and k_heavy_commit applies its finds after
 * the apply; 0: the pull after the apply), "blocked_clear_all" (1 default: wide blocked rounds clear every new word in
 * level 2; 0: level 1 clears the words it consumes).
 * Layout keys
 * apply at the next gossip_build_graph / gossip_load_csr ("list_cap": at the
 * next chain of needy-list rounds, never inside one).  GOSSIP_EINVAL: unknown key. */
gossip_status gossip_set_tuning(gossip_ctx* ctx, const char* key, int64_t value);

#ifdef __cplusplus
}
#endif
#endif
