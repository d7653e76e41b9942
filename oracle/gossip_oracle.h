/*
 * gossip_oracle.h -- CPU restatement of the reference's gossip hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libgossip_hip, the C++
 * drop-in surface, the Python host package) may include, link or load this.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the timed CPU baseline.
 *
 * The reference (PareenShah27/P2P-GossipProtocol @ 2025-02-25) compiles here
 * from its sources with the image's nlohmann/json 3.1.1 (oracle/Makefile ref;
 * its own Makefile is broken, F1), but its hot path cannot run: a peer stops
 * at its first receipt (peer.cpp:280->283->126, F3, observed in
 * tests/golden/ref_wire.json).  So this file restates the *intended*
 * semantics of peer.cpp as the deterministic round model of DESIGN.md
 * section 2 ("round contract").  Each function cites the reference lines it
 * follows.
 *
 * Parity pinning: Philox4x32-10 is pinned by the Random123 KATs
 * (tests/golden/philox_kat.json); the ref_bootstrap generator by the
 * structural known answer F8 (out-edges of peer i are a subset of {0..i-1});
 * the round driver by hand graphs with analytically known per-round counts
 * (tests/golden/hand_graphs.json) and by two independent drivers
 * (literal message-list driver vs 64-bit-mask driver) that must agree.
 * The NetworkConfig restatement is pinned against the real reference
 * config.cpp compiled into oracle/_ref/ (tests/golden/config_cases.json);
 * the seed registry and the wire and log formats of the surface against the
 * reference's seed.cpp / peer.cpp / info.hpp run here (tests/golden/
 * ref_wire.json).
 */
#ifndef GOSSIP_ORACLE_H
#define GOSSIP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Philox4x32-10 (Salmon et al. SC'11; Random123 constants) ---------- */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* Counter "purpose" words (ctr[0]); key = {rng_seed, peer}.  Must match
 * DESIGN.md section 3 and include/gossip/philox.h. */
enum {
    ORACLE_P_DEGREE = 1,  /* ctr {1, response, 0, 0}.x  -> k draw (peer.cpp:220-222) */
    ORACLE_P_TARGET = 2,  /* ctr {2, response, i>>2, 0}[i&3] -> candidate i (powerlaw) */
    ORACLE_P_SHUFFLE = 3, /* ctr {3, response, d>>2, 0}[d&3] -> Fisher-Yates draw d (peer.cpp:224-225) */
    ORACLE_P_CHURN = 4,   /* key {seed, v >> 2}, ctr {4, round, 0, 0}, lane v & 3 -> peer v dies if < churn_threshold */
    ORACLE_P_ORIGIN = 5,  /* key {seed, 0xFFFFFFFF}, ctr {5, k, attempt, 0}.x -> origin k */
    ORACLE_P_REBOOT = 6,  /* ctr {6, round, dead, 0}.x -> k draw; ctr {6, round, dead, 1+(i>>2)}[i&3] -> candidate i */
    ORACLE_P_REJOIN = 7   /* ctr {7, round, 0, 0}.x -> a dead peer restarts if < rejoin_threshold, .y -> k draw;
                             ctr {7, round, 1+(i>>2), 0}[i&3] -> candidate i */
};

/* Integer threshold for the reference's power-law pick
 *   numPeers = floor(L * U^(1/2.5))          (peer.cpp:219-222)
 * k >= j  <=>  x >= thr(j, L) = ceil(2^32 * (j/L)^2.5), computed exactly
 * (smallest x with x^2 * L^5 >= 2^64 * j^5).  Valid for 1 <= j < L <= 4096.
 * Returns 0xFFFFFFFF... as uint64 2^32 when j >= L. */
uint64_t oracle_threshold(uint32_t j, uint32_t L);

/* Skewed candidate pick for the scale overlay: c = floor(n * V^3) with
 * V = x / 2^32, computed by truncating 64-bit integer products.  Gives
 * Chung-Lu weights w_c ~ c^(-2/3), i.e. a degree power law with exponent
 * 2.5 (the reference's alpha, peer.cpp:219). */
uint32_t oracle_skew_pick(uint32_t x, uint64_t n);

/* ---- overlay generators (return malloc'd CSR; free with oracle_free) --- */
/* ref_bootstrap: the literal F8 bootstrap.  Peer i registers in arrival
 * order with seeds 0..q-1, q = n_seeds/2+1 (peer.cpp:63-72, config.cpp:76);
 * each seed returns its whole registry {0..i} (seed.cpp:117-125);
 * selectAndConnectPeers (peer.cpp:214-253) picks k by the power law,
 * Fisher-Yates shuffles, takes the first k, skips self.  Directed edges
 * i->c; union over responses.  n <= 4096. */
int oracle_gen_ref_bootstrap(uint32_t n, uint32_t n_seeds, uint32_t seed,
                             uint64_t** row_ptr, uint32_t** col, uint64_t* n_edges);
/* powerlaw: per peer one response of list_len i.i.d. skewed candidates,
 * k by the power law, skip self, symmetrised, deduplicated, rows sorted. */
int oracle_gen_powerlaw(uint64_t n, uint32_t list_len, uint32_t seed, int threads,
                        uint64_t** row_ptr, uint32_t** col, uint64_t* n_edges);
/* Philox-chosen distinct origins (used by configs 2-5). */
void oracle_pick_origins(uint64_t n, uint32_t seed, uint32_t count, uint32_t* out);
/* F10 (peer.cpp:186-210,62-78): peers of the literal bootstrap that start when
 * a peer reads at most list_cap bytes of a seed's peer_list (0 = no cap) */
uint64_t oracle_started_under_cap(uint64_t n, uint32_t list_cap);
void oracle_free(void* p);

/* ---- digest weight g(i) ------------------------- */
uint64_t oracle_digest_weight(uint64_t idx);
/* fixture checksums: sum_i g(i) * x[i] mod 2^64 (OpenMP) */
uint64_t oracle_hash_u64(const uint64_t* x, uint64_t n, int threads);
uint64_t oracle_hash_u32(const uint32_t* x, uint64_t n, int threads);
uint64_t oracle_hash_u8(const uint8_t* x, uint64_t n, int threads);

/* ---- round driver ------------------------------------------------------ */
typedef struct oracle_stats {
    uint32_t round;
    uint32_t flags;         /* bit0: ping round */
    uint64_t frontier;      /* |F_r| at push start */
    uint64_t traversals;    /* live out-edges scanned from F_r */
    uint64_t deliveries;    /* sum popcount(new[u]) over traversed edges, alive target */
    uint64_t undelivered;   /* same, dead target (send attempted, not delivered) */
    uint64_t new_receipts;  /* bits newly set in seen this round */
    uint64_t duplicates;    /* deliveries - new_receipts */
    uint64_t injected;      /* messages injected this round */
    uint64_t died;          /* peers that died this round */
    uint64_t reports;       /* dead-node reports emitted this round */
    uint64_t seed_removals; /* registry entries removed this round */
    uint64_t digest;        /* sum g(v*W+w) * seen[v][w] mod 2^64 at push start */
    uint64_t covered;       /* sum popcount(seen) at push start */
    uint64_t reconnects;    /* out-edges added by re-bootstrap this round (extra_cap > 0) */
    uint64_t rejoined;      /* dead peers restarted this round (rejoin_threshold > 0) */
} oracle_stats;

typedef struct oracle_report {
    uint32_t round, reporter, dead;
} oracle_report;

typedef struct oracle_sim_cfg {
    uint64_t n;
    uint32_t n_msgs;           /* M; words per peer W = ceil(M/64) */
    uint32_t seed;             /* rng_seed (churn) */
    uint32_t churn_threshold;  /* 0 = no churn; peer dies if philox.x < thr */
    uint32_t ping_every;       /* 0 = no liveness */
    uint32_t max_missed;       /* max_missed_pings (peer.cpp:337) */
    uint32_t max_rounds;
    uint32_t min_rounds;
    int threads;               /* fast driver OpenMP threads */
    int variant;               /* 0 fast (mask), 1 literal (message lists) */
    uint32_t extra_cap;        /* re-bootstrap after a death: up to this many extra out-edges per peer (0 = off) */
    uint32_t list_len;         /* re-bootstrap: candidates per seed response (powerlaw list_len) */
    uint64_t n_started;        /* peers >= n_started never start (failed registration, F10); 0 = all start */
    uint32_t rejoin_threshold; /* join churn: a dead peer restarts in round r if philox < threshold; 0 = never */
    uint32_t pad0;
} oracle_sim_cfg;

typedef struct oracle_sim oracle_sim;

oracle_sim* oracle_sim_create(const oracle_sim_cfg* cfg, const uint64_t* row_ptr, const uint32_t* col);
void oracle_sim_destroy(oracle_sim* s);
/* message m: origin[m], inject_round[m]; kills: peer kill_peer[i] dies at kill_round[i] */
int oracle_sim_schedule(oracle_sim* s, const uint32_t* origin, const uint32_t* inject_round,
                        uint32_t n_kills, const uint32_t* kill_peer, const uint32_t* kill_round);
/* one round; returns 1 if the run is finished after this round, 0 if not, <0 on error */
int oracle_sim_step(oracle_sim* s, oracle_stats* out);
/* runs to termination; per_round may be NULL; returns rounds executed */
int oracle_sim_run(oracle_sim* s, oracle_stats* per_round, uint32_t cap);
void oracle_sim_seen(const oracle_sim* s, uint64_t* out);          /* n*W words */
void oracle_sim_coverage(const oracle_sim* s, uint64_t* out);      /* M counts (current) */
uint64_t oracle_sim_reports(const oracle_sim* s, oracle_report* buf, uint64_t cap); /* sorted (round,u,v) */
void oracle_sim_alive(const oracle_sim* s, uint8_t* out);          /* n bytes */
void oracle_sim_extra(const oracle_sim* s, uint32_t* counts, uint32_t* cols); /* n, n*extra_cap */
void oracle_sim_registered(const oracle_sim* s, uint8_t* out);     /* n bytes */
uint64_t oracle_sim_sent_to_total(const oracle_sim* s);             /* literal variant: sum sentTo */

/* ---- partition emulation (multi-rank driver tests on CPU) --------------- */
/* One block [b, e) of a 1D partition: row_ptr is local (e-b+1 entries),
 * col holds global ids.  Per round: part_push(send) -> exchange ->
 * part_finish(recv) -> sum of the ranks' stats -> part_commit(global fresh).
 * part_finish's digest/covered are per-round increments. */
typedef struct oracle_part oracle_part;
oracle_part* oracle_part_create(const oracle_sim_cfg* cfg, uint64_t b, uint64_t e, const uint64_t* row_ptr,
                                const uint32_t* col);
void oracle_part_destroy(oracle_part* p);
int oracle_part_schedule(oracle_part* p, const uint32_t* origin, const uint32_t* inject_round, uint32_t n_kills,
                         const uint32_t* kill_peer, const uint32_t* kill_round);
int oracle_part_push(oracle_part* p, uint64_t* send);   /* begin(push) + push_compute */
int oracle_part_begin(oracle_part* p, int requested_pull); /* returns 1 if this round pulls */
void oracle_part_publish(oracle_part* p, uint64_t* gather);
int oracle_part_pull(oracle_part* p, const uint64_t* gather);
int oracle_part_push_compute(oracle_part* p, uint64_t* send);
void oracle_part_compact(oracle_part* p, uint64_t* send, uint64_t chunk, uint32_t world, uint64_t* seg,
                         uint64_t* counts);
int oracle_part_finish_records(oracle_part* p, const uint64_t* rec, uint64_t n_rec, oracle_stats* out);
int oracle_part_finish(oracle_part* p, const uint64_t* recv, uint32_t world, oracle_stats* out);
int oracle_part_commit(oracle_part* p, uint64_t global_new_receipts);
void oracle_part_reset(oracle_part* p);
void oracle_part_seen(const oracle_part* p, uint64_t* out);
uint64_t oracle_part_reports(const oracle_part* p, oracle_report* buf, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
