/*
 * gossip_oracle.c -- CPU restatement of the reference gossip hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see gossip_oracle.h).  Never linked into the
 * product.  Restates the intended semantics of:
 *   peer.cpp:214-253  selectAndConnectPeers   (overlay construction)
 *   peer.cpp:255-295  handleClient            (receive + Message-List dedup)
 *   peer.cpp:297-318  broadcastMessage        (push to every out-neighbour; F9)
 *   peer.cpp:320-355  pingLoop                (miss counters, 3 misses -> dead)
 *   peer.cpp:357-379  messageGenerationLoop   (origination)
 *   peer.cpp:381-405  handleDeadPeer          (drop edge)
 *   seed.cpp:130-138,158-167 handleDeadNode   (registry removal on report)
 * as the deterministic round model of DESIGN.md section 2.
 */
#include "gossip_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ */
/* Philox4x32-10                                                            */
/* ------------------------------------------------------------------------ */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline uint32_t philox_x(uint32_t seed, uint32_t peer, uint32_t a, uint32_t b, uint32_t c,
                                uint32_t d, int lane) {
    uint32_t ctr[4] = {a, b, c, d}, key[2] = {seed, peer}, out[4];
    oracle_philox4x32_10(ctr, key, out);
    return out[lane];
}

/* ------------------------------------------------------------------------ */
/* Power-law pick thresholds (peer.cpp:219-222)                             */
/* ------------------------------------------------------------------------ */
static int thr_ok(uint64_t x, uint32_t j, uint32_t L) {
    u128 l5 = (u128)L * L * L * L * L;
    u128 j5 = (u128)j * j * j * j * j;
    return (u128)x * x * l5 >= (j5 << 64);
}

uint64_t oracle_threshold(uint32_t j, uint32_t L) {
    if (j >= L) return (uint64_t)1 << 32;
    if (j == 0) return 0;
    double est = ldexp(pow((double)j / (double)L, 2.5), 32);
    uint64_t x = (uint64_t)ceil(est);
    if (x > ((uint64_t)1 << 32)) x = (uint64_t)1 << 32;
    while (x > 0 && thr_ok(x - 1, j, L)) --x;
    while (!thr_ok(x, j, L)) ++x;
    return x;
}

/* k = floor(L * U^(1/2.5)) with U = x/2^32, via the exact thresholds. */
static uint32_t pick_count(uint32_t x, uint32_t L, const uint64_t* thr) {
    uint32_t k = 0;
    for (uint32_t j = 1; j < L; ++j) k += ((uint64_t)x >= thr[j]);
    return k;
}

uint32_t oracle_skew_pick(uint32_t x, uint64_t n) {
    uint64_t a = ((uint64_t)x * x) >> 32;
    uint64_t b = (a * x) >> 32;
    return (uint32_t)((n * b) >> 32);
}

uint64_t oracle_digest_weight(uint64_t idx) {
    uint64_t z = (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z | 1ull;
}

void oracle_free(void* p) { free(p); }

/* Fixture checksums (tests/golden/make_fullsize_golden.py): sum_i g(i) * x[i]
 * mod 2^64 with the digest weights, so order and position matter. */
uint64_t oracle_hash_u64(const uint64_t* x, uint64_t n, int threads) {
    uint64_t h = 0;
    if (threads <= 0) threads = 1;
#pragma omp parallel for reduction(+ : h) schedule(static, 1 << 16) num_threads(threads)
    for (int64_t i = 0; i < (int64_t)n; ++i) h += oracle_digest_weight((uint64_t)i) * x[i];
    return h;
}

uint64_t oracle_hash_u32(const uint32_t* x, uint64_t n, int threads) {
    uint64_t h = 0;
    if (threads <= 0) threads = 1;
#pragma omp parallel for reduction(+ : h) schedule(static, 1 << 16) num_threads(threads)
    for (int64_t i = 0; i < (int64_t)n; ++i) h += oracle_digest_weight((uint64_t)i) * x[i];
    return h;
}

uint64_t oracle_hash_u8(const uint8_t* x, uint64_t n, int threads) {
    uint64_t h = 0;
    if (threads <= 0) threads = 1;
#pragma omp parallel for reduction(+ : h) schedule(static, 1 << 16) num_threads(threads)
    for (int64_t i = 0; i < (int64_t)n; ++i) h += oracle_digest_weight((uint64_t)i) * x[i];
    return h;
}

/* ------------------------------------------------------------------------ */
/* CSR assembly: sort rows, drop duplicates and self loops                  */
/* ------------------------------------------------------------------------ */
static int cmp_u32(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return (x > y) - (x < y);
}

static void sort_row(uint32_t* a, uint64_t len) {
    if (len < 32) {
        for (uint64_t i = 1; i < len; ++i) {
            uint32_t v = a[i];
            uint64_t j = i;
            while (j > 0 && a[j - 1] > v) { a[j] = a[j - 1]; --j; }
            a[j] = v;
        }
    } else {
        qsort(a, len, sizeof(uint32_t), cmp_u32);
    }
}

/* raw rows [rp_raw[v], rp_raw[v+1]) of col_raw -> sorted unique CSR without self loops */
static int finish_csr(uint64_t n, uint64_t* rp_raw, uint32_t* col_raw, int threads,
                      uint64_t** row_ptr, uint32_t** col, uint64_t* n_edges) {
    (void)threads;
    uint64_t* cnt = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    if (!cnt) return -1;
#pragma omp parallel for schedule(dynamic, 1024) num_threads(threads)
    for (int64_t v = 0; v < (int64_t)n; ++v) {
        uint32_t* a = col_raw + rp_raw[v];
        uint64_t len = rp_raw[v + 1] - rp_raw[v];
        sort_row(a, len);
        uint64_t m = 0;
        for (uint64_t i = 0; i < len; ++i) {
            if (a[i] == (uint32_t)v) continue;
            if (m > 0 && a[m - 1] == a[i]) continue;
            a[m++] = a[i];
        }
        cnt[v] = m;
    }
    uint64_t* rp = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    if (!rp) { free(cnt); return -1; }
    rp[0] = 0;
    for (uint64_t v = 0; v < n; ++v) rp[v + 1] = rp[v] + cnt[v];
    uint32_t* c = (uint32_t*)malloc((rp[n] ? rp[n] : 1) * sizeof(uint32_t));
    if (!c) { free(cnt); free(rp); return -1; }
#pragma omp parallel for schedule(dynamic, 1024) num_threads(threads)
    for (int64_t v = 0; v < (int64_t)n; ++v)
        memcpy(c + rp[v], col_raw + rp_raw[v], cnt[v] * sizeof(uint32_t));
    free(cnt);
    *row_ptr = rp;
    *col = c;
    *n_edges = rp[n];
    return 0;
}

/* ------------------------------------------------------------------------ */
/* ref_bootstrap: literal F8 overlay (peer.cpp:63-72, 214-253; seed.cpp:117) */
/* ------------------------------------------------------------------------ */
int oracle_gen_ref_bootstrap(uint32_t n, uint32_t n_seeds, uint32_t seed, uint64_t** row_ptr,
                             uint32_t** col, uint64_t* n_edges) {
    if (n == 0 || n > 4096 || n_seeds == 0) return -1;
    uint32_t q = n_seeds / 2 + 1; /* quorum, peer.cpp:64 / config.cpp:76 */
    uint64_t cap = (uint64_t)n * n;
    uint64_t* rp_raw = (uint64_t*)calloc((size_t)n + 1, sizeof(uint64_t));
    uint32_t* col_raw = (uint32_t*)malloc(cap * sizeof(uint32_t) + 4);
    uint32_t* perm = (uint32_t*)malloc((size_t)n * sizeof(uint32_t));
    uint8_t* chosen = (uint8_t*)malloc(n);
    uint64_t* thr = (uint64_t*)malloc((size_t)(n + 1) * sizeof(uint64_t));
    if (!rp_raw || !col_raw || !perm || !chosen || !thr) return -1;
    uint64_t w = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t L = i + 1; /* registry {0..i}, self included (seed.cpp:117-122) */
        for (uint32_t j = 0; j < L; ++j) thr[j] = oracle_threshold(j, L);
        memset(chosen, 0, L);
        for (uint32_t s = 0; s < q; ++s) {
            uint32_t x = philox_x(seed, i, ORACLE_P_DEGREE, s, 0, 0, 0);
            uint32_t k = pick_count(x, L, thr);
            for (uint32_t j = 0; j < L; ++j) perm[j] = j; /* list in registration order */
            uint32_t d = 0;
            for (uint32_t idx = L - 1; idx >= 1; --idx, ++d) { /* Fisher-Yates, peer.cpp:224-225 */
                uint32_t r = philox_x(seed, i, ORACLE_P_SHUFFLE, s, d >> 2, 0, (int)(d & 3));
                uint32_t jj = (uint32_t)(((uint64_t)r * (idx + 1)) >> 32);
                uint32_t t = perm[idx]; perm[idx] = perm[jj]; perm[jj] = t;
            }
            for (uint32_t t = 0; t < k; ++t) {          /* peer.cpp:227-230 */
                uint32_t c = perm[t];
                if (c == i) continue;                    /* self still consumes a slot */
                chosen[c] = 1;                           /* peer.cpp:242 map overwrite = union */
            }
        }
        rp_raw[i] = w;
        for (uint32_t c = 0; c < L; ++c)
            if (chosen[c]) col_raw[w++] = c;
    }
    rp_raw[n] = w;
    free(perm); free(chosen); free(thr);
    int rc = finish_csr(n, rp_raw, col_raw, 1, row_ptr, col, n_edges);
    free(rp_raw); free(col_raw);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* powerlaw: scale overlay, symmetrised                                     */
/* ------------------------------------------------------------------------ */
int oracle_gen_powerlaw(uint64_t n, uint32_t list_len, uint32_t seed, int threads, uint64_t** row_ptr,
                        uint32_t** col, uint64_t* n_edges) {
    if (n < 2 || n > 0x80000000ull || list_len < 2 || list_len > 64) return -1;
    if (threads <= 0) threads = 1;
    uint64_t thr[65];
    for (uint32_t j = 0; j <= list_len; ++j) thr[j] = oracle_threshold(j, list_len);
    uint64_t* deg = (uint64_t*)calloc(n + 1, sizeof(uint64_t));
    if (!deg) return -1;
    /* pass 1: count (u->c and c->u) */
#pragma omp parallel for schedule(static, 4096) num_threads(threads)
    for (int64_t u = 0; u < (int64_t)n; ++u) {
        uint32_t x = philox_x(seed, (uint32_t)u, ORACLE_P_DEGREE, 0, 0, 0, 0);
        uint32_t k = pick_count(x, list_len, thr);
        uint64_t mine = 0;
        for (uint32_t i = 0; i < k; ++i) {
            uint32_t t = philox_x(seed, (uint32_t)u, ORACLE_P_TARGET, 0, i >> 2, 0, (int)(i & 3));
            uint32_t c = oracle_skew_pick(t, n);
            if (c == (uint32_t)u) continue;
            ++mine;
            __atomic_fetch_add(&deg[c], 1, __ATOMIC_RELAXED);
        }
        __atomic_fetch_add(&deg[u], mine, __ATOMIC_RELAXED);
    }
    uint64_t* rp_raw = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    if (!rp_raw) { free(deg); return -1; }
    rp_raw[0] = 0;
    for (uint64_t v = 0; v < n; ++v) rp_raw[v + 1] = rp_raw[v] + deg[v];
    uint32_t* col_raw = (uint32_t*)malloc((rp_raw[n] ? rp_raw[n] : 1) * sizeof(uint32_t));
    if (!col_raw) { free(deg); free(rp_raw); return -1; }
    for (uint64_t v = 0; v < n; ++v) deg[v] = rp_raw[v]; /* cursors */
#pragma omp parallel for schedule(static, 4096) num_threads(threads)
    for (int64_t u = 0; u < (int64_t)n; ++u) {
        uint32_t x = philox_x(seed, (uint32_t)u, ORACLE_P_DEGREE, 0, 0, 0, 0);
        uint32_t k = pick_count(x, list_len, thr);
        for (uint32_t i = 0; i < k; ++i) {
            uint32_t t = philox_x(seed, (uint32_t)u, ORACLE_P_TARGET, 0, i >> 2, 0, (int)(i & 3));
            uint32_t c = oracle_skew_pick(t, n);
            if (c == (uint32_t)u) continue;
            uint64_t a = __atomic_fetch_add(&deg[u], 1, __ATOMIC_RELAXED);
            col_raw[a] = c;
            uint64_t b = __atomic_fetch_add(&deg[c], 1, __ATOMIC_RELAXED);
            col_raw[b] = (uint32_t)u;
        }
    }
    free(deg);
    int rc = finish_csr(n, rp_raw, col_raw, threads, row_ptr, col, n_edges);
    free(rp_raw); free(col_raw);
    return rc;
}

void oracle_pick_origins(uint64_t n, uint32_t seed, uint32_t count, uint32_t* out) {
    for (uint32_t k = 0; k < count; ++k) {
        for (uint32_t attempt = 0;; ++attempt) {
            uint32_t x = philox_x(seed, 0xFFFFFFFFu, ORACLE_P_ORIGIN, k, attempt, 0, 0);
            uint32_t o = (uint32_t)(((uint64_t)x * n) >> 32);
            int dup = 0;
            for (uint32_t i = 0; i < k; ++i) dup |= (out[i] == o);
            if (!dup || (uint64_t)k >= n) { out[k] = o; break; }
        }
    }
}

/* F10: PeerNode::connectToSeed reads one 4 KB recv (peer.cpp:186-190) and
 * json::parse fails on a truncated peer_list (:193-207); start() needs q
 * answers (:62-78).  Peer i's list at seeds 0..q-1 is the registry {0..i} in
 * registration order -- the compact sorted-key JSON the seed sends
 * (seed.cpp:117-125) -- built here entry by entry, with the build's address
 * mapping (127.0.0.1:5000+id up to 60000 peers, else 10.a.b.c:5000+(id>>24))
 * and a 10-digit lastSeen.  The first peer whose list exceeds list_cap bytes
 * fails at every one of those seeds; seeds q..S-1 cannot make up the quorum,
 * and every later list is longer still. */
uint64_t oracle_started_under_cap(uint64_t n, uint32_t list_cap) {
    if (!list_cap) return n;
    uint64_t bytes = strlen("{\"peers\":[") + strlen("],\"type\":\"peer_list\"}");
    char e[128];
    for (uint64_t i = 0; i < n; ++i) {
        char ip[32];
        unsigned port;
        if (n <= 60000) { snprintf(ip, sizeof ip, "127.0.0.1"); port = 5000u + (unsigned)i; }
        else {
            snprintf(ip, sizeof ip, "10.%u.%u.%u", (unsigned)((i >> 16) & 255), (unsigned)((i >> 8) & 255),
                     (unsigned)(i & 255));
            port = 5000u + (unsigned)(i >> 24);
        }
        const int len = snprintf(e, sizeof e, "%s{\"ip\":\"%s\",\"lastSeen\":%lld,\"port\":%u}", i ? "," : "", ip,
                                 1740441600LL, port);
        bytes += (uint64_t)len;
        if (bytes > list_cap) return i;
    }
    return n;
}

/* ------------------------------------------------------------------------ */
/* Round driver                                                             */
/* ------------------------------------------------------------------------ */
/* literal variant: per-peer Message-List (peer.hpp:52) keyed by message id,
 * with the MessageTracker.sentTo count (peer.hpp:23-26). */
typedef struct msg_list {
    uint32_t cap, size;
    uint32_t* key;     /* 0xFFFFFFFF = empty */
    uint64_t* sent_to; /* |sentTo| per message */
} msg_list;

struct oracle_sim {
    oracle_sim_cfg cfg;
    uint64_t n, e;
    uint32_t W, M;
    const uint64_t* rp;
    const uint32_t* col;
    uint8_t* alive;
    uint8_t* registered;
    uint8_t* masked; /* per edge */
    uint8_t* miss;   /* per edge, saturating */
    uint32_t round;
    int finished;
    /* schedule */
    uint32_t* origin;
    uint32_t* inject_round;
    uint32_t n_kills;
    uint32_t* kill_peer;
    uint32_t* kill_round;
    /* reports */
    oracle_report* rep;
    uint64_t n_rep, cap_rep;
    /* re-bootstrap overflow rows: extra out-edges, K per peer */
    uint32_t K;
    uint32_t* ex_col;
    uint32_t* ex_cnt;
    uint8_t* ex_masked;
    uint8_t* ex_miss;
    uint64_t thr[65];
    uint64_t sent_lost;  /* literal variant: sentTo counts of Message-Lists dropped by a restart */
    /* fast variant */
    uint64_t *seen, *nw, *nx;
    /* literal variant */
    msg_list* lists;
    uint32_t** outbox;   /* per peer: message ids to broadcast this round */
    uint32_t* outbox_n;
    uint32_t** nextbox;
    uint32_t* nextbox_n;
};

static int ml_find(const msg_list* l, uint32_t m) {
    if (!l->cap) return -1;
    uint32_t mask = l->cap - 1, h = (m * 0x9E3779B1u) & mask;
    for (;;) {
        if (l->key[h] == 0xFFFFFFFFu) return -1;
        if (l->key[h] == m) return (int)h;
        h = (h + 1) & mask;
    }
}

static int ml_insert(msg_list* l, uint32_t m) {
    if ((l->size + 1) * 2 > l->cap) {
        uint32_t ncap = l->cap ? l->cap * 2 : 8;
        uint32_t* nk = (uint32_t*)malloc(ncap * sizeof(uint32_t));
        uint64_t* ns = (uint64_t*)calloc(ncap, sizeof(uint64_t));
        memset(nk, 0xFF, ncap * sizeof(uint32_t));
        for (uint32_t i = 0; i < l->cap; ++i) {
            if (l->key[i] == 0xFFFFFFFFu) continue;
            uint32_t h = (l->key[i] * 0x9E3779B1u) & (ncap - 1);
            while (nk[h] != 0xFFFFFFFFu) h = (h + 1) & (ncap - 1);
            nk[h] = l->key[i];
            ns[h] = l->sent_to[i];
        }
        free(l->key); free(l->sent_to);
        l->key = nk; l->sent_to = ns; l->cap = ncap;
    }
    uint32_t h = (m * 0x9E3779B1u) & (l->cap - 1);
    while (l->key[h] != 0xFFFFFFFFu) h = (h + 1) & (l->cap - 1);
    l->key[h] = m;
    l->sent_to[h] = 0;
    l->size++;
    return (int)h;
}

oracle_sim* oracle_sim_create(const oracle_sim_cfg* cfg, const uint64_t* row_ptr, const uint32_t* col) {
    if (!cfg || cfg->n == 0 || cfg->n_msgs == 0) return NULL;
    oracle_sim* s = (oracle_sim*)calloc(1, sizeof(oracle_sim));
    s->cfg = *cfg;
    if (s->cfg.threads <= 0) s->cfg.threads = 1;
    if (s->cfg.max_rounds == 0) s->cfg.max_rounds = 1u << 20;
    s->n = cfg->n;
    s->e = row_ptr[cfg->n];
    s->M = cfg->n_msgs;
    s->W = (cfg->n_msgs + 63) / 64;
    s->rp = row_ptr;
    s->col = col;
    s->alive = (uint8_t*)malloc(s->n);
    s->registered = (uint8_t*)malloc(s->n);
    memset(s->alive, 1, s->n);
    memset(s->registered, 1, s->n);
    if (cfg->n_started && cfg->n_started < s->n)  /* failed registration: registered, never alive */
        memset(s->alive + cfg->n_started, 0, s->n - cfg->n_started);
    s->masked = (uint8_t*)calloc(s->e + 1, 1);
    s->miss = (uint8_t*)calloc(s->e + 1, 1);
    s->K = cfg->extra_cap;
    if (s->K) {
        if (cfg->list_len < 2 || cfg->list_len > 64) { free(s->alive); free(s->registered); free(s->masked);
                                                        free(s->miss); free(s); return NULL; }
        s->ex_col = (uint32_t*)calloc(s->n * s->K, sizeof(uint32_t));
        s->ex_cnt = (uint32_t*)calloc(s->n, sizeof(uint32_t));
        s->ex_masked = (uint8_t*)calloc(s->n * s->K, 1);
        s->ex_miss = (uint8_t*)calloc(s->n * s->K, 1);
        for (uint32_t j = 1; j < cfg->list_len; ++j) s->thr[j] = oracle_threshold(j, cfg->list_len);
    }
    s->origin = (uint32_t*)calloc(s->M, sizeof(uint32_t));
    s->inject_round = (uint32_t*)malloc(s->M * sizeof(uint32_t));
    for (uint32_t m = 0; m < s->M; ++m) s->inject_round[m] = 0xFFFFFFFFu; /* unscheduled */
    if (cfg->variant == 0) {
        s->seen = (uint64_t*)calloc(s->n * s->W, sizeof(uint64_t));
        s->nw = (uint64_t*)calloc(s->n * s->W, sizeof(uint64_t));
        s->nx = (uint64_t*)calloc(s->n * s->W, sizeof(uint64_t));
    } else {
        s->lists = (msg_list*)calloc(s->n, sizeof(msg_list));
        s->outbox = (uint32_t**)calloc(s->n, sizeof(uint32_t*));
        s->nextbox = (uint32_t**)calloc(s->n, sizeof(uint32_t*));
        s->outbox_n = (uint32_t*)calloc(s->n, sizeof(uint32_t));
        s->nextbox_n = (uint32_t*)calloc(s->n, sizeof(uint32_t));
        for (uint64_t v = 0; v < s->n; ++v) {
            s->outbox[v] = (uint32_t*)malloc(s->M * sizeof(uint32_t));
            s->nextbox[v] = (uint32_t*)malloc(s->M * sizeof(uint32_t));
        }
    }
    return s;
}

void oracle_sim_destroy(oracle_sim* s) {
    if (!s) return;
    free(s->alive); free(s->registered); free(s->masked); free(s->miss);
    free(s->origin); free(s->inject_round); free(s->kill_peer); free(s->kill_round);
    free(s->rep); free(s->seen); free(s->nw); free(s->nx);
    free(s->ex_col); free(s->ex_cnt); free(s->ex_masked); free(s->ex_miss);
    if (s->lists) {
        for (uint64_t v = 0; v < s->n; ++v) {
            free(s->lists[v].key); free(s->lists[v].sent_to);
            free(s->outbox[v]); free(s->nextbox[v]);
        }
        free(s->lists); free(s->outbox); free(s->nextbox); free(s->outbox_n); free(s->nextbox_n);
    }
    free(s);
}

int oracle_sim_schedule(oracle_sim* s, const uint32_t* origin, const uint32_t* inject_round, uint32_t n_kills,
                        const uint32_t* kill_peer, const uint32_t* kill_round) {
    for (uint32_t m = 0; m < s->M; ++m) {
        if (origin[m] >= s->n) return -1;
        s->origin[m] = origin[m];
        s->inject_round[m] = inject_round[m];
    }
    free(s->kill_peer); free(s->kill_round);
    s->n_kills = n_kills;
    s->kill_peer = (uint32_t*)malloc((n_kills + 1) * sizeof(uint32_t));
    s->kill_round = (uint32_t*)malloc((n_kills + 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < n_kills; ++i) {
        if (kill_peer[i] >= s->n) return -1;
        s->kill_peer[i] = kill_peer[i];
        s->kill_round[i] = kill_round[i];
    }
    return 0;
}

static int cmp_rep(const void* a, const void* b) {
    const oracle_report* x = (const oracle_report*)a;
    const oracle_report* y = (const oracle_report*)b;
    if (x->round != y->round) return x->round < y->round ? -1 : 1;
    if (x->reporter != y->reporter) return x->reporter < y->reporter ? -1 : 1;
    if (x->dead != y->dead) return x->dead < y->dead ? -1 : 1;
    return 0;
}

static void push_report(oracle_sim* s, uint32_t r, uint32_t u, uint32_t v) {
    if (s->n_rep == s->cap_rep) {
        s->cap_rep = s->cap_rep ? s->cap_rep * 2 : 1024;
        s->rep = (oracle_report*)realloc(s->rep, s->cap_rep * sizeof(oracle_report));
    }
    s->rep[s->n_rep].round = r;
    s->rep[s->n_rep].reporter = u;
    s->rep[s->n_rep].dead = v;
    s->n_rep++;
}

static int has_bit_fast(const oracle_sim* s, uint64_t v, uint32_t m) {
    return (int)((s->seen[v * s->W + (m >> 6)] >> (m & 63)) & 1u);
}

/* Join churn (the reference has no rejoin path): a peer
 * dead at the start of round r restarts at the same address -- PeerNode::start
 * again (peer.cpp:28-101): it re-registers with the seeds (seed.cpp:153-156),
 * its Message-List is empty and its old connections are gone (its row is
 * dropped), and it selects fresh out-edges from one seed response into its
 * overflow row (extra_cap > 0; none otherwise).  Edges other peers still hold
 * to its address deliver again; edges they already dropped stay dropped. */
static int has_out_edge(const oracle_sim* s, uint32_t u, uint32_t c);

static uint32_t* do_rejoin(oracle_sim* s, uint32_t r, uint64_t* n_rj) {
    *n_rj = 0;
    if (!s->cfg.rejoin_threshold) return NULL;
    const uint64_t n_boot = s->cfg.n_started && s->cfg.n_started < s->n ? s->cfg.n_started : s->n;
    uint32_t* list = NULL;
    uint64_t cap = 0;
    for (uint64_t v = 0; v < n_boot; ++v) {
        if (s->alive[v]) continue;
        if (philox_x(s->cfg.seed, (uint32_t)v, ORACLE_P_REJOIN, r, 0, 0, 0) >= s->cfg.rejoin_threshold) continue;
        if (*n_rj == cap) { cap = cap ? 2 * cap : 256; list = (uint32_t*)realloc(list, cap * sizeof(uint32_t)); }
        list[(*n_rj)++] = (uint32_t)v;
        s->alive[v] = 1;
        s->registered[v] = 1;
        if (s->cfg.variant == 0) {
            memset(s->seen + v * s->W, 0, s->W * sizeof(uint64_t));
            memset(s->nw + v * s->W, 0, s->W * sizeof(uint64_t));
        } else {
            msg_list* l = &s->lists[v];
            for (uint32_t i = 0; i < l->cap; ++i)
                if (l->key[i] != 0xFFFFFFFFu) { s->sent_lost += l->sent_to[i]; l->key[i] = 0xFFFFFFFFu; }
            l->size = 0;
            s->outbox_n[v] = 0;
        }
        for (uint64_t e = s->rp[v]; e < s->rp[v + 1]; ++e) s->masked[e] = 1;
        if (s->K) s->ex_cnt[v] = 0;
    }
    return list;
}

/* the restarted peers' selectAndConnectPeers (peer.cpp:214-253), after the
 * round's deaths: one response of L candidates keyed by the round; self, dead
 * and repeated candidates are skipped, at most K kept */
static void rejoin_select(oracle_sim* s, uint32_t r, const uint32_t* list, uint64_t n_rj, oracle_stats* st) {
    if (!s->K) return;
    const uint32_t L = s->cfg.list_len;
    for (uint64_t j = 0; j < n_rj; ++j) {
        const uint32_t v = list[j];
        if (!s->alive[v]) continue;  /* died again in the same round */
        const uint32_t k = pick_count(philox_x(s->cfg.seed, v, ORACLE_P_REJOIN, r, 0, 0, 1), L, s->thr);
        for (uint32_t i = 0; i < k; ++i) {
            const uint32_t c = oracle_skew_pick(philox_x(s->cfg.seed, v, ORACLE_P_REJOIN, r, 1 + (i >> 2), 0, i & 3), s->n);
            if (c == v || !s->alive[c] || has_out_edge(s, v, c) || s->ex_cnt[v] >= s->K) continue;
            const uint64_t slot = (uint64_t)v * s->K + s->ex_cnt[v]++;
            s->ex_col[slot] = c;
            s->ex_masked[slot] = 0;
            s->ex_miss[slot] = 0;
            st->reconnects++;
        }
    }
}

/* step 1: churn (A11) + kill list -- a dead peer stops receiving, forwarding, pinging */
static uint64_t do_churn(oracle_sim* s, uint32_t r) {
    uint64_t died = 0;
    for (uint32_t i = 0; i < s->n_kills; ++i) {
        uint32_t v = s->kill_peer[i];
        if (s->kill_round[i] == r && s->alive[v]) {
            s->alive[v] = 0;
            ++died;
        }
    }
    if (s->cfg.churn_threshold) {
        for (uint64_t v = 0; v < s->n; ++v) {
            if (!s->alive[v]) continue;
            uint32_t x = philox_x(s->cfg.seed, (uint32_t)(v >> 2), ORACLE_P_CHURN, r, 0, 0, (int)(v & 3));
            if (x < s->cfg.churn_threshold) { s->alive[v] = 0; ++died; }
        }
    }
    if (died) {
        for (uint64_t v = 0; v < s->n; ++v) {
            if (s->alive[v]) continue;
            if (s->cfg.variant == 0) memset(s->nw + v * s->W, 0, s->W * sizeof(uint64_t));
            else s->outbox_n[v] = 0;
        }
    }
    return died;
}

/* one ping of an out-edge (pingLoop peer.cpp:328-346); returns 1 when the
 * edge is dropped (handleDeadPeer :383-397) and reported to the seeds (:158-167) */
static int ping_one(oracle_sim* s, uint32_t r, uint32_t u, uint32_t v, uint8_t* masked, uint8_t* miss,
                    oracle_stats* st) {
    if (*masked) return 0;
    if (s->alive[v]) { *miss = 0; return 0; }               /* ping ok -> reset (:340-341) */
    if (*miss < 255) (*miss)++;                             /* failedAttempts++ (:336) */
    if (*miss < s->cfg.max_missed) return 0;                /* >= 3 -> dead (:337-338) */
    *masked = 1;                                            /* connectedPeers.erase (:388) */
    push_report(s, r, u, v);
    st->reports++;
    if (s->registered[v]) { s->registered[v] = 0; st->seed_removals++; } /* seed.cpp:162 */
    return 1;
}

/* u holds a connection to c: an unmasked entry of its sorted row or of its
 * overflow row (a dropped edge is erased from connectedPeers, peer.cpp:388) */
static int has_out_edge(const oracle_sim* s, uint32_t u, uint32_t c) {
    uint64_t lo = s->rp[u], hi = s->rp[u + 1];            /* rows are sorted */
    while (lo < hi) {
        uint64_t mid = (lo + hi) / 2;
        if (s->col[mid] < c) lo = mid + 1; else hi = mid;
    }
    if (lo < s->rp[u + 1] && s->col[lo] == c && !s->masked[lo]) return 1;
    for (uint32_t k = 0; k < s->ex_cnt[u]; ++k)
        if (s->ex_col[(uint64_t)u * s->K + k] == c && !s->ex_masked[(uint64_t)u * s->K + k]) return 1;
    return 0;
}

/* Re-bootstrap (handleDeadPeer :398-404 -> connectToSeed -> selectAndConnectPeers
 * :214-253): reporter u draws one seed response of L candidates keyed by
 * (round, dead peer) and connects to the first k (the power-law pick); a
 * candidate that is u, dead (connect() fails), already connected (the
 * connectedPeers map) or beyond the overflow row's capacity is skipped. */
static void rebootstrap(oracle_sim* s, uint32_t r, uint32_t u, uint32_t dead, oracle_stats* st) {
    const uint32_t L = s->cfg.list_len;
    const uint32_t k = pick_count(philox_x(s->cfg.seed, u, ORACLE_P_REBOOT, r, dead, 0, 0), L, s->thr);
    for (uint32_t i = 0; i < k; ++i) {
        const uint32_t x = philox_x(s->cfg.seed, u, ORACLE_P_REBOOT, r, dead, 1 + (i >> 2), i & 3);
        const uint32_t c = oracle_skew_pick(x, s->n);
        if (c == u || !s->alive[c] || has_out_edge(s, u, c)) continue;
        if (s->ex_cnt[u] >= s->K) continue;
        const uint64_t slot = (uint64_t)u * s->K + s->ex_cnt[u]++;
        s->ex_col[slot] = c;
        s->ex_masked[slot] = 0;
        s->ex_miss[slot] = 0;
        st->reconnects++;
    }
}

/* step 2: liveness (pingLoop peer.cpp:328-346 + handleDeadPeer :383-397 + seed :158-167) */
static void do_liveness(oracle_sim* s, uint32_t r, oracle_stats* st) {
    const uint64_t first = s->n_rep;
    for (uint64_t u = 0; u < s->n; ++u) {
        if (!s->alive[u]) continue;
        for (uint64_t e = s->rp[u]; e < s->rp[u + 1]; ++e)
            ping_one(s, r, (uint32_t)u, s->col[e], &s->masked[e], &s->miss[e], st);
        for (uint32_t k = 0; s->K && k < s->ex_cnt[u]; ++k) {
            const uint64_t x = u * s->K + k;
            ping_one(s, r, (uint32_t)u, s->ex_col[x], &s->ex_masked[x], &s->ex_miss[x], st);
        }
    }
    if (!s->K) return;
    /* this round's reports in (reporter, dead) order */
    if (s->n_rep > first) qsort(s->rep + first, s->n_rep - first, sizeof(oracle_report), cmp_rep);
    for (uint64_t i = first; i < s->n_rep; ++i) rebootstrap(s, r, s->rep[i].reporter, s->rep[i].dead, st);
}

static void stats_start_fast(oracle_sim* s, oracle_stats* st) {
    uint64_t frontier = 0, digest = 0, covered = 0;
    const uint32_t W = s->W;
    int T = s->cfg.threads;
    (void)T;
#pragma omp parallel for reduction(+ : frontier, digest, covered) schedule(static, 8192) num_threads(T)
    for (int64_t v = 0; v < (int64_t)s->n; ++v) {
        int act = 0;
        for (uint32_t w = 0; w < W; ++w) {
            uint64_t x = s->seen[v * W + w];
            act |= s->nw[v * W + w] != 0;
            covered += (uint64_t)__builtin_popcountll(x);
            digest += oracle_digest_weight((uint64_t)v * W + w) * x;
        }
        frontier += (uint64_t)act;
    }
    st->frontier = frontier;
    st->digest = digest;
    st->covered = covered;
}

static int step_fast(oracle_sim* s, oracle_stats* st) {
    const uint32_t W = s->W;
    const uint32_t r = s->round;
    /* 3: injection (messageGenerationLoop peer.cpp:359-374) */
    for (uint32_t m = 0; m < s->M; ++m) {
        if (s->inject_round[m] != r) continue;
        uint32_t o = s->origin[m];
        if (!s->alive[o]) continue;
        s->seen[o * W + (m >> 6)] |= 1ull << (m & 63);
        s->nw[o * W + (m >> 6)] |= 1ull << (m & 63);
        st->injected++;
    }
    stats_start_fast(s, st);
    /* 4: push (broadcastMessage :310-316 -> handleClient :277-285) */
    uint64_t trav = 0, deliv = 0, undeliv = 0, fresh_bits = 0;
    int T = s->cfg.threads;
    (void)T;
#pragma omp parallel for reduction(+ : trav, deliv, undeliv, fresh_bits) schedule(dynamic, 256) num_threads(T)
    for (int64_t u = 0; u < (int64_t)s->n; ++u) {
        const uint64_t* mk = s->nw + (uint64_t)u * W;
        int act = 0;
        uint64_t pc = 0;
        for (uint32_t w = 0; w < W; ++w) { act |= mk[w] != 0; pc += (uint64_t)__builtin_popcountll(mk[w]); }
        if (!act) continue;
        const uint64_t n_out = s->rp[u + 1] - s->rp[u] + (s->K ? s->ex_cnt[u] : 0);
        for (uint64_t i = 0; i < n_out; ++i) {   /* the row, then the re-bootstrap edges */
            const uint64_t e = s->rp[u] + i;
            const int base = e < s->rp[u + 1];
            const uint64_t x = base ? 0 : (uint64_t)u * s->K + (e - s->rp[u + 1]);
            if (base ? s->masked[e] : s->ex_masked[x]) continue;
            ++trav;
            uint32_t v = base ? s->col[e] : s->ex_col[x];
            if (!s->alive[v]) { undeliv += pc; continue; }
            deliv += pc;
            for (uint32_t w = 0; w < W; ++w) {
                if (!mk[w]) continue;
                uint64_t old = __atomic_fetch_or(&s->seen[(uint64_t)v * W + w], mk[w], __ATOMIC_RELAXED);
                uint64_t fr = mk[w] & ~old;
                if (fr) {
                    __atomic_fetch_or(&s->nx[(uint64_t)v * W + w], fr, __ATOMIC_RELAXED);
                    fresh_bits += (uint64_t)__builtin_popcountll(fr);
                }
            }
        }
    }
    st->traversals = trav;
    st->deliveries = deliv;
    st->undelivered = undeliv;
    st->new_receipts = fresh_bits;
    st->duplicates = deliv - fresh_bits;
    /* 5: advance */
    uint64_t* t = s->nw; s->nw = s->nx; s->nx = t;
    memset(s->nx, 0, s->n * W * sizeof(uint64_t));
    return 0;
}

static int step_literal(oracle_sim* s, oracle_stats* st) {
    const uint32_t r = s->round;
    const uint32_t W = s->W;
    for (uint32_t m = 0; m < s->M; ++m) {
        if (s->inject_round[m] != r) continue;
        uint32_t o = s->origin[m];
        if (!s->alive[o]) continue;
        if (ml_find(&s->lists[o], m) < 0) ml_insert(&s->lists[o], m); /* messageList[hash] = {msg,{}} (:371) */
        s->outbox[o][s->outbox_n[o]++] = m;                           /* broadcastMessage(msg) (:374) */
        st->injected++;
    }
    /* stats at push start, from the message lists */
    for (uint64_t v = 0; v < s->n; ++v) {
        const msg_list* l = &s->lists[v];
        st->frontier += s->outbox_n[v] > 0;
        for (uint32_t i = 0; i < l->cap; ++i) {
            uint32_t m = l->key[i];
            if (m == 0xFFFFFFFFu) continue;
            st->covered++;
            st->digest += oracle_digest_weight(v * W + (m >> 6)) * (1ull << (m & 63));
        }
    }
    /* push: every sender broadcasts every outbox message to every live out-edge */
    for (uint64_t u = 0; u < s->n; ++u) {
        if (!s->outbox_n[u]) continue;
        const uint64_t n_out = s->rp[u + 1] - s->rp[u] + (s->K ? s->ex_cnt[u] : 0);
        for (uint64_t i = 0; i < n_out; ++i) {   /* connectedPeers: the row, then the re-bootstrap edges */
            const uint64_t e = s->rp[u] + i;
            const int base = e < s->rp[u + 1];
            const uint64_t x = base ? 0 : (uint64_t)u * s->K + (e - s->rp[u + 1]);
            if (base ? s->masked[e] : s->ex_masked[x]) continue;
            st->traversals++;
            uint32_t v = base ? s->col[e] : s->ex_col[x];
            for (uint32_t i = 0; i < s->outbox_n[u]; ++i) {
                uint32_t m = s->outbox[u][i];
                if (!s->alive[v]) { st->undelivered++; continue; } /* send() fails: not in sentTo */
                st->deliveries++;
                int h = ml_find(&s->lists[u], m);
                s->lists[u].sent_to[h]++;                           /* sentTo.insert(peer) (:314) */
                /* receiver: handleClient dedup (:281-285) */
                if (ml_find(&s->lists[v], m) < 0) {
                    ml_insert(&s->lists[v], m);
                    s->nextbox[v][s->nextbox_n[v]++] = m;
                    st->new_receipts++;
                } else {
                    st->duplicates++;
                }
            }
        }
    }
    for (uint64_t v = 0; v < s->n; ++v) {
        uint32_t* t = s->outbox[v]; s->outbox[v] = s->nextbox[v]; s->nextbox[v] = t;
        s->outbox_n[v] = s->nextbox_n[v];
        s->nextbox_n[v] = 0;
    }
    return 0;
}

int oracle_sim_step(oracle_sim* s, oracle_stats* out) {
    if (s->finished) return 1;
    oracle_stats st;
    memset(&st, 0, sizeof(st));
    uint32_t r = s->round;
    st.round = r;
    uint64_t n_rj = 0;
    uint32_t* rj = do_rejoin(s, r, &n_rj);
    st.rejoined = n_rj;
    st.died = do_churn(s, r);
    rejoin_select(s, r, rj, n_rj, &st);
    free(rj);
    if (s->cfg.ping_every && r % s->cfg.ping_every == 0) {
        st.flags |= 1;
        do_liveness(s, r, &st);
    }
    if (s->cfg.variant == 0) step_fast(s, &st);
    else step_literal(s, &st);
    if (out) *out = st;
    s->round++;
    int pending = 0;
    for (uint32_t m = 0; m < s->M; ++m) pending |= (s->inject_round[m] != 0xFFFFFFFFu && s->inject_round[m] > r);
    if ((st.new_receipts == 0 && !pending && s->round >= s->cfg.min_rounds) || s->round >= s->cfg.max_rounds)
        s->finished = 1;
    return s->finished;
}

int oracle_sim_run(oracle_sim* s, oracle_stats* per_round, uint32_t cap) {
    int rounds = 0;
    while (!s->finished) {
        oracle_stats st;
        int rc = oracle_sim_step(s, &st);
        if (rc < 0) return rc;
        if (per_round && (uint32_t)rounds < cap) per_round[rounds] = st;
        ++rounds;
    }
    return rounds;
}

void oracle_sim_seen(const oracle_sim* s, uint64_t* out) {
    if (s->cfg.variant == 0) {
        memcpy(out, s->seen, s->n * s->W * sizeof(uint64_t));
        return;
    }
    memset(out, 0, s->n * s->W * sizeof(uint64_t));
    for (uint64_t v = 0; v < s->n; ++v) {
        const msg_list* l = &s->lists[v];
        for (uint32_t i = 0; i < l->cap; ++i) {
            uint32_t m = l->key[i];
            if (m != 0xFFFFFFFFu) out[v * s->W + (m >> 6)] |= 1ull << (m & 63);
        }
    }
}

void oracle_sim_coverage(const oracle_sim* s, uint64_t* out) {
    memset(out, 0, s->M * sizeof(uint64_t));
    for (uint64_t v = 0; v < s->n; ++v) {
        for (uint32_t m = 0; m < s->M; ++m) {
            if (s->cfg.variant == 0) out[m] += (uint64_t)has_bit_fast(s, v, m);
            else out[m] += ml_find(&s->lists[v], m) >= 0;
        }
    }
}


uint64_t oracle_sim_reports(const oracle_sim* s, oracle_report* buf, uint64_t cap) {
    if (s->n_rep) qsort(s->rep, s->n_rep, sizeof(oracle_report), cmp_rep);
    uint64_t k = s->n_rep < cap ? s->n_rep : cap;
    if (buf && k) memcpy(buf, s->rep, k * sizeof(oracle_report));
    return s->n_rep;
}

/* re-bootstrap edges: counts[n], cols[n * extra_cap] (bit 31 = dropped by liveness) */
void oracle_sim_extra(const oracle_sim* s, uint32_t* counts, uint32_t* cols) {
    for (uint64_t u = 0; u < s->n; ++u) {
        counts[u] = s->K ? s->ex_cnt[u] : 0;
        for (uint32_t k = 0; k < s->K; ++k) {
            const uint64_t x = u * s->K + k;
            cols[x] = k < s->ex_cnt[u] ? (s->ex_col[x] | (s->ex_masked[x] ? 0x80000000u : 0u)) : 0u;
        }
    }
}

void oracle_sim_alive(const oracle_sim* s, uint8_t* out) { memcpy(out, s->alive, s->n); }
void oracle_sim_registered(const oracle_sim* s, uint8_t* out) { memcpy(out, s->registered, s->n); }

uint64_t oracle_sim_sent_to_total(const oracle_sim* s) {
    if (!s->lists) return 0;
    uint64_t t = s->sent_lost;
    for (uint64_t v = 0; v < s->n; ++v)
        for (uint32_t i = 0; i < s->lists[v].cap; ++i)
            if (s->lists[v].key[i] != 0xFFFFFFFFu) t += s->lists[v].sent_to[i];
    return t;
}

/* ------------------------------------------------------------------------ */
/* Partition emulation: the same round model over one vertex block          */
/* [b, e) of a P-way 1D partition, with an explicit exchange step, so that  */
/* the multi-rank driver can be tested on CPU (gloo).  State that the       */
/* engine keeps globally (alive, registry view) is global here too.         */
/* ------------------------------------------------------------------------ */
struct oracle_part {
    oracle_sim_cfg cfg;
    uint64_t n, b, e, nl, E;
    uint32_t W, M;
    const uint64_t* rp;
    const uint32_t* col;
    uint8_t *alive, *registered, *masked, *miss;
    uint64_t *seen, *nw, *nx;
    uint32_t *origin, *inject_round, n_kills, *kill_peer, *kill_round;
    oracle_report* rep;
    uint64_t n_rep, cap_rep;
    uint32_t round;
    int finished;
    uint64_t prev_digest, prev_covered;
    int pull;
    oracle_stats cur;
};

oracle_part* oracle_part_create(const oracle_sim_cfg* cfg, uint64_t b, uint64_t e, const uint64_t* row_ptr,
                                const uint32_t* col) {
    if (!cfg || b >= e || e > cfg->n || cfg->extra_cap || cfg->rejoin_threshold || cfg->n_started)
        return NULL; /* no re-bootstrap, rejoin or failed registrations in the emulation */
    oracle_part* p = (oracle_part*)calloc(1, sizeof(oracle_part));
    p->cfg = *cfg;
    if (p->cfg.max_rounds == 0) p->cfg.max_rounds = 1u << 20;
    p->n = cfg->n; p->b = b; p->e = e; p->nl = e - b;
    p->E = row_ptr[p->nl];
    p->M = cfg->n_msgs; p->W = (cfg->n_msgs + 63) / 64;
    p->rp = row_ptr; p->col = col;
    p->alive = (uint8_t*)malloc(p->n); memset(p->alive, 1, p->n);
    p->registered = (uint8_t*)malloc(p->n); memset(p->registered, 1, p->n);
    p->masked = (uint8_t*)calloc(p->E + 1, 1);
    p->miss = (uint8_t*)calloc(p->E + 1, 1);
    p->seen = (uint64_t*)calloc(p->nl * p->W, 8);
    p->nw = (uint64_t*)calloc(p->nl * p->W, 8);
    p->nx = (uint64_t*)calloc(p->nl * p->W, 8);
    p->origin = (uint32_t*)calloc(p->M, 4);
    p->inject_round = (uint32_t*)malloc(p->M * 4);
    for (uint32_t m = 0; m < p->M; ++m) p->inject_round[m] = 0xFFFFFFFFu;
    return p;
}

void oracle_part_destroy(oracle_part* p) {
    if (!p) return;
    free(p->alive); free(p->registered); free(p->masked); free(p->miss);
    free(p->seen); free(p->nw); free(p->nx); free(p->origin); free(p->inject_round);
    free(p->kill_peer); free(p->kill_round); free(p->rep);
    free(p);
}

int oracle_part_schedule(oracle_part* p, const uint32_t* origin, const uint32_t* inject_round, uint32_t n_kills,
                         const uint32_t* kill_peer, const uint32_t* kill_round) {
    for (uint32_t m = 0; m < p->M; ++m) { p->origin[m] = origin[m]; p->inject_round[m] = inject_round[m]; }
    free(p->kill_peer); free(p->kill_round);
    p->n_kills = n_kills;
    p->kill_peer = (uint32_t*)malloc((n_kills + 1) * 4);
    p->kill_round = (uint32_t*)malloc((n_kills + 1) * 4);
    for (uint32_t i = 0; i < n_kills; ++i) { p->kill_peer[i] = kill_peer[i]; p->kill_round[i] = kill_round[i]; }
    return 0;
}

static int owned(const oracle_part* p, uint64_t v) { return v >= p->b && v < p->e; }

/* round phase 1: churn, liveness, injection, push-start stats; returns the
 * mode that will run (pull only if requested and nobody is dead -- the
 * overlay is assumed symmetric, as the powerlaw model is). */
int oracle_part_begin(oracle_part* p, int requested_pull) {
    const uint32_t W = p->W, r = p->round;
    oracle_stats* st = &p->cur;
    memset(st, 0, sizeof(*st));
    st->round = r;
    /* churn + kills over every peer (alive state is global) */
    for (uint32_t i = 0; i < p->n_kills; ++i) {
        uint32_t v = p->kill_peer[i];
        if (p->kill_round[i] == r && p->alive[v]) { p->alive[v] = 0; if (owned(p, v)) st->died++; }
    }
    if (p->cfg.churn_threshold) {
        for (uint64_t v = 0; v < p->n; ++v) {
            if (!p->alive[v]) continue;
            if (philox_x(p->cfg.seed, (uint32_t)(v >> 2), ORACLE_P_CHURN, r, 0, 0, (int)(v & 3)) < p->cfg.churn_threshold) {
                p->alive[v] = 0;
                if (owned(p, v)) st->died++;
            }
        }
    }
    for (uint64_t lv = 0; lv < p->nl; ++lv)
        if (!p->alive[p->b + lv]) memset(p->nw + lv * W, 0, W * 8);
    if (p->cfg.ping_every && r % p->cfg.ping_every == 0) {
        st->flags |= 1;
        for (uint64_t lu = 0; lu < p->nl; ++lu) {
            uint64_t u = p->b + lu;
            if (!p->alive[u]) continue;
            for (uint64_t e = p->rp[lu]; e < p->rp[lu + 1]; ++e) {
                if (p->masked[e]) continue;
                uint32_t v = p->col[e];
                if (p->alive[v]) { p->miss[e] = 0; continue; }
                if (p->miss[e] < 255) p->miss[e]++;
                if (p->miss[e] >= p->cfg.max_missed) {
                    p->masked[e] = 1;
                    if (p->n_rep == p->cap_rep) {
                        p->cap_rep = p->cap_rep ? 2 * p->cap_rep : 1024;
                        p->rep = (oracle_report*)realloc(p->rep, p->cap_rep * sizeof(oracle_report));
                    }
                    p->rep[p->n_rep].round = r; p->rep[p->n_rep].reporter = (uint32_t)u; p->rep[p->n_rep].dead = v;
                    p->n_rep++;
                    st->reports++;
                    if (p->registered[v]) { p->registered[v] = 0; st->seed_removals++; }
                }
            }
        }
    }
    for (uint32_t m = 0; m < p->M; ++m) {
        uint32_t o = p->origin[m];
        if (p->inject_round[m] != r || !owned(p, o) || !p->alive[o]) continue;
        p->seen[(o - p->b) * W + (m >> 6)] |= 1ull << (m & 63);
        p->nw[(o - p->b) * W + (m >> 6)] |= 1ull << (m & 63);
        st->injected++;
    }
    uint64_t digest = 0, covered = 0;
    for (uint64_t lv = 0; lv < p->nl; ++lv) {
        int act = 0;
        for (uint32_t w = 0; w < W; ++w) {
            uint64_t x = p->seen[lv * W + w];
            act |= p->nw[lv * W + w] != 0;
            covered += (uint64_t)__builtin_popcountll(x);
            digest += oracle_digest_weight((p->b + lv) * W + w) * x;
        }
        st->frontier += (uint64_t)act;
    }
    st->digest = digest - p->prev_digest;  /* increments, summed over ranks by the driver */
    st->covered = covered - p->prev_covered;
    p->prev_digest = digest;
    p->prev_covered = covered;
    int any_dead = 0;
    for (uint64_t v = 0; v < p->n && !any_dead; ++v) any_dead = !p->alive[v];
    p->pull = requested_pull && !any_dead;
    return p->pull;
}

/* pull: publish this block's new words at gather[b * W] (global peer index) */
void oracle_part_publish(oracle_part* p, uint64_t* gather) {
    memcpy(gather + p->b * p->W, p->nw, p->nl * p->W * 8);
}

/* pull round: every owned peer ORs its neighbours' new words (gather, indexed
 * by global peer); traversals/deliveries counted on the source side. */
int oracle_part_pull(oracle_part* p, const uint64_t* gather) {
    const uint32_t W = p->W;
    oracle_stats* st = &p->cur;
    for (uint64_t lu = 0; lu < p->nl; ++lu) {
        uint64_t pc = 0;
        for (uint32_t w = 0; w < W; ++w) pc += (uint64_t)__builtin_popcountll(p->nw[lu * W + w]);
        if (!pc) continue;
        const uint64_t deg = p->rp[lu + 1] - p->rp[lu];
        st->traversals += deg;
        st->deliveries += pc * deg;
    }
    for (uint64_t lv = 0; lv < p->nl; ++lv) {
        for (uint32_t w = 0; w < W; ++w) {
            uint64_t acc = 0;
            for (uint64_t e = p->rp[lv]; e < p->rp[lv + 1]; ++e) acc |= gather[(uint64_t)p->col[e] * W + w];
            const uint64_t fr = acc & ~p->seen[lv * W + w];
            if (!fr) continue;
            p->seen[lv * W + w] |= fr;
            p->nx[lv * W + w] |= fr;
            st->new_receipts += (uint64_t)__builtin_popcountll(fr);
        }
    }
    return 0;
}

/* push round: local push; masks for peers of other blocks are OR-ed into
 * send[v * W + w] (dense, global index). */
int oracle_part_push_compute(oracle_part* p, uint64_t* send) {
    const uint32_t W = p->W;
    oracle_stats* st = &p->cur;
    for (uint64_t lu = 0; lu < p->nl; ++lu) {
        const uint64_t* mk = p->nw + lu * W;
        uint64_t pc = 0;
        int act = 0;
        for (uint32_t w = 0; w < W; ++w) { act |= mk[w] != 0; pc += (uint64_t)__builtin_popcountll(mk[w]); }
        if (!act) continue;
        for (uint64_t e = p->rp[lu]; e < p->rp[lu + 1]; ++e) {
            if (p->masked[e]) continue;
            st->traversals++;
            uint32_t v = p->col[e];
            if (!p->alive[v]) { st->undelivered += pc; continue; }
            st->deliveries += pc;
            if (!owned(p, v)) {
                for (uint32_t w = 0; w < W; ++w) send[(uint64_t)v * W + w] |= mk[w];
                continue;
            }
            for (uint32_t w = 0; w < W; ++w) {
                uint64_t* s = &p->seen[(v - p->b) * W + w];
                uint64_t fr = mk[w] & ~*s;
                *s |= mk[w];
                if (fr) { p->nx[(v - p->b) * W + w] |= fr; st->new_receipts += (uint64_t)__builtin_popcountll(fr); }
            }
        }
    }
    return 0;
}

int oracle_part_push(oracle_part* p, uint64_t* send) {
    oracle_part_begin(p, 0);
    return oracle_part_push_compute(p, send);
}


/* sparse exchange: compact send (dense, global index) into per-destination
 * records {peer, words[W]} at seg + q*chunk*(1+W); clears send; counts[q] */
void oracle_part_compact(oracle_part* p, uint64_t* send, uint64_t chunk, uint32_t world, uint64_t* seg,
                         uint64_t* counts) {
    const uint32_t W = p->W;
    memset(counts, 0, world * sizeof(uint64_t));
    for (uint64_t v = 0; v < p->n; ++v) {
        int any = 0;
        for (uint32_t w = 0; w < W; ++w) any |= send[v * W + w] != 0;
        if (!any) continue;
        const uint64_t q = v / chunk;
        uint64_t* rec = seg + (q * chunk + counts[q]++) * (1 + W);
        rec[0] = v;
        for (uint32_t w = 0; w < W; ++w) { rec[1 + w] = send[v * W + w]; send[v * W + w] = 0; }
    }
}

/* sparse exchange, receiving side: test-and-set of the received records */
int oracle_part_finish_records(oracle_part* p, const uint64_t* rec, uint64_t n_rec, oracle_stats* out) {
    const uint32_t W = p->W;
    for (uint64_t i = 0; i < n_rec; ++i) {
        const uint64_t lv = rec[i * (1 + W)] - p->b;
        for (uint32_t w = 0; w < W; ++w) {
            const uint64_t fr = rec[i * (1 + W) + 1 + w] & ~p->seen[lv * W + w];
            if (!fr) continue;
            p->seen[lv * W + w] |= fr;
            p->nx[lv * W + w] |= fr;
            p->cur.new_receipts += (uint64_t)__builtin_popcountll(fr);
        }
    }
    p->cur.duplicates = p->cur.deliveries - p->cur.new_receipts;
    if (out) *out = p->cur;
    return 0;
}

/* test-and-set of the masks received from every block (recv: world x nl x W) */
int oracle_part_finish(oracle_part* p, const uint64_t* recv, uint32_t world, oracle_stats* out) {
    const uint32_t W = p->W;
    for (uint64_t lv = 0; recv && !p->pull && lv < p->nl; ++lv) {
        for (uint32_t w = 0; w < W; ++w) {
            uint64_t inc = 0;
            for (uint32_t q = 0; q < world; ++q) inc |= recv[((uint64_t)q * p->nl + lv) * W + w];
            uint64_t fr = inc & ~p->seen[lv * W + w];
            if (!fr) continue;
            p->seen[lv * W + w] |= fr;
            p->nx[lv * W + w] |= fr;
            p->cur.new_receipts += (uint64_t)__builtin_popcountll(fr);
        }
    }
    p->cur.duplicates = p->cur.deliveries - p->cur.new_receipts;
    if (out) *out = p->cur;
    return 0;
}

int oracle_part_commit(oracle_part* p, uint64_t global_new_receipts) {
    uint64_t* t = p->nw; p->nw = p->nx; p->nx = t;
    memset(p->nx, 0, p->nl * p->W * 8);
    uint32_t r = p->round++;
    int pending = 0;
    for (uint32_t m = 0; m < p->M; ++m) pending |= (p->inject_round[m] != 0xFFFFFFFFu && p->inject_round[m] > r);
    if ((global_new_receipts == 0 && !pending && p->round >= p->cfg.min_rounds) || p->round >= p->cfg.max_rounds)
        p->finished = 1;
    return p->finished;
}

void oracle_part_reset(oracle_part* p) {
    memset(p->alive, 1, p->n); memset(p->registered, 1, p->n);
    memset(p->masked, 0, p->E + 1); memset(p->miss, 0, p->E + 1);
    memset(p->seen, 0, p->nl * p->W * 8); memset(p->nw, 0, p->nl * p->W * 8); memset(p->nx, 0, p->nl * p->W * 8);
    p->n_rep = 0; p->round = 0; p->finished = 0; p->prev_digest = p->prev_covered = 0;
}

void oracle_part_seen(const oracle_part* p, uint64_t* out) { memcpy(out, p->seen, p->nl * p->W * 8); }

uint64_t oracle_part_reports(const oracle_part* p, oracle_report* buf, uint64_t cap) {
    if (p->n_rep) qsort(p->rep, p->n_rep, sizeof(oracle_report), cmp_rep);
    uint64_t k = p->n_rep < cap ? p->n_rep : cap;
    if (buf && k) memcpy(buf, p->rep, k * sizeof(oracle_report));
    return p->n_rep;
}
