/* oracle_stress.c -- CPU sanitizer harness for the oracle (TEST
 * INFRASTRUCTURE: oracle/gossip_oracle.c is the checker, never the product).
 * Built by tests/sanitize/Makefile with the oracle source under
 * Address+UB sanitizers; run by tests/test_sanitizers.py.
 *
 * Drives both overlay generators, the fast (OpenMP) and literal round
 * drivers on workloads with churn, kills, liveness, re-bootstrap and join
 * churn, and the partition emulation, and checks literal == fast. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/gossip_oracle.h"

static int run(const oracle_sim_cfg* cfg, const uint64_t* rp, const uint32_t* col, const uint32_t* origin,
               const uint32_t* rounds, uint32_t n_kills, const uint32_t* kp, const uint32_t* kr, oracle_stats* out,
               uint32_t cap, uint64_t* seen) {
    oracle_sim* s = oracle_sim_create(cfg, rp, col);
    if (!s) return -1;
    oracle_sim_schedule(s, origin, rounds, n_kills, kp, kr);
    const int nr = oracle_sim_run(s, out, cap);
    oracle_sim_seen(s, seen);
    uint64_t cnt = oracle_sim_reports(s, NULL, 0);
    oracle_report* rep = (oracle_report*)malloc((cnt + 1) * sizeof(oracle_report));
    oracle_sim_reports(s, rep, cnt);
    free(rep);
    oracle_sim_destroy(s);
    return nr;
}

static int compare(const char* what, uint64_t n, uint32_t M, const uint64_t* rp, const uint32_t* col,
                   oracle_sim_cfg cfg, const uint32_t* origin, const uint32_t* rounds, uint32_t n_kills,
                   const uint32_t* kp, const uint32_t* kr) {
    enum { CAP = 512 };
    static oracle_stats a[CAP], b[CAP];
    const uint32_t W = (M + 63) / 64;
    uint64_t* sa = (uint64_t*)calloc(n * W, 8);
    uint64_t* sb = (uint64_t*)calloc(n * W, 8);
    cfg.variant = 0;
    const int ra = run(&cfg, rp, col, origin, rounds, n_kills, kp, kr, a, CAP, sa);
    cfg.variant = 1;
    const int rb = run(&cfg, rp, col, origin, rounds, n_kills, kp, kr, b, CAP, sb);
    int ok = ra > 0 && ra == rb && !memcmp(a, b, (size_t)ra * sizeof(oracle_stats)) && !memcmp(sa, sb, n * W * 8);
    printf("%-28s rounds %d/%d %s\n", what, ra, rb, ok ? "ok" : "MISMATCH");
    free(sa);
    free(sb);
    return ok ? 0 : 1;
}

int main(void) {
    int fails = 0;
    uint64_t* rp = NULL;
    uint32_t* col = NULL;
    uint64_t m = 0;
    /* powerlaw overlay, 64 messages, churn + liveness + re-bootstrap */
    const uint64_t n = 3000;
    if (oracle_gen_powerlaw(n, 6, 0x5EED0005u, 4, &rp, &col, &m)) return 2;
    uint32_t origin[130], rounds[130], kp[4] = {0, 7, 100, 2999}, kr[4] = {1, 2, 4, 6};
    oracle_pick_origins(n, 0x5EED0005u, 130, origin);
    for (int i = 0; i < 130; ++i) rounds[i] = (uint32_t)(i % 4);
    oracle_sim_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.n = n;
    cfg.n_msgs = 130;
    cfg.seed = 0x5EED0005u;
    cfg.churn_threshold = 42949673u * 2;
    cfg.ping_every = 3;
    cfg.max_missed = 2;
    cfg.max_rounds = 200;
    cfg.min_rounds = 20;
    cfg.threads = 4;
    cfg.list_len = 6;
    fails += compare("powerlaw churn", n, 130, rp, col, cfg, origin, rounds, 4, kp, kr);
    cfg.extra_cap = 8;
    fails += compare("powerlaw re-bootstrap", n, 130, rp, col, cfg, origin, rounds, 4, kp, kr);
    cfg.rejoin_threshold = (uint32_t)(0.05 * 4294967296.0);
    fails += compare("powerlaw rejoin", n, 130, rp, col, cfg, origin, rounds, 4, kp, kr);
    /* partition emulation: two blocks, push rounds, exchange by hand */
    {
        oracle_sim_cfg pc = cfg;
        pc.extra_cap = 0;
        pc.rejoin_threshold = 0;
        pc.churn_threshold = 0;
        pc.ping_every = 0;
        pc.n_msgs = 64;
        const uint64_t half = n / 2, bnd[3] = {0, half, n};
        oracle_part* P[2];
        uint64_t* lrp[2];
        for (int p = 0; p < 2; ++p) {
            lrp[p] = (uint64_t*)malloc((bnd[p + 1] - bnd[p] + 1) * 8);
            for (uint64_t v = bnd[p]; v <= bnd[p + 1]; ++v) lrp[p][v - bnd[p]] = rp[v] - rp[bnd[p]];
            P[p] = oracle_part_create(&pc, bnd[p], bnd[p + 1], lrp[p], col + rp[bnd[p]]);
            oracle_part_schedule(P[p], origin, rounds, 0, kp, kr);
        }
        uint64_t* send[2] = {(uint64_t*)calloc(n, 8), (uint64_t*)calloc(n, 8)};
        uint64_t* recv[2] = {(uint64_t*)calloc(2 * half, 8), (uint64_t*)calloc(2 * (n - half), 8)};
        int fin = 0, r = 0;
        while (!fin && r++ < 100) {
            for (int p = 0; p < 2; ++p) {
                memset(send[p], 0, n * 8);
                oracle_part_push(P[p], send[p]);
            }
            for (int q = 0; q < 2; ++q)
                for (int p = 0; p < 2; ++p)
                    memcpy(recv[q] + (uint64_t)p * (bnd[q + 1] - bnd[q]), send[p] + bnd[q], (bnd[q + 1] - bnd[q]) * 8);
            oracle_stats st[2];
            for (int p = 0; p < 2; ++p) oracle_part_finish(P[p], recv[p], 2, &st[p]);
            const uint64_t fresh = st[0].new_receipts + st[1].new_receipts;
            fin = oracle_part_commit(P[0], fresh);
            oracle_part_commit(P[1], fresh);
        }
        printf("%-28s rounds %d %s\n", "partition emulation", r, fin ? "ok" : "NO TERMINATION");
        fails += !fin;
        for (int p = 0; p < 2; ++p) {
            oracle_part_destroy(P[p]);
            free(lrp[p]);
            free(send[p]);
            free(recv[p]);
        }
    }
    oracle_free(rp);
    oracle_free(col);
    /* literal bootstrap DAG (F8), config-1 style schedule with a kill */
    const uint32_t nb = 40;
    if (oracle_gen_ref_bootstrap(nb, 20, 0x5EED0001u, &rp, &col, &m)) return 2;
    uint32_t o2[400], r2[400], k1[1] = {3}, kr1[1] = {12};
    for (uint32_t i = 0; i < 400; ++i) {
        o2[i] = i / 10;
        r2[i] = (i % 10) * 5;
    }
    memset(&cfg, 0, sizeof cfg);
    cfg.n = nb;
    cfg.n_msgs = 400;
    cfg.seed = 0x5EED0001u;
    cfg.ping_every = 15;
    cfg.max_missed = 3;
    cfg.max_rounds = 400;
    cfg.min_rounds = 46;
    cfg.threads = 4;
    cfg.n_started = oracle_started_under_cap(nb, 1500);
    fails += compare("ref_bootstrap + F10 cap", nb, 400, rp, col, cfg, o2, r2, 1, k1, kr1);
    oracle_free(rp);
    oracle_free(col);
    printf("oracle_stress: %d failure(s)\n", fails);
    return fails ? 1 : 0;
}
