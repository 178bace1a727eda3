/* TEST INFRASTRUCTURE: the oracle's threaded paths under ThreadSanitizer (`make -C oracle
 * check_tsan`, tests/test_host_sanitizers.py): orc_update_batch_mt (the C3 CPU leg's concurrent
 * writers, each key's ops on one writer) against the single writer's orc_update_batch on a twin
 * table -- equal return codes and reads -- and the threaded read batch afterwards. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "stage_oracle.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

int main(void) {
    const uint64_t n = 30000;
    const uint32_t P = 1000, ROW = 8 + P, D = 100;
    orc_tree *a = orc_tree_new(64 * 1024, 16 * 1024, P), *b = orc_tree_new(64 * 1024, 16 * 1024, P);
    if (orc_load_ycsb(a, 0, n, 8, 1) != n || orc_load_ycsb(b, 0, n, 8, 1) != n) return 2;
    const uint64_t m = 6000;
    uint64_t *keys = malloc(m * 8);
    uint8_t *deltas = malloc(m * D), *rca = malloc(m), *rcb = malloc(m);
    uint32_t *wid = malloc(m * 4), *cid = malloc(m * 4);
    int fails = 0;
    uint32_t counter = 10;
    for (int ep = 0; ep < 3; ep++) {
        for (uint64_t i = 0; i < m; i++) {
            keys[i] = (i % 4 == 0) ? rnd() % 30 : rnd() % (n + 50); /* hot keys and absent ones */
            memset(deltas + i * D, (int)(rnd() % 4), D);
            wid[i] = counter + 2 * (uint32_t)i;
            cid[i] = (rnd() % 20 == 0 && keys[i] >= 30) ? 0 : wid[i] + 1; /* some left in flight */
        }
        counter += 2 * (uint32_t)m + 2;
        double sec = 0;
        const uint64_t oka = orc_update_batch_mt(a, keys, 8, m, 0, deltas, D, wid, cid, rca, 8, &sec);
        const uint64_t okb = orc_update_batch(b, keys, 8, m, 0, deltas, D, wid, cid, rcb);
        if (oka != okb || memcmp(rca, rcb, m) != 0) fails++;
    }
    const uint64_t q = 4096;
    uint64_t *pk = malloc(q * 8);
    uint32_t *rids = malloc(q * 4);
    for (uint64_t i = 0; i < q; i++) pk[i] = rnd() % (n + 10), rids[i] = (uint32_t)(rnd() % counter);
    orc_read_out *oa = calloc(q, sizeof(orc_read_out)), *ob = calloc(q, sizeof(orc_read_out));
    uint8_t *ra = calloc(q, ROW), *rb = calloc(q, ROW);
    orc_read_batch(a, pk, 8, rids, q, oa, ra, 8);
    orc_read_batch(b, pk, 8, rids, q, ob, rb, 1);
    for (uint64_t i = 0; i < q; i++)
        if (oa[i].status != ob[i].status || memcmp(ra + i * ROW, rb + i * ROW, ROW) != 0) fails++;
    orc_tree_free(a);
    orc_tree_free(b);
    free(keys), free(deltas), free(rca), free(rcb), free(wid), free(cid), free(pk), free(rids);
    free(oa), free(ob), free(ra), free(rb);
    printf("oracle_tsan: %s (%d mismatches)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
}
