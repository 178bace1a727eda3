/* TEST INFRASTRUCTURE: the oracle under AddressSanitizer + UndefinedBehaviorSanitizer
 * (`make -C oracle check`, tests/test_host_sanitizers.py).  Exercises the restatement's entry
 * points on small tables: sequential and parallel YCSB loads (same reads), threaded reads and
 * scans, index scans at old snapshots, random updates with commit / abort / finalize, deletes,
 * aborted inserts, batched epochs, read-only transactions, leaf-image export, locations. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "stage_oracle.h"

static int fails;
#define CHECK(c, msg)                                              \
    do {                                                           \
        if (!(c) && fails++ < 20) fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
    } while (0)

static uint64_t rng_state = 88172645463325252ull;
static uint64_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : 100000;
    const uint32_t P = 1000, ROW = 8 + P;
    orc_tree *a = orc_tree_new(64 * 1024, 16 * 1024, P);
    orc_tree *b = orc_tree_new(64 * 1024, 16 * 1024, P);
    orc_tree_set_merge_threshold(a, 32 * 1024);
    CHECK(orc_load_ycsb(a, 0, n, 8, 1) == n, "load");
    CHECK(orc_load_ycsb_parallel(b, 0, n, 8, 1, 4) == n, "parallel load");
    const uint64_t m = 4096;
    uint64_t *keys = malloc(m * 8);
    uint32_t *rids = malloc(m * 4), *counts = malloc(m * 4);
    for (uint64_t i = 0; i < m; i++) keys[i] = rnd() % (n + 100), rids[i] = 0xFFFFFFFEu;
    orc_read_out *oa = calloc(m, sizeof(orc_read_out)), *ob = calloc(m, sizeof(orc_read_out));
    uint8_t *ra = calloc(m, ROW), *rb = calloc(m, ROW);
    orc_read_batch(a, keys, 8, rids, m, oa, ra, 4);
    orc_read_batch(b, keys, 8, rids, m, ob, rb, 4);
    CHECK(!memcmp(oa, ob, m * sizeof(orc_read_out)) && !memcmp(ra, rb, (size_t)m * ROW), "parallel load reads");
    uint8_t *srecs = calloc((size_t)64 * 100, ROW);
    orc_scan_batch(a, keys, 8, 64, 100, counts, srecs, 4);
    /* random single-writer traffic on a */
    uint32_t tid = 10;
    uint8_t delta[16], payload[1000], st[100];
    for (uint64_t i = 0; i < n; i++) {
        uint64_t k = rnd() % (n + n / 4);
        const uint8_t *kb = (const uint8_t *)&k;
        int op = (int)(rnd() % 100);
        memset(delta, (int)i, sizeof delta);
        if (op < 40) {
            if (orc_update(a, kb, 8, (uint32_t)(rnd() % 900), delta, 16, ++tid) == 1) {
                int c = (int)(rnd() % 4);
                if (c == 0) orc_abort_update(a, kb, 8);
                else if (c == 1) orc_finalize_update(a, kb, 8, ++tid);
                else if (c == 2) orc_commit_update(a, kb, 8, ++tid, tid);
                /* c == 3: stays in flight until the next update of the key fails or commits */
            }
        } else if (op < 55) {
            memset(payload, (int)k, sizeof payload);
            if (orc_insert(a, kb, 8, payload, ++tid) == 1 && rnd() % 3 == 0) orc_abort_insert(a, kb, 8);
        } else if (op < 65) {
            orc_delete(a, kb, 8, ++tid);
        } else if (op < 75) {
            orc_read_out o;
            uint8_t rec[1008];
            orc_read(a, kb, 8, (uint32_t)(rnd() % (tid + 1)), &o, rec);
        } else if (op < 80) {
            orc_index_scan(a, kb, 8, 100, (uint32_t)(rnd() % (tid + 1)), srecs, st);
        } else if (op < 81) {
            uint64_t bk[32];
            uint32_t wid[32], cid[32];
            uint8_t d[32 * 8], rc[32];
            for (int j = 0; j < 32; j++) bk[j] = rnd() % n, wid[j] = ++tid, cid[j] = ++tid;
            bk[31] = bk[0]; /* one key twice */
            memset(d, 5, sizeof d);
            orc_update_batch(a, bk, 8, 32, 0, d, 8, wid, cid, rc);
        }
    }
    for (uint64_t i = 0; i < m; i++) rids[i] = (uint32_t)(rnd() % (tid + 1));
    orc_read_batch(a, keys, 8, rids, m, oa, ra, 4);
    orc_scan_batch(a, keys, 8, 64, 100, counts, srecs, 4);
    /* read-only transactions on b */
    double secs = 0;
    uint64_t res[3] = {0, 0, 0};
    orc_ycsb_txn_timed(b, keys, 8, 10, m / 10, 4, 1, &secs, res);
    CHECK(res[0] + res[1] > 0, "transactions ran");
    /* leaf images and locations of a */
    uint64_t stats[8] = {0};
    orc_stats(a, stats);
    const uint64_t nl = stats[2];
    uint8_t *blocks = malloc((size_t)nl * 64 * 1024);
    uint64_t *seps = malloc(nl * 8);
    uint16_t *sl = malloc(nl * 2);
    CHECK(orc_export_leaf_images(a, nl, blocks, seps, sl) == (int64_t)nl, "export");
    const uint64_t nloc = orc_location_count(a);
    uint64_t *h = malloc((nloc + 1) * 8);
    uint32_t *lf = malloc((nloc + 1) * 4);
    uint16_t *ls = malloc((nloc + 1) * 2);
    for (uint64_t i = 0; i < nloc; i++) h[i] = i + 1;
    orc_resolve_locations(a, h, nloc, lf, ls);
    printf("oracle_check: %llu rows, %llu leaves, %llu locations, %llu txns committed%s\n", (unsigned long long)n,
           (unsigned long long)nl, (unsigned long long)nloc, (unsigned long long)res[0], fails ? "" : ": ok");
    free(h), free(lf), free(ls), free(blocks), free(seps), free(sl);
    free(keys), free(rids), free(counts), free(oa), free(ob), free(ra), free(rb), free(srecs);
    orc_tree_free(a);
    orc_tree_free(b);
    return fails ? 1 : 0;
}
