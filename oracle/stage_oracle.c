/*
 * stage_oracle.c -- TEST INFRASTRUCTURE ONLY: the parity checker and the CPU baseline.
 *
 * A plain-C restatement of the reference's index-organized read path (and of the small
 * part of its write path needed to build the same leaf layouts and version chains).
 * Every function cites the reference file:line it follows (paths relative to the
 * reference checkout sheepTnT/Stage-IndexOrganized @ 2024-12-18).  Nothing here is
 * compiled into, linked with or called by the product library; the product path
 * (stage-indexorganized_amd/) is an independent implementation that is checked
 * against this one.
 *
 * Single writer: the reference's CAS/retry/freeze loops collapse to their
 * single-threaded outcome (every CAS succeeds, no node is frozen by another thread).
 */
#define _GNU_SOURCE
#include "stage_oracle.h"

#include <pthread.h>
#include <sys/mman.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define MAX_CID 0xFFFFFFFFu
#define INVALID_CID 0u

/* ---------------------------------------------------------------- key order */
/* my_memcmp, b_tree.h:99-106: plain char is signed on the reference's x86 target */
static int my_memcmp(const uint8_t *k1, const uint8_t *k2, uint32_t size) {
    for (uint32_t i = 0; i < size; i++) {
        signed char a = (signed char)k1[i], b = (signed char)k2[i];
        if (a != b) return (int)a - (int)b;
    }
    return 0;
}

/* BaseNode::KeyCompare, b_tree.h:116-134 (memcmp -- unsigned -- only from 16 bytes up) */
int orc_key_compare(const uint8_t *k1, uint32_t s1, const uint8_t *k2, uint32_t s2) {
    if (!k1) return -1;
    if (!k2) return 1;
    uint32_t m = s1 < s2 ? s1 : s2;
    int cmp = (m < 16) ? my_memcmp(k1, k2, m) : memcmp(k1, k2, m);
    if (cmp == 0) return (int)(s1 - s2);
    return cmp;
}

/* ---------------------------------------------------------------- metadata */
/* RecordMetadata masks, record_meta.h:66-70 */
#define M_CONTROL (1ull << 63)
#define M_VISIBLE (1ull << 62)
#define M_KEYLEN (0x2FFFull << 48)
#define M_OFFSET (0xFFFFull << 32)
#define M_TXN 0xFFFFFFFFull

static inline uint16_t m_keylen(uint64_t m) { return (uint16_t)((m & M_KEYLEN) >> 48); }
static inline uint16_t pad_key(uint32_t k) { return (uint16_t)((k + 7) / 8 * 8); } /* :89-91 */
static inline uint16_t m_padded(uint64_t m) { return pad_key(m_keylen(m)); }
static inline uint16_t m_offset(uint64_t m) { return (uint16_t)((m & M_OFFSET) >> 32); }
static inline int m_visible(uint64_t m) { return (m & M_VISIBLE) != 0; }
static inline int m_inserting(uint64_t m) { return m_visible(m) && (m & M_CONTROL); } /* :178-181 */
static inline uint32_t m_cstamp(uint64_t m) { return (uint32_t)(m & M_TXN); }
/* FinalizeForInsert(offset,key_len,commit_id), record_meta.h:128-137 */
static inline uint64_t m_finalize_insert(uint64_t off, uint64_t klen, uint64_t cid) {
    uint64_t m = (klen << 48) | (1ull << 62) | (off << 32) | cid;
    return m & ~M_CONTROL;
}

/* next_ptr handles: the reference stores raw pointers (copy-buffer location while an
 * update is in flight, TupleHeader* after commit).  Tagged here so a reader can tell
 * them apart (the reference cannot; see DESIGN.md "chain walk on a copy pointer"). */
#define NEXT_COPY 1ull
#define NEXT_TH 2ull
#define NEXT_KIND(x) ((x) & 3ull)
#define NEXT_PTR(x) ((void *)(uintptr_t)((x) & ~3ull))

typedef struct orc_loc { uint8_t *leaf; uint32_t slot; uint64_t id; } orc_loc; /* RecordLocation; id = allocation index */

typedef struct orc_copy { /* EphemeralPool::OverwriteVersionHeader, ephemeral_pool.h:26-150 */
    uint32_t cstamp, pstamp, rstamp, sstamp;
    uint64_t next; /* old TupleHeader chain at update time */
    uint64_t pre;
    uint16_t key_len;
    uint32_t payload_size;
    int live, waiting;
    int wr_count; /* readers counted by IncreaseWRCount / DecreaseWRCount (ephemeral_pool.cpp:194-239) */
    uint8_t *image; /* [key(key_len)][payload] (b_tree.cpp:1143-1144) */
    struct orc_copy *reg_next;
    uint32_t id;                /* allocation order (the copy id of a next handle) */
    uint32_t *readers;          /* AddReader (ephemeral_pool.h:61-65) */
    uint32_t nreaders, capreaders;
} orc_copy;

typedef struct orc_th { /* TupleHeader, version_store.h:28-155 */
    uint32_t begin_id, comm_id;
    uint64_t next;
    uint8_t *slot; /* [key(key_len)][payload] (transaction_manager.cpp:639-640) */
    uint16_t key_len;
    struct orc_th *reg_next;
    uint32_t id; /* allocation order (the version id of a next handle) */
} orc_th;

/* ---------------------------------------------------------------- leaf image */
/* sizeof(LeafNode) == 40: vptr(8) is_leaf(1,+7) NodeHeader{size u32, sorted_count u32,
 * next_record_slot u32 (+4), StatusWord u64} (b_tree.h:109-113, version_store.h:158-231) */
#define LEAF_HDR 40u
#define META_SZ 24u
#define OFF_ISLEAF 8
#define OFF_SIZE 16
#define OFF_SORTED 20
#define OFF_STATUS 32

typedef struct { uint64_t meta, next; orc_loc *loc; } orc_rmeta; /* 24 B */

static inline uint32_t *l_size(uint8_t *n) { return (uint32_t *)(n + OFF_SIZE); }
static inline uint32_t *l_sorted(uint8_t *n) { return (uint32_t *)(n + OFF_SORTED); }
static inline uint64_t *l_status(uint8_t *n) { return (uint64_t *)(n + OFF_STATUS); }
static inline orc_rmeta *l_meta(uint8_t *n, uint32_t i) { return (orc_rmeta *)(n + LEAF_HDR + META_SZ * i); }
/* StatusWord, version_store.h:167-214 */
static inline uint32_t st_count(uint64_t s) { return (uint32_t)((s >> 44) & 0xFFFF); }
static inline uint32_t st_block(uint64_t s) { return (uint32_t)((s >> 22) & 0x3FFFFF); }
static inline uint32_t st_deleted(uint64_t s) { return (uint32_t)(s & 0x3FFFFF); }
static inline int st_frozen(uint64_t s) { return (s >> 60) & 1; }
static inline uint64_t st_set_count(uint64_t s, uint32_t c) { return (s & ~(0xFFFFull << 44)) | ((uint64_t)c << 44); }
static inline uint64_t st_set_block(uint64_t s, uint32_t b) { return (s & ~(0x3FFFFFull << 22)) | ((uint64_t)b << 22); }
static inline uint64_t st_set_deleted(uint64_t s, uint32_t d) { return (s & ~0x3FFFFFull) | d; }
/* LeafNode::GetUsedSpace, b_tree.h:577-582 */
static inline uint32_t used_space(uint64_t s) { return LEAF_HDR + st_block(s) + st_count(s) * META_SZ; }
/* BaseNode::GetKey, b_tree.h:188-193 */
static inline const uint8_t *l_key(uint8_t *n, uint64_t m) { return m_visible(m) ? n + m_offset(m) : NULL; }

/* ---------------------------------------------------------------- inner node */
typedef struct orc_inner { /* InternalNode (b_tree.h:213-398): immutable once built */
    uint8_t hdr[16];       /* hdr[OFF_ISLEAF] == 0 */
    uint32_t size;         /* header.size == the node's allocation size */
    uint32_t count;        /* header.sorted_count */
    int frozen;
    uint16_t *klen;
    uint8_t **key;         /* NULL for the dummy slot-0 key */
    void **child;
    uint8_t *keybuf;
} orc_inner;

static inline int is_leaf(void *p) { return ((uint8_t *)p)[OFF_ISLEAF] != 0; }

struct orc_tree {
    uint32_t leaf_node_size, split_threshold, payload_size, merge_threshold;
    uint32_t key_pad; /* key bytes of a canonical tuple row (8, or the padded wide key width) */
    void *root;
    orc_copy *copies;
    orc_th *ths;
    orc_loc **locs;
    uint64_t nlocs, caplocs;
    void **garbage; /* nodes replaced during the current Insert (released after install) */
    uint64_t ngarbage, capgarbage;
    uint64_t retired;
    int bulk; /* orc_tree_set_bulk: a load of distinct keys, CheckUnique skipped */
    orc_copy **copy_by_id; /* copy id -> copy (ids in allocation order) */
    uint32_t ncopies, capcopies, nths;
};

typedef struct { orc_inner *node; uint32_t meta_index; } frame_t;
typedef struct { frame_t f[32]; uint32_t n; void *root; } stack_t_; /* Stack, b_tree.h:743-784 */

static void push(stack_t_ *s, orc_inner *n, uint32_t i) { s->f[s->n].node = n; s->f[s->n].meta_index = i; s->n++; }
static frame_t *pop(stack_t_ *s) { return s->n == 0 ? NULL : &s->f[--s->n]; }
static frame_t *top(stack_t_ *s) { return s->n == 0 ? NULL : &s->f[s->n - 1]; }

static void *xmalloc(size_t n) {
    void *p = malloc(n);
    if (!p) abort();
    return p;
}

/* leaf blocks come from a process-wide pool: leaves of one size carved from 1 GiB anonymous
 * mappings, freed leaves kept on a free list and reused by the next split, a freed tree's
 * leaves handed back to the kernel (MADV_DONTNEED).  malloc's heap fragments under the
 * loader's split pattern (10M rows held 2x their live leaves); a 100M-row table would not fit
 * the GPU box's per-command memory cap. */
#define POOL_CHUNK (1ull << 30)
typedef struct { uint32_t size; void *free_list; uint8_t *chunk; uint64_t left; } leaf_pool;
static leaf_pool g_pools[4];
static pthread_mutex_t g_pool_lock = PTHREAD_MUTEX_INITIALIZER;

static leaf_pool *pool_of(uint32_t size) {
    for (int i = 0; i < 4; i++) {
        if (g_pools[i].size == size) return &g_pools[i];
        if (g_pools[i].size == 0) {
            g_pools[i].size = size;
            return &g_pools[i];
        }
    }
    return NULL;
}

static void *leaf_block_alloc(uint32_t size) {
    pthread_mutex_lock(&g_pool_lock);
    leaf_pool *p = pool_of(size);
    void *b = NULL;
    if (p && p->free_list) {
        b = p->free_list;
        p->free_list = *(void **)b;
    } else if (p && size % 4096 == 0) {
        if (p->left < size) {
            void *c = mmap(NULL, POOL_CHUNK, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (c == MAP_FAILED) abort();
            p->chunk = c;
            p->left = POOL_CHUNK;
        }
        b = p->chunk;
        p->chunk += size;
        p->left -= size;
    }
    pthread_mutex_unlock(&g_pool_lock);
    if (!b) { /* sizes that are not page multiples: plain allocation */
        b = aligned_alloc(64, size);
        if (!b) abort();
    }
    return b;
}

static void leaf_block_free(uint32_t size, void *b, int release) {
    if (size % 4096) {
        free(b);
        return;
    }
    if (release) madvise(b, size, MADV_DONTNEED);
    pthread_mutex_lock(&g_pool_lock);
    leaf_pool *p = pool_of(size);
    *(void **)b = p->free_list;
    p->free_list = b;
    pthread_mutex_unlock(&g_pool_lock);
}

static void garbage_add(orc_tree *t, void *p) {
    if (t->ngarbage == t->capgarbage) {
        t->capgarbage = t->capgarbage ? 2 * t->capgarbage : 64;
        t->garbage = realloc(t->garbage, t->capgarbage * sizeof(void *));
    }
    t->garbage[t->ngarbage++] = p;
}

static void inner_free(orc_inner *n) {
    free(n->klen);
    free(n->key);
    free(n->child);
    free(n->keybuf);
    free(n);
}

static void garbage_release(orc_tree *t) {
    for (uint64_t i = 0; i < t->ngarbage; i++) {
        void *p = t->garbage[i];
        if (is_leaf(p)) leaf_block_free(t->leaf_node_size, p, 0);
        else inner_free((orc_inner *)p);
    }
    t->ngarbage = 0;
}

static orc_inner *inner_alloc(uint32_t cap, uint32_t keybytes) {
    orc_inner *n = xmalloc(sizeof(orc_inner));
    memset(n, 0, sizeof(*n));
    n->klen = xmalloc(sizeof(uint16_t) * cap);
    n->key = xmalloc(sizeof(uint8_t *) * cap);
    n->child = xmalloc(sizeof(void *) * cap);
    n->keybuf = xmalloc(keybytes ? keybytes : 1);
    return n;
}

typedef struct { uint32_t used; } kb_t;
static void inner_set(orc_inner *n, kb_t *kb, uint32_t idx, const uint8_t *key, uint16_t klen, void *child) {
    n->klen[idx] = klen;
    if (klen && key) {
        memcpy(n->keybuf + kb->used, key, klen);
        n->key[idx] = n->keybuf + kb->used;
        kb->used += klen;
    } else {
        n->key[idx] = NULL; /* GetRawRecord: zero-length key -> nullptr (b_tree.h:378-382) */
    }
    n->child[idx] = child;
}

static uint32_t inner_keybytes(orc_inner *src, uint32_t b, uint32_t nr, uint32_t extra) {
    uint32_t s = extra;
    if (src)
        for (uint32_t i = b; i < b + nr; i++) s += src->klen[i];
    return s;
}

/* InternalNode(node_size, key, key_size, left, right), b_tree.cpp:363-389; alloc b_tree.h:249-265 */
static orc_inner *inner_new_root(const uint8_t *key, uint16_t ks, void *left, void *right) {
    orc_inner *n = inner_alloc(2, ks);
    kb_t kb = {0};
    n->size = 48 + pad_key(ks) + 8 + 8 + 2 * META_SZ;
    inner_set(n, &kb, 0, NULL, 0, left);
    inner_set(n, &kb, 1, key, ks, right);
    n->count = 2;
    return n;
}

/* InternalNode(node_size, src, begin, nr, key, key_size, left, right, left_most),
 * b_tree.cpp:391-497 */
static void inner_build(orc_inner *n, orc_inner *src, uint32_t begin, uint32_t nr, const uint8_t *key,
                        uint16_t ks, void *left, void *right, void *left_most) {
    kb_t kb = {0};
    int need_insert_new = key != NULL;
    uint32_t idx = 0;
    if (left_most) {
        inner_set(n, &kb, 0, NULL, 0, left_most);
        idx++;
    }
    for (uint32_t i = begin; i < begin + nr; i++) {
        const uint8_t *mk = src->key[i];
        uint16_t mks = src->klen[i];
        if (!need_insert_new) {
            inner_set(n, &kb, idx, mk, mks, src->child[i]);
        } else {
            int cmp = orc_key_compare(mk, mks, key, ks);
            if (cmp > 0) {
                n->child[idx - 1] = left; /* previous key's payload := left child */
                inner_set(n, &kb, idx, key, ks, right);
                idx++;
                inner_set(n, &kb, idx, mk, mks, src->child[i]);
                need_insert_new = 0;
            } else {
                inner_set(n, &kb, idx, mk, mks, src->child[i]);
            }
        }
        idx++;
    }
    if (need_insert_new) { /* new key is the right-most */
        inner_set(n, &kb, idx, key, ks, right);
        n->child[idx - 1] = left;
        idx++;
    }
    n->count = idx;
}

/* InternalNode::New(src, key, ...) b_tree.h:230-246 */
static orc_inner *inner_new_insert(orc_inner *src, const uint8_t *key, uint16_t ks, void *left, void *right) {
    orc_inner *n = inner_alloc(src->count + 1, inner_keybytes(src, 0, src->count, ks));
    n->size = src->size + pad_key(ks) + 8 + META_SZ;
    inner_build(n, src, 0, src->count, key, ks, left, right, NULL);
    return n;
}

/* InternalNode::New(src, begin, nr, key, ...) b_tree.h:266-303 */
static orc_inner *inner_new_range(orc_inner *src, uint32_t begin, uint32_t nr, const uint8_t *key, uint16_t ks,
                                  void *left, void *right, void *left_most) {
    uint32_t alloc = 48;
    if (begin > 0) alloc += pad_key(src->klen[0]) + 8 + META_SZ;
    for (uint32_t i = begin; i < begin + nr; i++) alloc += pad_key(src->klen[i]) + 8 + META_SZ;
    if (key) alloc += pad_key(ks) + 8 + META_SZ;
    orc_inner *n = inner_alloc(nr + 2, inner_keybytes(src, begin, nr, key ? ks : 0));
    n->size = alloc;
    inner_build(n, src, begin, nr, key, ks, left, right, left_most);
    return n;
}

/* InternalNode::GetChildIndex, b_tree.cpp:664-702 (reproduced literally) */
static uint32_t get_child_index(orc_inner *n, const uint8_t *key, uint16_t ks, int get_le) {
    int32_t left = 0, right = (int32_t)n->count - 1, mid = 0;
    for (;;) {
        mid = (left + right) / 2;
        int cmp = orc_key_compare(key, ks, n->key[mid], n->klen[mid]);
        if (cmp == 0) return get_le ? (uint32_t)(mid - 1) : (uint32_t)mid;
        if (left > right) {
            if (cmp <= 0 && get_le) return (uint32_t)(mid - 1);
            return (uint32_t)mid;
        }
        if (cmp > 0) left = mid + 1;
        else right = mid - 1;
    }
}

/* BTree::TraverseToLeaf, b_tree.cpp:1804-1846 */
static uint8_t *traverse_to_leaf(orc_tree *t, stack_t_ *st, const uint8_t *key, uint16_t ks, int le_child) {
    void *node = t->root;
    if (st) st->root = node;
    while (!is_leaf(node)) {
        orc_inner *p = (orc_inner *)node;
        uint32_t idx = get_child_index(p, key, ks, le_child);
        node = p->child[idx];
        if (st) push(st, p, idx);
    }
    return (uint8_t *)node;
}

/* InternalNode::PrepareForSplit, b_tree.cpp:500-598 */
static orc_inner *inner_prepare_for_split(orc_tree *t, orc_inner *n, stack_t_ *st, const uint8_t *key,
                                          uint16_t ks, void *left, void *right) {
    uint32_t data_size = n->size + ks + 8 + META_SZ;
    uint32_t new_node_size = 48 + data_size;
    if (new_node_size < t->split_threshold) return inner_new_insert(n, key, ks, left, right);

    uint32_t n_left = n->count >> 1;
    const uint8_t *sep_key = n->key[n_left];
    uint16_t sep_ks = n->klen[n_left];
    void *sep_child = n->child[n_left];
    int cmp = orc_key_compare(key, ks, sep_key, sep_ks);
    if (cmp == 0) cmp = (int)ks - (int)sep_ks;
    orc_inner *l, *r;
    if (cmp < 0) {
        l = inner_new_range(n, 0, n_left, key, ks, left, right, NULL);
        r = inner_new_range(n, n_left + 1, n->count - n_left - 1, NULL, 0, NULL, NULL, sep_child);
    } else {
        l = inner_new_range(n, 0, n_left, NULL, 0, NULL, NULL, NULL);
        r = inner_new_range(n, n_left + 1, n->count - n_left - 1, key, ks, left, right, sep_child);
    }
    garbage_add(t, n); /* this node is replaced by l and r */
    pop(st);
    frame_t *pf = top(st);
    if (!pf) return inner_new_root(sep_key, sep_ks, l, r);
    pf->node->frozen = 1;
    return inner_prepare_for_split(t, pf->node, st, sep_key, sep_ks, l, r);
}

static uint8_t *leaf_new(orc_tree *t) { /* LeafNode::New, b_tree.cpp:791-797 */
    uint8_t *n = leaf_block_alloc(t->leaf_node_size);
    memset(n, 0, t->leaf_node_size);
    n[OFF_ISLEAF] = 1;
    *l_size(n) = t->leaf_node_size;
    return n;
}

/* A slot's meta word is read by every search of its leaf and, under orc_update_batch_mt,
 * written by the writer that owns its key while other writers search the same leaf: relaxed
 * atomic loads and stores (the reference CASes the word, b_tree.cpp:1106-1120) -- the other
 * writers' searches only need its visible bit and key length, which an update never changes. */
static inline uint64_t meta_load(const orc_rmeta *m) { return __atomic_load_n(&m->meta, __ATOMIC_RELAXED); }
static inline void meta_store(orc_rmeta *m, uint64_t v) { __atomic_store_n(&m->meta, v, __ATOMIC_RELAXED); }

/* BaseNode::SearchRecordMeta, b_tree.cpp:18-122 (called with check_concurrency == true by
 * LeafNode::Read because of the argument shift at b_tree.cpp:1044-1045). */
static int64_t search_record_meta(uint8_t *n, const uint8_t *key, uint16_t ks, int check_concurrency) {
    uint32_t sorted = *l_sorted(n);
    for (uint32_t i = 0; i < sorted; i++) {
        uint64_t m = meta_load(l_meta(n, i));
        if (m == 0) continue;
        const uint8_t *ck = l_key(n, m);
        int cmp = orc_key_compare(key, ks, ck, m_keylen(m));
        if (cmp == 0 && m_visible(m)) return i;
    }
    uint32_t cnt = st_count(*l_status(n));
    for (uint32_t i = sorted; i < cnt; i++) {
        uint64_t m = meta_load(l_meta(n, i));
        if (m_visible(m)) {
            uint16_t cs = m_keylen(m);
            if (cs == ks && orc_key_compare(key, ks, l_key(n, m), cs) == 0) return i;
        } else if (!check_concurrency) {
            return i;
        }
    }
    return -1;
}

/* LeafNode::Insert, b_tree.cpp:809-947 (single writer) */
static int leaf_insert(orc_tree *t, uint8_t *n, const uint8_t *key, uint16_t ks, const uint8_t *payload,
                       uint32_t commit_id, orc_loc *loc, orc_rmeta **out) {
    uint64_t status = *l_status(n);
    if (st_frozen(status)) return ORC_RET_NODE_FROZEN;
    /* CheckUnique, b_tree.cpp:1395-1417 (a bulk load of distinct keys cannot hit:
     * skipped, the resulting leaves are the same -- tests/test_oracle_golden.py) */
    int64_t hit = t->bulk ? -1 : search_record_meta(n, key, ks, 1);
    if (hit >= 0) {
        uint64_t m = l_meta(n, (uint32_t)hit)->meta;
        if (m_inserting(m)) return ORC_RET_INVALID; /* ReCheck vs an in-flight update: unsupported */
        if (orc_key_compare(key, ks, l_key(n, m), m_keylen(m)) == 0) return ORC_RET_KEY_EXISTS;
    }
    uint32_t new_size = used_space(status) + META_SZ + pad_key(ks) + t->payload_size;
    if (new_size >= t->leaf_node_size) return ORC_RET_NOT_ENOUGH_SPACE; /* split_threshold == leaf_node_size (:1869-1871) */
    uint32_t total = pad_key(ks) + t->payload_size;
    uint64_t desired = status + ((1ull << 44) + ((uint64_t)total << 22)); /* PrepareForInsert */
    uint32_t slot = st_count(status);
    orc_rmeta *mp = l_meta(n, slot);
    if (mp->meta != 0) return ORC_RET_RETRY_FAILURE;
    uint64_t offset = *l_size(n) - st_block(desired);
    /* PrepareForInsert(offset,key_len,commit_id), record_meta.h:114-120 */
    mp->meta = ((uint64_t)ks << 48) | (offset << 32) | commit_id | M_CONTROL | M_VISIBLE;
    *l_status(n) = desired;
    loc->leaf = n;
    loc->slot = slot;
    mp->loc = loc;
    memcpy(n + offset, key, ks);
    memcpy(n + offset + pad_key(ks), payload, t->payload_size);
    *out = mp;
    return ORC_RET_OK;
}

typedef struct { const uint8_t *k; uint16_t ks; orc_rmeta *m; } sortrec_t;
static int sortrec_cmp(const void *a, const void *b) {
    const sortrec_t *x = a, *y = b;
    int c = orc_key_compare(x->k, x->ks, y->k, y->ks);
    return (c > 0) - (c < 0);
}

/* LeafNode::CopyFrom, b_tree.cpp:1486-1545 */
static void leaf_copy_from(orc_tree *t, uint8_t *dst, uint8_t *src, sortrec_t *v, uint32_t nv) {
    uint32_t offset = *l_size(dst);
    uint32_t nrec = 0;
    for (uint32_t i = 0; i < nv; i++) {
        orc_rmeta mm = *v[i].m;
        if (mm.meta == 0) continue;
        if (m_padded(mm.meta) == 0) continue; /* GetRawRecord false */
        uint32_t total = m_padded(mm.meta) + t->payload_size;
        offset -= total;
        memcpy(dst + offset, src + m_offset(mm.meta), total);
        orc_rmeta *dm = l_meta(dst, nrec);
        orc_loc *loc = mm.loc;
        if (loc) {
            loc->leaf = dst;
            loc->slot = nrec;
        }
        dm->loc = loc;
        dm->next = mm.next;
        dm->meta = m_finalize_insert(offset, m_keylen(mm.meta), m_cstamp(mm.meta));
        nrec++;
    }
    uint64_t s = *l_status(dst);
    s = st_set_block(s, *l_size(dst) - offset);
    s = st_set_count(s, nrec);
    *l_status(dst) = s;
    *l_sorted(dst) = nrec;
}

/* LeafNode::PrepareForSplit, b_tree.cpp:1558-1690 */
static int leaf_prepare_for_split(orc_tree *t, uint8_t *n, stack_t_ *st, uint8_t **pl, uint8_t **pr,
                                  orc_inner **new_parent) {
    uint32_t cnt = st_count(*l_status(n));
    if (cnt < 3) return 0;
    uint8_t *l = leaf_new(t), *r = leaf_new(t);
    sortrec_t *v = xmalloc(sizeof(sortrec_t) * (cnt + 1));
    uint32_t nv = 0, total = 0;
    for (uint32_t i = 0; i < cnt; i++) {
        orc_rmeta *mp = l_meta(n, i);
        if (mp->meta == 0) continue;
        if (m_visible(mp->meta) && m_keylen(mp->meta) > 0) {
            v[nv].k = n + m_offset(mp->meta);
            v[nv].ks = m_keylen(mp->meta);
            v[nv].m = mp;
            nv++;
            total += m_padded(mp->meta) + t->payload_size;
        }
    }
    qsort(v, nv, sizeof(sortrec_t), sortrec_cmp); /* Sorter::Sort (unique keys -> same order as std::sort) */
    if (total == 0) {
        free(v);
        leaf_block_free(t->leaf_node_size, l, 0);
        leaf_block_free(t->leaf_node_size, r, 0);
        return 0;
    }
    for (uint32_t i = 0; i < cnt; i++) { /* CopyFrom drops these records: their locations dangle */
        orc_rmeta *mp = l_meta(n, i);
        if (!(mp->meta != 0 && m_visible(mp->meta) && m_keylen(mp->meta) > 0) && mp->loc) mp->loc->leaf = NULL;
    }
    int32_t left_size = (int32_t)(total / 2);
    uint32_t nleft = 0;
    for (uint32_t i = 0; i < nv; i++) {
        ++nleft;
        left_size -= (int32_t)(m_padded(v[i].m->meta) + t->payload_size);
        if (left_size <= 0) break;
    }
    leaf_copy_from(t, l, n, v, nleft);
    leaf_copy_from(t, r, n, v + nleft, nv - nleft);
    /* separator = last key of the left node (in the frozen old node) */
    const uint8_t *sep = v[nleft - 1].k;
    uint16_t sep_ks = v[nleft - 1].ks;
    frame_t *pf = top(st);
    if (!pf) {
        *new_parent = inner_new_root(sep, sep_ks, l, r);
    } else {
        pf->node->frozen = 1;
        *new_parent = inner_prepare_for_split(t, pf->node, st, sep, sep_ks, l, r);
    }
    free(v);
    *pl = l;
    *pr = r;
    return 1;
}

static orc_loc *new_loc(orc_tree *t) { /* BTree::RecordIndirectLocation */
    orc_loc *l = xmalloc(sizeof(orc_loc));
    l->leaf = NULL;
    l->slot = 0;
    l->id = t->nlocs;
    if (t->nlocs == t->caplocs) {
        t->caplocs = t->caplocs ? 2 * t->caplocs : 1024;
        t->locs = realloc(t->locs, t->caplocs * sizeof(orc_loc *));
    }
    t->locs[t->nlocs++] = l;
    return l;
}

/* BTree::Insert, b_tree.cpp:1849-2020 */
static int btree_insert(orc_tree *t, const uint8_t *key, uint16_t ks, const uint8_t *payload, uint32_t commit_id,
                        orc_rmeta **out) {
    stack_t_ st;
    for (int guard = 0; guard < 64; guard++) {
        st.n = 0;
        uint8_t *leaf = traverse_to_leaf(t, &st, key, ks, 1);
        orc_loc *loc = new_loc(t);
        int rc = leaf_insert(t, leaf, key, ks, payload, commit_id, loc, out);
        if (rc == ORC_RET_OK) return rc;
        if (rc == ORC_RET_KEY_EXISTS || rc == ORC_RET_RETRY_FAILURE || rc == ORC_RET_INVALID) return rc;
        /* NotEnoughSpace: freeze and split */
        *l_status(leaf) |= (1ull << 60);
        uint8_t *l = NULL, *r = NULL;
        orc_inner *np = NULL;
        if (!leaf_prepare_for_split(t, leaf, &st, &l, &r, &np)) return ORC_RET_RETRY_FAILURE;
        frame_t *f = pop(&st);
        orc_inner *old_parent = f ? f->node : NULL;
        f = pop(&st);
        orc_inner *grand = f ? f->node : NULL;
        if (grand) {
            grand->child[f->meta_index] = np; /* InternalNode::Update, b_tree.cpp:635-662 */
        } else {
            t->root = np; /* ChangeRoot */
        }
        garbage_add(t, leaf);
        if (old_parent) garbage_add(t, old_parent);
        garbage_release(t);
    }
    return ORC_RET_RETRY_FAILURE;
}

/* ---------------------------------------------------------------- public: build */
orc_tree *orc_tree_new(uint32_t leaf_node_size, uint32_t split_threshold, uint32_t payload_size) {
    orc_tree *t = xmalloc(sizeof(orc_tree));
    memset(t, 0, sizeof(*t));
    t->leaf_node_size = leaf_node_size;
    t->split_threshold = split_threshold;
    t->payload_size = payload_size;
    t->merge_threshold = 32 * 1024;
    t->key_pad = 8;
    t->root = leaf_new(t);
    return t;
}

void orc_tree_set_merge_threshold(orc_tree *t, uint32_t merge_threshold) { t->merge_threshold = merge_threshold; }
void orc_tree_set_key_pad(orc_tree *t, uint32_t key_pad) { t->key_pad = key_pad < 8 ? 8 : key_pad; }
void orc_tree_set_bulk(orc_tree *t, int bulk) { t->bulk = bulk; }

static void free_subtree(orc_tree *t, void *n) {
    if (is_leaf(n)) {
        leaf_block_free(t->leaf_node_size, n, 1);
        return;
    }
    orc_inner *p = n;
    for (uint32_t i = 0; i < p->count; i++) free_subtree(t, p->child[i]);
    inner_free(p);
}

void orc_tree_free(orc_tree *t) {
    if (!t) return;
    free_subtree(t, t->root);
    for (orc_copy *c = t->copies; c;) {
        orc_copy *nx = c->reg_next;
        free(c->image);
        free(c->readers);
        free(c);
        c = nx;
    }
    for (orc_th *h = t->ths; h;) {
        orc_th *nx = h->reg_next;
        free(h->slot);
        free(h);
        h = nx;
    }
    for (uint64_t i = 0; i < t->nlocs; i++) free(t->locs[i]);
    free(t->locs);
    free(t->garbage);
    free(t->copy_by_id);
    free(t);
}

int orc_insert(orc_tree *t, const uint8_t *key, uint32_t key_size, const uint8_t *payload, uint32_t commit_id) {
    orc_rmeta *mp = NULL;
    int rc = btree_insert(t, key, (uint16_t)key_size, payload, commit_id, &mp);
    if (rc == ORC_RET_OK) {
        /* BTree::FinalizeInsert, b_tree.cpp:2238-2251 */
        mp->meta = m_finalize_insert(m_offset(mp->meta), m_keylen(mp->meta), commit_id);
    }
    return rc;
}

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t orc_payload_word(uint64_t rowid, uint32_t j) { return splitmix64((rowid << 8) ^ j); }

void orc_fill_payload(uint64_t rowid, int mode, uint8_t *dst, uint32_t payload_size) {
    if (mode == 0) { /* memset(tuple.cols[i], rowid, ...) ycsb_loader.cpp:149-150 */
        memset(dst, (int)(rowid & 0xFF), payload_size);
        return;
    }
    for (uint32_t j = 0; j * 8 < payload_size; j++) {
        uint64_t w = orc_payload_word(rowid, j);
        uint32_t nb = payload_size - j * 8 < 8 ? payload_size - j * 8 : 8;
        memcpy(dst + j * 8, &w, nb);
    }
}

uint64_t orc_load_keys(orc_tree *t, const uint64_t *keys, uint64_t n, uint32_t key_size, int payload_mode) {
    uint8_t *payload = xmalloc(t->payload_size + 8);
    uint64_t ok = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t k = keys[i];
        orc_fill_payload(k, payload_mode, payload, t->payload_size);
        if (orc_insert(t, (const uint8_t *)&k, key_size, payload, INVALID_CID) == ORC_RET_OK) ok++;
    }
    free(payload);
    return ok;
}

uint64_t orc_load_rows(orc_tree *t, const uint8_t *keys, uint32_t key_stride, uint32_t key_size,
                       const uint8_t *payloads, uint32_t payload_stride, uint64_t n) {
    uint64_t ok = 0;
    for (uint64_t i = 0; i < n; i++)
        if (orc_insert(t, keys + i * key_stride, key_size, payloads + i * (uint64_t)payload_stride, INVALID_CID) ==
            ORC_RET_OK)
            ok++;
    return ok;
}

uint64_t orc_load_ycsb(orc_tree *t, uint64_t begin, uint64_t end, uint32_t key_size, int payload_mode) {
    uint8_t *payload = xmalloc(t->payload_size + 8);
    uint64_t ok = 0;
    for (uint64_t rowid = begin; rowid < end; rowid++) {
        uint64_t k = rowid; /* uint32_t k_ = rowid for the 4-byte driver (ycsb_loader.cpp:152) */
        orc_fill_payload(rowid, payload_mode, payload, t->payload_size);
        if (orc_insert(t, (const uint8_t *)&k, key_size, payload, INVALID_CID) == ORC_RET_OK) ok++;
    }
    free(payload);
    return ok;
}

/* ---------------------------------------------------------------- parallel load (CPU baseline)
 * LoadYCSBRows of rows [begin, end) built by several threads with the same LEAVES as the
 * single loader.  Leaves only ever split during inserts and a split depends only on the
 * leaf's own records, so once a leaf boundary exists it stays: after the first rows are
 * inserted sequentially, the leaves are cut into nthreads groups of consecutive leaves and
 * each thread inserts, in row order, the remaining rows that route into its group (into a
 * private tree holding just that group).  The inner levels are then rebuilt bottom-up over
 * all leaves with the split-time separators and the reference's observed fanout (273
 * children per inner node: 20,498 leaves under 75 bottom nodes at 1M rows):
 * routing is identical, inner node shapes are not (tests/test_oracle_golden.py). */
typedef struct { void **node; const uint8_t **sep; uint16_t *seplen; uint64_t n, cap; } node_list;

static void nl_push(node_list *L, void *node, const uint8_t *sep, uint16_t seplen) {
    if (L->n == L->cap) {
        L->cap = L->cap ? 2 * L->cap : 1024;
        L->node = realloc(L->node, L->cap * sizeof(void *));
        L->sep = realloc((void *)L->sep, L->cap * sizeof(uint8_t *));
        L->seplen = realloc(L->seplen, L->cap * sizeof(uint16_t));
        if (!L->node || !L->sep || !L->seplen) abort();
    }
    L->node[L->n] = node;
    L->sep[L->n] = sep;
    L->seplen[L->n] = seplen;
    L->n++;
}

/* leaves in key order, each with its lower separator (the inner key routing to it) */
static void collect_leaves(void *node, node_list *L, const uint8_t *lo, uint16_t lo_len) {
    if (is_leaf(node)) {
        nl_push(L, node, lo, lo_len);
        return;
    }
    orc_inner *p = node;
    for (uint32_t i = 0; i < p->count; i++)
        collect_leaves(p->child[i], L, i == 0 ? lo : p->key[i], i == 0 ? lo_len : p->klen[i]);
}

static void free_inner_only(void *node) {
    if (is_leaf(node)) return;
    orc_inner *p = node;
    for (uint32_t i = 0; i < p->count; i++) free_inner_only(p->child[i]);
    inner_free(p);
}

/* an inner node over entries [b, e) of L: slot 0 = dummy key, slot i = L->sep[b+i] */
static orc_inner *inner_over(node_list *L, uint64_t b, uint64_t e) {
    uint32_t nr = (uint32_t)(e - b), kbytes = 0, size = 48;
    for (uint64_t i = b + 1; i < e; i++) kbytes += L->seplen[i];
    orc_inner *n = inner_alloc(nr, kbytes);
    kb_t kb = {0};
    for (uint64_t i = b; i < e; i++) {
        int first = i == b;
        inner_set(n, &kb, (uint32_t)(i - b), first ? NULL : L->sep[i], first ? 0 : L->seplen[i], L->node[i]);
        size += pad_key(first ? 0 : L->seplen[i]) + 8 + META_SZ;
    }
    n->size = size;
    n->count = nr;
    return n;
}

/* bottom-up inner levels over a list of children; the list is consumed */
static void *build_levels(node_list *L, uint32_t fanout) {
    while (L->n > 1) {
        node_list up = {0};
        for (uint64_t b = 0; b < L->n; b += fanout) {
            uint64_t e = b + fanout < L->n ? b + fanout : L->n;
            nl_push(&up, inner_over(L, b, e), L->sep[b], L->seplen[b]);
        }
        free(L->node);
        free((void *)L->sep);
        free(L->seplen);
        *L = up;
    }
    void *root = L->node[0];
    free(L->node);
    free((void *)L->sep);
    free(L->seplen);
    return root;
}

typedef struct {
    orc_tree *sub;
    const uint8_t *part;
    uint8_t g;
    uint64_t begin, end;
    uint32_t ks;
    int mode;
    uint64_t ok;
} pload_t;

static void *pload_worker(void *arg) {
    pload_t *p = arg;
    uint8_t *payload = xmalloc(p->sub->payload_size + 8);
    for (uint64_t r = p->begin; r < p->end; r++) {
        if (p->part[r - p->begin] != p->g) continue;
        uint64_t k = r;
        orc_fill_payload(r, p->mode, payload, p->sub->payload_size);
        if (orc_insert(p->sub, (const uint8_t *)&k, p->ks, payload, INVALID_CID) == ORC_RET_OK) p->ok++;
    }
    free(payload);
    return NULL;
}

typedef struct {
    const uint8_t **bsep;
    const uint16_t *blen;
    uint32_t nb;
    uint8_t *part;
    uint64_t base, b, e;
    uint32_t ks;
} route_t;

static void *route_worker(void *arg) {
    route_t *r = arg;
    for (uint64_t i = r->b; i < r->e; i++) {
        uint64_t k = r->base + i;
        uint32_t lo = 0, hi = r->nb; /* groups g > 0 start above separator bsep[g-1] */
        while (lo < hi) {
            uint32_t mid = (lo + hi) / 2;
            if (orc_key_compare((const uint8_t *)&k, r->ks, r->bsep[mid], r->blen[mid]) > 0) lo = mid + 1;
            else hi = mid;
        }
        r->part[i] = (uint8_t)lo;
    }
    return NULL;
}

uint64_t orc_load_ycsb_parallel(orc_tree *t, uint64_t begin, uint64_t end, uint32_t key_size, int payload_mode,
                                int nthreads) {
    if (nthreads > 64) nthreads = 64;
    uint64_t seq_end = begin + 100000 < end ? begin + 100000 : end;
    uint64_t ok = orc_load_ycsb(t, begin, seq_end, key_size, payload_mode);
    node_list leaves = {0};
    collect_leaves(t->root, &leaves, NULL, 0);
    if (nthreads < 2 || seq_end == end || leaves.n < (uint64_t)nthreads) {
        free(leaves.node);
        free((void *)leaves.sep);
        free(leaves.seplen);
        return ok + orc_load_ycsb(t, seq_end, end, key_size, payload_mode);
    }
    int T = nthreads;
    uint64_t m = leaves.n;
    /* group g = leaves [m*g/T, m*(g+1)/T); boundary g-1 = lower separator of its first leaf */
    const uint8_t *bsep[64];
    uint16_t blen[64];
    orc_tree *sub[64];
    for (int g = 0; g < T; g++) {
        uint64_t b = m * (uint64_t)g / T, e = m * (uint64_t)(g + 1) / T;
        if (g > 0) {
            bsep[g - 1] = leaves.sep[b];
            blen[g - 1] = leaves.seplen[b];
        }
        sub[g] = orc_tree_new(t->leaf_node_size, t->split_threshold, t->payload_size);
        leaf_block_free(t->leaf_node_size, sub[g]->root, 0);
        sub[g]->merge_threshold = t->merge_threshold;
        sub[g]->key_pad = t->key_pad;
        sub[g]->bulk = t->bulk;
        sub[g]->root = e - b == 1 ? leaves.node[b] : (void *)inner_over(&leaves, b, e);
    }
    uint64_t rest = end - seq_end;
    uint8_t *part = xmalloc(rest ? rest : 1);
    pthread_t th[64];
    route_t rt[64];
    for (int i = 0; i < T; i++) {
        route_t r = {bsep, blen, (uint32_t)(T - 1), part, seq_end, rest * (uint64_t)i / T,
                     rest * (uint64_t)(i + 1) / T, key_size};
        rt[i] = r;
        pthread_create(&th[i], NULL, route_worker, &rt[i]);
    }
    for (int i = 0; i < T; i++) pthread_join(th[i], NULL);
    pload_t pl[64];
    for (int g = 0; g < T; g++) {
        pload_t p = {sub[g], part, (uint8_t)g, seq_end, end, key_size, payload_mode, 0};
        pl[g] = p;
        pthread_create(&th[g], NULL, pload_worker, &pl[g]);
    }
    for (int g = 0; g < T; g++) {
        pthread_join(th[g], NULL);
        ok += pl[g].ok;
    }
    free(part);
    /* every leaf in key order with its lower separator, then the inner levels */
    node_list all = {0};
    for (int g = 0; g < T; g++) {
        uint64_t first = all.n;
        collect_leaves(sub[g]->root, &all, g ? bsep[g - 1] : NULL, g ? blen[g - 1] : 0);
        (void)first;
    }
    void *old_root = t->root;
    t->root = build_levels(&all, 273);
    free_inner_only(old_root); /* the boundary separators lived here: copied by inner_set */
    for (int g = 0; g < T; g++) {
        orc_tree *s = sub[g];
        free_inner_only(s->root);
        for (uint64_t i = 0; i < s->nlocs; i++) {
            if (t->nlocs == t->caplocs) {
                t->caplocs = t->caplocs ? 2 * t->caplocs : 1024;
                t->locs = realloc(t->locs, t->caplocs * sizeof(orc_loc *));
            }
            s->locs[i]->id = t->nlocs; /* this build's allocation order differs from the single loader's */
            t->locs[t->nlocs++] = s->locs[i];
        }
        free(s->locs);
        free(s->garbage);
        free(s);
    }
    free(leaves.node);
    free((void *)leaves.sep);
    free(leaves.seplen);
    return ok;
}

/* ---------------------------------------------------------------- read path */
static orc_copy *copy_of(uint64_t next) {
    if (next == 0 || NEXT_KIND(next) != NEXT_COPY) return NULL;
    orc_copy *c = NEXT_PTR(next);
    return c->live ? c : NULL; /* EphemeralPool::GetOversionHeader (ephemeral_pool.cpp:110-123) */
}

/* canonical tuple row: [key padded to key_pad][payload] (key_pad = 8 for keys of <= 8 bytes,
 * the padded key width for wider fixed-width keys) */
static void emit_canonical(orc_tree *t, uint8_t *rec, const uint8_t *key, uint16_t ks, const uint8_t *payload) {
    if (!rec) return;
    memset(rec, 0, t->key_pad);
    memcpy(rec, key, ks > t->key_pad ? t->key_pad : ks);
    memcpy(rec + t->key_pad, payload, t->payload_size);
}

/* BTree::Read (b_tree.cpp:2066-2129) followed by the point-lookup branch of
 * IndexScanExecutor::Execute (executor.h:374-454), canonical output.
 * for_update: Read(..., is_for_update = true) -- the copy branch is taken only when
 * `meta->IsInserting() && !is_for_update` (:2087), so the writer reads its own in-flight record
 * from the leaf like any other (:2114-2120, cstamp = the reader's id, no AddReader); the
 * executor's rule is unchanged apart from skipping PerformRead (executor.h:388), which the
 * oracle's outputs do not model (the caller knows it asked for update). */
static int read_one_fu(orc_tree *t, const uint8_t *key, uint16_t ks, uint32_t read_id, int for_update,
                       orc_read_out *o, uint8_t *rec);
static int read_one(orc_tree *t, const uint8_t *key, uint16_t ks, uint32_t read_id, orc_read_out *o, uint8_t *rec) {
    return read_one_fu(t, key, ks, read_id, 0, o, rec);
}
static int read_one_fu(orc_tree *t, const uint8_t *key, uint16_t ks, uint32_t read_id, int for_update,
                       orc_read_out *o, uint8_t *rec) {
    memset(o, 0, sizeof(*o));
    o->copy_sstamp = MAX_CID;
    uint32_t rs = t->key_pad + t->payload_size;
    if (rec) memset(rec, 0, rs);
    uint8_t *leaf = traverse_to_leaf(t, NULL, key, ks, 1);
    int64_t slot = search_record_meta(leaf, key, ks, 1);
    if (slot < 0) {
        o->status = ORC_ST_NOT_FOUND;
        return 0;
    }
    orc_rmeta *mp = l_meta(leaf, (uint32_t)slot);
    uint64_t m = mp->meta;
    o->rec_cstamp = m_cstamp(m);
    orc_copy *pc = copy_of(mp->next); /* PerformRead's GetOversionHeader(meta.next_ptr) */
    if (pc) {
        o->copy_present = 1;
        o->copy_sstamp = pc->sstamp;
    }
    const uint8_t *rkey, *rpay;
    uint64_t next_tuple;
    int from_copy = 0;
    if (m_inserting(m) && !for_update) {
        orc_copy *c = pc;
        if (!c) { /* copy location 0 / header gone: Read returns nullptr */
            o->status = ORC_ST_NOT_FOUND;
            return 0;
        }
        rkey = c->image; /* Record::Neww: key(keylen) then payload */
        rpay = c->image + c->key_len;
        o->cstamp = c->rstamp;
        next_tuple = c->next;
        from_copy = 1;
    } else {
        rkey = leaf + m_offset(m);
        rpay = leaf + m_offset(m) + m_padded(m);
        o->cstamp = read_id;
        next_tuple = mp->next;
    }
    if (read_id >= o->rec_cstamp) {
        o->status = from_copy ? ORC_ST_COPY : ORC_ST_LATEST;
        emit_canonical(t, rec, rkey, m_keylen(m), rpay);
        return 0;
    }
    /* older snapshot: walk the TupleHeader chain (executor.h:407-449) */
    if (next_tuple == 0 || NEXT_KIND(next_tuple) != NEXT_TH) {
        o->status = ORC_ST_CHAIN_MISS;
        return 0;
    }
    orc_th *th = NEXT_PTR(next_tuple);
    for (;;) {
        o->hops++;
        if (th->begin_id == INVALID_CID || th->comm_id == INVALID_CID) {
            o->status = ORC_ST_FAIL_INVALID_TS;
            return 0;
        }
        if (read_id >= th->begin_id && read_id <= th->comm_id) {
            o->status = ORC_ST_OLD;
            o->cstamp = th->begin_id;
            emit_canonical(t, rec, th->slot, th->key_len, th->slot + th->key_len);
            return 0;
        }
        uint64_t nx = th->next;
        if (nx == 0 || nx == ~0ull || NEXT_KIND(nx) != NEXT_TH) {
            o->status = ORC_ST_CHAIN_MISS;
            return 0;
        }
        th = NEXT_PTR(nx);
    }
}

int orc_read(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t read_id, orc_read_out *out, uint8_t *rec) {
    return read_one(t, key, (uint16_t)key_size, read_id, out, rec);
}

int orc_read_fu(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t read_id, int for_update,
                orc_read_out *out, uint8_t *rec) {
    return read_one_fu(t, key, (uint16_t)key_size, read_id, for_update, out, rec);
}

typedef struct {
    orc_tree *t;
    const uint64_t *keys;
    uint32_t ks;
    const uint32_t *rids;
    uint64_t b, e;
    orc_read_out *outs;
    uint8_t *recs;
    uint32_t scan_size;
    uint32_t *counts;
    uint64_t sum;
    const uint8_t *kbytes; /* byte keys (kstride apart) instead of u64 keys */
    uint32_t kstride;
} job_t;

static const uint8_t *job_key(job_t *j, uint64_t i, uint64_t *tmp) {
    if (j->kbytes) return j->kbytes + i * j->kstride;
    *tmp = j->keys[i];
    return (const uint8_t *)tmp;
}

static void *read_worker(void *arg) {
    job_t *j = arg;
    uint32_t rs = j->t->key_pad + j->t->payload_size;
    for (uint64_t i = j->b; i < j->e; i++) {
        uint64_t k;
        read_one(j->t, job_key(j, i, &k), (uint16_t)j->ks, j->rids ? j->rids[i] : 0xFFFFFFFEu, &j->outs[i],
                 j->recs ? j->recs + i * rs : NULL);
    }
    return NULL;
}

static void run_jobs(void *(*fn)(void *), job_t *proto, uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[256];
    job_t jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = *proto;
        jobs[i].b = n * (uint64_t)i / nthreads;
        jobs[i].e = n * (uint64_t)(i + 1) / nthreads;
        jobs[i].sum = 0;
        pthread_create(&th[i], NULL, fn, &jobs[i]);
    }
    proto->sum = 0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        proto->sum += jobs[i].sum;
    }
}

int orc_read_batch(orc_tree *t, const uint64_t *keys, uint32_t key_size, const uint32_t *read_ids, uint64_t n,
                   orc_read_out *outs, uint8_t *recs, int nthreads) {
    job_t j = {t, keys, key_size, read_ids, 0, n, outs, recs, 0, NULL, 0, NULL, 0};
    run_jobs(read_worker, &j, n, nthreads);
    return 0;
}

int orc_read_batch_k(orc_tree *t, const uint8_t *keys, uint32_t key_stride, uint32_t key_size,
                     const uint32_t *read_ids, uint64_t n, orc_read_out *outs, uint8_t *recs, int nthreads) {
    job_t j = {t, NULL, key_size, read_ids, 0, n, outs, recs, 0, NULL, 0, keys, key_stride};
    run_jobs(read_worker, &j, n, nthreads);
    return 0;
}

/* CPU baseline worker: the reference's work per read -- traverse, leaf probe, heap Record
 * (Record::New, b_tree.h:407-428) and the executor's `new T` + memcpy (executor.h:396-401),
 * both freed afterwards -- without the txn bookkeeping. */
static void *timed_worker(void *arg) {
    job_t *j = arg;
    orc_tree *t = j->t;
    uint64_t sum = 0;
    orc_read_out o;
    for (uint64_t i = j->b; i < j->e; i++) {
        uint64_t k = j->keys[i];
        const uint8_t *key = (const uint8_t *)&k;
        uint16_t ks = (uint16_t)j->ks;
        uint32_t rid = j->rids ? j->rids[i] : 0xFFFFFFFEu;
        uint8_t *leaf = traverse_to_leaf(t, NULL, key, ks, 1);
        int64_t slot = search_record_meta(leaf, key, ks, 1);
        if (slot < 0) continue;
        orc_rmeta *mp = l_meta(leaf, (uint32_t)slot);
        uint64_t m = mp->meta;
        if (m_inserting(m)) { /* rare: fall back to the full restatement */
            uint8_t *rec = xmalloc(8 + t->payload_size);
            read_one(t, key, ks, rid, &o, rec);
            sum += rec[8];
            free(rec);
            continue;
        }
        size_t rsz = 48 + 4 + m_padded(m) + t->payload_size;
        uint8_t *r = xmalloc(rsz);
        memcpy(r + 52, leaf + m_offset(m), m_padded(m));
        memcpy(r + 52 + m_padded(m), leaf + m_offset(m) + m_padded(m), t->payload_size);
        if (rid >= m_cstamp(m)) {
            uint8_t *tup = xmalloc(4 + t->payload_size);
            memcpy(tup, r + 52, 4 + t->payload_size);
            sum += tup[4 + (i % t->payload_size)];
            free(tup);
        } else {
            read_one(t, key, ks, rid, &o, NULL);
            sum += o.status;
        }
        free(r);
    }
    j->sum = sum;
    return NULL;
}

uint64_t orc_read_batch_timed(orc_tree *t, const uint64_t *keys, uint32_t key_size, const uint32_t *read_ids,
                              uint64_t n, int nthreads, double *seconds) {
    job_t j = {t, keys, key_size, read_ids, 0, n, NULL, NULL, 0, NULL, 0, NULL, 0};
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    run_jobs(timed_worker, &j, n, nthreads);
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    return j.sum;
}

/* ---------------------------------------------------------------- full transactions
 * CPU baseline "full-txn" mode: RunMixed (benchmark/ycsb/ycsb_mixed.cpp:18-140) with every op
 * a read, through IndexScanExecutor (executor.h:374-454) and the Index-SSN read side:
 *   BeginTransaction     transaction_manager.cpp:280-309  read_id = tid_counter++, new context,
 *                                                         active_tids.Insert(read_id)
 *   PerformRead          transaction_manager.cpp:362-410  RecordRead (rw-set insert, hash on the
 *                        meta word, equality on loc_ptr: txn_context.h:16-24), SetPredecessor,
 *                        GetOversionHeader(next_ptr) -> IncreaseWRCount + SetSuccessor,
 *                        CheckExclusion
 *   CommitTransaction    transaction_manager.cpp:535-815  commit id = tid_counter++, FindMinSstamp
 *                        (:113-221) and FindMaxPstamp (:29-102) over copies of the rw-set,
 *                        post-commit READ entries (:749-764), active_tids.Insert(commit_id)
 * The reference never erases active_tids nor deletes contexts (EndTransaction is empty,
 * :311-322); here both are released after the timed region. */
typedef struct rw_node { orc_rmeta *loc; uint64_t meta; int type; struct rw_node *next; } rw_node;
typedef struct txn_ctx {
    uint32_t read_id, commit_id, pred, succ;
    int aborted, finished;
    rw_node *bucket[16]; /* rw_set_ (ReadWriteSet, txn_context.h:28) */
    uint32_t nrw;
} txn_ctx;

typedef struct tid_node { uint32_t tid; txn_ctx *ctx; struct tid_node *next; } tid_node;
#define TID_STRIPES 64
#define TID_BUCKETS (1u << 20)
typedef struct { /* active_tids: concurrent map tid -> context (transaction_manager.h) */
    pthread_mutex_t lock[TID_STRIPES];
    tid_node **b;
} tid_map;

static void tid_insert(tid_map *m, uint32_t tid, txn_ctx *ctx) {
    uint32_t h = (uint32_t)(((uint64_t)tid * 0x9ddfea08eb382d69ull) >> 44) & (TID_BUCKETS - 1);
    tid_node *n = xmalloc(sizeof(tid_node));
    n->tid = tid;
    n->ctx = ctx;
    pthread_mutex_t *l = &m->lock[h % TID_STRIPES];
    pthread_mutex_lock(l);
    n->next = m->b[h];
    m->b[h] = n;
    pthread_mutex_unlock(l);
}

static int tid_find(tid_map *m, uint32_t tid, txn_ctx **out) {
    uint32_t h = (uint32_t)(((uint64_t)tid * 0x9ddfea08eb382d69ull) >> 44) & (TID_BUCKETS - 1);
    pthread_mutex_t *l = &m->lock[h % TID_STRIPES];
    int found = 0;
    pthread_mutex_lock(l);
    for (tid_node *n = m->b[h]; n; n = n->next)
        if (n->tid == tid) {
            *out = n->ctx;
            found = 1;
            break;
        }
    pthread_mutex_unlock(l);
    return found;
}

static uint32_t rw_hash(uint64_t meta) { return (uint32_t)((meta * 0x9E3779B97F4A7C15ull) >> 60); }

/* TransactionContext::RecordRead, transaction_context.cpp:88-99 */
static int rw_record_read(txn_ctx *c, orc_rmeta *loc, uint64_t meta) {
    uint32_t h = rw_hash(meta);
    for (rw_node *n = c->bucket[h]; n; n = n->next)
        if (n->loc == loc) return 0;
    rw_node *n = xmalloc(sizeof(rw_node));
    n->loc = loc;
    n->meta = meta;
    n->type = 0; /* RWType::READ */
    n->next = c->bucket[h];
    c->bucket[h] = n;
    c->nrw++;
    return 1;
}

/* `auto rw_set = current_txn->GetReadWriteSet()` copies the map (FindMinSstamp :111,
 * FindMaxPstamp :30): flattened here into a per-call array */
static uint32_t rw_copy(txn_ctx *c, rw_node *out) {
    uint32_t k = 0;
    for (int b = 0; b < 16; b++)
        for (rw_node *n = c->bucket[b]; n; n = n->next) out[k++] = *n;
    return k;
}

typedef struct {
    orc_tree *t;
    const uint64_t *keys;
    uint32_t ks, ops;
    uint64_t b, e; /* transactions [b, e) */
    uint32_t *tid_counter;
    tid_map *tids;
    txn_ctx **ctxs;
    uint64_t sum, commits, aborts;
} txn_job_t;

static void *txn_worker(void *arg) {
    txn_job_t *j = arg;
    orc_tree *t = j->t;
    uint16_t ks = (uint16_t)j->ks;
    uint64_t sum = 0, commits = 0, aborts = 0;
    rw_node *copy = xmalloc(sizeof(rw_node) * (j->ops + 1));
    for (uint64_t x = j->b; x < j->e; x++) {
        txn_ctx *c = xmalloc(sizeof(txn_ctx));
        memset(c, 0, sizeof(*c));
        c->read_id = __atomic_fetch_add(j->tid_counter, 1, __ATOMIC_SEQ_CST);
        c->succ = MAX_CID;
        tid_insert(j->tids, c->read_id, c);
        j->ctxs[x] = c;
        int ok = 1;
        for (uint32_t op = 0; op < j->ops && ok; op++) {
            uint64_t k = j->keys[x * j->ops + op];
            const uint8_t *key = (const uint8_t *)&k;
            uint8_t *leaf = traverse_to_leaf(t, NULL, key, ks, 1);
            int64_t slot = search_record_meta(leaf, key, ks, 1);
            if (slot < 0) continue; /* Read -> nullptr: the executor returns true, no tuple */
            orc_rmeta *mp = l_meta(leaf, (uint32_t)slot);
            uint64_t m = mp->meta;
            /* BTree::Read: heap Record (Record::New, b_tree.h:407-428) */
            size_t rsz = 48 + 4 + m_padded(m) + t->payload_size;
            uint8_t *r = xmalloc(rsz);
            memcpy(r + 52, leaf + m_offset(m), m_padded(m) + t->payload_size);
            uint32_t cstamp = m_inserting(m) ? 0 : c->read_id;
            if (m_inserting(m)) {
                orc_copy *cp = copy_of(mp->next);
                if (cp) {
                    memcpy(r + 52, cp->image, cp->key_len + t->payload_size);
                    cstamp = cp->rstamp;
                }
            }
            if (c->read_id >= m_cstamp(m)) {
                /* PerformRead (transaction_manager.cpp:362-410) */
                if (rw_record_read(c, mp, m)) {
                    if (cstamp > c->pred) c->pred = cstamp;
                    orc_copy *hdr = copy_of(mp->next);
                    if (hdr) {
                        __atomic_fetch_add(&hdr->wr_count, 1, __ATOMIC_SEQ_CST); /* IncreaseWRCount */
                        if (hdr->sstamp != MAX_CID && hdr->sstamp < c->succ) c->succ = hdr->sstamp;
                    }
                    if (c->succ <= c->pred) { /* CheckExclusion */
                        c->aborted = 1;
                        ok = 0;
                    }
                }
                /* the executor's `new T` + memcpy (executor.h:396-401), deleted by the driver */
                uint8_t *tup = xmalloc(4 + t->payload_size);
                memcpy(tup, r + 52, 4 + t->payload_size);
                sum += tup[4 + (op % t->payload_size)];
                free(tup);
            } else {
                orc_read_out o;
                read_one(t, key, ks, c->read_id, &o, NULL);
                sum += o.status;
            }
            free(r);
        }
        if (!ok) {
            aborts++;
            continue;
        }
        /* CommitTransaction (:535-815) */
        c->commit_id = __atomic_fetch_add(j->tid_counter, 1, __ATOMIC_SEQ_CST);
        /* FindMinSstamp: successor starts at t_cstamp; READ entries overwritten since */
        if (c->commit_id < c->succ) c->succ = c->commit_id;
        uint32_t nc = rw_copy(c, copy);
        for (uint32_t i = 0; i < nc; i++) {
            if (copy[i].type != 0) continue;
            uint64_t cur = copy[i].loc->meta;
            uint32_t cur_c = m_cstamp(cur), old_c = m_cstamp(copy[i].meta);
            if (cur_c != old_c && cur_c < c->commit_id) {
                txn_ctx *w;
                if (cur_c != INVALID_CID && tid_find(j->tids, cur_c, &w) && !w->aborted && w->succ < c->succ)
                    c->succ = w->succ;
            } else {
                orc_copy *hc = copy_of(copy[i].loc->next);
                if (hc) {
                    txn_ctx *w;
                    if (tid_find(j->tids, hc->cstamp, &w) && w->finished && w->succ < c->succ) c->succ = w->succ;
                }
            }
        }
        /* FindMaxPstamp: UPDATE entries only (none in a read-only mix), over a second copy */
        nc = rw_copy(c, copy);
        for (uint32_t i = 0; i < nc; i++) sum += copy[i].type;
        c->finished = 1;
        /* post-commit, READ entries: v.pstamp = max(v.pstamp, t.cstamp), DecreaseWRCount */
        for (int b = 0; b < 16; b++)
            for (rw_node *n = c->bucket[b]; n; n = n->next) {
                orc_copy *hc = copy_of(n->loc->next);
                if (hc) {
                    if (hc->pstamp < c->commit_id) hc->pstamp = c->commit_id;
                    __atomic_fetch_sub(&hc->wr_count, 1, __ATOMIC_SEQ_CST);
                }
            }
        tid_insert(j->tids, c->commit_id, c);
        commits++;
    }
    free(copy);
    j->sum = sum;
    j->commits = commits;
    j->aborts = aborts;
    return NULL;
}

/* n_txns transactions of ops_per_txn reads each (keys[x*ops + op], u64 little-endian keys of
 * key_size bytes); results[0] = commits, results[1] = aborts, results[2] = checksum. */
void orc_ycsb_txn_timed(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint32_t ops_per_txn, uint64_t n_txns,
                        int nthreads, uint32_t first_tid, double *seconds, uint64_t *results) {
    tid_map m;
    for (int i = 0; i < TID_STRIPES; i++) pthread_mutex_init(&m.lock[i], NULL);
    m.b = calloc(TID_BUCKETS, sizeof(tid_node *));
    txn_ctx **ctxs = calloc(n_txns ? n_txns : 1, sizeof(txn_ctx *));
    uint32_t counter = first_tid;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((uint64_t)nthreads > n_txns) nthreads = n_txns ? (int)n_txns : 1;
    pthread_t th[256];
    txn_job_t jobs[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < nthreads; i++) {
        txn_job_t jj = {t, keys, key_size, ops_per_txn, n_txns * (uint64_t)i / nthreads,
                        n_txns * (uint64_t)(i + 1) / nthreads, &counter, &m, ctxs, 0, 0, 0};
        jobs[i] = jj;
        pthread_create(&th[i], NULL, txn_worker, &jobs[i]);
    }
    uint64_t commits = 0, aborts = 0, sum = 0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        commits += jobs[i].commits;
        aborts += jobs[i].aborts;
        sum += jobs[i].sum;
    }
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    if (results) {
        results[0] = commits;
        results[1] = aborts;
        results[2] = sum;
    }
    for (uint64_t x = 0; x < n_txns; x++) {
        txn_ctx *c = ctxs[x];
        if (!c) continue;
        for (int bb = 0; bb < 16; bb++)
            for (rw_node *n = c->bucket[bb]; n;) {
                rw_node *nx = n->next;
                free(n);
                n = nx;
            }
        free(c);
    }
    free(ctxs);
    for (uint32_t i = 0; i < TID_BUCKETS; i++)
        for (tid_node *n = m.b[i]; n;) {
            tid_node *nx = n->next;
            free(n);
            n = nx;
        }
    free(m.b);
    for (int i = 0; i < TID_STRIPES; i++) pthread_mutex_destroy(&m.lock[i]);
}

/* ---------------------------------------------------------------- scans */
typedef struct { uint8_t *leaf; uint32_t slot; const uint8_t *k; uint16_t ks; } scanrec_t;
static int scanrec_cmp(const void *a, const void *b) {
    const scanrec_t *x = a, *y = b;
    int c = orc_key_compare(x->k, x->ks, y->k, y->ks);
    return (c > 0) - (c < 0);
}

/* LeafNode::RangeScanBySize, b_tree.cpp:1261-1315: slot order, stop once > to_scan
 * collected, then sort by KeyCompare. */
static uint32_t range_scan_by_size(uint8_t *n, const uint8_t *key, uint16_t ks, uint32_t to_scan, scanrec_t *out) {
    if (to_scan == 0) return 0;
    uint32_t cnt = st_count(*l_status(n)), m = 0;
    for (uint32_t i = 0; i < cnt; i++) {
        if (m > to_scan) break;
        uint64_t mm = l_meta(n, i)->meta;
        if (m_visible(mm)) {
            int cmp = orc_key_compare(key, ks, l_key(n, mm), m_keylen(mm));
            if (cmp <= 0) {
                out[m].leaf = n;
                out[m].slot = i;
                out[m].k = n + m_offset(mm);
                out[m].ks = m_keylen(mm);
                m++;
            }
        }
    }
    qsort(out, m, sizeof(scanrec_t), scanrec_cmp);
    return m;
}

static void emit_scan_rec(orc_tree *t, uint8_t *dst, scanrec_t *r) {
    uint64_t mm = l_meta(r->leaf, r->slot)->meta;
    memset(dst, 0, t->key_pad);
    memcpy(dst, r->leaf + m_offset(mm), m_padded(mm) > t->key_pad ? t->key_pad : m_padded(mm));
    memcpy(dst + t->key_pad, r->leaf + m_offset(mm) + m_padded(mm), t->payload_size);
}

/* IndexScanExecutor::Execute range branch (executor.h:456-530), per iterator record: a
 * reader with txn_id >= the record's commit id reads the leaf record (PerformRead; for an
 * in-flight update that is the patched image); otherwise the TupleHeader chain from next_ptr
 * gives the version with begin <= txn_id <= end, and nothing is produced when begin or end is
 * INVALID_CID or the chain ends.  Deviations: the reference never leaves its chain loop after
 * a match (executor.h:500-508 re-tests the same header forever) -- here the match ends the
 * walk; a next_ptr that points at an overwrite copy (in-flight record) produces nothing.
 * status: 1 = latest, 3 = old version, 0 = nothing produced. */
static void emit_index_rec(orc_tree *t, uint8_t *dst, scanrec_t *r, uint32_t read_id, uint8_t *status) {
    orc_rmeta *mp = l_meta(r->leaf, r->slot);
    uint32_t rs = t->key_pad + t->payload_size;
    if (read_id >= m_cstamp(mp->meta)) {
        *status = ORC_ST_LATEST;
        if (dst) emit_scan_rec(t, dst, r);
        return;
    }
    *status = ORC_ST_NOT_FOUND;
    if (dst) memset(dst, 0, rs);
    uint64_t nx = mp->next;
    while (nx != 0 && nx != ~0ull && NEXT_KIND(nx) == NEXT_TH) {
        orc_th *th = NEXT_PTR(nx);
        if (th->begin_id == INVALID_CID || th->comm_id == INVALID_CID) return;
        if (read_id >= th->begin_id && read_id <= th->comm_id) {
            *status = ORC_ST_OLD;
            if (dst) emit_canonical(t, dst, th->slot, th->key_len, th->slot + th->key_len);
            return;
        }
        nx = th->next;
    }
}

/* TableScanExecutor::Execute (executor.h:620-639) driving Iterator::GetNext (b_tree.h:899-941);
 * with `status` non-NULL the IndexScanExecutor range branch above decides each record. */
static uint32_t scan_one_ex(orc_tree *t, const uint8_t *key, uint16_t ks, uint32_t scan_size, uint8_t *recs,
                            scanrec_t *buf, uint32_t bufcap, uint32_t read_id, uint8_t *status);
static uint32_t scan_one(orc_tree *t, const uint8_t *key, uint16_t ks, uint32_t scan_size, uint8_t *recs,
                         scanrec_t *buf, uint32_t bufcap) {
    return scan_one_ex(t, key, ks, scan_size, recs, buf, bufcap, 0, NULL);
}

static uint32_t scan_one_ex(orc_tree *t, const uint8_t *key, uint16_t ks, uint32_t scan_size, uint8_t *recs,
                            scanrec_t *buf, uint32_t bufcap, uint32_t read_id, uint8_t *status) {
    uint32_t rs = t->key_pad + t->payload_size, produced = 0;
    uint32_t remaining = scan_size;
    uint8_t lastkey[64];
    uint16_t lastks = 0;
    uint8_t *leaf = traverse_to_leaf(t, NULL, key, ks, 1);
    uint32_t m = range_scan_by_size(leaf, key, ks, scan_size < bufcap ? scan_size : bufcap - 1, buf);
    uint32_t head = 0;
    for (uint32_t scanned = 0; scanned < scan_size; scanned++) {
        /* GetNext */
        if (head >= m || remaining == 0) continue; /* nullptr -> fail_num++ */
        remaining -= 1;
        if (m - head > 1) {
            if (status) emit_index_rec(t, recs ? recs + (uint64_t)produced * rs : NULL, &buf[head], read_id,
                                       status + produced);
            else if (recs) emit_scan_rec(t, recs + (uint64_t)produced * rs, &buf[head]);
            produced++;
            head++;
            continue;
        }
        scanrec_t last = buf[head];
        head++;
        if (status) emit_index_rec(t, recs ? recs + (uint64_t)produced * rs : NULL, &last, read_id, status + produced);
        else if (recs) emit_scan_rec(t, recs + (uint64_t)produced * rs, &last);
        produced++;
        lastks = last.ks > 64 ? 64 : last.ks;
        memcpy(lastkey, last.k, lastks);
        uint8_t *nl = traverse_to_leaf(t, NULL, lastkey, lastks, 0);
        m = range_scan_by_size(nl, lastkey, lastks, remaining < bufcap ? remaining : bufcap - 1, buf);
        head = 0;
        if (m > 0 && orc_key_compare(buf[0].k, buf[0].ks, lastkey, lastks) == 0) m = 0; /* item_vec.clear() */
    }
    return produced;
}

uint32_t orc_index_scan(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t scan_size, uint32_t read_id,
                        uint8_t *recs, uint8_t *status) {
    uint32_t cap = 4096;
    scanrec_t *buf = xmalloc(sizeof(scanrec_t) * cap);
    uint32_t r = scan_one_ex(t, key, (uint16_t)key_size, scan_size, recs, buf, cap, read_id, status);
    free(buf);
    return r;
}

uint32_t orc_scan(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t scan_size, uint8_t *recs) {
    uint32_t cap = 4096;
    scanrec_t *buf = xmalloc(sizeof(scanrec_t) * cap);
    uint32_t r = scan_one(t, key, (uint16_t)key_size, scan_size, recs, buf, cap);
    free(buf);
    return r;
}

static void *scan_worker(void *arg) {
    job_t *j = arg;
    uint32_t cap = 4096;
    scanrec_t *buf = xmalloc(sizeof(scanrec_t) * cap);
    uint64_t rs = j->t->key_pad + j->t->payload_size, sum = 0;
    for (uint64_t i = j->b; i < j->e; i++) {
        uint64_t k;
        uint32_t c = scan_one(j->t, job_key(j, i, &k), (uint16_t)j->ks, j->scan_size,
                              j->recs ? j->recs + i * rs * j->scan_size : NULL, buf, cap);
        if (j->counts) j->counts[i] = c;
        sum += c;
    }
    free(buf);
    j->sum = sum;
    return NULL;
}

static void *scan_timed_worker(void *arg) {
    job_t *j = arg;
    uint32_t cap = 4096;
    scanrec_t *buf = xmalloc(sizeof(scanrec_t) * cap);
    uint64_t rs = 8 + j->t->payload_size, sum = 0;
    uint8_t *scratch = xmalloc(rs * (j->scan_size ? j->scan_size : 1));
    for (uint64_t i = j->b; i < j->e; i++) {
        uint64_t k = j->keys[i];
        sum += scan_one(j->t, (const uint8_t *)&k, (uint16_t)j->ks, j->scan_size, scratch, buf, cap);
    }
    free(scratch);
    free(buf);
    j->sum = sum;
    return NULL;
}

uint64_t orc_scan_batch_timed(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n, uint32_t scan_size,
                              int nthreads, double *seconds) {
    job_t j = {t, keys, key_size, NULL, 0, n, NULL, NULL, scan_size, NULL, 0, NULL, 0};
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    run_jobs(scan_timed_worker, &j, n, nthreads);
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    return j.sum;
}

uint64_t orc_scan_batch(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n, uint32_t scan_size,
                        uint32_t *counts, uint8_t *recs, int nthreads) {
    job_t j = {t, keys, key_size, NULL, 0, n, NULL, recs, scan_size, counts, 0, NULL, 0};
    run_jobs(scan_worker, &j, n, nthreads);
    return j.sum;
}

uint64_t orc_scan_batch_k(orc_tree *t, const uint8_t *keys, uint32_t key_stride, uint32_t key_size, uint64_t n,
                          uint32_t scan_size, uint32_t *counts, uint8_t *recs, int nthreads) {
    job_t j = {t, NULL, key_size, NULL, 0, n, NULL, recs, scan_size, counts, 0, keys, key_stride};
    run_jobs(scan_worker, &j, n, nthreads);
    return j.sum;
}

/* ---------------------------------------------------------------- traversal export */
static int64_t leaf_index_rec(void *node, uint8_t *target, int64_t *counter) {
    if (is_leaf(node)) {
        int64_t me = (*counter)++;
        return node == target ? me : -1;
    }
    orc_inner *p = node;
    for (uint32_t i = 0; i < p->count; i++) {
        int64_t r = leaf_index_rec(p->child[i], target, counter);
        if (r >= 0) return r;
    }
    return -1;
}

int64_t orc_traverse_leaf_index(orc_tree *t, const uint8_t *key, uint32_t key_size, int le_child) {
    uint8_t *leaf = traverse_to_leaf(t, NULL, key, (uint16_t)key_size, le_child);
    int64_t c = 0;
    return leaf_index_rec(t->root, leaf, &c);
}

typedef struct {
    uint32_t cap;
    uint64_t max, n;
    uint32_t *rc, *sc;
    uint64_t *meta, *keyw;
} export_t;

static void export_rec(void *node, export_t *e, uint64_t *stats, uint32_t depth) {
    if (is_leaf(node)) {
        uint8_t *n = node;
        uint32_t cnt = st_count(*l_status(n)), sorted = *l_sorted(n);
        if (stats) {
            if (depth + 1 > stats[0]) stats[0] = depth + 1;
            stats[2]++;
            for (uint32_t i = 0; i < cnt; i++)
                if (m_visible(l_meta(n, i)->meta)) {
                    stats[3]++;
                    if (i < sorted) stats[4]++;
                    else stats[5]++;
                }
            if (cnt > stats[6]) stats[6] = cnt;
        }
        if (e) {
            if (e->n < e->max) {
                e->rc[e->n] = cnt;
                e->sc[e->n] = sorted;
                for (uint32_t i = 0; i < e->cap; i++) {
                    uint64_t mm = i < cnt ? l_meta(n, i)->meta : 0;
                    uint64_t kw = 0;
                    if (mm) memcpy(&kw, n + m_offset(mm), m_keylen(mm) > 8 ? 8 : m_keylen(mm));
                    e->meta[e->n * (uint64_t)e->cap + i] = mm;
                    e->keyw[e->n * (uint64_t)e->cap + i] = kw;
                }
            }
            e->n++;
        }
        return;
    }
    orc_inner *p = node;
    if (stats) stats[1]++;
    for (uint32_t i = 0; i < p->count; i++) export_rec(p->child[i], e, stats, depth + 1);
}

/* Leaf-level snapshot in the reference's own block format (LeafNode, b_tree.h:571-740;
 * BaseNode{is_leaf, NodeHeader} b_tree.h:109-113; StatusWord version_store.h:158-231;
 * RecordMetadata{meta, next_ptr, loc_ptr} record_meta.h:30-60).  Canonical form: the process
 * pointers (next_ptr, loc_ptr) are written as 0 and record bytes no live metadata entry
 * references (deleted records) are zeroed.  Leaf i's separator is the inner-node key that
 * bounds it from above: child j of an inner node covers (key[j], key[j+1]] (GetChildIndex,
 * b_tree.cpp:664-702), the last child inherits its parent's bound; the last leaf gets
 * len 0xFFFF (+inf). */
typedef struct {
    uint64_t max, n;
    uint32_t block, payload;
    uint8_t *blocks;
    uint64_t *sep_key; /* kwords u64 words of key bytes per leaf */
    uint16_t *sep_len;
    uint32_t kwords;
} image_export_t;

static void image_rec(void *node, image_export_t *e, const uint8_t *ub, uint16_t ub_len, int ub_inf) {
    if (is_leaf(node)) {
        if (e->n < e->max) {
            uint8_t *n = node, *dst = e->blocks + e->n * (uint64_t)e->block;
            uint32_t cnt = st_count(*l_status(n));
            memcpy(dst, n, LEAF_HDR);
            memset(dst, 0, 8); /* vptr */
            memset(dst + LEAF_HDR, 0, e->block - LEAF_HDR);
            for (uint32_t i = 0; i < cnt; i++) {
                uint64_t m = l_meta(n, i)->meta;
                uint64_t lp = l_meta(n, i)->loc ? l_meta(n, i)->loc->id + 1 : 0; /* location handle */
                memcpy(dst + LEAF_HDR + META_SZ * i, &m, 8);
                memcpy(dst + LEAF_HDR + META_SZ * i + 16, &lp, 8);
                if (m) {
                    uint32_t off = m_offset(m), len = pad_key(m_keylen(m)) + e->payload;
                    memcpy(dst + off, n + off, len);
                }
            }
            if (e->sep_key) {
                uint64_t *kw = e->sep_key + e->n * (uint64_t)e->kwords;
                memset(kw, 0, 8 * e->kwords);
                if (!ub_inf) memcpy(kw, ub, ub_len > 8 * e->kwords ? 8 * e->kwords : ub_len);
                e->sep_len[e->n] = ub_inf ? 0xFFFF : ub_len;
            }
        }
        e->n++;
        return;
    }
    orc_inner *p = node;
    for (uint32_t i = 0; i < p->count; i++) {
        if (i + 1 < p->count) image_rec(p->child[i], e, p->key[i + 1], p->klen[i + 1], 0);
        else image_rec(p->child[i], e, ub, ub_len, ub_inf);
    }
}

int64_t orc_export_leaf_images_k(orc_tree *t, uint64_t max_leaves, uint8_t *blocks, uint64_t *sep_key,
                                 uint32_t kwords, uint16_t *sep_len) {
    image_export_t e = {max_leaves, 0, t->leaf_node_size, t->payload_size, blocks, sep_key, sep_len, kwords};
    image_rec(t->root, &e, NULL, 0, 1);
    return (int64_t)e.n;
}

int64_t orc_export_leaf_images(orc_tree *t, uint64_t max_leaves, uint8_t *blocks, uint64_t *sep_key,
                               uint16_t *sep_len) {
    return orc_export_leaf_images_k(t, max_leaves, blocks, sep_key, 1, sep_len);
}

void orc_stats(orc_tree *t, uint64_t *stats) {
    memset(stats, 0, 8 * sizeof(uint64_t));
    export_rec(t->root, NULL, stats, 0);
    stats[7] = t->retired;
}

int64_t orc_export_leaves(orc_tree *t, uint32_t cap, uint64_t max_leaves, uint32_t *rc, uint32_t *sc,
                          uint64_t *meta, uint64_t *keyw) {
    export_t e = {cap, max_leaves, 0, rc, sc, meta, keyw};
    export_rec(t->root, &e, NULL, 0);
    if (e.n > max_leaves) return -(int64_t)e.n;
    return (int64_t)e.n;
}

/* ---------------------------------------------------------------- write path (scenarios) */
static orc_rmeta *find_meta(orc_tree *t, const uint8_t *key, uint16_t ks, uint8_t **leafp) {
    uint8_t *leaf = traverse_to_leaf(t, NULL, key, ks, 1);
    int64_t slot = search_record_meta(leaf, key, ks, 1);
    if (leafp) *leafp = leaf;
    return slot < 0 ? NULL : l_meta(leaf, (uint32_t)slot);
}

/* Allocations of one writer thread of orc_update_batch_mt: the reference's EphemeralPool and
 * VersionStore are concurrent pools (ephemeral_pool.cpp:17-44, version_store.cpp); here each
 * writer keeps its own list and the lists join the tree's registry after the writers end. */
typedef struct {
    orc_copy **copies;
    uint32_t ncopies, capcopies;
    orc_th **ths;
    uint32_t nths, capths;
} alloc_sink;
static __thread alloc_sink *tl_sink;

static void sink_push(void ***arr, uint32_t *n, uint32_t *cap, void *p) {
    if (*n == *cap) {
        *cap = *cap ? 2 * *cap : 1024;
        *arr = realloc(*arr, sizeof(void *) * *cap);
        if (!*arr) abort();
    }
    (*arr)[(*n)++] = p;
}

static void register_copy(orc_tree *t, orc_copy *c) {
    c->reg_next = t->copies;
    t->copies = c;
    if (t->ncopies == t->capcopies) {
        t->capcopies = t->capcopies ? 2 * t->capcopies : 1024;
        t->copy_by_id = realloc(t->copy_by_id, sizeof(orc_copy *) * t->capcopies);
        if (!t->copy_by_id) abort();
    }
    c->id = t->ncopies;
    t->copy_by_id[t->ncopies++] = c;
}

static void register_th(orc_tree *t, orc_th *th) {
    th->reg_next = t->ths;
    t->ths = th;
    th->id = t->nths++;
    t->retired++;
}

static orc_copy *copy_alloc(orc_tree *t, const uint8_t *src_key, uint16_t klen, uint64_t next, uint32_t cstamp,
                            uint32_t rstamp) {
    /* EphemeralPool::Allocate, ephemeral_pool.cpp:17-44 */
    orc_copy *c = xmalloc(sizeof(orc_copy));
    memset(c, 0, sizeof(*c));
    c->cstamp = cstamp;
    c->pstamp = cstamp;
    c->rstamp = rstamp;
    c->sstamp = MAX_CID;
    c->next = next;
    c->key_len = klen;
    c->payload_size = t->payload_size;
    c->live = 1;
    c->image = xmalloc(klen + t->payload_size);
    memcpy(c->image, src_key, klen);                                   /* b_tree.cpp:1143 */
    memcpy(c->image + klen, src_key + pad_key(klen), t->payload_size); /* b_tree.cpp:1144 */
    if (tl_sink)
        sink_push((void ***)&tl_sink->copies, &tl_sink->ncopies, &tl_sink->capcopies, c);
    else
        register_copy(t, c);
    return c;
}

/* LeafNode::Update, b_tree.cpp:1061-1163 (is_for_update == false) */
int orc_update(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t payload_off, const uint8_t *delta,
               uint32_t delta_len, uint32_t writer_id) {
    uint16_t ks = (uint16_t)key_size;
    uint8_t *leaf;
    orc_rmeta *mp = find_meta(t, key, ks, &leaf);
    if (!mp) return ORC_RET_NOT_FOUND;
    if (m_inserting(mp->meta)) return ORC_RET_DIRTY;
    uint8_t *rk = leaf + m_offset(mp->meta);
    /* Catalog::get_field_index of a payload column = the key columns' width (8 for the YCSB
     * key column, 16/24/32 for TPC-C int64 key fields) + its offset inside the payload
     * (ComparePayload / CopyPayload, b_tree.h:661-695) */
    uint8_t *col = rk + m_padded(mp->meta) + payload_off;
    if (payload_off + delta_len > t->payload_size) return ORC_RET_INVALID;
    if (memcmp(col, delta, delta_len) == 0) return ORC_RET_NOT_NEEDED_UPDATE; /* ComparePayload */
    if (m_cstamp(mp->meta) > writer_id) return ORC_RET_NOT_NEEDED_UPDATE;
    uint64_t old = mp->meta;
    meta_store(mp, old | M_CONTROL | M_VISIBLE); /* PrepareForUpdate */
    orc_copy *c = copy_alloc(t, rk, m_keylen(old), mp->next, writer_id, m_cstamp(old));
    mp->next = (uint64_t)(uintptr_t)c | NEXT_COPY;
    memcpy(col, delta, delta_len); /* CopyPayload */
    return ORC_RET_OK;
}

/* LeafNode::Update, b_tree.cpp:1061-1163 with is_for_update == true: no WriteDirty refusal of an
 * inserting record (:1077), ComparePayload and the newer-writer check as above (:1086-1100),
 * then CopyPayload in place (:1101-1104) -- no copy, no PrepareForUpdate. */
int orc_update_owned(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t payload_off, const uint8_t *delta,
                     uint32_t delta_len, uint32_t writer_id) {
    uint16_t ks = (uint16_t)key_size;
    uint8_t *leaf;
    orc_rmeta *mp = find_meta(t, key, ks, &leaf);
    if (!mp) return ORC_RET_NOT_FOUND;
    uint8_t *col = leaf + m_offset(mp->meta) + m_padded(mp->meta) + payload_off;
    if (payload_off + delta_len > t->payload_size) return ORC_RET_INVALID;
    if (memcmp(col, delta, delta_len) == 0) return ORC_RET_NOT_NEEDED_UPDATE; /* ComparePayload */
    if (m_cstamp(mp->meta) > writer_id) return ORC_RET_NOT_NEEDED_UPDATE;
    memcpy(col, delta, delta_len); /* CopyPayload */
    return ORC_RET_OK;
}

/* CommitTransaction, UPDATE entry (transaction_manager.cpp:610-676) for a single writer
 * whose t_sstamp is `sstamp` (FindMinSstamp starts it at t_cstamp, :113-121). */
int orc_commit_update(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id, uint32_t sstamp) {
    orc_rmeta *mp = find_meta(t, key, (uint16_t)key_size, NULL);
    if (!mp || !m_inserting(mp->meta)) return ORC_RET_NOT_FOUND;
    orc_copy *c = copy_of(mp->next);
    if (!c) return ORC_RET_NOT_FOUND;
    orc_th *th = xmalloc(sizeof(orc_th)); /* AcquireVersion + PerformUpdate (:435-491) */
    memset(th, 0, sizeof(*th));
    th->next = c->next;
    th->begin_id = c->rstamp;
    c->sstamp = sstamp;
    c->waiting = 1;
    th->comm_id = c->sstamp;
    th->key_len = c->key_len;
    th->slot = xmalloc(c->key_len + t->payload_size);
    memcpy(th->slot, c->image, c->key_len + t->payload_size);
    if (tl_sink)
        sink_push((void ***)&tl_sink->ths, &tl_sink->nths, &tl_sink->capths, th);
    else
        register_th(t, th);
    c->pre = (uint64_t)(uintptr_t)th;
    uint64_t m = mp->meta;
    m = (m & ~M_TXN) | commit_id; /* FinalizeForUpdate(t_cstamp), record_meta.h:146-151 */
    m &= ~M_CONTROL;
    meta_store(mp, m);
    mp->next = (uint64_t)(uintptr_t)th | NEXT_TH;
    return ORC_RET_OK;
}

/* AbortTransaction, UPDATE entry (transaction_manager.cpp:846-921): the old image is copied
 * back from the overwrite copy into the record, FinalizeForUpdate() (control bit cleared, the
 * cstamp untouched), next_ptr := the chain the update found (the TupleHeader it reserved is
 * dropped -- this restatement reserves it only at commit), the copy header is released. */
int orc_abort_update(orc_tree *t, const uint8_t *key, uint32_t key_size) {
    uint16_t ks = (uint16_t)key_size;
    uint8_t *leaf;
    orc_rmeta *mp = find_meta(t, key, ks, &leaf);
    if (!mp || !m_inserting(mp->meta)) return ORC_RET_NOT_FOUND;
    orc_copy *c = copy_of(mp->next);
    if (!c) return ORC_RET_NOT_FOUND;
    uint8_t *rk = leaf + m_offset(mp->meta);
    memcpy(rk, c->image, c->key_len);                                        /* key */
    memcpy(rk + m_padded(mp->meta), c->image + c->key_len, t->payload_size); /* payload */
    mp->meta = (mp->meta & ~M_CONTROL) | M_VISIBLE;
    mp->next = c->next;
    c->live = 0;        /* no record reaches it any more */
    c->sstamp = MAX_CID; /* UpdateSs(MAX_CID), SetWaiting(true): the header stays in the pool */
    c->waiting = 1;
    return ORC_RET_OK;
}

/* AbortTransaction, INSERT entry (transaction_manager.cpp:949-979): FinalizeForDelete (meta
 * := 0, record_meta.h:167-172) and StatusWord::FailForInsert (record count - 1, block size -
 * record size, version_store.h:214-217).  FailForInsert drops the leaf's LAST slot, so the
 * aborted insert must be that slot (single writer); otherwise ORC_RET_INVALID. */
int orc_abort_insert(orc_tree *t, const uint8_t *key, uint32_t key_size) {
    uint16_t ks = (uint16_t)key_size;
    uint8_t *leaf;
    orc_rmeta *mp = find_meta(t, key, ks, &leaf);
    if (!mp) return ORC_RET_NOT_FOUND;
    uint64_t s = *l_status(leaf);
    uint32_t slot = (uint32_t)(((uint8_t *)mp - (leaf + LEAF_HDR)) / META_SZ);
    if (slot + 1 != st_count(s) || slot < *l_sorted(leaf)) return ORC_RET_INVALID;
    uint32_t total = m_padded(mp->meta) + t->payload_size;
    mp->meta = 0;
    mp->next = 0;
    if (mp->loc) mp->loc->leaf = NULL;
    mp->loc = NULL;
    *l_status(leaf) = s - ((1ull << 44) + ((uint64_t)total << 22));
    return ORC_RET_OK;
}

/* one transaction epoch of single-key writers, op by op in batch order (as tests/
 * test_gpu_write_path.py::oracle_epoch): orc_update, then orc_commit_update(cid, cid) when it
 * succeeded and cid[i] != 0 (cid 0 = left in flight); rc[i] = the last ReturnCode */
uint64_t orc_update_batch(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n, uint32_t payload_off,
                          const uint8_t *deltas, uint32_t delta_len, const uint32_t *wid, const uint32_t *cid,
                          uint8_t *rc) {
    uint64_t ok = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t k = keys[i];
        int r = orc_update(t, (const uint8_t *)&k, key_size, payload_off, deltas + i * delta_len, delta_len, wid[i]);
        if (r == ORC_RET_OK && cid[i]) r = orc_commit_update(t, (const uint8_t *)&k, key_size, cid[i], cid[i]);
        if (rc) rc[i] = (uint8_t)r;
        ok += r == ORC_RET_OK;
    }
    return ok;
}

/* The same epoch with T concurrent writers (the CPU baseline of C3's write share).  RunMixed's
 * writer threads each run LeafNode::Update with CASes on the record's own meta and next words
 * (b_tree.cpp:1061-1163) and commit their own records (transaction_manager.cpp:610-676): no
 * update touches another record's bytes, splits never happen on this path, and the leaf status
 * word is CASed to its own value.  Writer g takes the ops whose key hashes to g, in batch order,
 * so every key's op sequence -- hence every rc and the final state of every record -- is the
 * single writer's.  Copy and version allocations go to per-writer lists (alloc_sink) joined to
 * the tree after the writers end; copy / version ids then follow writer order, not batch order
 * (ids are handles only; no read result depends on them). */
typedef struct {
    orc_tree *t;
    const uint64_t *keys;
    uint32_t key_size, payload_off, delta_len, g, T;
    uint64_t n;
    const uint8_t *deltas;
    const uint32_t *wid, *cid;
    uint8_t *rc;
    uint64_t ok;
    alloc_sink sink;
} upd_job;

static inline uint32_t writer_of(uint64_t k, uint32_t T) { return (uint32_t)(splitmix64(k) % T); }

static void *upd_worker(void *arg) {
    upd_job *j = arg;
    tl_sink = &j->sink;
    uint64_t ok = 0;
    for (uint64_t i = 0; i < j->n; i++) {
        uint64_t k = j->keys[i];
        if (writer_of(k, j->T) != j->g) continue;
        int r = orc_update(j->t, (const uint8_t *)&k, j->key_size, j->payload_off, j->deltas + i * j->delta_len,
                           j->delta_len, j->wid[i]);
        if (r == ORC_RET_OK && j->cid[i])
            r = orc_commit_update(j->t, (const uint8_t *)&k, j->key_size, j->cid[i], j->cid[i]);
        if (j->rc) j->rc[i] = (uint8_t)r;
        ok += r == ORC_RET_OK;
    }
    tl_sink = NULL;
    j->ok = ok;
    return NULL;
}

uint64_t orc_update_batch_mt(orc_tree *t, const uint64_t *keys, uint32_t key_size, uint64_t n, uint32_t payload_off,
                             const uint8_t *deltas, uint32_t delta_len, const uint32_t *wid, const uint32_t *cid,
                             uint8_t *rc, int nthreads, double *seconds) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    upd_job *jobs = calloc((size_t)nthreads, sizeof(upd_job));
    pthread_t th[256];
    if (!jobs) abort();
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int g = 0; g < nthreads; g++) {
        jobs[g] = (upd_job){t, keys, key_size, payload_off, delta_len, (uint32_t)g, (uint32_t)nthreads, n,
                            deltas, wid, cid, rc, 0, {0}};
        pthread_create(&th[g], NULL, upd_worker, &jobs[g]);
    }
    for (int g = 0; g < nthreads; g++) pthread_join(th[g], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    uint64_t ok = 0;
    for (int g = 0; g < nthreads; g++) {
        alloc_sink *s = &jobs[g].sink;
        for (uint32_t i = 0; i < s->ncopies; i++) register_copy(t, s->copies[i]);
        for (uint32_t i = 0; i < s->nths; i++) register_th(t, s->ths[i]);
        free(s->copies);
        free(s->ths);
        ok += jobs[g].ok;
    }
    free(jobs);
    return ok;
}

/* BTree::FinalizeUpdate, b_tree.cpp:2252-2268: cstamp := commit_id, next_ptr untouched */
/* InsertExecutor of a transaction that has not committed yet: BTree::Insert leaves the record
 * PrepareForInsert (control + visible, cstamp = the writer's read id, b_tree.cpp:860-864; next
 * pointer 0), so a reader's BTree::Read finds it inserting without an overwrite copy and returns
 * nullptr (b_tree.cpp:2087-2095). */
int orc_insert_inflight(orc_tree *t, const uint8_t *key, uint32_t key_size, const uint8_t *payload,
                        uint32_t writer_id) {
    orc_rmeta *mp = NULL;
    return btree_insert(t, key, (uint16_t)key_size, payload, writer_id, &mp);
}

/* CommitTransaction INSERT entry (transaction_manager.cpp:677-695):
 * FinalizeForInsert(offset, key_len, t_cstamp) -- visible, control cleared, cstamp = commit id */
int orc_commit_insert(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id) {
    orc_rmeta *mp = find_meta(t, key, (uint16_t)key_size, NULL);
    if (!mp || !m_inserting(mp->meta)) return ORC_RET_NOT_FOUND;
    mp->meta = m_finalize_insert(m_offset(mp->meta), m_keylen(mp->meta), commit_id);
    return ORC_RET_OK;
}

int orc_finalize_update(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id) {
    orc_rmeta *mp = find_meta(t, key, (uint16_t)key_size, NULL);
    if (!mp) return ORC_RET_NOT_FOUND;
    uint64_t m = mp->meta;
    m = (m & ~M_TXN) | commit_id;
    m &= ~M_CONTROL;
    mp->meta = m;
    return ORC_RET_OK;
}

/* LeafNode::Delete (b_tree.cpp:1171-1251, is_for_update == false) + BTree::FinalizeDelete
 * (:2275-2310).  BaseNode::CheckMerge (:150-318) is not restated: a delete that would merge
 * siblings returns ORC_RET_INVALID after deleting. */
int orc_delete(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t commit_id) {
    (void)commit_id;
    uint16_t ks = (uint16_t)key_size;
    uint8_t *leaf;
    orc_rmeta *mp = find_meta(t, key, ks, &leaf);
    if (!mp) return ORC_RET_NOT_FOUND;
    if (m_inserting(mp->meta)) return ORC_RET_DIRTY;
    uint8_t *rk = leaf + m_offset(mp->meta);
    orc_copy *c = copy_alloc(t, rk, m_keylen(mp->meta), mp->next, commit_id, m_cstamp(mp->meta));
    uint32_t padded = m_padded(mp->meta);
    mp->next = (uint64_t)(uintptr_t)c | NEXT_COPY;
    mp->meta = 0;
    uint64_t s = *l_status(leaf);
    *l_status(leaf) = st_set_deleted(s, st_deleted(s) + padded + t->payload_size);
    /* CheckMerge gate (b_tree.cpp:155-173) */
    s = *l_status(leaf);
    uint32_t valid = used_space(s) - st_deleted(s);
    if (leaf != t->root && valid <= t->merge_threshold)
        return ORC_RET_INVALID;
    return ORC_RET_OK;
}

/* LeafNode::Delete with is_for_update == true (b_tree.cpp:1210-1220): meta := 0 (the copy the
 * reference allocates at :1195-1203 is reachable from nothing and is not restated); no
 * PerformDelete, hence no FinalizeDelete and no deleted-size change; the merge gate as orc_delete. */
int orc_delete_owned(orc_tree *t, const uint8_t *key, uint32_t key_size) {
    uint16_t ks = (uint16_t)key_size;
    uint8_t *leaf;
    orc_rmeta *mp = find_meta(t, key, ks, &leaf);
    if (!mp) return ORC_RET_NOT_FOUND;
    mp->meta = 0;
    uint64_t s = *l_status(leaf);
    uint32_t valid = used_space(s) - st_deleted(s);
    if (leaf != t->root && valid <= t->merge_threshold) return ORC_RET_INVALID;
    return ORC_RET_OK;
}

/* ---------------------------------------------------------------- record locations */
/* RecordLocation (record_location.h:13-42) of handle h (= allocation index + 1) -> (leaf index
 * in key order, slot); leaf 0xFFFFFFFF = the location dangles (dropped by a split, aborted). */
static int ptr_cmp(const void *a, const void *b) {
    uintptr_t x = *(const uintptr_t *)a, y = *(const uintptr_t *)b;
    return (x > y) - (x < y);
}

static void leaves_in_order(void *node, uintptr_t *out, uint64_t *n) {
    if (is_leaf(node)) {
        out[(*n)++] = (uintptr_t)node;
        return;
    }
    orc_inner *p = node;
    for (uint32_t i = 0; i < p->count; i++) leaves_in_order(p->child[i], out, n);
}

void orc_resolve_locations(orc_tree *t, const uint64_t *handles, uint64_t n, uint32_t *leaf, uint16_t *slot) {
    uint64_t stats[8];
    orc_stats(t, stats);
    uint64_t nl = 0;
    uintptr_t *ord = xmalloc(sizeof(uintptr_t) * (stats[2] + 1));
    leaves_in_order(t->root, ord, &nl);
    /* (pointer, key-order index) pairs sorted by pointer */
    uintptr_t *pairs = xmalloc(sizeof(uintptr_t) * 2 * (nl + 1));
    for (uint64_t i = 0; i < nl; i++) {
        pairs[2 * i] = ord[i];
        pairs[2 * i + 1] = i;
    }
    qsort(pairs, nl, 2 * sizeof(uintptr_t), ptr_cmp);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t h = handles[i];
        orc_loc *l = (h == 0 || h > t->nlocs) ? NULL : t->locs[h - 1];
        uintptr_t key = l ? (uintptr_t)l->leaf : 0;
        uintptr_t *hit = key ? bsearch(&key, pairs, nl, 2 * sizeof(uintptr_t), ptr_cmp) : NULL;
        leaf[i] = hit ? (uint32_t)hit[1] : 0xFFFFFFFFu;
        slot[i] = hit ? (uint16_t)l->slot : 0xFFFF;
    }
    free(pairs);
    free(ord);
}

uint64_t orc_location_count(orc_tree *t) { return t->nlocs; }

/* ---------------------------------------------------------------- transaction-manager facts
 * What the kept SSNTransactionManager reads through a Record and its pool (the checker side of
 * stage_hip.h's stage_probe_ident / stage_location_cell / stage_copy_*):
 *   next handle   RecordMetadata::next_ptr named canonically: 0, ORC_NEXT_COPY | copy id (the
 *                 EphemeralPool location of an in-flight update), ORC_NEXT_TH | version id
 *   loc handle    RecordMetadata::loc_ptr = the RecordLocation's allocation index + 1
 *   location meta *GetLocationPtr()->record_meta_ptr now (tm.cpp:37, 123, 605)
 *   copy state    OverwriteVersionHeader cstamp / pstamp / rstamp / sstamp / readers / count /
 *                 waiting (ephemeral_pool.h:26-150) and AddReader (b_tree.cpp:2105),
 *                 IncreaseWRCount / DecreaseWRCount (ephemeral_pool.cpp:69-103), UpdatePs (:194-205) */
#define ORC_NEXT_COPY 0x40000000u
#define ORC_NEXT_TH 0x80000000u

static uint32_t next_handle(uint64_t next) {
    if (next == 0) return 0;
    if (NEXT_KIND(next) == NEXT_COPY) return ORC_NEXT_COPY | ((orc_copy *)NEXT_PTR(next))->id;
    if (NEXT_KIND(next) == NEXT_TH) return ORC_NEXT_TH | ((orc_th *)NEXT_PTR(next))->id;
    return 0;
}

int orc_read_ident(orc_tree *t, const uint8_t *key, uint32_t key_size, uint32_t read_id, orc_read_out *out,
                   uint8_t *rec, uint64_t *meta, uint32_t *loc, uint32_t *next) {
    read_one(t, key, (uint16_t)key_size, read_id, out, rec);
    *meta = 0;
    *loc = 0;
    *next = 0;
    if (out->status == ORC_ST_NOT_FOUND) return 0;
    uint8_t *leaf = traverse_to_leaf(t, NULL, key, (uint16_t)key_size, 1);
    int64_t slot = search_record_meta(leaf, key, (uint16_t)key_size, 1);
    if (slot < 0) return -1;
    orc_rmeta *mp = l_meta(leaf, (uint32_t)slot);
    *meta = mp->meta;
    *loc = mp->loc ? (uint32_t)(mp->loc->id + 1) : 0;
    *next = next_handle(mp->next);
    return 0;
}

/* the key's record now (BTree::Update's meta_upt_, b_tree.cpp:2144-2155): 0 = found, -1 = none */
int orc_record_meta(orc_tree *t, const uint8_t *key, uint32_t key_size, uint64_t *meta, uint32_t *loc, uint32_t *next) {
    *meta = 0;
    *loc = 0;
    *next = 0;
    orc_rmeta *mp = find_meta(t, key, (uint16_t)key_size, NULL);
    if (!mp) return -1;
    *meta = mp->meta;
    *loc = mp->loc ? (uint32_t)(mp->loc->id + 1) : 0;
    *next = next_handle(mp->next);
    return 0;
}

int orc_location_meta(orc_tree *t, uint64_t handle, uint64_t *meta, uint32_t *next) {
    *meta = 0;
    *next = 0;
    if (handle == 0 || handle > t->nlocs) return -1;
    orc_loc *l = t->locs[handle - 1];
    if (!l || !l->leaf) return 0; /* dangling: dropped by a split or an aborted insert */
    orc_rmeta *mp = l_meta(l->leaf, l->slot);
    *meta = mp->meta;
    *next = next_handle(mp->next);
    return 0;
}

static orc_copy *copy_by(orc_tree *t, uint32_t id) { return id < t->ncopies ? t->copy_by_id[id] : NULL; }

int orc_copy_state(orc_tree *t, uint32_t copy_id, uint32_t *st /* cstamp pstamp rstamp sstamp nreaders count waiting */) {
    orc_copy *c = copy_by(t, copy_id);
    if (!c) return -1;
    st[0] = c->cstamp;
    st[1] = c->pstamp;
    st[2] = c->rstamp;
    st[3] = c->sstamp;
    st[4] = c->nreaders;
    st[5] = (uint32_t)(uint16_t)c->wr_count;
    st[6] = (uint32_t)c->waiting;
    return 0;
}

uint32_t orc_copy_readers(orc_tree *t, uint32_t copy_id, uint32_t *out, uint32_t max) {
    orc_copy *c = copy_by(t, copy_id);
    if (!c) return 0;
    for (uint32_t i = 0; i < c->nreaders && i < max; i++) out[i] = c->readers[i];
    return c->nreaders;
}

int orc_copy_add_reader(orc_tree *t, uint32_t copy_id, uint32_t read_id) {
    orc_copy *c = copy_by(t, copy_id);
    if (!c) return -1;
    if (c->nreaders == c->capreaders) {
        c->capreaders = c->capreaders ? 2 * c->capreaders : 8;
        c->readers = realloc(c->readers, sizeof(uint32_t) * c->capreaders);
        if (!c->readers) abort();
    }
    c->readers[c->nreaders++] = read_id;
    return 0;
}

/* delta +1: IncreaseWRCount -> AddCount, refused (0) once the header is waiting; -1:
 * DecreaseWRCount -> SubCount (a uint16_t count) */
int orc_copy_wr_count(orc_tree *t, uint32_t copy_id, int delta) {
    orc_copy *c = copy_by(t, copy_id);
    if (!c) return -1;
    if (delta > 0) {
        if (c->waiting) return 0;
        c->wr_count = (uint16_t)(c->wr_count + 1);
        return 1;
    }
    c->wr_count = (uint16_t)(c->wr_count - 1);
    return 1;
}

int orc_copy_update_ps(orc_tree *t, uint32_t copy_id, uint32_t pstamp) {
    orc_copy *c = copy_by(t, copy_id);
    if (!c) return -1;
    c->pstamp = pstamp;
    return 0;
}

/* ---------------------------------------------------------------- murmur */
/* MurmurHash64A, misc/murmur/MurmurHash2.cpp:99-147 (little-endian, unaligned) */
uint64_t orc_murmur64a(const void *key, int len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = seed ^ ((uint64_t)(int64_t)len * m);
    const uint8_t *p = key;
    int nblocks = len / 8;
    for (int i = 0; i < nblocks; i++) {
        uint64_t k;
        memcpy(&k, p + 8 * i, 8);
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
    }
    const uint8_t *d2 = p + 8 * nblocks;
    switch (len & 7) {
    case 7: h ^= (uint64_t)d2[6] << 48; /* fallthrough */
    case 6: h ^= (uint64_t)d2[5] << 40; /* fallthrough */
    case 5: h ^= (uint64_t)d2[4] << 32; /* fallthrough */
    case 4: h ^= (uint64_t)d2[3] << 24; /* fallthrough */
    case 3: h ^= (uint64_t)d2[2] << 16; /* fallthrough */
    case 2: h ^= (uint64_t)d2[1] << 8;  /* fallthrough */
    case 1:
        h ^= (uint64_t)d2[0];
        h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}

void orc_murmur64a_batch(const uint64_t *keys, uint64_t n, int len, uint64_t seed, uint64_t *out) {
    for (uint64_t i = 0; i < n; i++) out[i] = orc_murmur64a(&keys[i], len, seed);
}

/* ---------------------------------------------------------------- TPC-C stock-level */
/* tpcc_stock_level.cpp:37-180 over DISTRICT / ORDER_LINE / STOCK trees (keys of int64
 * fields, payloads starting with D_NEXT_O_ID / OL_I_ID / S_QUANTITY as int32):
 * returns the number of distinct S_I_IDs below the threshold, -1 if the transaction aborts. */
static int32_t rd_i32(const uint8_t *p) { int32_t v; memcpy(&v, p, 4); return v; }
static int64_t rd_i64(const uint8_t *p) { int64_t v; memcpy(&v, p, 8); return v; }

int32_t orc_stock_level(orc_tree *dist, orc_tree *ol, orc_tree *stock, int64_t w, int64_t d, int32_t threshold,
                        uint32_t read_id) {
    orc_read_out o;
    uint8_t drow[16 + 4096], srow[16 + 4096], olrows[10 * (32 + 4096)], st[10];
    int64_t dk[2] = {w, d};
    read_one(dist, (const uint8_t *)dk, 16, read_id, &o, drow);
    if (o.status != ORC_ST_LATEST && o.status != ORC_ST_COPY && o.status != ORC_ST_OLD) return -1;
    int32_t next = rd_i32(drow + dist->key_pad);
    int32_t items[20];
    int nitems = 0;
    uint32_t ors = ol->key_pad + ol->payload_size;
    scanrec_t *buf = xmalloc(sizeof(scanrec_t) * 4096);
    for (int32_t oid = next - 20; oid < next; oid++) {
        int64_t ok[4] = {w, d, oid, 5};
        uint32_t c = scan_one_ex(ol, (const uint8_t *)ok, 32, 10, olrows, buf, 4096, read_id, st);
        int found = 0;
        int32_t item = 0;
        for (uint32_t j = 0; j < c && !found; j++) {
            if (st[j] != ORC_ST_LATEST && st[j] != ORC_ST_OLD) continue;
            const uint8_t *r = olrows + (uint64_t)j * ors;
            if (rd_i64(r + 16) == oid && rd_i64(r) == w && rd_i64(r + 8) == d) {
                found = 1;
                item = rd_i32(r + ol->key_pad);
            }
        }
        if (!found) continue;
        int64_t sk[2] = {w, item};
        read_one(stock, (const uint8_t *)sk, 16, read_id, &o, srow);
        if (o.status == ORC_ST_FAIL_INVALID_TS) { free(buf); return -1; }
        if (o.status != ORC_ST_LATEST && o.status != ORC_ST_COPY && o.status != ORC_ST_OLD) continue;
        if (rd_i32(srow + stock->key_pad) < threshold) {
            int32_t sid = (int32_t)rd_i64(srow + 8), dup = 0;
            for (int k = 0; k < nitems; k++) dup |= items[k] == sid;
            if (!dup) items[nitems++] = sid;
        }
    }
    free(buf);
    return nitems;
}

typedef struct {
    orc_tree *dist, *ol, *stock;
    const int64_t *w, *d;
    const int32_t *thr;
    const uint32_t *rid;
    int32_t *res;
    uint64_t b, e;
} sl_job_t;

static void *sl_worker(void *arg) {
    sl_job_t *j = arg;
    for (uint64_t i = j->b; i < j->e; i++)
        j->res[i] = orc_stock_level(j->dist, j->ol, j->stock, j->w[i], j->d[i], j->thr[i],
                                    j->rid ? j->rid[i] : 0xFFFFFFFEu);
    return NULL;
}

void orc_stock_level_batch(orc_tree *dist, orc_tree *ol, orc_tree *stock, const int64_t *w, const int64_t *d,
                           const int32_t *thr, const uint32_t *rid, uint64_t n, int32_t *res, int nthreads,
                           double *seconds) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    sl_job_t jobs[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = (sl_job_t){dist, ol, stock, w, d, thr, rid, res, n * (uint64_t)i / nthreads,
                             n * (uint64_t)(i + 1) / nthreads};
        pthread_create(&th[i], NULL, sl_worker, &jobs[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* ---------------------------------------------------------------- CH-benCHmark Q2 */
/* RunQuery2 (benchmark/tpcc/tpcc_new_order.cpp:608-982) over REGION / NATION / SUPPLIER /
 * ITEM / STOCK trees (tpcc_record.h:160-200, 417-500, 773-880: 8-byte keys, STOCK {w, i}
 * 16 bytes; payloads R_NAME.. / N_REGIONKEY.. / SU_NATIONKEY.. / I_IM_ID, I_NAME, I_PRICE,
 * I_DATA / S_QUANTITY, S_YTD, S_ORDER_CNT, S_REMOTE_CNT..), with the driver's pre-built
 * supplier -> stocks map (tpcc_workload.cpp:398-404) as CSR: map_off[10001], (map_w, map_i)
 * in push order.  One record per supplier the query visits, in visiting order; *aborted = 1
 * where the reference aborts (a FAILURE read, or a STOCK / ITEM lookup that yields no tuple).
 * Nothing is written: out[k].update marks the stock update the transaction would make
 * (PointUpdateExecutor of S_QUANTITY..S_REMOTE_CNT = q + 50, ytd, order_cnt, remote_cnt). */
static const char *const q2_regions[] = {"AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"}; /* tpcc_record.h:931 */

typedef struct { int64_t supp, nation; } q2_supp_t;

/* TableScanExecutor with scan_sz == -1 (executor.h:580-612): ScanLeafNode over every leaf,
 * slots in slot order, raw records (no visibility).  Empty (meta == 0) slots are skipped. */
static void q2_scan_leaves(void *node, q2_supp_t *out, uint64_t *n, uint64_t cap) {
    if (is_leaf(node)) {
        uint8_t *l = node;
        uint32_t cnt = st_count(*l_status(l));
        for (uint32_t i = 0; i < cnt && *n < cap; i++) {
            uint64_t m = l_meta(l, i)->meta;
            if (!m) continue;
            const uint8_t *k = l + m_offset(m);
            out[*n].supp = rd_i64(k);
            out[*n].nation = rd_i64(k + pad_key(m_keylen(m)));
            (*n)++;
        }
        return;
    }
    orc_inner *p = node;
    for (uint32_t i = 0; i < p->count; i++) q2_scan_leaves(p->child[i], out, n, cap);
}

static int q2_produced(uint8_t st) { return st == ORC_ST_LATEST || st == ORC_ST_COPY || st == ORC_ST_OLD; }

int64_t orc_ch_query2(orc_tree *region, orc_tree *nation, orc_tree *supplier, orc_tree *item, orc_tree *stock,
                      const uint32_t *map_off, const int32_t *map_w, const int32_t *map_i, int target_region,
                      uint32_t read_id, orc_q2_rec *out, uint64_t max_out, int *aborted) {
    *aborted = 0;
    uint64_t nout = 0;
    uint32_t rrow = region->key_pad + region->payload_size, nrow = nation->key_pad + nation->payload_size;
    uint8_t *regs = xmalloc((uint64_t)rrow * 6), *nats = xmalloc((uint64_t)nrow * 65);
    scanrec_t *buf = xmalloc(sizeof(scanrec_t) * 4096);
    uint64_t zero = 0;
    uint32_t nreg = scan_one(region, (const uint8_t *)&zero, 8, 6, regs, buf, 4096);   /* :650-661 */
    uint32_t nnat = scan_one(nation, (const uint8_t *)&zero, 8, 65, nats, buf, 4096);  /* :731-742 */
    free(buf);
    q2_supp_t *supps = xmalloc(sizeof(q2_supp_t) * 20000);
    uint64_t nsupp = 0;
    q2_scan_leaves(supplier->root, supps, &nsupp, 20000);                             /* :783-797 */
    uint8_t irow[8 + 4096], srow[16 + 4096];
    orc_read_out o;
    for (uint32_t r = 0; r < nreg && !*aborted; r++) {
        const uint8_t *rr = regs + (uint64_t)r * rrow;
        char rname[56];
        memcpy(rname, rr + region->key_pad, 55);
        rname[55] = 0;
        if (strcmp(rname, q2_regions[target_region]) != 0) continue;                     /* :772 */
        int64_t rkey = rd_i64(rr);
        for (uint32_t a = 0; a < nnat && !*aborted; a++) {
            const uint8_t *nr = nats + (uint64_t)a * nrow;
            if (rd_i64(nr + nation->key_pad) != rkey) continue;                           /* :778 */
            int64_t nkey = rd_i64(nr);
            for (uint64_t s = 0; s < nsupp && !*aborted; s++) {                           /* :801 */
                if (supps[s].nation != nkey) continue;                                    /* :806 */
                int64_t sk = supps[s].supp;
                /* the "min" never moves (min_qty is not updated, :848): the last stock wins */
                int64_t w0 = 0, i0 = 0;
                int32_t q[4] = {0, 0, 0, 0};
                if (sk >= 0 && sk < 10000)
                    for (uint32_t e = map_off[sk]; e < map_off[sk + 1]; e++) {            /* :815 */
                        int64_t key[2] = {map_w[e], map_i[e]};
                        read_one(stock, (const uint8_t *)key, 16, read_id, &o, srow);
                        if (!q2_produced(o.status)) { *aborted = 1; break; }               /* :840-851 */
                        w0 = rd_i64(srow);
                        i0 = rd_i64(srow + 8);
                        for (int c = 0; c < 4; c++) q[c] = rd_i32(srow + stock->key_pad + 4 * c);
                    }
                if (*aborted) break;
                uint64_t ik = (uint64_t)i0;                                                /* :863 */
                read_one(item, (const uint8_t *)&ik, 8, read_id, &o, irow);
                if (!q2_produced(o.status)) { *aborted = 1; break; }                       /* :879-887 */
                /* std::string(I_DATA).find('b') (:890-892): I_DATA = payload bytes 44..107,
                 * up to its first NUL */
                const uint8_t *idata = irow + item->key_pad + 44;
                uint8_t has_b = 0;
                for (int c = 0; c < 64 && idata[c]; c++) has_b |= idata[c] == 'b';
                if (nout < max_out) {
                    orc_q2_rec *x = &out[nout];
                    memset(x, 0, sizeof(*x));
                    x->supp_key = sk;
                    x->s_w_id = w0;
                    x->s_i_id = i0;
                    x->s_quantity = q[0];
                    x->s_ytd = q[1];
                    x->s_order_cnt = q[2];
                    x->s_remote_cnt = q[3];
                    x->item_has_b = has_b;
                    x->update = !has_b && q[0] < 10;                                       /* :893-897 */
                }
                nout++;
            }
        }
    }
    free(regs);
    free(nats);
    free(supps);
    return (int64_t)nout;
}

typedef struct {
    orc_tree *r, *n, *s, *i, *k;
    const uint32_t *off;
    const int32_t *w, *it;
    int target;
    uint32_t rid;
    uint64_t b, e, recs;
    int aborts;
} q2_job_t;

static void *q2_worker(void *arg) {
    q2_job_t *j = arg;
    orc_q2_rec *tmp = xmalloc(sizeof(orc_q2_rec) * 16384);
    for (uint64_t x = j->b; x < j->e; x++) {
        int ab = 0;
        j->recs += (uint64_t)orc_ch_query2(j->r, j->n, j->s, j->i, j->k, j->off, j->w, j->it, j->target, j->rid, tmp,
                                           16384, &ab);
        j->aborts += ab;
    }
    free(tmp);
    return NULL;
}

/* count read-only Q2 transactions on nthreads threads (CPU baseline); returns records visited */
uint64_t orc_ch_query2_timed(orc_tree *region, orc_tree *nation, orc_tree *supplier, orc_tree *item, orc_tree *stock,
                             const uint32_t *map_off, const int32_t *map_w, const int32_t *map_i, int target_region,
                             uint32_t read_id, uint64_t count, int nthreads, double *seconds) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    q2_job_t jobs[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (q2_job_t){region, nation, supplier, item, stock, map_off, map_w, map_i, target_region, read_id,
                             count * (uint64_t)t / nthreads, count * (uint64_t)(t + 1) / nthreads, 0, 0};
        pthread_create(&th[t], NULL, q2_worker, &jobs[t]);
    }
    uint64_t recs = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        recs += jobs[t].recs;
    }
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    return recs;
}
