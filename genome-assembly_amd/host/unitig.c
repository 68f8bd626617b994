/*
 * unitig.c -- the reference's unitig extension, find_kmer_extensions
 * (binning.c:659-783, with find_kmer_extension / more_kmer_extension :477-649,
 * extend_kmers / further_extend_kmers / merge_lists / merge_keys :151-276,
 * merge_sorted_list llist.c:46-81), replayed EXACTLY on the materialised
 * tables without the reference's all-pairs candidate scan.
 *
 * What the reference does.  For mmer scores from getscore("CTT..T") up to
 * score_limit = getbp('A') * MMER_SIZE = 65 M (binning.c:672; the mmer string
 * wraps from AA..A to TT..T, next_smaller_mmer :129-145), it walks that mmer's
 * level-2 table bucket by bucket and chain by chain (:684-776).  For each
 * entry it looks for the unique entry overlapping it by K-1 bases, among the
 * <= 4 tables of the mmers one base off its end whose score is <= the current
 * one (:500-518), by iterating EVERY entry of those tables (:521-546) -- the
 * walk is quadratic in the table sizes (C2's reads at M = 4: 13 min for the
 * first 20 K reads, profiles/r06/unitig/).  A unique candidate is merged
 * (keys, per-base read-id lists), both entries unlinked, and the merged key
 * extended again (:734-766) until no unique candidate is left; it is then
 * zhash_set into the current table (:768).
 *
 * What makes "exact" non-trivial, and how each is reproduced:
 *  - iteration ORDER decides which of several candidates is found first and
 *    where a multiple-candidate scan stops.  Order within a table is (bucket,
 *    chain position); chains only ever lose entries or gain them at the head
 *    (zhash_set, zhash.c:64-66; no rehash can happen, every merge removes at
 *    least one entry first), so a per-entry (bucket, seq) with seq decreasing
 *    for every inserted entry IS the chain order;
 *  - iterate_level_two_hash's cursor is function-static (binning.c:389-392):
 *    a scan that breaks on a second candidate (:534-540, :624-630) leaves it
 *    inside that table, and the NEXT iterate call on the same table RESUMES
 *    from there instead of starting over.  The model keeps (table, link,
 *    index) exactly as the reference's statics and resumes the same way
 *    (reading the live link, which a zhash_set at the bucket head may have
 *    changed); on return it leaves the reference's own iterator in the same
 *    state when the program has one (the drop-in: print_kmers resumes too);
 *  - the deletion statements (:698-731, :745-765) are executed as written on
 *    the real chains, including their quirks (the second branch at :710 is
 *    the first one's test; :762-764 frees an entry without its key; none of
 *    :745-765 decrements entry_count; a "predecessor" match at :752 with both
 *    links NULL moves the walk's link into another chain);
 *  - one branch is a use-after-free in the reference: at :721-731 when the
 *    extension is the kmer's chain successor, the extension's link lives in
 *    the kmer entry just freed, so the extension is freed but stays linked.
 *    What glibc does next is undefined (its key field is then a free-list
 *    pointer); the replay keeps it linked and readable (the outcome of an
 *    allocator that does not reuse the block), counts it (u1_events in the
 *    trace) and gives it an empty per-base list.  None of the tested inputs
 *    reach it.
 *
 * Candidates come from two hash indexes, (table, first K-1 bases) and (table,
 * last K-1 bases), built once per table set and updated as entries merge;
 * a query costs <= 4 probes plus the (few) entries with that overlap.
 * Keys outside ACGT (not produced by the engine, which rejects them) fall
 * back to string lookups and byte compares.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/binning_gpu.h"

typedef unsigned __int128 u128;

#ifndef KMER_SIZE
#define KMER_SIZE 31 /* binning.c:11 */
#endif
#ifndef MMER_SIZE
#define MMER_SIZE 4 /* binning.c:10 */
#endif

/* K and M: binning_gpu.c's kbh_configure state when it is linked, else (this
 * file alone over the reference's own tables) the compile-time values */
__attribute__((weak)) void kbh_get_config(int *K, int *M, int *cutoff)
{
    if (K) *K = KMER_SIZE;
    if (M) *M = MMER_SIZE;
    if (cutoff) *cutoff = 1;
}

#define NONE UINT32_MAX

/* the reference's bucket ladder (zhash.c:13-17; binning.c:20-23 copies it) */
static const size_t UT_LADDER[23] = {
    53, 101, 211, 503, 1553, 3407, 6803, 12503, 25013, 50261, 104729, 250007,
    500009, 1000003, 2000029, 4000037, 10000019, 25000009, 50000047, 104395301,
    217645177, 512927357, 1000000007};

/* the reference's level-2 iterator, when the program links one (the drop-in:
 * binning.c:387-460); its static cursor is synchronised on return */
extern void *iterate_level_two_hash(struct ZHashTable *hash_table, bool indirection, bool remove_current)
    __attribute__((weak));

typedef struct {
    struct ZHashEntry *e;
    u128 pre, suf;      /* first / last K-1 bases, getval digits, first base high */
    int64_t seq;        /* chain order inside the bucket (ascending) */
    uint32_t tab, bucket;
    uint32_t npre, nsuf;/* next entry with the same (table, prefix) / (table, suffix) */
    uint32_t klen;
    uint8_t live, zombie, indexed;
} ut_ent;

typedef struct {
    uint32_t idx;
    struct ZHashEntry **link;
} ut_hit;

static struct {
    struct ZHashTable *level1;
    int K, M, general;            /* general: some key outside ACGT */
    ut_ent *ent;
    uint32_t n, cap;
    uintptr_t *pk;                /* entry pointer -> index (open addressing) */
    uint32_t *pv;
    uint64_t pcap, pused;
    uint32_t *cpre, *csuf;        /* (table, overlap) -> chain head */
    uint64_t ccap, cused_pre, cused_suf;
    struct ZHashTable **tabs;     /* level-2 tables */
    uint32_t *tab_val;            /* their mmer's getscore value */
    uint32_t ntab;
    int32_t *tab_of;              /* [4^M] value -> table, -1 none */
    int64_t next_seq;
    /* iterate_level_two_hash's statics (binning.c:389-392): table, entry, index */
    int it_valid;
    uint32_t it_tab;
    struct ZHashEntry **it_link;
    size_t it_index;
    struct ZHashTable *ref_it_table; /* where the reference's own cursor was left */
    uint64_t sig;                 /* the tables' counts when the last call returned */
    kbh_unitig_stats st;
} U;

/* ---- small helpers ---- */

static void *ut_alloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p) exit(EXIT_FAILURE); /* zhash.c:236 convention */
    return p;
}

static double ut_now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static inline uint64_t ut_mix(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

static inline int ut_acgt(char c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; }

/* getval (binning.c:91-111) */
static inline unsigned ut_val(char c)
{
    switch (c) {
    case 'T': return 0;
    case 'G': return 1;
    case 'C': return 2;
    default: return 3;
    }
}

static inline u128 ut_code(const char *s, int n)
{
    u128 c = 0;
    for (int j = 0; j < n; j++) c = (c << 2) | ut_val(s[j]);
    return c;
}

static void ut_fail(const char *what)
{
    fprintf(stderr, "kbin unitig: internal: %s\n", what);
    exit(EXIT_FAILURE);
}

/* ---- entry pointer -> index ---- */

static void ut_pmap_grow(void);

static void ut_pmap_put(struct ZHashEntry *e, uint32_t i)
{
    if ((U.pused + 1) * 2 > U.pcap) ut_pmap_grow();
    uint64_t s = ut_mix((uintptr_t)e) & (U.pcap - 1);
    while (U.pk[s] && U.pk[s] != (uintptr_t)e) s = (s + 1) & (U.pcap - 1);
    if (!U.pk[s]) U.pused++;
    U.pk[s] = (uintptr_t)e; /* a freed block reused by a new entry: overwritten */
    U.pv[s] = i;
}

static void ut_pmap_grow(void)
{
    uintptr_t *ok = U.pk;
    uint32_t *ov = U.pv;
    const uint64_t oc = U.pcap;
    U.pcap = oc ? oc * 2 : 1024;
    U.pk = calloc(U.pcap, sizeof *U.pk);
    U.pv = ut_alloc(U.pcap * sizeof *U.pv);
    if (!U.pk) exit(EXIT_FAILURE);
    U.pused = 0;
    for (uint64_t s = 0; s < oc; s++)
        if (ok[s]) ut_pmap_put((struct ZHashEntry *)ok[s], ov[s]);
    free(ok);
    free(ov);
}

static uint32_t ut_pmap_get(const struct ZHashEntry *e)
{
    uint64_t s = ut_mix((uintptr_t)e) & (U.pcap - 1);
    while (U.pk[s] != (uintptr_t)e) {
        if (!U.pk[s]) ut_fail("entry not indexed");
        s = (s + 1) & (U.pcap - 1);
    }
    return U.pv[s];
}

/* ---- (table, overlap) -> entries ---- */

static inline uint64_t ut_chash(uint32_t tab, u128 code)
{
    return ut_mix((uint64_t)code ^ ut_mix((uint64_t)(code >> 64) + 0x9e3779b97f4a7c15ull * (tab + 1)));
}

/* slot of (tab, code) in map (pre: by prefix, else suffix): the chain head,
 * or the empty slot where it goes */
static inline uint64_t ut_cslot(const uint32_t *map, int pre, uint32_t tab, u128 code)
{
    uint64_t s = ut_chash(tab, code) & (U.ccap - 1);
    for (;;) {
        const uint32_t h = map[s];
        if (h == NONE) return s;
        const ut_ent *x = &U.ent[h];
        if (x->tab == tab && (pre ? x->pre : x->suf) == code) return s;
        s = (s + 1) & (U.ccap - 1);
    }
}

static void ut_cmap_link(uint32_t i)
{
    ut_ent *x = &U.ent[i];
    uint64_t s = ut_cslot(U.cpre, 1, x->tab, x->pre);
    if (U.cpre[s] == NONE) U.cused_pre++;
    x->npre = U.cpre[s];
    U.cpre[s] = i;
    s = ut_cslot(U.csuf, 0, x->tab, x->suf);
    if (U.csuf[s] == NONE) U.cused_suf++;
    x->nsuf = U.csuf[s];
    U.csuf[s] = i;
}

static void ut_cmap_rebuild(uint64_t cap)
{
    free(U.cpre);
    free(U.csuf);
    U.ccap = cap;
    U.cpre = ut_alloc(cap * sizeof(uint32_t));
    U.csuf = ut_alloc(cap * sizeof(uint32_t));
    memset(U.cpre, 0xff, cap * sizeof(uint32_t));
    memset(U.csuf, 0xff, cap * sizeof(uint32_t));
    U.cused_pre = U.cused_suf = 0;
    for (uint32_t i = 0; i < U.n; i++)
        if (U.ent[i].indexed) ut_cmap_link(i);
}

/* a new entry (the initial tables, or a merged key zhash_set at :768) */
static uint32_t ut_add(struct ZHashEntry *e, uint32_t tab, uint32_t bucket, int64_t seq)
{
    if (U.n == U.cap) {
        U.cap = U.cap ? U.cap * 2 : 4096;
        U.ent = realloc(U.ent, (size_t)U.cap * sizeof(ut_ent));
        if (!U.ent) exit(EXIT_FAILURE);
    }
    const uint32_t i = U.n++;
    ut_ent *x = &U.ent[i];
    memset(x, 0, sizeof *x);
    x->e = e;
    x->tab = tab;
    x->bucket = bucket;
    x->seq = seq;
    x->live = 1;
    x->npre = x->nsuf = NONE;
    const size_t len = strlen(e->key);
    x->klen = (uint32_t)len;
    const int o = U.K - 1;
    for (size_t j = 0; j < len && !U.general; j++)
        if (!ut_acgt(e->key[j])) U.general = 1;
    if (len >= (size_t)o) { /* (shorter keys never overlap anything: compare_overlap reads K-1 bytes) */
        x->pre = ut_code(e->key, o);
        x->suf = ut_code(e->key + len - o, o);
        x->indexed = 1;
    }
    ut_pmap_put(e, i);
    return i;
}

static void ut_index_new(uint32_t i)
{
    if (!U.ent[i].indexed) return;
    if ((U.cused_pre + 1) * 2 > U.ccap || (U.cused_suf + 1) * 2 > U.ccap)
        ut_cmap_rebuild(U.ccap * 2);
    else
        ut_cmap_link(i);
}

static void ut_reset(void)
{
    free(U.ent);
    free(U.pk);
    free(U.pv);
    free(U.cpre);
    free(U.csuf);
    free(U.tabs);
    free(U.tab_val);
    free(U.tab_of);
    memset(&U, 0, sizeof U);
}

/* ---- the initial index, built by worker threads (the tables are read-only
 * here): entries per table counted, then filled at their offsets (codes,
 * positions), then the pointer map and the two candidate maps filled
 * lock-free (compare-and-swap on a slot; every key distinct) ---- */

typedef struct {
    uint32_t *cnt;   /* [ntab] entries per table, then offsets */
    uint32_t n_work, next;
    int phase;       /* 0 count, 1 fill, 2 pointer map, 3 candidate maps */
    uint64_t used_pre, used_suf;
    int general;
} ut_job;

static long ut_threads(void)
{
    long nt = sysconf(_SC_NPROCESSORS_ONLN);
    const char *env = getenv("KBH_THREADS");
    if (env && atol(env) > 0) nt = atol(env);
    if (nt < 1) nt = 1;
    return nt > 16 ? 16 : nt;
}

/* push entry i onto map's chain of its (table, code), lock-free */
static int ut_cmap_push(uint32_t *map, int pre, uint32_t i)
{
    ut_ent *x = &U.ent[i];
    const u128 code = pre ? x->pre : x->suf;
    uint64_t s = ut_chash(x->tab, code) & (U.ccap - 1);
    for (;;) {
        uint32_t h = __atomic_load_n(&map[s], __ATOMIC_ACQUIRE);
        if (h == NONE) {
            if (pre) x->npre = NONE; else x->nsuf = NONE;
            if (__atomic_compare_exchange_n(&map[s], &h, i, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return 1;
            continue; /* (someone took the slot: look again) */
        }
        const ut_ent *y = &U.ent[h];
        if (y->tab == x->tab && (pre ? y->pre : y->suf) == code) {
            if (pre) x->npre = h; else x->nsuf = h;
            if (__atomic_compare_exchange_n(&map[s], &h, i, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return 0;
            continue;
        }
        s = (s + 1) & (U.ccap - 1);
    }
}

static void *ut_index_worker(void *arg)
{
    ut_job *j = arg;
    uint64_t up = 0, us = 0;
    int general = 0;
    const int o = U.K - 1;
    const uint32_t CH = 4096; /* (entries per work item in phases 2-3) */
    for (;;) {
        const uint32_t w = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (w >= j->n_work) break;
        if (j->phase <= 1) {
            struct ZHashTable *T = U.tabs[w];
            if (!T) continue;
            const size_t m2 = UT_LADDER[T->size_index];
            uint32_t k = j->phase ? j->cnt[w] : 0;
            for (size_t b = 0; b < m2; b++) {
                int64_t p = 0;
                for (struct ZHashEntry *ke = T->entries[b]; ke; ke = ke->next, p++, k++) {
                    if (!j->phase) continue;
                    ut_ent *x = &U.ent[k];
                    memset(x, 0, sizeof *x);
                    x->e = ke;
                    x->tab = w;
                    x->bucket = (uint32_t)b;
                    x->seq = p;
                    x->live = 1;
                    x->npre = x->nsuf = NONE;
                    const char *key = ke->key;
                    const size_t len = strlen(key);
                    x->klen = (uint32_t)len;
                    for (size_t c = 0; c < len && !general; c++) general |= !ut_acgt(key[c]);
                    if (len >= (size_t)o) {
                        x->pre = ut_code(key, o);
                        x->suf = ut_code(key + len - o, o);
                        x->indexed = 1;
                    }
                }
            }
            if (!j->phase) j->cnt[w] = k;
        } else {
            const uint32_t a = w * CH, e = a + CH < U.n ? a + CH : U.n;
            for (uint32_t i = a; i < e; i++) {
                if (j->phase == 2) {
                    const uintptr_t key = (uintptr_t)U.ent[i].e;
                    uint64_t s = ut_mix(key) & (U.pcap - 1);
                    for (;;) {
                        uintptr_t cur = 0;
                        if (__atomic_compare_exchange_n(&U.pk[s], &cur, key, 0, __ATOMIC_ACQ_REL,
                                                        __ATOMIC_ACQUIRE)) {
                            U.pv[s] = i;
                            break;
                        }
                        s = (s + 1) & (U.pcap - 1);
                    }
                } else if (U.ent[i].indexed) {
                    up += (uint64_t)ut_cmap_push(U.cpre, 1, i);
                    us += (uint64_t)ut_cmap_push(U.csuf, 0, i);
                }
            }
        }
    }
    __atomic_fetch_add(&j->used_pre, up, __ATOMIC_RELAXED);
    __atomic_fetch_add(&j->used_suf, us, __ATOMIC_RELAXED);
    if (general) __atomic_store_n(&j->general, 1, __ATOMIC_RELAXED);
    return NULL;
}

static void ut_run(ut_job *j, int phase, uint32_t n_work)
{
    j->phase = phase;
    j->next = 0;
    j->n_work = n_work;
    long nt = ut_threads();
    if ((uint64_t)nt > n_work) nt = n_work ? (long)n_work : 1;
    pthread_t th[16];
    int started[16] = {0};
    for (long t = 1; t < nt; t++) started[t] = pthread_create(&th[t], NULL, ut_index_worker, j) == 0;
    ut_index_worker(j);
    for (long t = 1; t < nt; t++)
        if (started[t]) pthread_join(th[t], NULL);
}

static void ut_index_tables(void)
{
    ut_job j;
    memset(&j, 0, sizeof j);
    j.cnt = ut_alloc(((size_t)U.ntab + 1) * sizeof(uint32_t));
    ut_run(&j, 0, U.ntab);
    uint64_t tot = 0;
    for (uint32_t t = 0; t < U.ntab; t++) {
        const uint32_t c = j.cnt[t];
        j.cnt[t] = (uint32_t)tot;
        tot += c;
    }
    if (tot >= NONE) ut_fail("more than 2^32 entries");
    if (tot + 4096 > U.cap) {
        U.cap = (uint32_t)(tot + tot / 4 + 4096);
        U.ent = realloc(U.ent, (size_t)U.cap * sizeof(ut_ent));
        if (!U.ent) exit(EXIT_FAILURE);
    }
    ut_run(&j, 1, U.ntab);
    U.n = (uint32_t)tot;
    if (j.general) U.general = 1;
    /* pointer map and candidate maps at <= 1/2 load (new entries grow them) */
    uint64_t pc = 1024;
    while (pc < 2 * ((uint64_t)U.n + U.n / 4 + 1)) pc *= 2;
    if (pc > U.pcap) {
        free(U.pk);
        free(U.pv);
        U.pcap = pc;
        U.pk = calloc(U.pcap, sizeof *U.pk);
        U.pv = ut_alloc(U.pcap * sizeof *U.pv);
        if (!U.pk) exit(EXIT_FAILURE);
    }
    U.pused = U.n;
    const uint32_t chunks = (U.n + 4095) / 4096;
    ut_run(&j, 2, chunks);
    U.ccap = pc;
    free(U.cpre);
    free(U.csuf);
    U.cpre = ut_alloc(U.ccap * sizeof(uint32_t));
    U.csuf = ut_alloc(U.ccap * sizeof(uint32_t));
    memset(U.cpre, 0xff, U.ccap * sizeof(uint32_t));
    memset(U.csuf, 0xff, U.ccap * sizeof(uint32_t));
    ut_run(&j, 3, chunks);
    U.cused_pre = j.used_pre;
    U.cused_suf = j.used_suf;
    free(j.cnt);
}

/* index every level-2 entry of level1 (the first call on a table set) */
static void ut_build(struct ZHashTable *level1, int K, int M)
{
    ut_reset();
    U.level1 = level1;
    U.K = K;
    U.M = M;
    U.next_seq = -1;
    const size_t nv = (size_t)1 << (2 * M);
    U.tab_of = ut_alloc(nv * sizeof(int32_t));
    for (size_t v = 0; v < nv; v++) U.tab_of[v] = -1;
    const size_t m1 = UT_LADDER[level1->size_index];
    uint32_t nt = 0;
    uint64_t ne = 0;
    for (size_t b = 0; b < m1; b++)
        for (struct ZHashEntry *me = level1->entries[b]; me; me = me->next) {
            nt++;
            if (me->val) ne += ((struct ZHashTable *)me->val)->entry_count;
        }
    U.tabs = ut_alloc((nt + 1) * sizeof *U.tabs);
    U.tab_val = ut_alloc((nt + 1) * sizeof *U.tab_val);
    U.cap = (uint32_t)(ne + ne / 4 + 4096);
    U.ent = ut_alloc((size_t)U.cap * sizeof(ut_ent));
    U.pcap = 1024;
    while (U.pcap < 2 * (ne + ne / 4 + 1)) U.pcap *= 2;
    U.pk = calloc(U.pcap, sizeof *U.pk);
    U.pv = ut_alloc(U.pcap * sizeof *U.pv);
    if (!U.pk) exit(EXIT_FAILURE);
    for (size_t b = 0; b < m1; b++)
        for (struct ZHashEntry *me = level1->entries[b]; me; me = me->next) {
            const size_t ml = strlen(me->key);
            int ok = ml == (size_t)M;
            for (size_t j = 0; j < ml; j++) ok &= ut_acgt(me->key[j]);
            if (!ok) U.general = 1;
            const uint32_t v = (uint32_t)ut_code(me->key, (int)(ml < 16 ? ml : 16)) & (uint32_t)(nv - 1);
            if (ok && me->val && U.tab_of[v] < 0) U.tab_of[v] = (int32_t)U.ntab;
            U.tabs[U.ntab] = me->val;
            U.tab_val[U.ntab] = v;
            U.ntab++;
        }
    ut_index_tables();
}

/* the table of mmer string s (zhash_get(hash_table, compare_mmer), :514) */
static int32_t ut_table_of(const char *s, uint32_t value)
{
    if (!U.general) return U.tab_of[value];
    struct ZHashTable *t = zhash_get(U.level1, (char *)s);
    if (!t) return -1;
    for (uint32_t i = 0; i < U.ntab; i++)
        if (U.tabs[i] == t) return (int32_t)i;
    return -1;
}

/* the link through which the iterator reaches entry i (its chain predecessor's
 * next field, or the bucket slot) */
static struct ZHashEntry **ut_link_to(uint32_t i)
{
    const ut_ent *x = &U.ent[i];
    struct ZHashEntry **l = &U.tabs[x->tab]->entries[x->bucket];
    while (*l != x->e) {
        if (!*l) ut_fail("entry not in its chain");
        l = &(*l)->next;
    }
    return l;
}

static inline int ut_before(uint32_t b0, int64_t s0, uint32_t b1, int64_t s1)
{
    return b0 < b1 || (b0 == b1 && s0 < s1);
}

/*
 * find_kmer_extension (:477-559) / more_kmer_extension (:572-649): the unique
 * entry whose first (forward) or last (backward) K-1 bases equal q[0..K-1),
 * in the <= 4 tables one base off the key's end with score <= mmer_score,
 * skipping `self` (only find_kmer_extension has that test, :524).  Returns 1
 * with the entry and the link the iterator returned for it, else 0; the
 * iterator model is advanced exactly as the reference's scans advance its
 * static cursor.
 */
static int ut_query(int forward, u128 code, const char *q, const struct ZHashEntry *self, long mmer_score,
                    ut_hit *out)
{
    const int K = U.K, M = U.M;
    const uint32_t mm = (uint32_t)((1u << (2 * (M - 1))) - 1u);
    const uint32_t cm = forward ? (uint32_t)code & mm : (uint32_t)(code >> (2 * (K - M))) & mm;
    char cms[16];
    if (U.general) { /* compare_mmer as the reference builds it (:484-492, :503-506) */
        if (forward)
            memcpy(cms, q + (K - 1) - (M - 1), (size_t)(M - 1));
        else
            memcpy(cms + 1, q, (size_t)(M - 1));
        cms[M] = '\0';
    }
    uint32_t have = NONE;
    for (unsigned i = 0; i < 4; i++) {
        const uint32_t v = forward ? (cm << 2) | i : (i << (2 * (M - 1))) | cm;
        if ((long)v > mmer_score) continue; /* :508 (getscore maps other bytes to 3, as v does) */
        if (U.general) cms[forward ? M - 1 : 0] = "TGCA"[i];
        const int32_t t = ut_table_of(cms, v);
        if (t < 0) continue; /* :514 */
        /* an iterate_level_two_hash call on table t (:521): resumes when the
         * static cursor was left inside t (:403-427), else starts over */
        uint32_t sb = 0;
        int64_t ss = INT64_MIN;
        if (U.it_valid && U.it_tab == (uint32_t)t) {
            struct ZHashEntry *cur = *U.it_link;
            if (!cur) ut_fail("stale cursor on an empty link");
            struct ZHashEntry *s = cur->next;
            if (s) {
                const ut_ent *y = &U.ent[ut_pmap_get(s)];
                if (y->bucket + 1 != U.it_index) ut_fail("cursor chain and index disagree");
                sb = y->bucket;
                ss = y->seq;
            } else {
                sb = (uint32_t)U.it_index;
            }
            U.st.resumes++;
        }
        U.it_valid = 0;
        /* the first two matches at or after the start, in iteration order */
        uint32_t best[2] = {NONE, NONE};
        const uint32_t *map = forward ? U.cpre : U.csuf;
        const uint64_t slot = ut_cslot(map, forward, (uint32_t)t, code);
        for (uint32_t c = map[slot]; c != NONE; c = forward ? U.ent[c].npre : U.ent[c].nsuf) {
            const ut_ent *x = &U.ent[c];
            U.st.candidates++;
            if (!x->live || x->e == self) continue;
            if (ut_before(x->bucket, x->seq, sb, ss)) continue;
            if (U.general && memcmp(forward ? x->e->key : x->e->key + x->klen - (K - 1), q, (size_t)(K - 1)))
                continue; /* compare_overlap, :197-218 */
            if (best[0] == NONE || ut_before(x->bucket, x->seq, U.ent[best[0]].bucket, U.ent[best[0]].seq)) {
                best[1] = best[0];
                best[0] = c;
            } else if (best[1] == NONE ||
                       ut_before(x->bucket, x->seq, U.ent[best[1]].bucket, U.ent[best[1]].seq)) {
                best[1] = c;
            }
        }
        for (int j = 0; j < 2 && best[j] != NONE; j++) {
            if (have != NONE) { /* a second candidate: the scan breaks here (:534-540) */
                U.it_valid = 1;
                U.it_tab = (uint32_t)t;
                U.it_link = ut_link_to(best[j]);
                U.it_index = (size_t)U.ent[best[j]].bucket + 1;
                U.st.multiple++;
                return 0;
            }
            have = best[j];
        }
        /* (the scan ran to the table's end: cursor reset, :445-449) */
    }
    if (have == NONE) return 0;
    out->idx = have;
    out->link = ut_link_to(have);
    return 1;
}

/* ---- keys (merge_keys, :223-241) ---- */

typedef struct {
    char *buf;
    size_t cap, head, len; /* the key is buf[head .. head + len) */
} ut_key;

static void ut_key_init(ut_key *k, const char *s, size_t n)
{
    if (k->cap < 2 * n + 64) {
        free(k->buf);
        k->cap = 2 * n + 64;
        k->buf = ut_alloc(k->cap);
    }
    k->head = (k->cap - n) / 2;
    k->len = n;
    memcpy(k->buf + k->head, s, n);
}

static void ut_key_room(ut_key *k, size_t front, size_t back)
{
    if (k->head >= front && k->cap - k->head - k->len >= back + 1) return;
    const size_t nc = 2 * (k->len + front + back) + 64;
    char *nb = ut_alloc(nc);
    const size_t nh = front + (nc - k->len - front - back) / 2;
    memcpy(nb + nh, k->buf + k->head, k->len);
    free(k->buf);
    k->buf = nb;
    k->cap = nc;
    k->head = nh;
}

/* forward: key + b[K-1:]; backward: b + key[K-1:] == b[: len(b) - (K-1)] + key */
static void ut_key_merge(ut_key *k, const char *b, size_t bl, int forward)
{
    const size_t o = (size_t)U.K - 1, add = bl - o;
    if (forward) {
        ut_key_room(k, 0, add);
        memcpy(k->buf + k->head + k->len, b + o, add);
    } else {
        ut_key_room(k, add, 0);
        k->head -= add;
        memcpy(k->buf + k->head, b, add);
    }
    k->len += add;
}

/* ---- per-base read-id lists (merge_lists :154-195, merge_sorted_list llist.c:46-81) ---- */

static ll_node *ut_merge_sorted(ll_node *a, ll_node *b)
{
    ll_node *sorted = NULL, **t = &sorted;
    while (a && b) {
        if (a->read_id > b->read_id) {
            *t = a;
            a = a->next;
        } else if (a->read_id < b->read_id) {
            *t = b;
            b = b->next;
        } else { /* equal ids: b's node freed (llist.c:60-66) */
            *t = a;
            a = a->next;
            ll_node *d = b;
            b = b->next;
            free(d);
        }
        t = &(*t)->next;
    }
    if (a) *t = a;
    if (b) *t = b;
    return sorted;
}

/* merge_lists(a_len, b_len, a, b, forward); *skip (forward, growing list):
 * the node at a_len - (K-1) when known, updated to the merged list's */
static ll_node *ut_merge_lists(size_t a_len, size_t b_len, ll_node *a, ll_node *b, int forward, ll_node **skip)
{
    const size_t o = (size_t)U.K - 1;
    if (!forward) {
        ll_node *t = a;
        a = b;
        b = t;
        size_t tl = a_len;
        a_len = b_len;
        b_len = tl;
    }
    ll_node *new_list = a;
    if (forward && skip && *skip) {
        a = *skip;
    } else {
        for (size_t i = 0; i + o < a_len; i++) a = a->next;
    }
    ll_node *first = a;
    for (size_t i = 0; i < o; i++) {
        a->item = ut_merge_sorted(a->item, b->item);
        ll_node *d = b;
        b = b->next;
        free(d);
        if (i == o - 1)
            a->next = b;
        else
            a = a->next;
    }
    if (forward && skip) { /* the next merge's skip node: b_len - (K-1) further */
        ll_node *s = first;
        for (size_t i = 0; i + o < b_len; i++) s = s->next;
        *skip = s;
    }
    return new_list;
}

/* a fresh per-base list of n nodes with empty id lists (the U1 zombie's) */
static ll_node *ut_empty_list(size_t n)
{
    ll_node *h = NULL, **t = &h;
    for (size_t i = 0; i < n; i++) {
        ll_node *nd = ut_alloc(sizeof *nd);
        nd->next = NULL;
        nd->item = NULL;
        *t = nd;
        t = &nd->next;
    }
    return h;
}

/* ---- deletions ---- */

static void ut_drop(uint32_t i, int with_key)
{
    ut_ent *x = &U.ent[i];
    x->live = 0;
    if (with_key)
        zfree_entry(x->e, false); /* zhash.c:163-169 */
    else
        free(x->e); /* :764 leaves the key */
    U.st.deleted++;
}

/* leave the reference's own iterator (when linked) where the model's is */
static void ut_sync_ref_iterator(void)
{
    if (!iterate_level_two_hash) return;
    if (U.ref_it_table) { /* run the cursor we left earlier to its end: reset */
        while (iterate_level_two_hash(U.ref_it_table, true, false)) {
        }
        U.ref_it_table = NULL;
    }
    if (!U.it_valid) return;
    struct ZHashTable *X = U.tabs[U.it_tab];
    void *r;
    while ((r = iterate_level_two_hash(X, true, false)) != NULL && r != (void *)U.it_link) {
    }
    if (r != (void *)U.it_link) ut_fail("reference iterator out of step");
    U.ref_it_table = X;
}

static int g_trace = -1;

/* entry counts of every table: a later call on the same level-1 table reuses
 * the index only when nothing else changed the tables in between */
static uint64_t ut_signature(struct ZHashTable *level1)
{
    uint64_t h = ut_mix(level1->entry_count + 0x100 * level1->size_index);
    const size_t m1 = UT_LADDER[level1->size_index];
    for (size_t b = 0; b < m1; b++)
        for (struct ZHashEntry *me = level1->entries[b]; me; me = me->next) {
            const struct ZHashTable *t = me->val;
            h = ut_mix(h ^ (uintptr_t)t ^ (t ? (t->entry_count << 8 | t->size_index) : 0));
        }
    return h;
}

/* binning.c:659-783 */
void find_kmer_extensions(struct ZHashTable *hash_table, bool forward)
{
    int K, M;
    kbh_get_config(&K, &M, NULL);
    const double t0 = ut_now_ms();
    if (g_trace < 0) g_trace = getenv("KBH_TRACE") != NULL;
    if (K < 2 || M < 1 || M > 8 || M > K) ut_fail("K, M out of range");
    const long start = 2L << (2 * (M - 1)); /* getscore("CTT..T"), :663-668 */
    const long limit = 65L * M;             /* getbp('A') * MMER_SIZE, :672 */
    if (start > limit) { /* M >= 5: the loop at :678 never runs */
        U.st.calls++;
        return;
    }
    if (U.level1 != hash_table || U.K != K || U.M != M || U.sig != ut_signature(hash_table))
        ut_build(hash_table, K, M);
    const double t1 = ut_now_ms();
    U.st.index_ms += t1 - t0;
    U.st.calls++;
    const size_t o = (size_t)K - 1;
    const uint32_t vmask = (uint32_t)((1u << (2 * M)) - 1u);
    ut_key key = {0};
    for (long score = start; score <= limit; score++) {
        const uint32_t v = (uint32_t)score & vmask; /* the wrapped mmer string (:129-145) */
        char ms[16];
        for (int j = 0; j < M; j++) ms[j] = "TGCA"[(v >> (2 * (M - 1 - j))) & 3u];
        ms[M] = '\0';
        const int32_t t = ut_table_of(ms, v); /* :681 */
        if (t < 0) continue;
        struct ZHashTable *T = U.tabs[t];
        for (size_t ai = 0; ai < UT_LADDER[T->size_index]; ai++) { /* :685 */
            struct ZHashEntry **kL = &T->entries[ai];
            while (*kL) { /* :688 */
                struct ZHashEntry *Kp = *kL;
                const uint32_t ki = ut_pmap_get(Kp);
                ut_hit h;
                U.st.queries++;
                if (!U.ent[ki].indexed ||
                    !ut_query(forward, forward ? U.ent[ki].suf : U.ent[ki].pre,
                              forward ? Kp->key + U.ent[ki].klen - o : Kp->key, Kp, score, &h)) {
                    kL = &Kp->next; /* :772 */
                    continue;
                }
                U.st.unitigs++;
                /* extend_kmers (:246-258) */
                uint32_t ei = h.idx;
                struct ZHashEntry *E = U.ent[ei].e, **eL = h.link;
                size_t cur_len = U.ent[ki].klen;
                ll_node *skip = NULL;
                ll_node *cur = ut_merge_lists(cur_len, U.ent[ei].klen, Kp->val, E->val, forward, &skip);
                ut_key_init(&key, Kp->key, cur_len);
                ut_key_merge(&key, E->key, U.ent[ei].klen, forward);
                cur_len += U.ent[ei].klen - o;
                uint32_t end = ei;
                U.st.merges++;
                /* unlink both (:698-731) */
                if (E->next == Kp) { /* :698 (and :710, the same test) */
                    kL = eL;
                    *kL = E->next;
                    ut_drop(ei, 1);
                    *kL = Kp->next;
                    ut_drop(ki, 1);
                    T->entry_count -= 2;
                } else { /* :721-731 */
                    const int u1 = eL == &Kp->next;
                    *kL = Kp->next;
                    ut_drop(ki, 1);
                    T->entry_count--;
                    if (u1) { /* the extension's link was inside the entry just freed */
                        if (!U.st.u1_events++)
                            fprintf(stderr, "kbin unitig: warning: binning.c:721-731 frees the extension through a link "
                                            "inside the entry it just freed (a use-after-free; the reference crashes "
                                            "here); the extension is kept linked\n");
                        U.ent[ei].zombie = 1;
                        E->val = ut_empty_list(U.ent[ei].klen);
                    } else {
                        *eL = E->next;
                        ut_drop(ei, 1);
                    }
                    U.tabs[U.ent[ei].tab]->entry_count--;
                }
                /* keep extending (:734-766) */
                for (;;) {
                    const char *q = forward ? key.buf + key.head + key.len - o : key.buf + key.head;
                    U.st.queries++;
                    if (!ut_query(forward, forward ? U.ent[end].suf : U.ent[end].pre, q, NULL, score, &h)) break;
                    ei = h.idx;
                    E = U.ent[ei].e;
                    eL = h.link;
                    /* further_extend_kmers (:263-276) */
                    cur = ut_merge_lists(cur_len, U.ent[ei].klen, cur, E->val, forward, &skip);
                    ut_key_merge(&key, E->key, U.ent[ei].klen, forward);
                    cur_len += U.ent[ei].klen - o;
                    end = ei;
                    U.st.merges++;
                    if (E == *kL) { /* :745-750 */
                        *kL = E->next;
                        ut_drop(ei, 1);
                    } else if (E->next == *kL) { /* :752-758 */
                        kL = eL;
                        *kL = E->next;
                        ut_drop(ei, 1);
                    } else { /* :760-765 */
                        *eL = E->next;
                        ut_drop(ei, 0);
                    }
                }
                /* :768 zhash_set(mmer_hash, key, lists) -- copies the key */
                key.buf[key.head + key.len] = '\0';
                const size_t before = T->entry_count, si = T->size_index;
                zhash_set(T, key.buf + key.head, cur);
                if (T->size_index != si) ut_fail("level-2 table grew during the walk");
                if (T->entry_count != before) { /* created at its bucket's head */
                    const size_t b = zgenerate_hash(T, key.buf + key.head);
                    const uint32_t ni = ut_add(T->entries[b], (uint32_t)t, (uint32_t)b, U.next_seq--);
                    ut_index_new(ni);
                    U.st.inserted++;
                } else {
                    U.st.set_existing++;
                }
            }
        }
    }
    free(key.buf);
    ut_sync_ref_iterator();
    U.sig = ut_signature(hash_table);
    U.st.walk_ms += ut_now_ms() - t1;
    if (g_trace)
        fprintf(stderr,
                "{\"find_kmer_extensions_ms\": %.3f, \"forward\": %d, \"index_ms\": %.3f, \"entries\": %u, "
                "\"queries\": %llu, \"unitigs\": %llu, \"merges\": %llu, \"multiple\": %llu, \"resumes\": %llu, "
                "\"u1_events\": %llu}\n",
                ut_now_ms() - t0, forward ? 1 : 0, U.st.index_ms, U.n, (unsigned long long)U.st.queries,
                (unsigned long long)U.st.unitigs, (unsigned long long)U.st.merges,
                (unsigned long long)U.st.multiple, (unsigned long long)U.st.resumes,
                (unsigned long long)U.st.u1_events);
}

int kbh_unitig_stats_get(kbh_unitig_stats *out)
{
    if (!out) return KB_EINVAL;
    *out = U.st;
    return KB_OK;
}

/*
 * print_kmers (binning.c:827-843): every level-2 key, level-1 and level-2
 * tables in iteration order -- the first level-2 table RESUMES from the
 * static cursor the unitig walk may have left in it (binning.c:403-427),
 * exactly as the reference's iterator does.  The cursor is then reset.
 */
int kbh_print_kmers(struct ZHashTable *hash_table, FILE *out)
{
    const size_t m1 = UT_LADDER[hash_table->size_index];
    int first = 1;
    for (size_t b1 = 0; b1 < m1; b1++)
        for (struct ZHashEntry *me = hash_table->entries[b1]; me; me = me->next) {
            struct ZHashTable *T = me->val;
            if (!T) continue;
            size_t b2 = 0;
            struct ZHashEntry *from = NULL;
            if (first && U.level1 == hash_table && U.it_valid && U.tabs[U.it_tab] == T) {
                from = (*U.it_link)->next;
                b2 = U.it_index;
            }
            first = 0;
            U.it_valid = 0;
            for (struct ZHashEntry *ke = from; ke; ke = ke->next) {
                fputs(ke->key, out);
                fputc('\n', out);
            }
            for (; b2 < UT_LADDER[T->size_index]; b2++)
                for (struct ZHashEntry *ke = T->entries[b2]; ke; ke = ke->next) {
                    fputs(ke->key, out);
                    fputc('\n', out);
                }
        }
    U.it_valid = 0;
    return ferror(out) ? KB_EINVAL : KB_OK;
}

/* forget the index (the tables were freed or will be rebuilt) */
void kbh_unitig_reset(void) { ut_reset(); }
