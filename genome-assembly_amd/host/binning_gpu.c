/*
 * binning_gpu.c -- host C shim: the reference's process_read / prune_data
 * surface (binning.c:902, 1130) over the libkbin.so C-ABI (include/kbin.h).
 *
 * process_read() only copies the read into a staging batch (the hot work runs
 * on the GPU in prune_data); prune_data() flushes, runs kb_finalize and
 * materialises the surviving (mmer, kmer) entries into the caller's level-1
 * table as reference-layout ZHashTable / ll_node structures.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/binning_gpu.h"
#include "../../include/kbin.h"

#ifndef KMER_SIZE
#define KMER_SIZE 31        /* binning.c:11 */
#endif
#ifndef MMER_SIZE
#define MMER_SIZE 4         /* binning.c:10 */
#endif
#ifndef ABUNDANCE_CUTOFF
#define ABUNDANCE_CUTOFF 1  /* binning.c:12 */
#endif
/* batches small enough that kb_submit's asynchronous H2D + pack of one
 * batch overlaps the caller's read loop filling the next */
#ifndef KBH_BATCH_READS
#define KBH_BATCH_READS (1u << 16)
#endif
#ifndef KBH_BATCH_BYTES
#define KBH_BATCH_BYTES (16u << 20)
#endif

/* bucket counts of the level tables (zhash.c:13-17 ladder; the reference keeps
 * it file-static, so the walker carries its own copy) */
static const size_t LADDER[23] = {
    53, 101, 211, 503, 1553, 3407, 6803, 12503, 25013, 50261, 104729, 250007,
    500009, 1000003, 2000029, 4000037, 10000019, 25000009, 50000047, 104395301,
    217645177, 512927357, 1000000007};

static int g_K = KMER_SIZE, g_M = MMER_SIZE, g_cutoff = ABUNDANCE_CUTOFF, g_device = 0;
static kbh_times g_times;

static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

int kbh_last_times(kbh_times *out)
{
    if (!out) return KB_EINVAL;
    *out = g_times;
    return KB_OK;
}

/* one engine context per level-1 table the caller uses */
typedef struct {
    struct ZHashTable *table;
    kb_ctx *ctx;
    char *bases;
    uint32_t *lens;
    int32_t *ids;
    uint64_t n, nbytes, cap_reads, cap_bytes;
} binding_t;

#define MAX_BINDINGS 64
static binding_t g_bind[MAX_BINDINGS];

static void die(const char *what)
{
    fprintf(stderr, "kbin: %s: %s\n", what, kb_last_error());
    exit(EXIT_FAILURE); /* zhash.c:236/247 convention */
}

static void *xmalloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p) exit(EXIT_FAILURE);
    return p;
}

int kbh_configure(int K, int M, int cutoff, int device)
{
    g_K = K;
    g_M = M;
    g_cutoff = cutoff;
    g_device = device;
    return 0;
}

static binding_t *binding(struct ZHashTable *t, int create)
{
    binding_t *free_slot = NULL;
    for (int i = 0; i < MAX_BINDINGS; i++) {
        if (g_bind[i].table == t) return &g_bind[i];
        if (!g_bind[i].table && !free_slot) free_slot = &g_bind[i];
    }
    if (!create) return NULL;
    if (!free_slot) {
        fprintf(stderr, "kbin: more than %d live tables\n", MAX_BINDINGS);
        exit(EXIT_FAILURE);
    }
    kb_params p;
    memset(&p, 0, sizeof p);
    p.K = g_K;
    p.M = g_M;
    p.cutoff = g_cutoff;
    p.max_read_len = 65535;
    p.device = g_device;
    p.flags = KB_TRACK_FIRST;
    if (kb_create(&p, &free_slot->ctx) != KB_OK) die("kb_create");
    free_slot->table = t;
    free_slot->cap_reads = 4096;
    free_slot->cap_bytes = 1 << 20;
    free_slot->bases = xmalloc(free_slot->cap_bytes);
    free_slot->lens = xmalloc(free_slot->cap_reads * sizeof(uint32_t));
    free_slot->ids = xmalloc(free_slot->cap_reads * sizeof(int32_t));
    free_slot->n = free_slot->nbytes = 0;
    return free_slot;
}

static void flush(binding_t *b)
{
    if (!b->n) return;
    if (kb_submit_ids(b->ctx, b->bases, b->lens, b->n, b->ids) != KB_OK) die("kb_submit_ids");
    b->n = b->nbytes = 0;
}

/* binning.c:902 */
struct ZHashTable *process_read(struct ZHashTable *hash_table, char *read, int read_id)
{
    binding_t *b = binding(hash_table, 1);
    size_t len = strlen(read); /* binning.c:904 */
    if (b->n == b->cap_reads) {
        b->cap_reads *= 2;
        b->lens = realloc(b->lens, b->cap_reads * sizeof(uint32_t));
        b->ids = realloc(b->ids, b->cap_reads * sizeof(int32_t));
        if (!b->lens || !b->ids) exit(EXIT_FAILURE);
    }
    if (b->nbytes + len > b->cap_bytes) {
        while (b->nbytes + len > b->cap_bytes) b->cap_bytes *= 2;
        b->bases = realloc(b->bases, b->cap_bytes);
        if (!b->bases) exit(EXIT_FAILURE);
    }
    memcpy(b->bases + b->nbytes, read, len); /* `read` is borrowed for this call only */
    b->nbytes += len;
    b->lens[b->n] = (uint32_t)len;
    b->ids[b->n] = read_id;
    b->n++;
    if (b->n >= KBH_BATCH_READS || b->nbytes >= KBH_BATCH_BYTES) flush(b);
    return hash_table; /* binning.c:1075 */
}

static const char BP[4] = {'T', 'G', 'C', 'A'}; /* getbp, binning.c:69-88 */

static void code_to_str(uint64_t hi, uint64_t lo, int n, char *s)
{
    for (int j = n - 1; j >= 0; j--) {
        s[j] = BP[lo & 3u];
        lo = (lo >> 2) | (hi << 62);
        hi >>= 2;
    }
    s[n] = '\0';
}

/* the entries in first-occurrence order: LSD radix sort of the 48-bit
 * (call ordinal << 16 | position) keys, 16-bit digits, stable */
static uint64_t *first_order(const kb_csr *r)
{
    const uint64_t n = r->n_entries;
    uint64_t *idx = xmalloc(n * sizeof(uint64_t)), *tmp = xmalloc(n * sizeof(uint64_t));
    uint64_t *cnt = xmalloc(65537 * sizeof(uint64_t));
    for (uint64_t e = 0; e < n; e++) idx[e] = e;
    if (r->first) {
        for (int sh = 0; sh < 48; sh += 16) {
            memset(cnt, 0, 65537 * sizeof(uint64_t));
            for (uint64_t e = 0; e < n; e++) cnt[((r->first[idx[e]] >> sh) & 0xFFFF) + 1]++;
            for (int d = 0; d < 65536; d++) cnt[d + 1] += cnt[d];
            for (uint64_t e = 0; e < n; e++) tmp[cnt[(r->first[idx[e]] >> sh) & 0xFFFF]++] = idx[e];
            uint64_t *t = idx;
            idx = tmp;
            tmp = t;
        }
    }
    free(tmp);
    free(cnt);
    return idx;
}

static long n_threads(void)
{
    long nt = sysconf(_SC_NPROCESSORS_ONLN);
    if (nt < 1) nt = 1;
    return nt > 16 ? 16 : nt;
}

/* run fn(arg) on up to 16 threads (the caller is one of them) */
static void run_workers(void *(*fn)(void *), void *arg, long nt)
{
    pthread_t th[16];
    int started[16] = {0};
    for (long t = 1; t < nt; t++) started[t] = pthread_create(&th[t], NULL, fn, arg) == 0;
    fn(arg);
    for (long t = 1; t < nt; t++)
        if (started[t]) pthread_join(th[t], NULL);
}

/* One level-2 table per mmer, filled by several threads (the tables are
 * independent: zhash.c keeps no mutable global state).  A table's keys go in
 * first-occurrence order -- binning.c:1045-1057 inserts a key at its first
 * occurrence -- so its bucket chains, size and rehash history are the
 * reference's.  Values are the id lists as plain malloc'd ll_node chains
 * (list order = stored order, reverse call order), so downstream reference
 * code may free() or relink them (llist.c:59-64, binning.c:174-181).  With
 * `skip`, entries the prune is about to delete (count <= cutoff,
 * binning.c:1102) get no list: their keys still enter the table, so the
 * insertion history is exact, and prune_materialised then unlinks them. */
typedef struct {
    const kb_csr *r;
    const uint64_t *grouped;     /* entries grouped by mmer, each group in first-occurrence order */
    const uint64_t *gstart;      /* [n_groups + 1] */
    const uint32_t *gmmer;       /* mmer of each group */
    struct ZHashTable **l2;      /* level-2 table per mmer code */
    uint64_t n_groups, next;     /* next: the group counter (atomic) */
    uint64_t nodes;              /* (atomic) */
    int skip;
} fill_job;

static void *fill_tables(void *arg)
{
    fill_job *j = arg;
    char ks[129];
    uint64_t nodes = 0;
    for (;;) {
        const uint64_t g = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (g >= j->n_groups) break;
        struct ZHashTable *level2 = j->l2[j->gmmer[g]];
        for (uint64_t o = j->gstart[g]; o < j->gstart[g + 1]; o++) {
            const uint64_t e = j->grouped[o];
            ll_node *head = NULL, **tail = &head;
            if (!(j->skip && (int)j->r->count[e] <= g_cutoff)) {
                for (uint64_t k = j->r->offset[e]; k < j->r->offset[e + 1]; k++) {
                    *tail = create_node_num(j->r->ids[k]);
                    tail = &(*tail)->next;
                }
                nodes += j->r->count[e];
            }
            code_to_str(j->r->kmer_hi[e], j->r->kmer_lo[e], g_K, ks);
            zhash_set(level2, ks, head);
        }
    }
    __atomic_fetch_add(&j->nodes, nodes, __ATOMIC_RELAXED);
    return NULL;
}

/* Rebuild the reference's two-level table from the CSR: level 1 (mmer ->
 * level-2 table) in the order the reference creates its entries (the first
 * occurrence of any key of that mmer), then every level-2 table as above. */
static void materialise(struct ZHashTable *level1, const kb_csr *r, int prune)
{
    char ms[17];
    const uint64_t n = r->n_entries;
    const size_t nm = (size_t)1 << (2 * g_M);
    double t = now_ms();
    uint64_t *order = first_order(r);
    g_times.order_ms = now_ms() - t;
    t = now_ms();
    /* stable grouping by mmer, groups in first-sight order */
    uint32_t *gid = malloc(nm * sizeof(uint32_t));
    struct ZHashTable **l2 = calloc(nm, sizeof(struct ZHashTable *));
    if (!gid || !l2) exit(EXIT_FAILURE);
    memset(gid, 0xFF, nm * sizeof(uint32_t));
    uint64_t ng = 0;
    uint32_t *gmmer = xmalloc((n ? n : 1) * sizeof(uint32_t));
    uint64_t *gcnt = xmalloc((n + 1) * sizeof(uint64_t));
    for (uint64_t o = 0; o < n; o++) {
        const uint32_t m = r->mmer[order[o]];
        if (gid[m] == 0xFFFFFFFFu) {
            gid[m] = (uint32_t)ng;
            gmmer[ng] = m;
            gcnt[ng++] = 0;
            code_to_str(0, m, g_M, ms);
            struct ZHashTable *level2 = zhash_get(level1, ms);
            if (!level2) {
                level2 = zcreate_hash_table();
                zhash_set(level1, ms, level2);
            }
            l2[m] = level2;
        }
        gcnt[gid[m]]++;
    }
    uint64_t *gstart = xmalloc((ng + 1) * sizeof(uint64_t)), *grouped = xmalloc((n ? n : 1) * sizeof(uint64_t));
    gstart[0] = 0;
    for (uint64_t g = 0; g < ng; g++) gstart[g + 1] = gstart[g] + gcnt[g];
    for (uint64_t g = 0; g < ng; g++) gcnt[g] = gstart[g];
    for (uint64_t o = 0; o < n; o++) grouped[gcnt[gid[r->mmer[order[o]]]]++] = order[o];
    fill_job j = {r, grouped, gstart, gmmer, l2, ng, 0, 0, prune};
    g_times.group_ms = now_ms() - t;
    t = now_ms();
    run_workers(fill_tables, &j, n_threads());
    g_times.fill_ms = now_ms() - t;
    g_times.nodes += j.nodes;
    free(grouped);
    free(gstart);
    free(gcnt);
    free(gmmer);
    free(gid);
    free(l2);
    free(order);
}

/* prune_kmers / prune_data semantics on the materialised table
 * (binning.c:1085-1144): unlink every entry whose list has <= cutoff nodes
 * without resizing (the reference deletes through its iterators, which never
 * rehash), then drop emptied level-2 tables and their level-1 entries.  The
 * level-2 tables are independent: several threads prune them; the level-1
 * walk stays sequential. */
typedef struct {
    struct ZHashTable **tabs;
    uint64_t n, next;
} prune_job;

static void prune_level2(struct ZHashTable *level2, int cutoff)
{
    const size_t m2 = LADDER[level2->size_index];
    for (size_t b2 = 0; b2 < m2; b2++) {
        struct ZHashEntry **l2 = &level2->entries[b2];
        while (*l2) {
            int cnt = 0;
            for (ll_node *t = (*l2)->val; t && cnt <= cutoff; t = t->next) cnt++;
            if (cnt <= cutoff) {
                struct ZHashEntry *dead = *l2;
                *l2 = dead->next;
                free_llist(dead->val);
                zfree_entry(dead, false);
                level2->entry_count--;
            } else {
                l2 = &(*l2)->next;
            }
        }
    }
}

static void *prune_tables(void *arg)
{
    prune_job *j = arg;
    for (;;) {
        const uint64_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n) break;
        prune_level2(j->tabs[i], g_cutoff);
    }
    return NULL;
}

static void prune_materialised(struct ZHashTable *level1, int cutoff)
{
    (void)cutoff;
    const size_t m1 = LADDER[level1->size_index];
    prune_job j = {xmalloc((level1->entry_count + 1) * sizeof(struct ZHashTable *)), 0, 0};
    for (size_t b1 = 0; b1 < m1; b1++)
        for (struct ZHashEntry *me = level1->entries[b1]; me; me = me->next) j.tabs[j.n++] = me->val;
    run_workers(prune_tables, &j, n_threads());
    free(j.tabs);
    for (size_t b1 = 0; b1 < m1; b1++) {
        struct ZHashEntry **l1 = &level1->entries[b1];
        while (*l1) {
            struct ZHashTable *level2 = (*l1)->val;
            if (level2->entry_count == 0) {
                struct ZHashEntry *dead = *l1;
                *l1 = dead->next;
                free(level2->entries);
                free(level2);
                zfree_entry(dead, false);
                level1->entry_count--;
            } else {
                l1 = &(*l1)->next;
            }
        }
    }
}

static struct ZHashTable *finish(struct ZHashTable *hash_table, int prune)
{
    binding_t *b = binding(hash_table, 1);
    memset(&g_times, 0, sizeof g_times);
    double t = now_ms(), t0 = t;
    flush(b);
    /* every key, pruned ones included, takes part in the insertion history */
    if (kb_finalize(b->ctx, 0) != KB_OK) die("kb_finalize");
    g_times.finalize_ms = now_ms() - t;
    t = now_ms();
    kb_csr r;
    if (kb_export(b->ctx, &r) != KB_OK) die("kb_export");
    g_times.export_ms = now_ms() - t;
    g_times.entries = r.n_entries;
    g_times.ids = r.n_ids;
    t = now_ms();
    materialise(hash_table, &r, prune);
    g_times.materialise_ms = now_ms() - t;
    t = now_ms();
    if (prune) prune_materialised(hash_table, g_cutoff);
    g_times.prune_ms = now_ms() - t;
    kbh_release(hash_table);
    g_times.total_ms = now_ms() - t0;
    return hash_table;
}

/* binning.c:1130 */
struct ZHashTable *prune_data(struct ZHashTable *hash_table) { return finish(hash_table, 1); }

struct ZHashTable *kbh_finish_unpruned(struct ZHashTable *hash_table) { return finish(hash_table, 0); }

void kbh_release(struct ZHashTable *hash_table)
{
    binding_t *b = binding(hash_table, 0);
    if (!b) return;
    kb_destroy(b->ctx);
    free(b->bases);
    free(b->lens);
    free(b->ids);
    memset(b, 0, sizeof *b);
}

/* binning.c:1150-1166 */
int kbh_read_fgets(const char *path, int read_length, char **bases_out, uint32_t **lens_out,
                   uint64_t *n_out)
{
    FILE *f = fopen(path, "r");
    if (!f || read_length < 2) {
        if (f) fclose(f);
        return KB_EINVAL;
    }
    char *buf = xmalloc((size_t)read_length + 1);
    uint64_t cap_b = 1 << 20, nb = 0, cap_r = 1 << 14, nr = 0;
    char *bases = xmalloc(cap_b);
    uint32_t *lens = xmalloc(cap_r * sizeof(uint32_t));
    while (fgets(buf, read_length, f) != NULL) {
        size_t len = strlen(buf);
        buf[--len] = '\0'; /* strips whatever the last byte is (binning.c:1162-1163) */
        if (nb + len > cap_b) {
            while (nb + len > cap_b) cap_b *= 2;
            bases = realloc(bases, cap_b);
            if (!bases) exit(EXIT_FAILURE);
        }
        if (nr == cap_r) {
            cap_r *= 2;
            lens = realloc(lens, cap_r * sizeof(uint32_t));
            if (!lens) exit(EXIT_FAILURE);
        }
        memcpy(bases + nb, buf, len);
        nb += len;
        lens[nr++] = (uint32_t)len;
    }
    fclose(f);
    free(buf);
    *bases_out = bases;
    *lens_out = lens;
    *n_out = nr;
    return KB_OK;
}

void kbh_free_reads(char *bases, uint32_t *lens)
{
    free(bases);
    free(lens);
}

static int cmp_line(const void *a, const void *b)
{
    return strcmp(*(char *const *)a, *(char *const *)b);
}

int kbh_dump_table(struct ZHashTable *level1, FILE *out)
{
    size_t cap = 1024, n = 0;
    char **lines = xmalloc(cap * sizeof(char *));
    const size_t m1 = LADDER[level1->size_index];
    for (size_t b1 = 0; b1 < m1; b1++) {
        for (struct ZHashEntry *me = level1->entries[b1]; me; me = me->next) {
            struct ZHashTable *level2 = me->val;
            const size_t m2 = LADDER[level2->size_index];
            for (size_t b2 = 0; b2 < m2; b2++) {
                for (struct ZHashEntry *ke = level2->entries[b2]; ke; ke = ke->next) {
                    size_t cnt = 0, sz = strlen(me->key) + strlen(ke->key) + 32;
                    for (ll_node *t = ke->val; t; t = t->next) { cnt++; sz += 12; }
                    char *ln = xmalloc(sz);
                    int w = snprintf(ln, sz, "%s\t%s\t%zu\t", me->key, ke->key, cnt);
                    for (ll_node *t = ke->val; t; t = t->next)
                        w += snprintf(ln + w, sz - (size_t)w, t->next ? "%d," : "%d", t->read_id);
                    if (n == cap) {
                        cap *= 2;
                        lines = realloc(lines, cap * sizeof(char *));
                        if (!lines) exit(EXIT_FAILURE);
                    }
                    lines[n++] = ln;
                }
            }
        }
    }
    qsort(lines, n, sizeof(char *), cmp_line);
    for (size_t i = 0; i < n; i++) {
        fputs(lines[i], out);
        fputc('\n', out);
        free(lines[i]);
    }
    free(lines);
    return 0;
}
