/*
 * binning_gpu.c -- host C shim: the reference's process_read / prune_data
 * surface (binning.c:902, 1130) over the libkbin.so C-ABI (include/kbin.h).
 *
 * process_read() only copies the read into a staging batch (the hot work runs
 * on the GPU in prune_data); prune_data() flushes, runs kb_finalize and
 * materialises the surviving (mmer, kmer) entries into the caller's level-1
 * table as reference-layout ZHashTable / ll_node structures.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
#ifndef KBH_BATCH_READS
#define KBH_BATCH_READS (1u << 20)
#endif
#ifndef KBH_BATCH_BYTES
#define KBH_BATCH_BYTES (256u << 20)
#endif

/* bucket counts of the level tables (zhash.c:13-17 ladder; the reference keeps
 * it file-static, so the walker carries its own copy) */
static const size_t LADDER[23] = {
    53, 101, 211, 503, 1553, 3407, 6803, 12503, 25013, 50261, 104729, 250007,
    500009, 1000003, 2000029, 4000037, 10000019, 25000009, 50000047, 104395301,
    217645177, 512927357, 1000000007};

static int g_K = KMER_SIZE, g_M = MMER_SIZE, g_cutoff = ABUNDANCE_CUTOFF, g_device = 0;

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

static const uint64_t *g_first; /* qsort context */

static int cmp_first(const void *a, const void *b)
{
    const uint64_t x = g_first[*(const uint64_t *)a], y = g_first[*(const uint64_t *)b];
    return x < y ? -1 : x > y;
}

/* Rebuild the reference's two-level table from the CSR.  Keys are inserted in
 * the order the reference inserts them -- first occurrence (call ordinal,
 * k-mer position), binning.c:1045-1057 -- so bucket chains, table sizes and
 * rehash history come out identical; level-2 values are the id lists in
 * stored order (reverse call order). */
static void materialise(struct ZHashTable *level1, const kb_csr *r)
{
    char ms[17], ks[129];
    uint64_t *order = xmalloc(r->n_entries * sizeof(uint64_t));
    for (uint64_t e = 0; e < r->n_entries; e++) order[e] = e;
    if (r->first) {
        g_first = r->first;
        qsort(order, r->n_entries, sizeof(uint64_t), cmp_first);
    }
    for (uint64_t o = 0; o < r->n_entries; o++) {
        const uint64_t e = order[o];
        code_to_str(0, r->mmer[e], g_M, ms);
        code_to_str(r->kmer_hi[e], r->kmer_lo[e], g_K, ks);
        struct ZHashTable *level2 = zhash_get(level1, ms);
        if (!level2) {
            level2 = zcreate_hash_table();
            zhash_set(level1, ms, level2);
        }
        ll_node *head = NULL, **tail = &head;
        for (uint64_t k = r->offset[e]; k < r->offset[e + 1]; k++) {
            *tail = create_node_num(r->ids[k]);
            tail = &(*tail)->next;
        }
        zhash_set(level2, ks, head);
    }
    free(order);
}

/* prune_kmers / prune_data semantics on the materialised table
 * (binning.c:1085-1144): unlink every entry whose list has <= cutoff nodes
 * without resizing (the reference deletes through its iterators, which never
 * rehash), drop emptied level-2 tables and their level-1 entries. */
static void prune_materialised(struct ZHashTable *level1, int cutoff)
{
    const size_t m1 = LADDER[level1->size_index];
    for (size_t b1 = 0; b1 < m1; b1++) {
        struct ZHashEntry **l1 = &level1->entries[b1];
        while (*l1) {
            struct ZHashTable *level2 = (*l1)->val;
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
    flush(b);
    /* every key, pruned ones included, takes part in the insertion history */
    if (kb_finalize(b->ctx, 0) != KB_OK) die("kb_finalize");
    kb_csr r;
    if (kb_export(b->ctx, &r) != KB_OK) die("kb_export");
    materialise(hash_table, &r);
    if (prune) prune_materialised(hash_table, g_cutoff);
    kbh_release(hash_table);
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
