/*
 * binning_gpu.c -- host C shim: the reference's process_read / prune_data
 * surface (binning.c:902, 1130) over the libkbin.so C-ABI (include/kbin.h).
 *
 * process_read() only copies the read into a staging batch (the hot work runs
 * on the GPU in prune_data); prune_data() flushes, runs kb_finalize and
 * materialises the surviving (mmer, kmer) entries into the caller's level-1
 * table as reference-layout ZHashTable / ll_node structures.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE /* RTLD_DEFAULT */
#endif
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#if defined(__GLIBC__)
#include <malloc.h> /* mallopt (heap_pad_begin) */
#endif
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
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
/* multi-GPU (kbh_configure_gpus, else KBH_GPUS in the environment: a count
 * "8" or a device list "0,1,2,3"): one kb_group over these devices */
#define KBH_MAX_GPUS 64
static int g_ngpus = 0, g_gpus[KBH_MAX_GPUS], g_gpus_set = 0;
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

/* one engine context (or multi-GPU group) per level-1 table the caller uses */
typedef struct {
    struct ZHashTable *table;
    kb_ctx *ctx;
    kb_group *grp;          /* G > 1: the reads stay here until prune_data */
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

void kbh_get_config(int *K, int *M, int *cutoff)
{
    if (K) *K = g_K;
    if (M) *M = g_M;
    if (cutoff) *cutoff = g_cutoff;
}

int kbh_configure_gpus(int n_gpus, const int *devices)
{
    if (n_gpus < 1 || n_gpus > KBH_MAX_GPUS) return KB_EINVAL;
    g_ngpus = n_gpus;
    for (int i = 0; i < n_gpus; i++) g_gpus[i] = devices ? devices[i] : i;
    g_gpus_set = 1;
    return KB_OK;
}

/* KBH_GPUS: "<count>" (devices 0 .. count-1) or "<d0>,<d1>,..." (a device may
 * repeat: virtual shards on one GPU) */
static void gpus_from_env(void)
{
    const char *e = getenv("KBH_GPUS");
    if (g_gpus_set || !e || !*e) return;
    g_gpus_set = 1;
    if (!strchr(e, ',')) {
        const int n = atoi(e);
        if (n > 1 && n <= KBH_MAX_GPUS) {
            g_ngpus = n;
            for (int i = 0; i < n; i++) g_gpus[i] = i;
        }
        return;
    }
    int n = 0;
    for (const char *q = e; *q && n < KBH_MAX_GPUS;) {
        g_gpus[n++] = atoi(q);
        q = strchr(q, ',');
        if (!q) break;
        q++;
    }
    g_ngpus = n;
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
    gpus_from_env();
    if (g_ngpus > 1) {
        if (kb_group_create(&p, g_ngpus, g_gpus, &free_slot->grp) != KB_OK) die("kb_group_create");
    } else if (kb_create(&p, &free_slot->ctx) != KB_OK) {
        die("kb_create");
    }
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
    /* (a group splits the reads into contiguous per-GPU ranges at prune_data) */
    if (!b->grp && (b->n >= KBH_BATCH_READS || b->nbytes >= KBH_BATCH_BYTES)) flush(b);
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
    const char *env = getenv("KBH_THREADS");
    if (env && atol(env) > 0) nt = atol(env);
    if (nt < 1) nt = 1;
    return nt > 16 ? 16 : nt;
}

/* The tables and lists are ~10^8-10^9 small malloc blocks built by several
 * threads: grow the arenas in 64 MB steps rather than 128 KB ones (each
 * growth is a syscall under the process's address-space lock, which the
 * other workers' page faults also take), then put glibc's default pad back.
 * Side effect (glibc): any M_TOP_PAD call also switches off the dynamic
 * mmap threshold for the rest of the process, so later large blocks
 * (>= 128 KiB) are always mmapped -- allocation speed only, never results.
 * KBH_NO_TOP_PAD=1 leaves malloc's tuning untouched. */
static void heap_pad_begin(void)
{
#if defined(__GLIBC__) && defined(M_TOP_PAD)
    if (!getenv("KBH_NO_TOP_PAD")) mallopt(M_TOP_PAD, 64 << 20);
#endif
}

static void heap_pad_end(void)
{
#if defined(__GLIBC__) && defined(M_TOP_PAD)
    if (!getenv("KBH_NO_TOP_PAD")) mallopt(M_TOP_PAD, 128 << 10);
#endif
}

/* Transparent huge pages for the arenas the worker threads fill: a glibc
 * thread arena is a 64 MiB-aligned 64 MiB mapping (HEAP_MAX_SIZE), so the
 * first block a thread gets in a new one names it; madvise(MADV_HUGEPAGE)
 * on it is a paging hint only (512x fewer page faults while ~10^9 small
 * blocks are written, and a faster unmap at exit).  KBH_NO_THP=1: off. */
#define ARENA_SPAN ((uintptr_t)64 << 20)
static void thp_hint(const void *p, uintptr_t *last)
{
#if defined(__linux__) && defined(MADV_HUGEPAGE)
    const uintptr_t base = (uintptr_t)p & ~(ARENA_SPAN - 1);
    if (base != *last) {
        *last = base;
        static int off = -1;
        if (off < 0) off = getenv("KBH_NO_THP") != NULL;
        if (!off) (void)madvise((void *)base, ARENA_SPAN, MADV_HUGEPAGE);
    }
#else
    (void)p;
    (void)last;
#endif
}

/* List-node arena.  The drop-in's ~10^9-10^10 list nodes (the prune's
 * materialised lists, create_node_num; expand_read_id_list's copies,
 * duplicate_llist) are 16-B blocks that glibc rounds up to 32-B chunks, one
 * locked-arena malloc each.  When this file's free() is the process's free
 * (the drop-in executable links it: a strong definition in the executable
 * interposes libc's for every library), nodes are instead bumped out of
 * per-thread 64 MiB chunks of one reserved mapping (huge-page hinted, 16 B
 * per node), and free() of a pointer inside it is a no-op -- the reference's
 * own frees of nodes (free_llist, merge_lists: llist.c:101-108,
 * binning.c:174-181) stay valid, the memory returns at exit.  Every other
 * pointer goes to the free() this one shadows (RTLD_NEXT: a preloaded
 * allocator's, else glibc's).  Loaded any other way (a ctypes
 * library, RTLD_LOCAL) the process's free is libc's, the arena stays off and
 * nodes are malloc'd.  KBH_NODE_ARENA=0: off. */
#define NODE_ARENA_RESERVE ((uint64_t)512 << 30)
#define NODE_ARENA_CHUNK ((uint64_t)64 << 20)
static char *volatile g_node_base; /* set once, before any node exists */
static uint64_t g_node_next;
static pthread_once_t g_node_once = PTHREAD_ONCE_INIT;
extern void __libc_free(void *);

/* the free() this one shadows: the next definition in lookup order (an
 * LD_PRELOADed allocator's, else glibc's), resolved once; until then, and if
 * the lookup fails, glibc's own */
static void (*volatile g_next_free)(void *);
static int g_next_state; /* 0 unresolved, 1 resolving, 2 done */

static void node_free(void *p)
{
    char *const b = g_node_base;
    if (b && (char *)p >= b && (char *)p < b + NODE_ARENA_RESERVE) return;
    void (*f)(void *) = g_next_free;
    if (!f) {
        int expect = 0;
        if (__atomic_compare_exchange_n(&g_next_state, &expect, 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
            void *(*const d)(void *, const char *) = dlsym; /* (may free: those go to glibc meanwhile) */
            void (*nf)(void *) = (void (*)(void *))d(RTLD_NEXT, "free");
            g_next_free = nf ? nf : __libc_free;
            __atomic_store_n(&g_next_state, 2, __ATOMIC_RELEASE);
        }
        f = g_next_free ? g_next_free : __libc_free;
    }
    f(p);
}
void free(void *p) __attribute__((alias("node_free")));

/* resolve the shadowed free at load time, before the program can start threads
 * (a free() racing the lazy lookup went to glibc even when an
 * LD_PRELOADed allocator owns the pointer); frees inside dlsym itself, during
 * this single-threaded load, still take the fallback */
__attribute__((constructor)) static void node_free_resolve(void)
{
    int expect = 0;
    if (!__atomic_compare_exchange_n(&g_next_state, &expect, 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return;
    void *(*const d)(void *, const char *) = dlsym;
    void (*nf)(void *) = (void (*)(void *))d(RTLD_NEXT, "free");
    g_next_free = nf ? nf : __libc_free;
    __atomic_store_n(&g_next_state, 2, __ATOMIC_RELEASE);
}

static void node_arena_init(void)
{
#if defined(__linux__)
    const char *e = getenv("KBH_NODE_ARENA");
    if (e && *e == '0') return;
    void *(*const d)(void *, const char *) = dlsym;
    if ((void *)d(RTLD_DEFAULT, "free") != (void *)node_free) return; /* not the process's free */
    void *m = mmap(NULL, NODE_ARENA_RESERVE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                   -1, 0);
    if (m == MAP_FAILED) return;
#if defined(MADV_HUGEPAGE)
    if (!getenv("KBH_NO_THP")) (void)madvise(m, NODE_ARENA_RESERVE, MADV_HUGEPAGE);
#endif
    g_node_base = m;
#endif
}

int kbh_node_arena_active(void)
{
    pthread_once(&g_node_once, node_arena_init);
    return g_node_base != NULL;
}

typedef struct {
    char *cur, *end;
    uintptr_t thp; /* (the malloc path's huge-page hint) */
} node_alloc_t;

static inline ll_node *node_new(node_alloc_t *a)
{
    if (a->cur == a->end) {
        pthread_once(&g_node_once, node_arena_init);
        const uint64_t off = g_node_base ? __atomic_fetch_add(&g_node_next, NODE_ARENA_CHUNK, __ATOMIC_RELAXED)
                                         : NODE_ARENA_RESERVE;
        if (off + NODE_ARENA_CHUNK > NODE_ARENA_RESERVE) { /* no arena (or it is spent): malloc */
            ll_node *nd = xmalloc(sizeof *nd);
            thp_hint(nd, &a->thp);
            return nd;
        }
        a->cur = g_node_base + off;
        a->end = a->cur + NODE_ARENA_CHUNK;
    }
    ll_node *nd = (ll_node *)a->cur;
    a->cur += sizeof(ll_node);
    return nd;
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

/* REPLAY: rebuild the reference's two-level table from the CSR by calling
 * zhash_set in the reference's insertion order -- level 1 (mmer -> level-2
 * table) in the order the reference creates its entries (the first occurrence
 * of any key of that mmer), then every level-2 table as above.  Used when the
 * caller's table already holds entries, and by the tests as the check on the
 * direct layout below (kbh_materialise_csr). */
static void materialise_replay(struct ZHashTable *level1, const kb_csr *r, int prune)
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


/* DIRECT layout (the default): the final shape of every table -- size step,
 * bucket chains and their order -- is a function of the keys' insertion order
 * alone, so it is computed on integer codes and only the SURVIVING entries are
 * allocated and linked; no strings are hashed, no table is ever rehashed in
 * memory and pruned keys cost no allocation.
 *
 *   bucket (zhash.c:171-182): h = fold (17 h + c) mod m over the key's chars,
 *     i.e. the key's base-17 value P mod m; P is split into 15-char chunks
 *     (each < 2^64 for chars <= 'T'), h = sum_t (chunk_t mod m)(17^15t mod m)
 *     mod m;
 *   zhash_set (zhash.c:53-76): push on the chain head; after the insert, if
 *     entry_count > m / 2 rehash to the next ladder step;
 *   zhash_rehash (zhash.c:184-214): walk the old buckets 0..m-1, each chain
 *     head to tail, pushing every entry onto the head of its new chain;
 *   the prune (binning.c:1085-1144) unlinks entries through iterators, which
 *     never resize: survivors keep their relative chain order, a level-2
 *     table left empty is dropped from level 1, and level 1 keeps the size of
 *     its full history.
 * Each table's history is replayed on int32 chains (the ladder steps it
 * passes through), then its final chains are walked once to allocate and link
 * the survivors.  Tables are independent: worker threads take them largest
 * first. */
#define CHUNK_CHARS 15
#define MAX_CHUNKS 5 /* K <= 63 */
#define LADDER_TOP 23

static uint64_t g_pw[LADDER_TOP][MAX_CHUNKS]; /* 17^(15 t) mod m_s */

static void init_powers(void)
{
    for (int s = 0; s < LADDER_TOP; s++) {
        const uint64_t m = LADDER[s];
        uint64_t p15 = 1;
        for (int i = 0; i < CHUNK_CHARS; i++) p15 = p15 * 17 % m;
        uint64_t p = 1 % m;
        for (int t = 0; t < MAX_CHUNKS; t++) {
            g_pw[s][t] = p;
            p = p * p15 % m;
        }
    }
}

/* base-17 chunks of the key string for the 2-bit code (char j of the string
 * is code bits 2(n-1-j)); chunk t holds powers 17^(15t .. 15t+14) */
static int key_chunks(uint64_t hi, uint64_t lo, int n, uint64_t *ch)
{
    const int nc = (n + CHUNK_CHARS - 1) / CHUNK_CHARS;
    for (int t = 0; t < nc; t++) ch[t] = 0;
    for (int p = n - 1; p >= 0; p--) { /* p = power of 17 = distance from the end */
        const unsigned c2 = p >= 32 ? (unsigned)(hi >> (2 * (p - 32))) & 3u : (unsigned)(lo >> (2 * p)) & 3u;
        uint64_t *a = &ch[p / CHUNK_CHARS];
        *a = *a * 17 + (unsigned char)BP[c2];
    }
    return nc;
}

static inline uint32_t bucket_at(const uint64_t *ch, int nc, int s)
{
    const uint64_t m = LADDER[s];
    uint64_t h = 0;
    for (int t = 0; t < nc; t++) h += (ch[t] % m) * g_pw[s][t];
    return (uint32_t)(h % m);
}

static int final_step(uint64_t n)
{
    int s = 0;
    for (uint64_t c = 1; c <= n; c++)
        if (c > LADDER[s] / 2 && s + 1 < LADDER_TOP) s++;
    return s;
}

/* per-thread scratch of the replay */
typedef struct {
    uint64_t *ch;   /* [n * nc] key chunks */
    int32_t *next;  /* [n] chain links */
    int32_t *head, *nhead;
    uint64_t cap_n, cap_m;
} replay_buf;

static void replay_reserve(replay_buf *b, uint64_t n, int nc, uint64_t m)
{
    if (n > b->cap_n) {
        free(b->ch);
        free(b->next);
        b->cap_n = n + n / 2;
        b->ch = xmalloc(b->cap_n * MAX_CHUNKS * sizeof(uint64_t));
        b->next = xmalloc(b->cap_n * sizeof(int32_t));
    }
    if (m > b->cap_m) {
        free(b->head);
        free(b->nhead);
        b->cap_m = m;
        b->head = xmalloc(m * sizeof(int32_t));
        b->nhead = xmalloc((m + 1) * sizeof(int32_t));
    }
    (void)nc;
}

/* Replays n inserts (key i's chunks at ch + i*nc); returns the final step and
 * leaves the final chains in b->head[0..m) / b->next (-1 terminated). */
static int replay(replay_buf *b, uint64_t n, int nc)
{
    int s = 0;
    uint64_t m = LADDER[0];
    memset(b->head, 0xFF, m * sizeof(int32_t));
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t h = bucket_at(b->ch + i * nc, nc, s);
        b->next[i] = b->head[h];
        b->head[h] = (int32_t)i;
        if (i + 1 > m / 2 && s + 1 < LADDER_TOP) {
            const uint64_t nm = LADDER[s + 1];
            memset(b->nhead, 0xFF, nm * sizeof(int32_t));
            for (uint64_t bk = 0; bk < m; bk++) {
                for (int32_t j = b->head[bk]; j >= 0;) {
                    const int32_t nx = b->next[j];
                    const uint32_t h2 = bucket_at(b->ch + (uint64_t)j * nc, nc, s + 1);
                    b->next[j] = b->nhead[h2];
                    b->nhead[h2] = j;
                    j = nx;
                }
            }
            int32_t *t = b->head;
            b->head = b->nhead;
            b->nhead = t;
            s++;
            m = nm;
        }
    }
    return s;
}

static struct ZHashTable *new_table(int s, uint64_t count)
{
    struct ZHashTable *t = xmalloc(sizeof *t);
    t->size_index = (size_t)s;
    t->entry_count = count;
    t->entries = calloc(LADDER[s], sizeof(struct ZHashEntry *));
    if (!t->entries) exit(EXIT_FAILURE);
    return t;
}

static struct ZHashEntry *new_entry(const char *key, size_t klen, void *val)
{
    struct ZHashEntry *e = xmalloc(sizeof *e);
    e->key = xmalloc(klen + 1);
    memcpy(e->key, key, klen + 1);
    e->val = val;
    e->next = NULL;
    return e;
}

/* an entry as the replay and the linking need it, gathered once by the
 * grouping scatter (sequential reads of the CSR): insertion stamp, list start
 * with the survivor flag in bit 63, list length, k-mer code */
typedef struct {
    uint64_t first, o0, len, lo, hi;
} key_rec;
#define REC_ALIVE (1ull << 63)

typedef struct {
    const kb_csr *r;
    key_rec *grouped;         /* entries grouped by mmer */
    const uint64_t *gstart;   /* [nm + 1] */
    const uint32_t *work;     /* mmers, largest group first */
    struct ZHashTable **l2;   /* [nm] out: level-2 table (NULL: none survives) */
    uint64_t *gfirst;         /* [nm] out: first sight of the mmer */
    uint64_t n_work, next, nodes, kept;
} direct_job;

/* in-place sort of a group by insertion stamp (stamps are distinct) */
static void sort_recs(key_rec *a, int64_t n)
{
    while (n > 24) {
        const uint64_t x = a[0].first, y = a[n / 2].first, z = a[n - 1].first;
        const uint64_t piv = x < y ? (y < z ? y : (x < z ? z : x)) : (x < z ? x : (y < z ? z : y));
        int64_t i = 0, k = n - 1;
        for (;;) {
            while (a[i].first < piv) i++;
            while (a[k].first > piv) k--;
            if (i >= k) break;
            const key_rec t = a[i];
            a[i++] = a[k];
            a[k--] = t;
        }
        /* [0, k] <= piv <= [k + 1, n): recurse on the smaller side */
        if (k + 1 < n - k - 1) {
            sort_recs(a, k + 1);
            a += k + 1;
            n -= k + 1;
        } else {
            sort_recs(a + k + 1, n - k - 1);
            n = k + 1;
        }
    }
    for (int64_t i = 1; i < n; i++) {
        const key_rec t = a[i];
        int64_t k = i;
        for (; k > 0 && a[k - 1].first > t.first; k--) a[k] = a[k - 1];
        a[k] = t;
    }
}

static void *direct_tables(void *arg)
{
    direct_job *j = arg;
    const kb_csr *r = j->r;
    const int nc = (g_K + CHUNK_CHARS - 1) / CHUNK_CHARS;
    replay_buf b = {0};
    uint64_t nodes = 0, kept = 0;
    node_alloc_t na = {0, 0, 0};
    char ks[129];
    for (;;) {
        const uint64_t w = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (w >= j->n_work) break;
        const uint32_t mm = j->work[w];
        const uint64_t g0 = j->gstart[mm], n = j->gstart[mm + 1] - g0;
        key_rec *fk = j->grouped + g0;
        uint64_t alive = 0;
        for (uint64_t i = 0; i < n; i++) alive += fk[i].o0 >> 63;
        sort_recs(fk, (int64_t)n); /* insertion order */
        j->gfirst[mm] = fk[0].first;
        if (!alive) continue; /* the prune drops the whole table */
        replay_reserve(&b, n, nc, LADDER[final_step(n)]);
        for (uint64_t i = 0; i < n; i++) key_chunks(fk[i].hi, fk[i].lo, g_K, b.ch + i * nc);
        const int s = replay(&b, n, nc);
        struct ZHashTable *t = new_table(s, alive);
        /* survivors in chain order, per bucket (in the scratch the replay
         * no longer needs: the chunks and the spare head array) */
        int32_t *ord = (int32_t *)b.ch, q = 0;
        uint32_t *bstart = (uint32_t *)b.nhead;
        for (uint64_t bk = 0; bk < LADDER[s]; bk++) {
            bstart[bk] = (uint32_t)q;
            for (int32_t i = b.head[bk]; i >= 0; i = b.next[i])
                if (fk[i].o0 & REC_ALIVE) ord[q++] = i;
        }
        bstart[LADDER[s]] = (uint32_t)q;
        for (uint64_t bk = 0; bk < LADDER[s]; bk++) {
            struct ZHashEntry **tail = &t->entries[bk];
            for (uint32_t p = bstart[bk]; p < bstart[bk + 1]; p++) {
                const key_rec *kr = &fk[ord[p]];
                if (p + 4 < (uint32_t)q) __builtin_prefetch(&r->ids[fk[ord[p + 4]].o0 & ~REC_ALIVE]);
                const uint64_t o0 = kr->o0 & ~REC_ALIVE, o1 = o0 + kr->len;
                ll_node *head = NULL, **lt = &head;
                for (uint64_t k = o0; k < o1; k++) {
                    ll_node *nd = node_new(&na); /* create_node_num, llist.c:6-11 */
                    nd->next = NULL;
                    nd->read_id = r->ids[k];
                    *lt = nd;
                    lt = &nd->next;
                }
                nodes += o1 - o0;
                code_to_str(kr->hi, kr->lo, g_K, ks);
                *tail = new_entry(ks, (size_t)g_K, head);
                tail = &(*tail)->next;
            }
        }
        kept += alive;
        j->l2[mm] = t;
    }
    free(b.ch);
    free(b.next);
    free(b.head);
    free(b.nhead);
    __atomic_fetch_add(&j->nodes, nodes, __ATOMIC_RELAXED);
    __atomic_fetch_add(&j->kept, kept, __ATOMIC_RELAXED);
    return NULL;
}

typedef struct {
    const kb_csr *r;
    uint64_t lo, hi;
    uint64_t *cnt; /* [nm] this slice's histogram, then its scatter cursors */
    key_rec *grouped;
    int prune;
} group_slice;

static void *slice_count(void *arg)
{
    group_slice *g = arg;
    for (uint64_t e = g->lo; e < g->hi; e++) g->cnt[g->r->mmer[e]]++;
    return NULL;
}

/* survivor test of the prune (binning.c:1093-1102: fewer than cutoff + 1
 * list nodes) */
static void *slice_scatter(void *arg)
{
    group_slice *g = arg;
    const kb_csr *r = g->r;
    for (uint64_t e = g->lo; e < g->hi; e++) {
        key_rec *k = &g->grouped[g->cnt[r->mmer[e]]++];
        const int alive = !g->prune ||
                          ((int)r->count[e] > g_cutoff && (int64_t)(r->offset[e + 1] - r->offset[e]) > g_cutoff);
        k->first = r->first ? r->first[e] : e;
        k->o0 = r->offset[e] | (alive ? REC_ALIVE : 0);
        k->len = r->offset[e + 1] - r->offset[e];
        k->lo = r->kmer_lo[e];
        k->hi = r->kmer_hi[e];
    }
    return NULL;
}

static void run_slices(void *(*fn)(void *), group_slice *sl, long nt)
{
    pthread_t th[16];
    int started[16] = {0};
    for (long t = 1; t < nt; t++) started[t] = pthread_create(&th[t], NULL, fn, &sl[t]) == 0;
    fn(&sl[0]);
    for (long t = 1; t < nt; t++)
        if (started[t]) pthread_join(th[t], NULL);
        else fn(&sl[t]);
}

static const uint64_t *g_sort_first; /* level-1 order: qsort has no context argument */
static int cmp_mmer_first(const void *a, const void *b)
{
    const uint64_t x = g_sort_first[*(const uint32_t *)a], y = g_sort_first[*(const uint32_t *)b];
    return x < y ? -1 : x > y;
}

static const uint64_t *g_sort_size;
static int cmp_mmer_size(const void *a, const void *b)
{
    const uint64_t x = g_sort_size[*(const uint32_t *)a], y = g_sort_size[*(const uint32_t *)b];
    return x > y ? -1 : x < y;
}

static void materialise_direct(struct ZHashTable *level1, const kb_csr *r, int prune)
{
    static pthread_once_t once = PTHREAD_ONCE_INIT;
    pthread_once(&once, init_powers);
    const uint64_t n = r->n_entries;
    const uint32_t nm = 1u << (2 * g_M);
    const long nt = n_threads();
    double t = now_ms();
    /* 1. entries grouped by mmer: per-slice histograms, then a stable scatter */
    group_slice sl[16];
    key_rec *grouped = xmalloc((n ? n : 1) * sizeof(key_rec));
    uint64_t *gstart = calloc((size_t)nm + 1, sizeof(uint64_t));
    if (!gstart) exit(EXIT_FAILURE);
    for (long s = 0; s < nt; s++) {
        sl[s].r = r;
        sl[s].lo = n * (uint64_t)s / (uint64_t)nt;
        sl[s].hi = n * (uint64_t)(s + 1) / (uint64_t)nt;
        sl[s].cnt = calloc(nm, sizeof(uint64_t));
        if (!sl[s].cnt) exit(EXIT_FAILURE);
        sl[s].grouped = grouped;
        sl[s].prune = prune;
    }
    run_slices(slice_count, sl, nt);
    uint64_t run = 0;
    for (uint32_t m = 0; m < nm; m++) {
        gstart[m] = run;
        for (long s = 0; s < nt; s++) {
            const uint64_t c = sl[s].cnt[m];
            sl[s].cnt[m] = run;
            run += c;
        }
    }
    gstart[nm] = run;
    run_slices(slice_scatter, sl, nt);
    for (long s = 0; s < nt; s++) free(sl[s].cnt);
    uint32_t *work = xmalloc(nm * sizeof(uint32_t)), nw = 0;
    uint64_t *gsize = xmalloc(nm * sizeof(uint64_t));
    for (uint32_t m = 0; m < nm; m++) {
        gsize[m] = gstart[m + 1] - gstart[m];
        if (gsize[m]) work[nw++] = m;
    }
    g_sort_size = gsize;
    qsort(work, nw, sizeof(uint32_t), cmp_mmer_size);
    g_times.order_ms = now_ms() - t;
    /* 2. level-2 tables (worker threads) */
    t = now_ms();
    direct_job j = {r, grouped, gstart, work, calloc(nm, sizeof(struct ZHashTable *)),
                    xmalloc(nm * sizeof(uint64_t)), nw, 0, 0, 0};
    if (!j.l2) exit(EXIT_FAILURE);
    heap_pad_begin();
    run_workers(direct_tables, &j, nt);
    heap_pad_end();
    g_times.fill_ms = now_ms() - t;
    g_times.nodes += j.nodes;
    /* 3. level 1: every mmer in first-sight order, survivors linked */
    t = now_ms();
    g_sort_first = j.gfirst;
    qsort(work, nw, sizeof(uint32_t), cmp_mmer_first);
    replay_buf b = {0};
    replay_reserve(&b, nw ? nw : 1, 1, LADDER[final_step(nw)]);
    for (uint32_t i = 0; i < nw; i++) key_chunks(0, work[i], g_M, b.ch + i);
    const int s1 = replay(&b, nw, 1);
    uint64_t kept1 = 0;
    for (uint32_t i = 0; i < nw; i++) kept1 += j.l2[work[i]] != NULL;
    free(level1->entries);
    level1->size_index = (size_t)s1;
    level1->entry_count = kept1;
    level1->entries = calloc(LADDER[s1], sizeof(struct ZHashEntry *));
    if (!level1->entries) exit(EXIT_FAILURE);
    char ms[17];
    for (uint64_t bk = 0; bk < LADDER[s1]; bk++) {
        struct ZHashEntry **tail = &level1->entries[bk];
        for (int32_t i = b.head[bk]; i >= 0; i = b.next[i]) {
            struct ZHashTable *l2 = j.l2[work[i]];
            if (!l2) continue;
            code_to_str(0, work[i], g_M, ms);
            *tail = new_entry(ms, (size_t)g_M, l2);
            tail = &(*tail)->next;
        }
    }
    free(b.ch);
    free(b.next);
    free(b.head);
    free(b.nhead);
    g_times.group_ms = now_ms() - t;
    free(j.l2);
    free(j.gfirst);
    free(work);
    free(gsize);
    free(gstart);
    free(grouped);
}

/* direct layout for a fresh table (the reference path: prune_data on the
 * table process_read filled), replay otherwise */
static int materialise(struct ZHashTable *level1, const kb_csr *r, int prune)
{
    if (level1->entry_count == 0 && level1->size_index == 0 && g_M <= CHUNK_CHARS && getenv("KBH_REPLAY") == NULL) {
        materialise_direct(level1, r, prune);
        return 1; /* already pruned */
    }
    materialise_replay(level1, r, prune);
    return 0;
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

/* ---- the rest of the reference's calling surface (north_star: the host keeps
 * the getbp/getval 2-bit encoding and the prune API), for a host that links
 * only libkbin_host + libkbin.  Weak: in the drop-in the reference's own
 * binning.o defines the same symbols, and its strong ones win. */

/* binning.c:69-88: 0..3 -> T, G, C, A; anything else -> 'A' */
__attribute__((weak)) char getbp(int bp) { return bp >= 0 && bp < 4 ? BP[bp] : 'A'; }

/* binning.c:91-111: T, G, C, A -> 0..3; any other byte -> 3 (as 'A') */
__attribute__((weak)) int getval(char c)
{
    switch (c) {
    case 'T': return 0;
    case 'G': return 1;
    case 'C': return 2;
    default: return 3;
    }
}

/* binning.c:114-124: the base-4 value, first character most significant
 * (int arithmetic; long strings wrap as the reference's -O2 build does) */
__attribute__((weak)) int getscore(char *string)
{
    unsigned score = 0;
    for (; *string != '\0'; string++) score = score * 4u + (unsigned)getval(*string);
    return (int)score;
}

/* binning.c:1085-1123 on one level-2 (kmer) table: every entry whose id list
 * holds <= ABUNDANCE_CUTOFF (kbh_configure's cutoff) nodes is unlinked and
 * freed, the table is never resized (the reference's iterator deletes in
 * place), and an emptied table is freed and NULL returned.  (The reference
 * frees only a pruned list's head node, :1106; the whole list is freed here.) */
__attribute__((weak)) struct ZHashTable *prune_kmers(struct ZHashTable *hash_table)
{
    prune_level2(hash_table, g_cutoff);
    if (hash_table->entry_count == 0) {
        free(hash_table->entries);
        free(hash_table);
        return NULL;
    }
    return hash_table;
}

/* Multi-GPU: the reads of the whole loop, cut into G contiguous ranges (rank
 * g's reads all precede rank g+1's, so arrival order at every receiver is the
 * call order), each submitted with its call ORDINALS as ids -- lists then come
 * out in reverse call order whatever ids the caller used, and first
 * occurrences carry call ordinals as on one GPU.  After the group's exchange
 * and binning, the G disjoint results are concatenated into one host CSR and
 * ordinals mapped back to the caller's ids. */
typedef struct {
    uint32_t *mmer, *count;
    uint64_t *hi, *lo, *offset, *first;
    int32_t *ids;
} merged_csr;

static void group_finish(binding_t *b, kb_csr *r, merged_csr *m)
{
    int G = 0, nl = 0;
    if (kb_group_info(b->grp, &G, &nl, NULL, NULL) != KB_OK) die("kb_group_info");
    uint64_t byte0 = 0, r0 = 0;
    int32_t *ord = xmalloc((b->n ? b->n : 1) * sizeof(int32_t));
    for (uint64_t i = 0; i < b->n; i++) ord[i] = (int32_t)i;
    for (int g = 0; g < nl; g++) {
        const uint64_t r1 = b->n * (uint64_t)(g + 1) / (uint64_t)nl;
        uint64_t nb = 0;
        for (uint64_t i = r0; i < r1; i++) nb += b->lens[i];
        if (r1 > r0 && kb_group_submit_ids(b->grp, g, b->bases + byte0, b->lens + r0, r1 - r0, ord + r0) != KB_OK)
            die("kb_group_submit_ids");
        byte0 += nb;
        r0 = r1;
    }
    /* every key, pruned ones included, takes part in the insertion history */
    if (kb_group_finalize(b->grp, 0) != KB_OK) die("kb_group_finalize");
    free(ord);
    kb_csr part[KBH_MAX_GPUS];
    uint64_t ne = 0, ni = 0, nk = 0, nd = 0;
    for (int g = 0; g < nl; g++) {
        if (kb_export(kb_group_ctx(b->grp, g), &part[g]) != KB_OK) die("kb_export");
        ne += part[g].n_entries;
        ni += part[g].n_ids;
        nk += part[g].n_kmers;
        nd += part[g].n_distinct;
    }
    m->mmer = xmalloc((ne + 1) * sizeof(uint32_t));
    m->count = xmalloc((ne + 1) * sizeof(uint32_t));
    m->hi = xmalloc((ne + 1) * sizeof(uint64_t));
    m->lo = xmalloc((ne + 1) * sizeof(uint64_t));
    m->first = xmalloc((ne + 1) * sizeof(uint64_t));
    m->offset = xmalloc((ne + 1) * sizeof(uint64_t));
    m->ids = xmalloc((ni + 1) * sizeof(int32_t));
    uint64_t e0 = 0, i0 = 0;
    for (int g = 0; g < nl; g++) {
        const kb_csr *q = &part[g];
        const uint64_t n = q->n_entries;
        memcpy(m->mmer + e0, q->mmer, n * sizeof(uint32_t));
        memcpy(m->count + e0, q->count, n * sizeof(uint32_t));
        memcpy(m->hi + e0, q->kmer_hi, n * sizeof(uint64_t));
        memcpy(m->lo + e0, q->kmer_lo, n * sizeof(uint64_t));
        if (q->first) memcpy(m->first + e0, q->first, n * sizeof(uint64_t));
        else die("group result without first occurrences");
        for (uint64_t e = 0; e < n; e++) m->offset[e0 + e] = i0 + q->offset[e];
        for (uint64_t k = 0; k < q->n_ids; k++) m->ids[i0 + k] = b->ids[q->ids[k]]; /* ordinal -> caller id */
        e0 += n;
        i0 += q->n_ids;
    }
    m->offset[ne] = ni;
    memset(r, 0, sizeof *r);
    r->n_entries = ne;
    r->n_ids = ni;
    r->n_kmers = nk;
    r->n_distinct = nd;
    r->mmer = m->mmer;
    r->kmer_hi = m->hi;
    r->kmer_lo = m->lo;
    r->count = m->count;
    r->offset = m->offset;
    r->ids = m->ids;
    r->first = m->first;
}

static struct ZHashTable *finish(struct ZHashTable *hash_table, int prune)
{
    binding_t *b = binding(hash_table, 1);
    memset(&g_times, 0, sizeof g_times);
    double t = now_ms(), t0 = t;
    kb_csr r;
    merged_csr m = {0};
    if (b->grp) {
        group_finish(b, &r, &m);
        g_times.finalize_ms = now_ms() - t;
    } else {
        flush(b);
        /* every key, pruned ones included, takes part in the insertion history */
        if (kb_finalize(b->ctx, 0) != KB_OK) die("kb_finalize");
        g_times.finalize_ms = now_ms() - t;
        t = now_ms();
        if (kb_export(b->ctx, &r) != KB_OK) die("kb_export");
    }
    g_times.export_ms = now_ms() - t;
    g_times.entries = r.n_entries;
    g_times.ids = r.n_ids;
    t = now_ms();
    const int done = materialise(hash_table, &r, prune);
    g_times.materialise_ms = now_ms() - t;
    t = now_ms();
    if (prune && !done) prune_materialised(hash_table, g_cutoff);
    g_times.prune_ms = now_ms() - t;
    t = now_ms();
    kbh_release(hash_table);
    free(m.mmer);
    free(m.count);
    free(m.hi);
    free(m.lo);
    free(m.first);
    free(m.offset);
    free(m.ids);
    g_times.release_ms = now_ms() - t;
    g_times.total_ms = now_ms() - t0;
    if (getenv("KBH_TRACE")) /* (the drop-in binaries: no caller reads kbh_last_times) */
        fprintf(stderr,
                "{\"prune_data_ms\": %.3f, \"finalize_ms\": %.3f, \"export_ms\": %.3f, \"materialise_ms\": %.3f, "
                "\"release_ms\": %.3f, \"entries\": %llu, \"ids\": %llu, \"nodes\": %llu}\n",
                g_times.total_ms, g_times.finalize_ms, g_times.export_ms, g_times.materialise_ms,
                g_times.release_ms, (unsigned long long)g_times.entries, (unsigned long long)g_times.ids,
                (unsigned long long)g_times.nodes);
    return hash_table;
}

int kbh_materialise_csr(struct ZHashTable *hash_table, const kb_csr *r, int prune, int replay_only)
{
    if (!hash_table || !r) return KB_EINVAL;
    memset(&g_times, 0, sizeof g_times);
    int done;
    if (replay_only) {
        materialise_replay(hash_table, r, prune);
        done = 0;
    } else {
        done = materialise(hash_table, r, prune);
    }
    if (prune && !done) prune_materialised(hash_table, g_cutoff);
    return KB_OK;
}

static uint64_t mix64(uint64_t x)
{
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

static uint64_t str_hash(const char *s)
{
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (; *s; s++) h = mix64(h ^ (unsigned char)*s);
    return h;
}

uint64_t kbh_layout_digest(struct ZHashTable *level1)
{
    uint64_t h = mix64(level1->size_index * 1000003u + level1->entry_count);
    const size_t m1 = LADDER[level1->size_index];
    for (size_t b1 = 0; b1 < m1; b1++) {
        for (struct ZHashEntry *me = level1->entries[b1]; me; me = me->next) {
            struct ZHashTable *level2 = me->val;
            h = mix64(h ^ b1 ^ str_hash(me->key));
            h = mix64(h ^ (level2->size_index << 40) ^ level2->entry_count);
            const size_t m2 = LADDER[level2->size_index];
            for (size_t b2 = 0; b2 < m2; b2++) {
                for (struct ZHashEntry *ke = level2->entries[b2]; ke; ke = ke->next) {
                    h = mix64(h ^ (b2 << 1) ^ str_hash(ke->key));
                    for (ll_node *t = ke->val; t; t = t->next) h = mix64(h ^ (uint32_t)t->read_id);
                    h = mix64(h + 1);
                }
            }
        }
    }
    return h;
}

/* binning.c:1130 */
struct ZHashTable *prune_data(struct ZHashTable *hash_table) { return finish(hash_table, 1); }

/* expand_read_id_list (binning.c:857-888): every kmer entry's id list becomes
 * a list of strlen(key) list nodes (create_node_item, llist.c:13-18) whose
 * items are the original list followed by strlen(key) - 1 fresh copies of it
 * (duplicate_llist, llist.c:83-99).  The result depends on each entry alone,
 * so the level-2 tables are expanded by worker threads, largest first.  Every
 * node stays an individual malloc block, as the reference's are: downstream
 * reference code frees and relinks them (merge_lists / free_llist at
 * binning.c:174-181, llist.c:101-108).  The reference walks the tables with
 * its static-cursor iterators (binning.c:298-460) to the end, which leaves
 * them reset; this walk does not touch them. */
typedef struct {
    struct ZHashTable **tabs;
    uint64_t n, next, nodes;
} expand_job;

static void *expand_tables(void *arg)
{
    expand_job *j = arg;
    uint64_t nodes = 0;
    int *ids = NULL;
    size_t cap = 0;
    node_alloc_t na = {0, 0, 0};
    for (;;) {
        const uint64_t w = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (w >= j->n) break;
        struct ZHashTable *level2 = j->tabs[w];
        const size_t m2 = LADDER[level2->size_index];
        for (size_t b2 = 0; b2 < m2; b2++) {
            for (struct ZHashEntry *ke = level2->entries[b2]; ke; ke = ke->next) {
                ll_node *const list = ke->val;
                const size_t klen = strlen(ke->key);
                /* the list's ids once, then every copy from them */
                size_t n = 0;
                for (const ll_node *s = list; s; s = s->next) {
                    if (n == cap) {
                        cap = cap ? 2 * cap : 1024;
                        ids = realloc(ids, cap * sizeof(int));
                        if (!ids) exit(EXIT_FAILURE);
                    }
                    ids[n++] = s->read_id;
                }
                ll_node *outer = NULL, **ot = &outer;
                for (size_t i = 0; i < klen; i++) {
                    ll_node *copy = list;
                    if (i) { /* duplicate_llist */
                        ll_node **ct = &copy;
                        for (size_t q = 0; q < n; q++) {
                            ll_node *nd = node_new(&na);
                            nd->next = NULL;
                            nd->read_id = ids[q];
                            *ct = nd;
                            ct = &nd->next;
                        }
                        nodes += n;
                        *ct = NULL;
                    }
                    ll_node *o = node_new(&na); /* create_node_item */
                    o->next = NULL;
                    o->item = copy;
                    *ot = o;
                    ot = &o->next;
                    nodes++;
                }
                if (klen) ke->val = outer; /* (an empty key: the reference reads an unset pointer) */
            }
        }
    }
    free(ids);
    __atomic_fetch_add(&j->nodes, nodes, __ATOMIC_RELAXED);
    return NULL;
}

static int cmp_table_size(const void *a, const void *b)
{
    const size_t x = (*(struct ZHashTable *const *)a)->entry_count, y = (*(struct ZHashTable *const *)b)->entry_count;
    return x > y ? -1 : x < y;
}

/* KBH_TRACE: when exit() starts (after the caller's main has returned), so a
 * parent can split the drop-in's tail into printing and process teardown */
static void trace_exit(void) { fprintf(stderr, "{\"t_exit_s\": %.6f}\n", now_ms() * 1e-3); }

void expand_read_id_list(struct ZHashTable *hashtable)
{
    static int traced = 0;
    if (getenv("KBH_TRACE") && !traced) traced = atexit(trace_exit) == 0;
    double t = now_ms();
    const size_t m1 = LADDER[hashtable->size_index];
    uint64_t nt2 = 0;
    for (size_t b1 = 0; b1 < m1; b1++)
        for (struct ZHashEntry *me = hashtable->entries[b1]; me; me = me->next) nt2 += me->val != NULL;
    expand_job j = {xmalloc((nt2 + 1) * sizeof(struct ZHashTable *)), 0, 0, 0};
    for (size_t b1 = 0; b1 < m1; b1++)
        for (struct ZHashEntry *me = hashtable->entries[b1]; me; me = me->next)
            if (me->val) j.tabs[j.n++] = me->val;
    qsort(j.tabs, j.n, sizeof(struct ZHashTable *), cmp_table_size);
    heap_pad_begin();
    run_workers(expand_tables, &j, n_threads());
    heap_pad_end();
    free(j.tabs);
    g_times.expand_ms = now_ms() - t;
    g_times.expand_nodes = j.nodes;
    if (getenv("KBH_TRACE")) /* (t_end_s: CLOCK_MONOTONIC, so a parent can time what follows) */
        fprintf(stderr, "{\"expand_ms\": %.3f, \"expand_nodes\": %llu, \"t_end_s\": %.6f}\n", g_times.expand_ms,
                (unsigned long long)j.nodes, now_ms() * 1e-3);
}

struct ZHashTable *kbh_finish_unpruned(struct ZHashTable *hash_table) { return finish(hash_table, 0); }

void kbh_release(struct ZHashTable *hash_table)
{
    binding_t *b = binding(hash_table, 0);
    if (!b) return;
    kb_destroy(b->ctx);
    kb_group_destroy(b->grp);
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
