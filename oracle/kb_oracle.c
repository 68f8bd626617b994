/*
 * kb_oracle.c -- TEST INFRASTRUCTURE ONLY.  This is the parity oracle: a
 * clean-room CPU restatement of the reference hot path (twitu/genome-assembly
 * binning.c `process_read` + `prune_data`).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / the
 * CPU baseline -- the product (libkbin.so) never links or calls it.
 *
 * Parity pinning: the canonical dumps this file writes are checked against the
 * eight known-answer sha256 digests of SURVEY.md §8(c) (tests/golden/digests.json)
 * and against the compiled reference (oracle/_ref, built by build_ref.sh) on
 * seeded random inputs -- see tests/test_oracle.py.
 *
 * Algorithm, restated character by character:
 *   - base encoding getval/getbp: binning.c:69-111 (T0 G1 C2 A3, other -> 3 / 'A')
 *   - signature: binning.c:918-1021, including the "sticky" recompute rule
 *     (`kmer > signature`, binning.c:922) and the incremental branch that is
 *     dead for K >= 2M (loop bound at binning.c:997) -- restated verbatim so the
 *     oracle also matches the reference for K < 2M;
 *   - key build + complement (no reversal): binning.c:1023-1040;
 *   - two-level insert with list *prepend* (reverse call order, duplicates
 *     kept): binning.c:1042-1069.  The chained string hash (zhash.c) is only an
 *     associative container; its bucket order is not part of the contract, so
 *     the oracle groups equal keys by sorting records instead;
 *   - prune: keep an entry iff its list length > cutoff (binning.c:1085-1123);
 *     mmers left empty disappear with their entries (binning.c:1130-1144).
 *   - read loop: fgets(buf, READ_LENGTH) + unconditional strip of the last byte
 *     + read_id++ per chunk (binning.c:1150-1166) in kbo_read_fgets().
 *
 * Output order is the canonical dump order: bytewise (mmer, kmer) ascending.
 * With the reference digit order (A=3 > C=2 > G=1 > T=0) that is DESCENDING
 * numeric code order.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kb_oracle.h"

/* binning.c:17 */
static const int power_val[] = {1, 4, 16, 64, 256, 1024, 4096, 16384};

/* binning.c:69-88 */
static char o_getbp(int bp)
{
    switch (bp) {
    case 0: return 'T';
    case 1: return 'G';
    case 2: return 'C';
    case 3: return 'A';
    default: return 'A';
    }
}

/* binning.c:91-111 */
static int o_getval(char c)
{
    switch (c) {
    case 'T': return 0;
    case 'G': return 1;
    case 'C': return 2;
    case 'A': return 3;
    default: return 3;
    }
}

typedef struct {
    uint64_t hi, lo;   /* k-mer code, first base most significant */
    uint16_t mmer;     /* mmer code (M <= 8) */
    uint16_t pos;      /* k-mer position in the read (reads < 64 K bases) */
    uint32_t ord;      /* call ordinal of the read */
} rec_t;

typedef struct {
    rec_t *r;
    uint64_t n, cap;
} recvec_t;

static int push(recvec_t *v, rec_t x)
{
    if (v->n == v->cap) {
        uint64_t nc = v->cap ? v->cap * 2 : 1024;
        rec_t *p = realloc(v->r, nc * sizeof(rec_t));
        if (!p) return -1;
        v->r = p;
        v->cap = nc;
    }
    v->r[v->n++] = x;
    return 0;
}

/* 2-bit code of a key string, first char most significant (matches getscore,
 * binning.c:114-124, extended to 128 bits). */
static void pack_code(const char *s, int n, uint64_t *hi, uint64_t *lo)
{
    uint64_t h = 0, l = 0;
    for (int j = 0; j < n; j++) {
        h = (h << 2) | (l >> 62);
        l = (l << 2) | (uint64_t)o_getval(s[j]);
    }
    *hi = h;
    *lo = l;
}

/* where scan_read's records go: the record vector (kbo_bin), or a caller's
 * function (the streaming digest below) */
typedef struct sink {
    recvec_t *vec;
    int (*put)(struct sink *, const rec_t *);
} sink_t;

/* process_read restated (binning.c:902-1076).  Emits one record per k-mer. */
static int scan_read(const char *read, int read_len, int K, int M, uint32_t ord,
                     const uint8_t *mmer_mask, sink_t *out, uint64_t *n_kmers, int *alphabet_ok)
{
    const char *kmer = read;
    const char *signature = NULL; /* binning.c:906 */
    char kmer_key[129];
    char mmer[17];
    char signature_cpy[17];
    /* binning.c:913: int arithmetic; the dead branch (K < 2M) can overflow, the
     * reference's gcc build wraps -- emulate with uint32 and cast back. */
    int32_t score = 0, rev_score = 0, max_score = 0;
    int is_rev = 0;
    int msb = 0;
    int i, j;

    for (i = 0; i < read_len; i++) {
        char c = read[i];
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T') *alphabet_ok = 0;
    }

    for (i = 0; i < read_len - K + 1; i++) {                   /* binning.c:918 */
        if (kmer > signature) {                                /* binning.c:922 */
            score = 0; rev_score = 0; max_score = 0;           /* binning.c:926-928 */
            for (j = 0; j < M; j++) {                          /* binning.c:931-936 */
                mmer[j] = kmer[j];
                score = (int32_t)((uint32_t)score * 4u + (uint32_t)o_getval(kmer[j]));
                rev_score = (int32_t)((uint32_t)rev_score * 4u + 3u - (uint32_t)o_getval(kmer[j]));
            }
            mmer[M] = '\0';
            if (score > rev_score) { max_score = score; is_rev = 0; }   /* 940-949 */
            else { max_score = rev_score; is_rev = 1; }
            signature = kmer;
            msb = 0;
            j = M;
            while (j < K) {                                    /* binning.c:955-988 */
                score = (int32_t)(((uint32_t)score - (uint32_t)(o_getval(mmer[msb]) * power_val[M - 1])) * 4u);
                score = (int32_t)((uint32_t)score + (uint32_t)o_getval(kmer[j]));
                rev_score = (int32_t)(((uint32_t)rev_score - (uint32_t)((3 - o_getval(mmer[msb])) * power_val[M - 1])) * 4u);
                rev_score = (int32_t)((uint32_t)rev_score + 3u - (uint32_t)o_getval(kmer[j]));
                mmer[msb] = kmer[j];
                msb = (msb + 1) % M;
                j++;
                int32_t mx = score > rev_score ? score : rev_score;
                if (mx > max_score) {                          /* binning.c:972 (strict: leftmost wins) */
                    if (score > rev_score) { max_score = score; is_rev = 0; }
                    else { max_score = rev_score; is_rev = 1; }
                    signature = &kmer[j] - M;                  /* binning.c:986 */
                }
            }
        } else {
            /* binning.c:992-1021: runs zero iterations whenever K >= 2M */
            for (j = K - M; j < M; j++) {
                mmer[j] = kmer[j];
                score = (int32_t)((uint32_t)score * 4u + (uint32_t)o_getval(kmer[j]));
                rev_score = (int32_t)((uint32_t)rev_score * 4u + 3u - (uint32_t)o_getval(kmer[j]));
            }
            mmer[M] = '\0';
            int32_t mx = score > rev_score ? score : rev_score;
            if (mx > max_score) {
                if (score > rev_score) { max_score = score; is_rev = 0; }
                else { max_score = rev_score; is_rev = 1; }
                signature = &kmer[K - M];                      /* binning.c:1019 */
            }
        }

        /* binning.c:1023-1040: copy, then complement in place (no reversal);
         * (the test-side mmer filter looks at the signature before the k-mer
         * key is built: a filtered-out key's string is never needed) */
        memcpy(signature_cpy, signature, (size_t)M);
        signature_cpy[M] = '\0';
        if (is_rev)
            for (j = 0; j < M; j++) signature_cpy[j] = o_getbp(3 - o_getval(signature_cpy[j]));

        rec_t r;
        uint64_t mh, ml;
        pack_code(signature_cpy, M, &mh, &ml);
        r.mmer = (uint16_t)ml;
        r.pos = (uint16_t)i;
        (*n_kmers)++;
        if (!mmer_mask || mmer_mask[r.mmer]) { /* test-side partition filter */
            memcpy(kmer_key, kmer, (size_t)K);
            kmer_key[K] = '\0';
            if (is_rev)
                for (j = 0; j < K; j++) kmer_key[j] = o_getbp(3 - o_getval(kmer_key[j]));
            pack_code(kmer_key, K, &r.hi, &r.lo);
            r.ord = ord;
            if (out->put ? out->put(out, &r) : push(out->vec, r)) return -1;
        }
        kmer++;                                                /* binning.c:1072 */
    }
    return 0;
}

/* Canonical order: (mmer, kmer) descending codes == ascending strings; inside a
 * key the list is in reverse call order (prepend, binning.c:1065-1068). */
static int cmp_rec(const void *a, const void *b)
{
    const rec_t *x = a, *y = b;
    if (x->mmer != y->mmer) return x->mmer > y->mmer ? -1 : 1;
    if (x->hi != y->hi) return x->hi > y->hi ? -1 : 1;
    if (x->lo != y->lo) return x->lo > y->lo ? -1 : 1;
    if (x->ord != y->ord) return x->ord > y->ord ? -1 : 1;
    return 0;
}

int kbo_bin(const char *bases, const uint64_t *read_off, uint64_t n_reads,
            const int32_t *read_ids, int K, int M, int cutoff, int prune,
            kbo_result *out)
{
    return kbo_bin_masked(bases, read_off, n_reads, read_ids, K, M, cutoff, prune, NULL, out);
}

int kbo_bin_masked(const char *bases, const uint64_t *read_off, uint64_t n_reads,
                   const int32_t *read_ids, int K, int M, int cutoff, int prune,
                   const uint8_t *mmer_mask, kbo_result *out)
{
    memset(out, 0, sizeof(*out));
    if (K < 1 || K > 64 || M < 1 || M > 8 || M > K) return KBO_EINVAL;
    recvec_t v = {0};
    sink_t sk = {&v, NULL};
    int alphabet_ok = 1;
    uint64_t n_kmers = 0;
    for (uint64_t r = 0; r < n_reads; r++) {
        int len = (int)(read_off[r + 1] - read_off[r]);
        if (scan_read(bases + read_off[r], len, K, M, (uint32_t)r, mmer_mask, &sk, &n_kmers, &alphabet_ok)) {
            free(v.r);
            return KBO_ENOMEM;
        }
    }
    out->n_kmers = n_kmers;
    out->alphabet_ok = alphabet_ok;
    if (v.n) qsort(v.r, v.n, sizeof(rec_t), cmp_rec);

    /* group */
    uint64_t n_ent = 0, n_ids = 0;
    for (uint64_t a = 0; a < v.n;) {
        uint64_t b = a + 1;
        while (b < v.n && v.r[b].mmer == v.r[a].mmer && v.r[b].hi == v.r[a].hi &&
               v.r[b].lo == v.r[a].lo)
            b++;
        uint64_t c = b - a;
        if (!prune || c > (uint64_t)cutoff) { n_ent++; n_ids += c; }
        a = b;
    }
    out->n_entries = n_ent;
    out->mmer = malloc((n_ent ? n_ent : 1) * sizeof(uint32_t));
    out->kmer_hi = malloc((n_ent ? n_ent : 1) * sizeof(uint64_t));
    out->kmer_lo = malloc((n_ent ? n_ent : 1) * sizeof(uint64_t));
    out->count = malloc((n_ent ? n_ent : 1) * sizeof(uint32_t));
    out->offset = malloc((n_ent + 1) * sizeof(uint64_t));
    out->ids = malloc((n_ids ? n_ids : 1) * sizeof(int32_t));
    out->first = malloc((n_ent ? n_ent : 1) * sizeof(uint64_t));
    if (!out->mmer || !out->kmer_hi || !out->kmer_lo || !out->count || !out->offset || !out->ids || !out->first) {
        free(v.r);
        kbo_free(out);
        return KBO_ENOMEM;
    }
    uint64_t e = 0, p = 0;
    out->offset[0] = 0;
    for (uint64_t a = 0; a < v.n;) {
        uint64_t b = a + 1;
        while (b < v.n && v.r[b].mmer == v.r[a].mmer && v.r[b].hi == v.r[a].hi &&
               v.r[b].lo == v.r[a].lo)
            b++;
        uint64_t c = b - a;
        if (!prune || c > (uint64_t)cutoff) {
            out->mmer[e] = v.r[a].mmer;
            out->kmer_hi[e] = v.r[a].hi;
            out->kmer_lo[e] = v.r[a].lo;
            out->count[e] = (uint32_t)c;
            uint64_t first = UINT64_MAX; /* the key's first occurrence: the reference's insertion order */
            for (uint64_t k = a; k < b; k++) {
                out->ids[p++] = read_ids ? read_ids[v.r[k].ord] : (int32_t)v.r[k].ord;
                const uint64_t st = (uint64_t)v.r[k].ord << 16 | v.r[k].pos;
                if (st < first) first = st;
            }
            out->first[e] = first;
            e++;
            out->offset[e] = p;
        }
        a = b;
    }
    free(v.r);
    return KBO_OK;
}

void kbo_free(kbo_result *r)
{
    if (!r) return;
    free(r->mmer); free(r->kmer_hi); free(r->kmer_lo);
    free(r->count); free(r->offset); free(r->ids); free(r->first);
    memset(r, 0, sizeof(*r));
}

/* unpack a code into its key string (getbp, binning.c:69-88) */
static void unpack(uint64_t hi, uint64_t lo, int n, char *s)
{
    for (int j = n - 1; j >= 0; j--) {
        s[j] = o_getbp((int)(lo & 3));
        lo = (lo >> 2) | (hi << 62);
        hi >>= 2;
    }
    s[n] = '\0';
}

int kbo_write_dump(const kbo_result *r, int K, int M, const char *path)
{
    FILE *f = (path && strcmp(path, "-")) ? fopen(path, "w") : stdout;
    if (!f) return KBO_EIO;
    char ms[17], ks[129];
    for (uint64_t e = 0; e < r->n_entries; e++) {
        unpack(0, r->mmer[e], M, ms);
        unpack(r->kmer_hi[e], r->kmer_lo[e], K, ks);
        fprintf(f, "%s\t%s\t%u\t", ms, ks, r->count[e]);
        for (uint64_t k = r->offset[e]; k < r->offset[e + 1]; k++)
            fprintf(f, k + 1 < r->offset[e + 1] ? "%d," : "%d", r->ids[k]);
        fputc('\n', f);
    }
    if (f != stdout) fclose(f);
    return KBO_OK;
}

/* binning.c:1150-1166: fgets(buf, READ_LENGTH) chunking, strip of the last
 * byte (whatever it is), one id per chunk -- empty chunks included. */
int kbo_read_fgets(const char *path, int read_length, char **bases_out,
                   uint64_t **off_out, uint64_t *n_out)
{
    FILE *f = fopen(path, "r");
    if (!f) return KBO_EIO;
    char *buf = malloc((size_t)read_length + 1);
    uint64_t cap_b = 1 << 20, nb = 0, cap_r = 1 << 16, nr = 0;
    char *bases = malloc(cap_b);
    uint64_t *off = malloc(cap_r * sizeof(uint64_t));
    if (!buf || !bases || !off) { fclose(f); free(buf); free(bases); free(off); return KBO_ENOMEM; }
    off[0] = 0;
    while (fgets(buf, read_length, f) != NULL) {
        int len = (int)strlen(buf);
        buf[--len] = '\0';
        if (nb + (uint64_t)len > cap_b) {
            while (nb + (uint64_t)len > cap_b) cap_b *= 2;
            bases = realloc(bases, cap_b);
        }
        if (nr + 2 > cap_r) { cap_r *= 2; off = realloc(off, cap_r * sizeof(uint64_t)); }
        memcpy(bases + nb, buf, (size_t)len);
        nb += (uint64_t)len;
        off[++nr] = nb;
    }
    fclose(f);
    free(buf);
    *bases_out = bases;
    *off_out = off;
    *n_out = nr;
    return KBO_OK;
}

void kbo_free_reads(char *bases, uint64_t *off)
{
    free(bases);
    free(off);
}

/* ------------------------------------------------------------------------
 * The bench's synthetic reads on the CPU, and the kb_digest of a result too
 * large to hold (C3: 100 M reads, 12 G k-mer occurrences, 2 G ids), computed
 * by this oracle's own scan_read -- so the full-size digests bench.py asserts
 * come from the oracle, not from the GPU's history.
 * ------------------------------------------------------------------------ */

/* splitmix64 finaliser: the generator's and the digest's mixer (the product's
 * kbin_device.h mix64, restated) */
static uint64_t o_mix64(uint64_t x)
{
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

static uint64_t o_rng(uint64_t stream, uint64_t ctr)
{
    return o_mix64(stream * 0x9E3779B97F4A7C15ull + ctr + 0x632BE59BD9B4E019ull);
}

/* CPU twin of the device generator (kb_generate_reads_device_at; its kernel
 * mirrors generate_reads.py:93-112: an iid uniform genome of genome_len
 * bases, a uniform start per read, the forward strand, substitutions at
 * err_ppm per million bases, each to one of the three other bases) -- reads
 * read_base .. read_base + n_reads - 1 of the stream `seed` defines, as ASCII
 * (getbp: 0 T, 1 G, 2 C, 3 A), read_len bytes each.  A GPU test pins it
 * against the device on prefixes. */
void kbo_gen_reads(uint64_t n_reads, uint32_t L, uint64_t genome_len, uint32_t err_ppm, uint64_t seed,
                   uint64_t read_base, char *out)
{
    const uint64_t s_genome = o_mix64(seed ^ 0x1111111111111111ull);
    const uint64_t s_start = o_mix64(seed ^ 0x2222222222222222ull);
    const uint64_t s_err = o_mix64(seed ^ 0x3333333333333333ull);
    for (uint64_t r = 0; r < n_reads; r++) {
        const uint64_t rg = read_base + r;
        const uint64_t start = o_rng(s_start, rg) % (genome_len - L + 1);
        char *o = out + r * L;
        for (uint32_t b = 0; b < L; b++) {
            const uint64_t pos = start + b;
            uint32_t v = (uint32_t)(o_rng(s_genome, pos >> 5) >> (2 * (pos & 31))) & 3u;
            if (err_ppm) {
                const uint64_t u = o_rng(s_err, rg * (uint64_t)L + b);
                if ((uint32_t)(u % 1000000ull) < err_ppm) v = (v + 1u + (uint32_t)((u >> 32) % 3ull)) & 3u;
            }
            o[b] = o_getbp((int)v);
        }
    }
}

/* kb_digest's terms (kbin_digest.hip, kbin.result_digest): per kept key
 * mix64(key ^ count << 1); per list position j (1-based, the list in reverse
 * call order) mix64(key ^ (j << 32 | (uint32) id)); key = mix64(mix64(mix64(
 * mmer) ^ hi) ^ lo); sums mod 2^64 */
static uint64_t o_dkey(uint32_t mmer, uint64_t hi, uint64_t lo)
{
    return o_mix64(o_mix64(o_mix64((uint64_t)mmer) ^ hi) ^ lo);
}

/* one worker's keys: an open-addressed table of (mmer, hi, lo) -> count, then
 * (second pass) the list position left to hand out */
typedef struct {
    uint64_t *hi, *lo;
    uint32_t *mm;   /* mmer + 1 (0: empty slot) */
    uint32_t *cnt;
    uint64_t mask, n;
} dtab_t;

typedef struct {
    sink_t sk;      /* (first: scan_read's sink) */
    dtab_t t;
    int pass;       /* 1: count, 2: list terms */
    uint32_t cur_id;
    int cutoff, prune;
    uint64_t dl, ids, err;
} dwork_t;

static uint64_t *dslot(dtab_t *t, const rec_t *r, int insert, int *fresh)
{
    uint64_t h = o_dkey(r->mmer, r->hi, r->lo) & t->mask;
    for (;;) {
        if (t->mm[h] == 0) {
            if (!insert) return NULL;
            t->mm[h] = r->mmer + 1u;
            t->hi[h] = r->hi;
            t->lo[h] = r->lo;
            t->cnt[h] = 0;
            t->n++;
            *fresh = 1;
            return &t->hi[h];
        }
        if ((t->mm[h] & 0x7FFFFFFFu) == r->mmer + 1u && t->lo[h] == r->lo && t->hi[h] == r->hi) return &t->hi[h];
        h = (h + 1) & t->mask;
    }
}

static int dput(sink_t *s, const rec_t *r)
{
    dwork_t *w = (dwork_t *)s;
    int fresh = 0;
    uint64_t *p = dslot(&w->t, r, w->pass == 1, &fresh);
    if (!p) { w->err = 1; return -1; }
    const uint64_t h = (uint64_t)(p - w->t.hi);
    if (w->pass == 1) {
        if (w->t.n * 10 > (w->t.mask + 1) * 8) { w->err = 2; return -1; }  /* > 80 % full */
        w->t.cnt[h]++;
        return 0;
    }
    /* second pass: the occurrence's list position, counted down from the key's
     * count (call order t = 0 .. c - 1 sits at position c - t: prepend,
     * binning.c:1065-1068) */
    const uint32_t j = w->t.cnt[h]--;
    if (!w->prune || (w->t.mm[h] >> 31) == 0) {  /* (bit 31 of mm: a pruned key, set after pass 1) */
        w->dl += o_mix64(o_dkey(r->mmer, r->hi, r->lo) ^ (((uint64_t)j << 32) | w->cur_id));
        w->ids++;
    }
    return 0;
}

typedef struct {
    const char *reads;      /* n_reads x L ASCII, or NULL: */
    const uint64_t *packed; /* n_reads x ceil(L / 32) words, 2-bit codes first base high (the device layout) */
    uint64_t n_reads;
    uint32_t L;
    int K, M, cutoff, prune;
    int32_t id0;
    int nw, w;              /* worker w of nw: the mmers with owner(m) == w */
    uint64_t cap_log2;
    uint64_t out[5];        /* entries, ids, key sum, list sum, k-mers */
    int rc;
} djob_t;

static int owner_of(uint32_t m, int nw) { return (int)(o_mix64((uint64_t)m + 0x5bd1e995ull) % (uint64_t)nw); }

#include <pthread.h>
static void *dworker(void *arg)
{
    djob_t *jb = arg;
    const uint32_t nm = 1u << (2 * jb->M);
    uint8_t *mask = calloc(nm, 1);
    char *buf = malloc((size_t)jb->L + 1);
    dwork_t w;
    memset(&w, 0, sizeof w);
    w.sk.put = dput;
    w.cutoff = jb->cutoff;
    w.prune = jb->prune;
    const uint64_t cap = 1ull << jb->cap_log2;
    w.t.mask = cap - 1;
    w.t.hi = malloc(cap * 8);
    w.t.lo = malloc(cap * 8);
    w.t.mm = calloc(cap, 4);
    w.t.cnt = malloc(cap * 4);
    if (!mask || !buf || !w.t.hi || !w.t.lo || !w.t.mm || !w.t.cnt) { jb->rc = KBO_ENOMEM; goto done; }
    for (uint32_t m = 0; m < nm; m++) mask[m] = owner_of(m, jb->nw) == jb->w;
    for (w.pass = 1; w.pass <= 2; w.pass++) {
        uint64_t nk = 0;
        int aok = 1;
        const uint32_t RW = (jb->L + 31u) / 32u;
        for (uint64_t r = 0; r < jb->n_reads; r++) {
            w.cur_id = (uint32_t)(jb->id0 + (int32_t)r);
            const char *rd = jb->reads ? jb->reads + r * jb->L : buf;
            if (!jb->reads)
                for (uint32_t b = 0; b < jb->L; b++)
                    buf[b] = o_getbp((int)((jb->packed[r * RW + b / 32u] >> (62u - 2u * (b % 32u))) & 3u));
            if (scan_read(rd, (int)jb->L, jb->K, jb->M, (uint32_t)r, mask, &w.sk, &nk, &aok)) {
                jb->rc = w.err == 2 ? KBO_ENOMEM : KBO_EINVAL;
                goto done;
            }
        }
        jb->out[4] = nk;
        if (w.pass == 1) {  /* the kept keys' terms; pruned keys marked */
            uint64_t dk = 0, ent = 0;
            for (uint64_t h = 0; h < cap; h++) {
                if (!w.t.mm[h]) continue;
                const uint32_t c = w.t.cnt[h];
                if (jb->prune && c <= (uint32_t)jb->cutoff) { w.t.mm[h] |= 0x80000000u; continue; }
                dk += o_mix64(o_dkey(w.t.mm[h] - 1u, w.t.hi[h], w.t.lo[h]) ^ ((uint64_t)c << 1));
                ent++;
            }
            jb->out[0] = ent;
            jb->out[2] = dk;
        }
    }
    jb->out[1] = w.ids;
    jb->out[3] = w.dl;
done:
    free(mask);
    free(buf);
    free(w.t.hi); free(w.t.lo); free(w.t.mm); free(w.t.cnt);
    return NULL;
}

/* kb_digest of binning n_reads ASCII reads of length L (ids id0, id0 + 1, ...)
 * in one pass: entries, ids, key sum, list sum, and the k-mers scanned.
 * n_workers threads each own the mmers of one hash class (and scan every
 * read); a worker's table holds 2^cap_log2 keys at most 80 % full. */
static int stream_digest(const char *reads, const uint64_t *packed, uint64_t n_reads, uint32_t L, int K, int M,
                         int cutoff, int prune, int32_t id0, int n_workers, int cap_log2, uint64_t out[5])
{
    if (K < 1 || K > 64 || M < 1 || M > 8 || M > K || n_workers < 1 || n_workers > 256) return KBO_EINVAL;
    djob_t *jobs = calloc((size_t)n_workers, sizeof(djob_t));
    pthread_t *th = calloc((size_t)n_workers, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return KBO_ENOMEM; }
    for (int i = 0; i < n_workers; i++) {
        jobs[i] = (djob_t){reads, packed, n_reads, L, K, M, cutoff, prune, id0, n_workers, i, (uint64_t)cap_log2,
                           {0}, 0};
        pthread_create(&th[i], NULL, dworker, &jobs[i]);
    }
    int rc = KBO_OK;
    memset(out, 0, 5 * sizeof(uint64_t));
    for (int i = 0; i < n_workers; i++) {
        pthread_join(th[i], NULL);
        if (jobs[i].rc) rc = jobs[i].rc;
        for (int k = 0; k < 4; k++) out[k] += jobs[i].out[k];
        out[4] = jobs[i].out[4];
    }
    free(jobs);
    free(th);
    return rc;
}

int kbo_stream_digest(const char *reads, uint64_t n_reads, uint32_t L, int K, int M, int cutoff, int prune,
                      int32_t id0, int n_workers, int cap_log2, uint64_t out[5])
{
    return stream_digest(reads, NULL, n_reads, L, K, M, cutoff, prune, id0, n_workers, cap_log2, out);
}

/* the generator's reads packed 2-bit (first base high, the device layout) */
typedef struct {
    uint64_t *w;
    uint64_t r0, r1, read_base, genome_len, seed;
    uint32_t L, err_ppm;
} gjob_t;

static void *gworker(void *arg)
{
    gjob_t *g = arg;
    const uint32_t RW = (g->L + 31u) / 32u;
    char *buf = malloc(g->L);
    for (uint64_t r = g->r0; r < g->r1; r++) {
        kbo_gen_reads(1, g->L, g->genome_len, g->err_ppm, g->seed, g->read_base + r, buf);
        for (uint32_t k = 0; k < RW; k++) g->w[r * RW + k] = 0;
        for (uint32_t b = 0; b < g->L; b++)
            g->w[r * RW + b / 32u] |= (uint64_t)o_getval(buf[b]) << (62u - 2u * (b % 32u));
    }
    free(buf);
    return NULL;
}

/* kbo_stream_digest of the generator's reads read_base .. + n_reads - 1
 * (kbo_gen_reads), ids id0 + read index: the full-size C3 digest from the
 * oracle (tools/oracle_digest.py) */
int kbo_gen_stream_digest(uint64_t n_reads, uint32_t L, uint64_t genome_len, uint32_t err_ppm, uint64_t seed,
                          uint64_t read_base, int K, int M, int cutoff, int prune, int32_t id0, int n_workers,
                          int cap_log2, uint64_t out[5])
{
    const uint32_t RW = (L + 31u) / 32u;
    uint64_t *w = malloc(n_reads * RW * sizeof(uint64_t) + 8);
    gjob_t *g = calloc((size_t)n_workers, sizeof(gjob_t));
    pthread_t *th = calloc((size_t)n_workers, sizeof(pthread_t));
    if (!w || !g || !th) { free(w); free(g); free(th); return KBO_ENOMEM; }
    for (int i = 0; i < n_workers; i++) {
        g[i] = (gjob_t){w, n_reads * (uint64_t)i / (uint64_t)n_workers, n_reads * (uint64_t)(i + 1) / (uint64_t)n_workers,
                        read_base, genome_len, seed, L, err_ppm};
        pthread_create(&th[i], NULL, gworker, &g[i]);
    }
    for (int i = 0; i < n_workers; i++) pthread_join(th[i], NULL);
    free(g);
    free(th);
    const int rc = stream_digest(NULL, w, n_reads, L, K, M, cutoff, prune, id0, n_workers, cap_log2, out);
    free(w);
    return rc;
}

#ifdef KBO_MAIN
/* kb_oracle <reads-file> <K> <M> <READ_LENGTH> <cutoff> <prune 0|1>
 * prints the canonical (sorted) dump */
int main(int argc, char **argv)
{
    if (argc < 7) {
        fprintf(stderr, "usage: %s <reads> <K> <M> <READ_LENGTH> <cutoff> <prune>\n", argv[0]);
        return 2;
    }
    char *bases; uint64_t *off, n;
    if (kbo_read_fgets(argv[1], atoi(argv[4]), &bases, &off, &n)) { perror(argv[1]); return 2; }
    kbo_result r;
    int rc = kbo_bin(bases, off, n, NULL, atoi(argv[2]), atoi(argv[3]), atoi(argv[5]), atoi(argv[6]), &r);
    if (rc) { fprintf(stderr, "kbo_bin failed: %d\n", rc); return 1; }
    kbo_write_dump(&r, atoi(argv[2]), atoi(argv[3]), "-");
    kbo_free(&r);
    kbo_free_reads(bases, off);
    return 0;
}
#endif
