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
    uint32_t mmer;     /* mmer code */
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

/* process_read restated (binning.c:902-1076).  Emits one record per k-mer. */
static int scan_read(const char *read, int read_len, int K, int M, uint32_t ord,
                     const uint8_t *mmer_mask, recvec_t *out, uint64_t *n_kmers, int *alphabet_ok)
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

        /* binning.c:1023-1040: copy, then complement in place (no reversal) */
        memcpy(signature_cpy, signature, (size_t)M);
        memcpy(kmer_key, kmer, (size_t)K);
        signature_cpy[M] = '\0';
        kmer_key[K] = '\0';
        if (is_rev) {
            for (j = 0; j < M; j++) signature_cpy[j] = o_getbp(3 - o_getval(signature_cpy[j]));
            for (j = 0; j < K; j++) kmer_key[j] = o_getbp(3 - o_getval(kmer_key[j]));
        }

        rec_t r;
        uint64_t mh, ml;
        pack_code(signature_cpy, M, &mh, &ml);
        r.mmer = (uint32_t)ml;
        (*n_kmers)++;
        if (!mmer_mask || mmer_mask[r.mmer]) { /* test-side partition filter */
            pack_code(kmer_key, K, &r.hi, &r.lo);
            r.ord = ord;
            if (push(out, r)) return -1;
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
    int alphabet_ok = 1;
    uint64_t n_kmers = 0;
    for (uint64_t r = 0; r < n_reads; r++) {
        int len = (int)(read_off[r + 1] - read_off[r]);
        if (scan_read(bases + read_off[r], len, K, M, (uint32_t)r, mmer_mask, &v, &n_kmers, &alphabet_ok)) {
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
    if (!out->mmer || !out->kmer_hi || !out->kmer_lo || !out->count || !out->offset || !out->ids) {
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
            for (uint64_t k = a; k < b; k++)
                out->ids[p++] = read_ids ? read_ids[v.r[k].ord] : (int32_t)v.r[k].ord;
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
    free(r->count); free(r->offset); free(r->ids);
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
