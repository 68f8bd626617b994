/* kb_oracle.h -- TEST INFRASTRUCTURE ONLY (parity oracle; see kb_oracle.c). */
#ifndef KB_ORACLE_H
#define KB_ORACLE_H
#include <stdint.h>

#define KBO_OK 0
#define KBO_EINVAL 1
#define KBO_ENOMEM 2
#define KBO_EIO 3

typedef struct {
    uint64_t n_entries;
    uint32_t *mmer;     /* mmer code per entry */
    uint64_t *kmer_hi;  /* k-mer code, high 64 bits (0 when K <= 32) */
    uint64_t *kmer_lo;  /* k-mer code, low 64 bits */
    uint32_t *count;    /* list length (occurrences, duplicates kept) */
    uint64_t *offset;   /* n_entries + 1 */
    int32_t *ids;       /* read ids per entry, reverse call order */
    uint64_t n_kmers;   /* k-mer occurrences scanned */
    int alphabet_ok;    /* 0 if any byte outside ACGT was seen */
    uint64_t *first;    /* per entry: first occurrence, call ordinal << 16 | k-mer
                           position (kbin.h KB_TRACK_FIRST's stamp) */
} kbo_result;

int kbo_bin(const char *bases, const uint64_t *read_off, uint64_t n_reads,
            const int32_t *read_ids, int K, int M, int cutoff, int prune,
            kbo_result *out);
/* kbo_bin restricted to the keys whose canonical mmer code m has
 * mmer_mask[m] != 0 (4^M bytes; NULL = all): checks one partition of a large
 * input without sorting the rest.  n_kmers still counts every k-mer. */
int kbo_bin_masked(const char *bases, const uint64_t *read_off, uint64_t n_reads,
                   const int32_t *read_ids, int K, int M, int cutoff, int prune,
                   const uint8_t *mmer_mask, kbo_result *out);
void kbo_free(kbo_result *r);
int kbo_write_dump(const kbo_result *r, int K, int M, const char *path);
int kbo_read_fgets(const char *path, int read_length, char **bases_out,
                   uint64_t **off_out, uint64_t *n_out);
void kbo_free_reads(char *bases, uint64_t *off);

/* the device generator's reads (kb_generate_reads_device_at) on the CPU:
 * n_reads x L ASCII bytes, reads read_base .. of the stream `seed` defines */
void kbo_gen_reads(uint64_t n_reads, uint32_t L, uint64_t genome_len, uint32_t err_ppm, uint64_t seed,
                   uint64_t read_base, char *out);
/* kb_digest (kbin.h) of binning reads too many to hold as a result, from this
 * oracle's scan: out = {entries, ids, key sum, list sum, k-mers}.  Reads are
 * n_reads x L ASCII with ids id0 + index; n_workers threads own the mmers of
 * one hash class each, each table 2^cap_log2 keys (<= 80 % full, else
 * KBO_ENOMEM). */
int kbo_stream_digest(const char *reads, uint64_t n_reads, uint32_t L, int K, int M, int cutoff, int prune,
                      int32_t id0, int n_workers, int cap_log2, uint64_t out[5]);
/* the same over kbo_gen_reads' reads, generated and held 2-bit packed */
int kbo_gen_stream_digest(uint64_t n_reads, uint32_t L, uint64_t genome_len, uint32_t err_ppm, uint64_t seed,
                          uint64_t read_base, int K, int M, int cutoff, int prune, int32_t id0, int n_workers,
                          int cap_log2, uint64_t out[5]);

#endif
