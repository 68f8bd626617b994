/*
 * binning_gpu.h -- the reference's host-side C surface, backed by libkbin.so.
 *
 * Drop-in replacements (identical signatures and argument meaning):
 *   struct ZHashTable *process_read(struct ZHashTable *, char *read, int read_id)
 *       binning.c:902.  Copies `read` (borrowed for the call only, as main
 *       reuses one stack buffer, binning.c:1154/1158) into a staging batch of
 *       the context bound to `hash_table`; full batches go to kb_submit_ids.
 *       Returns `hash_table` (binning.c:1075).
 *   struct ZHashTable *prune_data(struct ZHashTable *)
 *       binning.c:1130.  Flushes, runs the device scan/insert/prune
 *       (kb_finalize), and MATERIALISES the surviving entries into
 *       `hash_table` as real level-1 mmer -> level-2 kmer -> ll_node tables
 *       (zhash.h / llist.h layout), so downstream reference code
 *       (expand_read_id_list, find_kmer_extensions, print_kmers) runs
 *       unchanged.  Returns `hash_table` (the reference has no return,
 *       binning.c:1144).
 *   void expand_read_id_list(struct ZHashTable *)
 *       binning.c:857-888.  The same nodes the reference builds (an outer
 *       create_node_item list of strlen(key) nodes per kmer entry: the
 *       original id list, then duplicate_llist copies), every node its own
 *       malloc block, built by worker threads over the level-2 tables.
 *
 * Error convention: like the reference (zhash.c:236/247 exit on OOM), any
 * engine failure prints kb_last_error() to stderr and calls exit(EXIT_FAILURE).
 *
 * Configuration (the reference's compile-time #defines, binning.c:10-13):
 * build with -DKMER_SIZE=.. -DMMER_SIZE=.. -DABUNDANCE_CUTOFF=.. matching the
 * caller, or call kbh_configure() before the first process_read.
 */
#ifndef BINNING_GPU_H
#define BINNING_GPU_H

#include <stdint.h>
#include <stdio.h>

#include "kb_zhash.h"
#include "kbin.h"

#ifdef __cplusplus
extern "C" {
#endif

struct ZHashTable *process_read(struct ZHashTable *hash_table, char *read, int read_id);
struct ZHashTable *prune_data(struct ZHashTable *hash_table);
/* binning.c:857-888: every kmer's id list -> strlen(key) list nodes holding
 * the original list and strlen(key) - 1 malloc'd copies (worker threads) */
void expand_read_id_list(struct ZHashTable *hashtable);

/* The rest of binning.c's calling surface, same semantics, exported weak (a
 * drop-in that links the reference's binning.o keeps the reference's own):
 *   getbp     binning.c:69-88    0..3 -> 'T','G','C','A' (else 'A')
 *   getval    binning.c:91-111   'T','G','C','A' -> 0..3 (else 3)
 *   getscore  binning.c:114-124  base-4 value of a string, first char high
 *   prune_kmers binning.c:1085-1123  one level-2 table: entries with <=
 *             cutoff ids removed in place (no resize); NULL (table freed)
 *             when it empties -- prune_data runs it over every mmer */
char getbp(int bp);
int getval(char c);
int getscore(char *string);
struct ZHashTable *prune_kmers(struct ZHashTable *hash_table);

/* explicit configuration (else the compile-time defaults); device = HIP ordinal */
int kbh_configure(int K, int M, int cutoff, int device);

/* Several GPUs behind the same process_read / prune_data surface: the reads
 * are kept on the host until prune_data, cut into n_gpus contiguous ranges and
 * binned by one multi-GPU group (kb_group_create: mmer-sharded, records
 * exchanged over RCCL); the tables materialised are identical to one GPU's.
 * devices: NULL = 0 .. n_gpus-1 (a device may repeat: virtual shards).  The
 * unchanged reference program gets the same from KBH_GPUS in the
 * environment ("8", or "0,1,2,3"). */
int kbh_configure_gpus(int n_gpus, const int *devices);

/* like prune_data but without the prune (every key kept) */
struct ZHashTable *kbh_finish_unpruned(struct ZHashTable *hash_table);

/* wall-clock phases of the last prune_data / kbh_finish_unpruned */
typedef struct {
    double finalize_ms;     /* flush + kb_finalize (device binning, every key) */
    double export_ms;       /* kb_export: D2H of the CSR */
    double materialise_ms;  /* zhash / ll_node tables in first-occurrence order */
    double prune_ms;        /* prune_kmers semantics on the tables */
    double total_ms;
    uint64_t entries;       /* keys materialised (all, before the prune) */
    uint64_t ids;           /* ids exported */
    uint64_t nodes;         /* ll_nodes allocated (kept keys only when pruning) */
    double order_ms;        /* materialise: entries grouped by mmer (direct layout;
                               replay: first-occurrence radix sort) */
    double group_ms;        /* materialise: level 1 */
    double fill_ms;         /* materialise: level-2 tables and lists (worker threads) */
    double release_ms;      /* kbh_release: the engine context's device and pinned memory */
    double expand_ms;       /* the last expand_read_id_list */
    uint64_t expand_nodes;  /* ll_nodes it allocated (outer nodes + list copies) */
} kbh_times;
int kbh_last_times(kbh_times *out);

/* Materialise a CSR (kb_export layout, `first` = insertion order) into
 * hash_table exactly as prune_data does (prune: the cutoff set by
 * kbh_configure).  replay_only: build it by zhash_set in insertion order (the
 * slow, obviously-reference path) instead of the direct layout -- the two
 * must give identical tables (kbh_layout_digest). */
int kbh_materialise_csr(struct ZHashTable *hash_table, const kb_csr *r, int prune, int replay_only);
/* 1 when list nodes come from the node arena (binning_gpu.c: this library's
 * free() is the process's, KBH_NODE_ARENA not 0), else 0 (malloc'd nodes) */
int kbh_node_arena_active(void);
/* digest of a two-level table's exact layout: size steps, counts, bucket
 * index and chain order of every entry, keys, list contents and order */
uint64_t kbh_layout_digest(struct ZHashTable *hash_table);

/* drop the engine context bound to hash_table (the tables stay) */
void kbh_release(struct ZHashTable *hash_table);

/* binning.c:1150-1166 read loop: fgets(buf, read_length) chunks, strip of the
 * last byte, one id per chunk (empty chunks included).  Returns concatenated
 * bases + lengths (malloc'd; free with kbh_free_reads). */
int kbh_read_fgets(const char *path, int read_length, char **bases, uint32_t **lens,
                   uint64_t *n_reads);
void kbh_free_reads(char *bases, uint32_t *lens);

/* the configuration in effect (kbh_configure, else the compile-time defaults) */
void kbh_get_config(int *K, int *M, int *cutoff);

/* binning.c:659-783: the reference's unitig extension, exact (same merges, same
 * keys, same per-base read-id lists, same table and iterator state after it),
 * without its all-pairs candidate scan (genome-assembly_amd/host/unitig.c).
 * A strong definition: a drop-in that links the reference's binning.o weakens
 * the reference's copy (oracle/build_ref.sh dropin).  Works on
 * any level-1 table laid out as zhash.h (ours or the reference's own), after
 * expand_read_id_list as in the reference's main (binning.c:1171-1177). */
void find_kmer_extensions(struct ZHashTable *hash_table, bool forward);
typedef struct {
    uint64_t calls, queries, unitigs, merges, multiple, resumes, candidates;
    uint64_t deleted, inserted, set_existing;
    uint64_t u1_events; /* binning.c:721-731 with the extension the kmer's chain
                           successor: a use-after-free in the reference (unitig.c) */
    double index_ms, walk_ms;
} kbh_unitig_stats;
int kbh_unitig_stats_get(kbh_unitig_stats *out);
/* print_kmers (binning.c:827-843), including the first level-2 table's resume
 * from the iterator cursor find_kmer_extensions may leave (binning.c:403-427) */
int kbh_print_kmers(struct ZHashTable *hash_table, FILE *out);
void kbh_unitig_reset(void);

/* canonical dump of a materialised two-level table:
 * "mmer\tkmer\tcount\tid1,id2,...\n", lines sorted bytewise */
int kbh_dump_table(struct ZHashTable *hash_table, FILE *out);

#ifdef __cplusplus
}
#endif
#endif
