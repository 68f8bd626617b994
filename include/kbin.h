/*
 * kbin.h -- C-ABI of the MI355X k-mer binning engine (libkbin.so).
 *
 * This is the device-side replacement for the reference hot path
 *   binning.c:902-1076  struct ZHashTable *process_read(struct ZHashTable*, char *read, int read_id)
 *   binning.c:1085-1144 prune_kmers / prune_data
 * and for the containers it drives (zhash.c chained string hash, llist.c
 * read-id lists).  The host keeps the reference's C surface (see
 * include/binning_gpu.h); that shim batches reads and forwards here.
 *
 * Plain C types only: pointers, sizes, status codes.  One host thread per
 * context; all device work runs on the context's own HIP stream and is
 * synchronised inside kb_finalize / kb_export.
 *
 * Semantics:
 *   - encoding getval: T=0 G=1 C=2 A=3 (binning.c:91-111); bytes outside ACGT
 *     are rejected with KB_EALPHABET (the reference silently maps them to 'A'
 *     for scoring but keeps them verbatim in forward keys -- not representable
 *     in 2 bits);
 *   - signature = complement-canonical mmer, leftmost strict argmax, "sticky"
 *     recompute only when the k-mer start passes it (binning.c:922-989);
 *   - key = (mmer, kmer), both complemented (no reversal) when the complement
 *     wins (binning.c:1029-1040);
 *   - per key the read ids in REVERSE CALL ORDER with duplicates
 *     (binning.c:1061-1068);
 *   - prune: keep a key iff its list length > cutoff (binning.c:1094-1102).
 *
 * Codes: a key string s of n bases is exported as the 2n-bit integer
 * sum_j getval(s[j]) * 4^(n-1-j) (getscore order, binning.c:114-124), split
 * into (hi, lo) 64-bit words for k-mers.
 */
#ifndef KBIN_H
#define KBIN_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define KB_OK 0
#define KB_EINVAL 1      /* bad argument / parameter combination */
#define KB_ENOMEM 2      /* device or host allocation failed */
#define KB_EDEVICE 3     /* HIP runtime error */
#define KB_EALPHABET 4   /* a read byte outside {A,C,G,T} */
#define KB_ETOOLONG 5    /* a read longer than max_read_len */
#define KB_ESTATE 6      /* call out of order (e.g. export before finalize) */
#define KB_EOVERFLOW 7   /* k-mer count beyond the 32-bit occurrence index */

/* kb_params.flags */
#define KB_TRACK_FIRST 1 /* keep (call ordinal << 16 | k-mer position) of every
                            key's first occurrence -- the order in which the
                            reference inserts keys (binning.c:1045-1057), needed
                            to rebuild its exact zhash layout */
#define KB_ENGINE_TABLE 2  /* force the global-table engine                      */
#define KB_ENGINE_BINNED 4 /* force the binned engine where it applies (the
                              default): K <= 31 always; K <= 63 on reads of
                              <= 512 bp (or received super-k-mers).  Elsewhere
                              the table engine runs.  Neither flag: KB_ENGINE=table|binned from
                              the environment (A/B runs), else binned.
                              Results are identical either way. */

/* kb_timing.engine */
#define KB_ENG_TABLE 1   /* scan + global find-or-insert + sort by slot + runs  */
#define KB_ENG_BINNED 2  /* super-k-mers + sort by mmer + one LDS table per bin */

typedef struct kb_ctx kb_ctx;

typedef struct {
    int32_t K;              /* KMER_SIZE       (binning.c:11); M <= K <= 63      */
    int32_t M;              /* MMER_SIZE       (binning.c:10); 1 <= M <= 8 (K < 2M:
                               the live incremental branch, one GPU, binned engine) */
    int32_t cutoff;         /* ABUNDANCE_CUTOFF (binning.c:12); >= 0            */
    int32_t max_read_len;   /* longest read accepted (READ_LENGTH-2 for fgets)  */
    int32_t device;         /* HIP device ordinal                               */
    int32_t flags;          /* KB_TRACK_FIRST: record each key's first occurrence */
    uint64_t table_slots;   /* hash-table slots hint (power of two); 0 = auto   */
} kb_params;

/* Exported result (CSR).  Entry order is unspecified (hash order), exactly as
 * the reference's bucket order is not part of its contract. */
typedef struct {
    uint64_t n_entries;     /* surviving (mmer, kmer) keys                      */
    uint64_t n_ids;         /* sum of counts                                    */
    uint64_t n_kmers;       /* k-mer occurrences scanned (all submitted reads)  */
    uint64_t n_distinct;    /* distinct keys before the prune                   */
    const uint32_t *mmer;   /* [n_entries] canonical mmer code                  */
    const uint64_t *kmer_hi;/* [n_entries] k-mer code bits 64..127 (0 if K<=32) */
    const uint64_t *kmer_lo;/* [n_entries] k-mer code bits 0..63                */
    const uint32_t *count;  /* [n_entries] list length (duplicates kept)        */
    const uint64_t *offset; /* [n_entries+1] into ids                           */
    const int32_t *ids;     /* [n_ids] read ids, reverse call order per entry   */
    const uint64_t *first;  /* [n_entries] first occurrence (ordinal << 16 | i)
                               with KB_TRACK_FIRST, else NULL                    */
} kb_csr;

/* per-phase device time of the last kb_finalize (HIP events on the context
 * stream; only filled when timing is enabled) */
typedef struct {
    float scan_insert_ms;   /* table: fused signature scan + find-or-insert;
                               binned: super-k-mer extraction (count + write)  */
    float sort_ms;          /* table: radix sort by slot; binned: by mmer + bins */
    float runs_ms;          /* table: runs/prune/CSR; binned: per-bin kernel    */
    float emit_ms;          /* read-id emission / totals                        */
    float total_ms;         /* first to last event of the finalize              */
    uint32_t scan_insert_launches;
    uint32_t sort_passes;
    uint64_t table_slots;   /* table: global slots; binned: LDS slots per bin   */
    uint32_t engine;        /* KB_ENG_TABLE or KB_ENG_BINNED                     */
    uint32_t n_bins;        /* binned: non-empty mmer bins                       */
    uint64_t n_superkmers;  /* binned: super-k-mer records                       */
    float bin_kernel_ms;    /* binned: bin_kernel alone (runs_ms also holds the
                               heavy-bin kernels and bins_final)                */
    /* binned: which paths the last finalize took (filled with or without
     * timing; tests assert on them) */
    uint32_t heavy_bins;    /* bins turned into flat per-partition lists       */
    uint32_t split_bins;    /* light bins split across workgroups              */
    uint64_t partitions;    /* LDS-table partitions swept to their prune       */
    uint64_t offset_partitions; /* of those, split by minimizer offset range   */
    uint64_t flat_partitions;   /* of those, swept from a heavy bin's flat list */
    uint32_t max_depth;     /* deepest split of one bin (log2 of its tables)   */
    uint32_t overflow_redos;/* partitions redone split after overflowing       */
    uint64_t prefiltered;   /* keys seen once, counted but kept out of the
                               tables by the singleton pre-filter              */
    uint32_t long_lists;    /* lists of 257..4096 ids (bucketed list sort)     */
    uint32_t clustered_lists; /* of those, lists sorted by the full network    */
    uint32_t split_mmers;   /* mmers whose bins were split into context
                               sub-bins (the bucket map the pass used)         */
    uint32_t tail_reruns;   /* binned: 1 when this finalize left the tail kernels
                               out (the last one needed none) and then ran them
                               after all (a heavy bin published, lists queued) */
    uint32_t light_prefilter_bins; /* two-word keys: bins kept light by the
                               singleton pre-filter (an LDS sketch per bin) */
    uint32_t ranked_bins;   /* bins whose records were ranked by call ordinal
                               (long lists: the last finalize's mean >= 64) */
    uint32_t bitmap_partitions; /* partitions whose lists were emitted from
                               per-key bitmaps over the ranks (no sort) */
} kb_timing;

/* Create a context (kb_create replaces zcreate_hash_table for the level-1
 * table, zhash.c:19-35). */
int kb_create(const kb_params *params, kb_ctx **out);
void kb_destroy(kb_ctx *ctx);

/* Append a batch of reads from host memory.  Reads are concatenated in
 * `bases`, `lens[r]` bytes each; read r gets id first_id + r and call ordinal
 * (its position in the stream of all submitted reads).  The bytes are copied
 * into one of two pinned staging slots before return (the caller may reuse its
 * buffer, as binning.c:1154/1158 does); the H2D copy and the 2-bit pack run
 * asynchronously on the context's stream while the caller prepares the next
 * batch (a submit waits only for the slot it reuses, two submits back).  Batch
 * memory comes from a per-context device pool that kb_reset rewinds.
 * A byte outside ACGT is reported as KB_EALPHABET by a later kb_submit or, at
 * the latest, by kb_finalize; the context then stays failed until kb_reset.
 * Replaces the per-call process_read(hash, read, id) (binning.c:902). */
int kb_submit(kb_ctx *ctx, const char *bases, const uint32_t *lens,
              uint64_t n_reads, int32_t first_id);

/* Same, with an explicit id per read (process_read's caller-supplied id). */
int kb_submit_ids(kb_ctx *ctx, const char *bases, const uint32_t *lens,
                  uint64_t n_reads, const int32_t *ids);

/* Append reads already resident in device memory in the engine's packed
 * layout: read r occupies words_per_read uint64 words at d_words + r*wpr, base
 * j of the read in word j/32 at bits [62-2(j%32), 63-2(j%32)] (getval codes,
 * first base most significant); d_lens[r] bases.  The device buffers are
 * referenced, not copied, until kb_reset/kb_destroy. */
int kb_submit_packed_device(kb_ctx *ctx, const uint64_t *d_words,
                            const uint32_t *d_lens, uint64_t n_reads,
                            uint32_t words_per_read, int32_t first_id);

/* Scan + insert + count, prune (keep count > cutoff when prune != 0), place
 * and order the read ids.  Replaces the insert half of process_read and
 * prune_data (binning.c:1130-1144). */
int kb_finalize(kb_ctx *ctx, int prune);

/* Copy the result to host memory owned by the context (valid until the next
 * kb_finalize / kb_reset / kb_destroy). */
int kb_export(kb_ctx *ctx, kb_csr *out);

/* Device pointers of the same result (no copy). */
int kb_export_device(kb_ctx *ctx, kb_csr *out);

/* Order-independent digest of the last result, for comparing results too
 * large to dump: out[0] entries, out[1] ids,
 * out[2] = sum_e mix(key_e ^ count_e << 1), out[3] = sum over every list
 * position j of mix(key_e ^ ((j + 1) << 32 | id)), sums mod 2^64, key_e =
 * mix(mix(mix(mmer) ^ kmer_hi) ^ kmer_lo), mix = the splitmix64 finaliser.
 * Independent of entry order, sensitive to list order; digests of disjoint
 * results (partitioned passes, ranks) add up to the digest of their union. */
int kb_digest(kb_ctx *ctx, uint64_t out[4]);
/* Drop all submitted reads and results; keeps allocations for reuse. */
int kb_reset(kb_ctx *ctx);

/* Per-phase timing of the last finalize (enable before kb_finalize):
 * 0 off, KB_TIMING_ALL every phase event, KB_TIMING_KERNEL (binned engine)
 * only the two events around bin_kernel (bin_kernel_ms; the phase fields read
 * 0) -- each event record idles the GPU for a few microseconds. */
#define KB_TIMING_ALL 1
#define KB_TIMING_KERNEL 2
int kb_set_timing(kb_ctx *ctx, int enable);
int kb_get_timing(kb_ctx *ctx, kb_timing *out);

/* Synthetic reads generated on device (mirroring
 * generate_reads.py:93-112: iid uniform genome, uniform start, forward strand,
 * iid substitutions at rate err_per_million/1e6), written in the packed
 * layout above into caller-owned device buffers.  Deterministic in seed
 * (splitmix64 counters).  d_words needs n_reads*ceil(read_len/32) words. */
int kb_generate_reads_device(int device, uint64_t *d_words, uint32_t *d_lens,
                             uint64_t n_reads, uint32_t read_len,
                             uint64_t genome_len, uint32_t err_per_million,
                             uint64_t seed);

/* The same generator from read index read_base on: reads read_base ..
 * read_base + n_reads - 1 of the one read stream that seed defines (the genome
 * depends on seed only).  Ranks r = 0..G-1 of a sharded job call it with
 * read_base = r * n_reads and together hold the first G * n_reads reads of
 * ONE genome (BASELINE C4/C5: one genome, reads split by id range, SURVEY
 * §8(e)); kb_generate_reads_device is read_base 0. */
int kb_generate_reads_device_at(int device, uint64_t *d_words, uint32_t *d_lens,
                                uint64_t n_reads, uint32_t read_len,
                                uint64_t genome_len, uint32_t err_per_million,
                                uint64_t seed, uint64_t read_base);

/* Unpack device packed reads to host ASCII (bases concatenated, lens). */
int kb_unpack_reads_to_host(int device, const uint64_t *d_words,
                            const uint32_t *d_lens, uint64_t n_reads,
                            uint32_t words_per_read, char *h_bases,
                            uint32_t *h_lens);

/* ---- multi-GPU routing ------------------------------
 * The canonical-mmer space shards: a super-k-mer (a run of consecutive k-mers
 * of one read sharing a signature) is owned by GPU owner(mmer) of n_dest
 * (kb_owner_table).
 * Sender: kb_route_plan counts the records per destination for every read
 * batch submitted so far; kb_route_pack writes them, destination-major and in
 * read order, into d_send (sum(counts) * kb_record_words u64 words) and marks
 * those batches as shipped.  The caller moves the buffers (RCCL all-to-all,
 * kbin/dist.py).  Receiver: kb_submit_superkmers_device adopts the records it
 * got, concatenated by source rank, and kb_finalize bins them.  Record ids are
 * the senders' read ids: across all ranks they must increase with call order
 * (rank r's ids below rank r+1's) and be >= 0; they are the list order key. */
int kb_record_words(kb_ctx *ctx, uint32_t *out);
/* owner(mmer) for n_dest ranks in pass (part, n_parts) of kb_set_partition
 * (n_parts 1: one pass): out[i] is the rank of canonical mmer 2^(2M-1) + i,
 * for i < 2^(2M-1).  Each pass's canonical mmers are packed onto the ranks,
 * heaviest expected load first (the signature frequency on uniform sequence,
 * ((i + 1) / 2^(2M-1))^(K-M)), each onto the least-loaded rank -- so every
 * rank and process derives the same table from (K, M, n_dest, part,
 * n_parts) alone.  K < 2M codes (not canonical) go to a hash of the code
 * instead.  Host only (no device needed). */
int kb_owner_table(int K, int M, uint32_t n_dest, uint32_t part, uint32_t n_parts, uint8_t *out);
int kb_route_plan(kb_ctx *ctx, uint32_t n_dest, uint64_t *h_counts);
int kb_route_pack(kb_ctx *ctx, uint64_t *d_send);
int kb_submit_superkmers_device(kb_ctx *ctx, const uint64_t *d_records, uint64_t n_records);

/* One-pass sender (binned engine only: K <= 63, reads of <= 512 bp).  Writes every record of the read batches
 * submitted so far into d_regions: destination d's records at
 * d_regions + d * region_cap * kb_record_words, h_counts[d] of them, in no
 * particular order (the binned receiver orders lists by read id, not by
 * arrival).  Returns KB_EOVERFLOW, with h_counts holding the counts needed
 * and the batches left unshipped, when a destination gets more than
 * region_cap records: call again with a larger region_cap.  Returns
 * KB_EINVAL when the binned engine does not apply (use plan/pack). */
int kb_route_scatter(kb_ctx *ctx, uint32_t n_dest, uint64_t *d_regions,
                     uint64_t region_cap, uint64_t *h_counts);

/* kb_route_scatter with the destinations being the n_parts passes of
 * kb_set_partition instead of ranks: ONE super-k-mer pass over the reads
 * serves every partitioned pass.  Region p goes to a context that calls
 * kb_set_partition(p, n_parts), kb_submit_superkmers_device(region p) and
 * kb_finalize; the passes' union is the single-pass result (read ids are the
 * list order key, as for routed records).  Replaces the reference's single
 * process_read loop (binning.c:1150-1166) at scales one finalize cannot hold. */
int kb_split_passes(kb_ctx *ctx, uint32_t n_parts, uint64_t *d_regions,
                    uint64_t region_cap, uint64_t *h_counts);

/* ---- partitioned passes (capacity) -------------
 * One context holds at most 2^32 - 1 k-mer occurrences per finalize.  Larger
 * inputs are binned in passes over disjoint slices of the canonical-mmer
 * space: after kb_set_partition(ctx, p, P) the next kb_finalize (and
 * kb_route_plan / kb_route_pack / kb_route_scatter) covers only the k-mers
 * whose signature mmer falls in partition p of P (a fixed hash of the mmer,
 * independent of the rank owner hash).  A key belongs to exactly one
 * partition (its mmer is part of the key), so the P results are disjoint and
 * their union is the single-pass result, entry for entry and list for list;
 * kb_csr.n_kmers counts the pass's occurrences.  The call drops received
 * super-k-mer batches and the last result, keeps the submitted read batches
 * (and re-arms shipped ones), and may be called any number of times;
 * kb_reset returns to one full pass.  Binned engine only (KB_EINVAL for
 * K > 31 or a forced table engine). */
int kb_set_partition(kb_ctx *ctx, uint32_t part, uint32_t n_parts);
/* Stream used by the context (hipStream_t as void*), for callers that want
 * to order their own work against the engine. */
void *kb_stream(kb_ctx *ctx);

/* ---- multi-GPU groups (SURVEY.md §8(b) kb_create(..., n_gpus, ...), §8(e))
 * A group of G ranks bins one job sharded by canonical mmer: every rank's
 * reads are scanned where they are, each super-k-mer record goes to rank
 * owner(mmer) (kb_route_scatter), the records move in ONE exchange -- the
 * per-destination counts (ncclAllGather), then grouped ncclSend/ncclRecv,
 * over RCCL / xGMI, called from C, each peer message in pieces of at most
 * KB_GROUP_CHUNK words (default 2^25 = 256 MB; the same on every rank: the
 * pieces are matched in order; a rank's own records by a device copy) -- and
 * every rank bins what it received
 * (kb_submit_superkmers_device + kb_finalize).  The ranks' results are
 * disjoint; their union is the single-GPU result, entry for entry and list
 * for list, provided read ids increase with the global call order (rank r's
 * ids below rank r+1's) and are >= 0: they are the reverse-call-order key of
 * the lists (binning.c:1061-1068).
 *   kb_group_create: every rank in this process, one per device of
 *     devices[0..n_gpus) (NULL: 0..n_gpus-1); RCCL communicators from
 *     ncclCommInitAll.  Devices listed more than once (virtual shards, tests
 *     on one GPU) -- or KB_GROUP_TRANSPORT=local -- move the records with
 *     device copies instead, on the same code path.
 *   kb_group_create_rank: one rank per process (params->device is this
 *     rank's device); every process passes the same 128-byte unique id, made
 *     once by kb_group_unique_id and distributed by the caller.
 * Reads go to a LOCAL rank (0 .. n_local-1) with kb_group_submit_ids /
 * kb_group_submit_packed_device and stay until kb_group_reset, so partitioned
 * passes (kb_group_set_partition, then send/receive per pass) reuse them.
 * kb_group_send routes and starts the exchange of the reads' records (the
 * pass's partition only) and returns once it is in flight; kb_group_receive
 * bins the oldest unit in flight on every local rank.  Two units may be in
 * flight, so a caller can send unit i+1 before receiving unit i (the
 * exchange overlaps the binning).  kb_group_send_async returns at once: the
 * unit's routing, count exchange and record sends run on the group's own
 * sender thread, in send order, so the caller's kb_group_receive of unit i
 * bins while unit i+1 routes (kb_group_receive / _discard wait for their
 * unit's send stage and return its failure; kb_group_reset, _submit_* and
 * _set_partition wait until no unit is routing).  kb_group_discard waits
 * for the oldest unit's records and drops them unbinned.  kb_group_finalize
 * = send + receive.  kb_group_reset drops the submitted reads (units in
 * flight keep their records).  A rank whose routing fails still takes part
 * in the counts all-gather, with its status: every rank then fails that unit
 * (no peer is left waiting in a collective).
 * h_counts (optional, G*G): records from rank s to rank d at [s*G + d];
 * kb_group_unit_counts gives the same for the last unit received or
 * discarded (the async sender's counts).
 * Each local rank's result is its receiver context (kb_group_ctx): kb_export,
 * kb_export_device, kb_digest and kb_get_timing apply.  Errors: status codes,
 * message in kb_last_error(). */
typedef struct kb_group kb_group;
#define KB_TRANSPORT_RCCL 1
#define KB_TRANSPORT_LOCAL 2
#define KB_TRANSPORT_HOST 3
/* kb_group_create_rank_host: one rank per process whose counts and records
 * move through the caller's collectives over host memory (e.g. a gloo process
 * group rehearsing several ranks on one GPU, where RCCL refuses a shared
 * device); routing, count bookkeeping, offsets and receivers are the group's
 * own.  Called from the group's sender thread, in send order, on every rank:
 *   allgather: every rank's n words, concatenated by rank, into all;
 *   alltoallv: send holds send_bytes[d] bytes for rank d, packed by d; recv
 *              gets recv_bytes[s] bytes from rank s, packed by s.
 * Each returns 0 on success. */
typedef struct {
    void *user;
    int (*allgather)(void *user, const uint64_t *mine, uint64_t n, uint64_t *all);
    int (*alltoallv)(void *user, const void *send, const uint64_t *send_bytes, void *recv,
                     const uint64_t *recv_bytes);
} kb_group_host_transport;
int kb_group_unique_id(void *out, size_t len);
int kb_group_create(const kb_params *params, int n_gpus, const int *devices, kb_group **out);
int kb_group_create_rank(const kb_params *params, int rank, int n_ranks, const void *unique_id, size_t len,
                         kb_group **out);
int kb_group_create_rank_host(const kb_params *params, int rank, int n_ranks, const kb_group_host_transport *t,
                              kb_group **out);
/* destroy: receive or discard every sent unit first (all ranks).  Units still
 * queued are dropped unsent (their collectives never start, so a peer that
 * has gone cannot block the teardown); a unit whose send stage is already in
 * its collectives is waited for; a warning goes to stderr either way. */
void kb_group_destroy(kb_group *grp);
int kb_group_info(kb_group *grp, int *n_ranks, int *n_local, int *rank0, int *transport);
int kb_group_submit_ids(kb_group *grp, int local, const char *bases, const uint32_t *lens, uint64_t n_reads,
                        const int32_t *ids);
int kb_group_submit_packed_device(kb_group *grp, int local, const uint64_t *d_words, const uint32_t *d_lens,
                                  uint64_t n_reads, uint32_t words_per_read, int32_t first_id);
int kb_group_set_partition(kb_group *grp, uint32_t part, uint32_t n_parts);
int kb_group_send(kb_group *grp, uint64_t *h_counts);
int kb_group_send_async(kb_group *grp);
int kb_group_unit_counts(kb_group *grp, uint64_t *h_counts);
int kb_group_receive(kb_group *grp, int prune);
int kb_group_finalize(kb_group *grp, int prune);
int kb_group_discard(kb_group *grp);
int kb_group_reset(kb_group *grp);
kb_ctx *kb_group_ctx(kb_group *grp, int local);

/* Message for the last failing call on this thread. */
const char *kb_last_error(void);

/* ABI version (bumped on incompatible change): 3 = kb_timing with the ranked-bin
 * counters (ranked_bins, bitmap_partitions, ...) and the kb_group_* calls */
int kb_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KBIN_H */
