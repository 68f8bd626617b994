// kbin_internal.h -- shared declarations between the HIP kernels
// (kbin_kernels.hip) and the host C-ABI (kbin_api.hip).  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kb {

// Slot layouts of the open-addressed (mmer, kmer) table.  EMPTY slot = all 0.
//  KW=1 (K <= 31):  w0 = kmer_code + 1 (claim word, CAS), w1 = tag | cnt << 32
//  KW=2 (K <= 63):  w0 = (code >> 63) + 1 (claim), w1 = (code & 2^63-1) | PUB,
//                   w2 = tag | cnt << 32, w3 = pad
// tag = mmer_code + 1 (non-zero marks it published).  Every non-claim word
// carries its own "published" marker, so readers never need cross-word
// ordering ("Table protocol").
constexpr uint64_t PUB = 1ull << 63;
constexpr uint32_t NONE = 0xFFFFFFFFu;

// status bits written by kernels
constexpr uint32_t ST_TABLE_FULL = 1u;   // distinct keys exceeded the load limit
constexpr uint32_t ST_PROBE_LIMIT = 2u;  // a probe sequence exceeded max_probe
constexpr uint32_t ST_ALPHABET = 4u;     // byte outside ACGT in packed input
constexpr uint32_t ST_NEG_ID = 8u;       // a routed read id < 0 (the binned receiver orders lists by id)
constexpr uint32_t ST_BUCKET_FULL = 16u; // a local bucket holds more mmers than bucket_kernel maps

struct ScanArgs {
    const uint64_t* words;     // packed reads, RW words per read
    const uint32_t* lens;      // bases per read
    const uint64_t* kmer_base; // [n_reads+1] first occurrence index of read r (batch-local)
    uint64_t n_reads;
    uint64_t* table;           // slots * SW words
    uint64_t mask;             // slots - 1
    uint64_t* occ;             // [n_occ_total] records (slot << 32 | ordinal), reversed
    uint64_t occ_base;         // first occurrence index of this batch
    uint64_t n_occ_total;
    uint32_t ord_base;         // call ordinal of the batch's first read
    uint64_t* first;           // [slots] min(ordinal << 16 | i) per key, or null
    uint32_t* n_distinct;      // global distinct-key counter
    uint32_t* status;
    uint32_t max_distinct;
    uint32_t max_probe;
    int RW;                    // words per read
    int K, M;
};

struct RouteArgs {
    const uint64_t* words;
    const uint32_t* lens;
    const int32_t* ids;        // read ids (carried in the records)
    uint64_t n_reads;
    uint32_t* offs;            // [G][n_reads] counts (count pass) / scanned offsets (pack pass)
    const uint64_t* adj;       // [G] per-destination base adjustment (pack pass)
    uint64_t* out;             // send buffer (pack pass)
    uint32_t G;
    uint32_t part, part_n;     // kb_set_partition: route only this mmer partition's records
    int rec_words;
    int RW, K, M;
    const uint8_t* owner_map;  // canonical mmer - 2^(2M-1) -> owner rank (kb_owner_table; null: the hash)
};

struct SkArgs {
    const uint64_t* recs;      // received super-k-mer records
    const uint32_t* rec_base;  // [n_rec] first occurrence index of each record (batch-local)
    uint64_t n_rec;
    int rec_words;
    uint64_t* table;
    uint64_t mask;
    uint64_t* occ;
    uint64_t occ_base;
    uint64_t n_occ_total;
    uint64_t* first;
    uint32_t* n_distinct;
    uint32_t* status;
    uint32_t max_distinct;
    uint32_t max_probe;
    int K, M;
};

// ---- binned engine (kbin_bins.hip)

struct SkScanArgs {
    const uint64_t* words;
    const uint32_t* lens;
    uint64_t n_reads;
    uint32_t* seg_count;       // count pass: segments per read
    unsigned long long* n_kmers;  // count pass: [sk_blocks()] per-block k-mer sums
    const uint32_t* rec_base;  // write pass: exclusive scan of seg_count
    unsigned long long* rec_ctr;  // write pass without count pass (thread kernel): records
                                  // allocated per block from this counter, any order; the
                                  // k-mer sums go to n_kmers as in the count pass
    uint64_t* pay;             // [3R] {ord | n << 32 | sig_off << 38 | rev << 44, span w0, w1}
    uint64_t* keys;            // [R] canonical mmer << 38 | (63 - n) << 32 | record index:
                               // bins in mmer order, records of a bin longest first
                               // (a wavefront's 64 records have near-equal k-mer counts)
    uint32_t ord_base;
    int RW, K, M;
    // region mode (thread kernel, with rec_ctr == nullptr): records go to
    // regions + (dest * region_cap + i) * rw, dest = hash(mmer + dest_salt) % G:
    // routing (ranks, routed format with the read id) or local buckets
    // (binned_fmt: the pay layout with the ordinal, rw = 1 + span words:
    // 3 for K <= 31, 5 for K <= 63)
    uint64_t* regions;
    uint64_t region_cap;
    const uint64_t* region_base;   // [G + 1] or null: destination d's records at region_base[d]
                                   // (exact layout after a counting pass), else at d * region_cap
    unsigned long long* dest_ctr;  // [G] records per destination (zeroed)
    const int32_t* read_ids;       // ordinal -> id (null: affine, id = ordinal + id_off)
    uint32_t id_off;
    uint32_t G;                    // <= 1024
    uint64_t dest_salt;
    int rw;
    int binned_fmt;
    // local buckets only: canonical mmer - 2^(2M-1) -> bucket map entry
    // (bm_* below), balanced by the host from the bins of earlier passes (null:
    // hash of the mmer); a split mmer's records are cut into their context
    // sub-bins (at most two pieces each) on the way into the buckets
    const uint32_t* bucket_map;
    const uint16_t* sub_map;
    int sub_stamp;             // the map splits mmers: bucket records carry their sub-bin (sub_room)
    // routing to ranks only: canonical mmer - 2^(2M-1) -> owner rank
    // (kb_owner_table; null: the owner hash, and always for K < 2M codes)
    const uint8_t* owner_map;
    // partitioned passes (kb_set_partition): only super-k-mers whose mmer is in
    // partition part of part_n are emitted and counted (part_n <= 1: all)
    uint32_t part, part_n;
};

// local buckets: every record of a bin lands in bucket dest_of(mmer, NB, BUCKET_SALT);
// bucket_kernel then orders each bucket's records by (mmer, 63 - n)
struct BucketArgs {
    const uint64_t* regions;   // NB regions of cap records, pay layout (1 + spw words)
    uint64_t cap;
    const uint64_t* rbase;     // [NB + 1] or null: region d at rbase[d], rbase[d+1]-rbase[d] records
    const unsigned long long* bfill;  // [NB] records per bucket
    int M;
    uint64_t* hdr;             // [2R] output (header, span word 0) pairs, bins contiguous, longest first
    uint64_t* w1;              // [R] span word 1 (K <= 31), or [2R] (word 1, word 2) pairs (spw = 4)
    uint64_t* w3;              // [R] span word 3 (spw = 4)
    int spw;                   // span words per record: 2 (K <= 31) or 4 (K <= 63)
    uint64_t* bbase;           // [NB + 1] output base of each bucket (bucket_bases_kernel)
    int bases_ready;           // bbase already written (bucket_stats_kernel after the record pass)
    int sub;                   // records carry their context sub-bin (sub_room): group by (mmer, sub-bin)
    uint32_t* bocc;            // [max_bins] k-mer occurrences of the bin (0: not counted), or null
    unsigned long long* bin_ctr;   // bins (zeroed; = totals[2])
    uint32_t* bstart;          // [max_bins] first record of bin
    uint32_t* bcount;          // [max_bins] records of bin
    uint32_t* bmmer;           // [max_bins] the bin's canonical mmer
    uint64_t max_bins;
    int ablate;                // KB_BIN_ABL builds: KB_BK_ABLATE (1: no placement stores, 2: no
                               // placement pass) -- results wrong by design
    uint32_t* status;          // ST_BUCKET_FULL: a bucket holds too many bins
    uint64_t rcap;             // records the hdr / w1 / w3 layout holds (0: every one; a speculative launch)
};

// region d of a record region set: fixed stride cap, or exact bases
__device__ __forceinline__ uint64_t region_off(const uint64_t* base, uint64_t cap, uint32_t d) {
    return base ? base[d] : (uint64_t)d * cap;
}
__device__ __forceinline__ uint64_t region_room(const uint64_t* base, uint64_t cap, uint32_t d) {
    return base ? base[d + 1] - base[d] : cap;
}

// ---- context sub-bins.  The reference's level-1 key is the signature mmer
// (binning.c:1045) and every (mmer, kmer) entry lives in one mmer bin, but a
// bin can hold far more distinct keys than one LDS table (few mmers per rank
// at N GPUs, high coverage).  A finer partition of a bin that is a function of
// the KEY and constant along a super-k-mer: for the k-mer starting o bases
// before its signature (o = sig - i; o is the first occurrence of the
// canonical mmer string in the key's k-mer, bin_body), the b bases right
// after the mmer lie inside the k-mer whenever o <= K - M - b, and they are
// the read's bases sig + M .. sig + M + b - 1 for every k-mer of the record
// (complemented with it, binning.c:1029-1040).  So sub-bin 1 + ctx holds the
// keys with o <= K - M - b and context ctx (4^b of them), sub-bin 0 (the
// "edge") the keys with o > K - M - b: a record is at most cut in two, its
// first so - (K - M - b) k-mers into the edge.  (Measured on uniform reads at
// K31 M7: b = 2 leaves 1.2 % of the occurrences in the edge and cuts 9.5 % of
// the records; the 16 context sub-bins hold 0.76..1.10 x their mean.)
// (round 5 tried depth 5, 1025 sub-bins, for C5's giant mmers with an 11-bit
// stamp -- K63 M7 leaves 9 spare bases, so the record has room: 2.9 x the
// bins, 6 x the light pre-filtered ones, but 35 % more heavy ones and the C5
// share 490 -> 637 ms per step (gpurun_out r5g5); depth 4 stays)
constexpr uint32_t SUB_MAX_B = 4;                      // 257 sub-bins at most
constexpr uint32_t SUB_BITS = 9;                       // sub-bin index bits (2 SUB_MAX_B + 1)
__host__ __device__ inline uint32_t sub_count(uint32_t b) { return b ? (1u << (2 * b)) + 1u : 1u; }

// Bucket map entry (u32 per canonical mmer - 2^(2M-1)):
//   bit 31 clear: the mmer's one bin lives in bucket (entry & 1023)
//   bit 31 set:   the mmer is split into sub_count(b) context sub-bins,
//                 b = (entry >> 28) & 7 in 1..SUB_MAX_B; sub-bin s lives in
//                 bucket sub_map[(entry & 0x0FFFFFFF) + s]
constexpr uint32_t BM_SPLIT = 0x80000000u;
// The bucket map covers the canonical mmer codes [2^(2M-1), 4^M) only
// (bucket_map[canon - 2^(2M-1)]).  A record whose code is below that -- a
// K < 2M signature (binning.c:992-1021: the host turns the map off for those
// passes) or a malformed received record -- has no entry and takes the hash
// route every map-less pass takes; no kernel indexes below the map
// (the r5g38 fault's class).
__host__ __device__ __forceinline__ bool bm_has_entry(uint32_t canon, int M) { return canon >= (1u << (2 * M - 1)); }

// Routed super-k-mer record header: id | i0 << 32 | n << 48 | sig_off << 54 |
// rev << 60.  rev is the complement flag (binning.c:1029-1040's is_rev).  For
// K >= 2M it is a function of the span -- the signature's code is below half
// exactly when the complement won -- and receivers rederive it; for K < 2M the
// incremental branch (binning.c:992-1021) sets is_rev from scores polluted by
// appended bases, so the sender's flag is the only source
constexpr int ROUTED_REV_BIT = 60;
__host__ __device__ __forceinline__ bool routed_rev(uint64_t h, uint32_t sm, int K, int M) {
    return K < 2 * M ? ((h >> ROUTED_REV_BIT) & 1u) != 0 : sm < (1u << (2 * M - 1));
}
__device__ __forceinline__ uint32_t bm_depth(uint32_t e) { return (e & BM_SPLIT) ? (e >> 28) & 7u : 0u; }
__device__ __forceinline__ uint32_t bm_bucket(uint32_t e, const uint16_t* sub_map, uint32_t sub) {
    return (e & BM_SPLIT) ? (uint32_t)sub_map[(e & 0x0FFFFFFFu) + sub] : (e & 1023u);
}
// A bucket record carries its sub-bin in the low SUB_BITS of its last span
// word: the span holds n + K - 1 <= 2K - M bases of its 32 x spw, and those
// bits (the last 5.5 base positions) lie past every k-mer the bin kernels
// read.  Splitting needs that room (and the bucket ordering then groups the
// records by (mmer, sub-bin) without the map).  K31 M7 and K63 M7 leave 9
// spare bases, the reference's K31 M4 six.
__host__ __device__ inline bool sub_room(int K, int M, int spw) { return 32 * spw - (2 * K - M) >= 5; }
static_assert(2 * SUB_MAX_B + 1 <= SUB_BITS, "the stamp holds every sub-bin index");
constexpr uint64_t SUB_MASK = (1ull << SUB_BITS) - 1ull;

// k-mers of a record (sig offset so, n k-mers) in the edge of depth b: its first ones
__device__ __forceinline__ int sub_edge(int so, int n, int K, int M, uint32_t b) {
    const int e = so - (K - M - (int)b);
    return e <= 0 ? 0 : (e < n ? e : n);
}
// sub-bin of a piece whose k-mers all lie on one side: w = 64-bit window of
// the read (or span) at the signature + M, rev = the complement won
__device__ __forceinline__ uint32_t sub_ctx(int so, int K, int M, uint32_t b, uint64_t w, bool rev) {
    if (!b || so > K - M - (int)b) return 0u;
    const uint32_t m = (1u << (2 * b)) - 1u;
    return 1u + (((uint32_t)(w >> (64 - 2 * b)) ^ (rev ? m : 0u)) & m);
}

constexpr uint32_t KB_FLAT_MAX = 16384;  // partitions of one heavy bin's flat lists (kbin_bins.hip FLAT_MAX)

// The bin kernels read BinArgs through a pointer (launch_bins): pointers loaded
// from device memory are generic to the compiler, so every access through them
// became a FLAT instruction -- counted in lgkmcnt as well, so each LDS wait
// (every barrier) also waited for the global stores in flight.  In device code
// the fields are global-address-space pointers (the layout is the host's) --
// in kbin_bins.hip's device pass, where the bin kernels live (KB_BINS_TU): the
// other files' host code assigns the fields from generic pointers, which the
// device pass of those files also type-checks.
#if defined(__HIP_DEVICE_COMPILE__) && defined(KB_BINS_TU)
#define KB_G __attribute__((address_space(1)))
#else
#define KB_G
#endif
struct BinArgs {
    KB_G const uint64_t* hdr;       // [2R] bin-ordered (header, span bases 0..31) pairs (header: SkScanArgs::pay)
    KB_G const uint64_t* w1;        // [R] span bases 32..63, or [2R] (32..63, 64..95) pairs (K > 31)
    KB_G const uint64_t* w3;        // [R] span bases 96..127 (K > 31: two-word k-mers)
    KB_G const uint32_t* bstart;    // [nbins] first record of bin
    KB_G const uint32_t* bcount;    // [nbins] records of bin
    KB_G const uint32_t* bmmer;     // [nbins] canonical mmer of bin
    KB_G const uint32_t* bocc;      // [nbins] its k-mer occurrences (0 or null: count them)
    uint64_t max_bins;         // capacity of the descriptors (nbins never exceeds it)
    KB_G unsigned long long* stage_ctr;  // stage allocation (zeroed): each bin takes its occurrences
    KB_G const uint32_t* order;     // [nbins] processing order (largest bins first)
    KB_G const uint4* bdesc;        // [2 nbins] or null: per processing slot {bin, start, count, mmer},
                               // {occurrences, stage base lo, hi, 0} (bins_desc_kernel)
    KB_G unsigned long long* work;  // work counter (zeroed)
    KB_G uint64_t* stage;           // [N] (LDS slot << 48 | position << 32 | ordinal) per occurrence
    // light bins of the first phase without first-occurrence tracking: the
    // stage as two arrays, 6 B per occurrence (null: the 8-B stage everywhere)
    KB_G uint32_t* stage_ord;       // [N] ordinal
    KB_G uint16_t* stage_slot;      // [N] LDS slot + 1 (0: not in the table)
    KB_G uint64_t* kstage;          // [KW N] heavy bins: the k-mer's table key per occurrence, parallel to stage
    uint32_t flat_l;           // heavy bin: initial partition depth >= flat_l (0 = never)
    // heavy bins, two launches: phase 0 bins every light bin and turns each heavy
    // bin into flat per-partition lists (published below); phase 1 sweeps the
    // published partitions, any block any partition
    KB_G uint32_t* flat_list;            // [max_bins] published heavy bins
    KB_G unsigned long long* flat_n;     // (zeroed) [0] published bins [1] pool [2] build items,
                                    // claims: [3] count [4] scatter [5] phase 1
    KB_G uint32_t* flat_next;            // [max_bins] next partition to claim
    KB_G uint32_t* flat_l0;              // [max_bins] partition depth
    KB_G unsigned long long* flat_sbase; // [max_bins] stage base
    KB_G unsigned long long* flat_obase; // [max_bins] the bin's range of flat_off
    KB_G uint32_t* flat_off;             // pool of list offsets, np + 1 per heavy (or split) bin
    KB_G uint32_t* flat_cur;             // the same layout: scatter cursors (flat bins)
    KB_G uint32_t* flat_chunk;           // [max_bins] first build item (record chunk) of the bin
    KB_G uint32_t* pool_bin;             // [flat_off] bin of an offset-pool entry (phase 1 items)
    KB_G uint32_t* chunk_bin;            // [R / 1024 + max_bins] bin of a build item
    KB_G unsigned long long* flat_octr;  // (zeroed) pool allocation
    // split bins (light bins above a fair share of one block): published like
    // heavy bins (flat_l0 | SPLIT_BIT), their partitions binned from the records
    uint64_t n_occ;                 // occurrences of this finalize
    uint32_t split_div;             // split above n_occ / (blocks x split_div) (0 = never)
    uint64_t split_occ;             // (set at launch)
    uint32_t big_div;               // flat lists for a multi-table bin above n_occ / (blocks x big_div)
    uint64_t big_occ;               // (set at launch; 0 = by depth only)
    KB_G const uint64_t* totals;    // totals[2] = nbins
    int K, M;
    uint32_t keep_gt;
    uint32_t ts_log2;
    float rho;                 // expected distinct keys per occurrence
    KB_G const float* rho_dev;      // cold pass: rho estimated on the device (hll_finish_kernel); else null
    float fill;                // target table load when choosing the partition depth
    uint32_t ringfree;         // unpartitioned bins expand without the per-wave ring (KB_BIN_RINGFREE)
    // offset partitions: a light bin of initial depth 1 <= l <= opart is split by
    // the minimizer's offset inside the k-mer (a function of the key, see
    // bin_body) instead of by a key hash, so each partition expands only its own
    // k-mers of every record; range r of depth l is [ocut[l][r], ocut[l][r + 1])
    uint32_t opart;            // deepest offset-partitioned depth (0: hash partitions only; KB_BIN_OPART)
    float fill_light;          // table load the depth of an offset-partitioned bin aims at
    uint32_t osplit;           // big light bins split by offset range across blocks (KB_BIN_OSPLIT; experimental)
    uint8_t ocut[5][17];
    uint32_t fsl_run;          // LDS-staged flat lists below this many entries per partition per chunk
    uint32_t win_heavy;        // LDS id windows in the heavy bins' partitions too (KB_BIN_WIN_HEAVY; bit 1: two-word keys)
    uint64_t heavy_hint;       // heavy / split bins the last finalize published (0: small grids for their kernels)
    int ablate;                // diagnostic builds (KB_BIN_PROF / KB_BIN_ABL) only: 1 expansion only,
                               // 2 no staging, 3 no id windows, 4 windows without sorts
    KB_G unsigned long long* gcount;  // [0] entries << 32 | ids  [2] distinct keys before prune
    KB_G uint32_t* status;
    KB_G uint32_t* e_mmer;
    KB_G uint64_t* e_hi;
    KB_G uint64_t* e_lo;
    KB_G uint32_t* e_cnt;
    KB_G uint64_t* e_off;
    KB_G uint64_t* e_first;         // KB_TRACK_FIRST: (ordinal << 16 | position) of each key's first occurrence
    KB_G uint32_t* ids_ord;
    KB_G int32_t* ids_out;
    KB_G const int32_t* read_ids;
    uint32_t id_off;
    uint64_t max_entries, max_ids;
    // list items for lists_kernel: (first entry << 16 | entries <= 256) of every
    // partition whose ids took the global path (and one-entry items for lists
    // > 256 of the LDS path); the LDS path leaves its lists final in ids_out.
    // null: the global path for every partition, lists_kernel over all entries
    KB_G uint64_t* lq_items;
    KB_G unsigned long long* lq_n;  // (zeroed) items
    uint64_t lq_cap;
    // singleton pre-filter of heavy (flat) bins: a partition's k-mers first
    // go through a 2-bit "seen twice" sketch in LDS; keys seen once are
    // counted (distinct) but never enter the table, the stage or sweep 2
    // (with cutoff >= 1 they are pruned anyway: exact).  Partitions are then
    // sized by the keys that do enter the table (rho_tab) and by the sketch
    uint32_t pf;               // 1: pre-filter the flat bins (prune, cutoff >= 1, no first-occurrence tracking)
    uint32_t pf_light;         // 1 (two-word keys, with pf): a bin the pre-filter brings under the flat
                               // depth stays light, its singles screened by a per-bin LDS sketch
    uint32_t fs_lds;           // 1: heavy bins with 9..2048 partitions write their lists LDS-staged
    float rho_tab;             // expected table keys per occurrence under the pre-filter
    KB_G unsigned long long* tab_keys;  // (zeroed) keys that entered a table
    // (zeroed) path counters for kb_timing, one atomic per bin or partition:
    // [0] heavy bins published as flat lists [1] split bins published
    // [2] partitions swept to their prune [3] partitions redone split (overflow)
    // [4] deepest partition depth (max) [5] keys kept out by the pre-filter
    // [6] offset-range partitions [7] partitions swept from flat lists
    // [8] light pre-filtered bins [9] ranked bins [10] partitions emitted from rank bitmaps
    KB_G unsigned long long* pstat;
    uint32_t ts_adapt;         // 1: one-table light bins take the smallest table for their keys (KB_BIN_TS_ADAPT)
    uint32_t ldsbar;           // 1: barriers that order LDS only skip the global-store drain (KB_BIN_LDSBAR)
    uint32_t corrupt;          // diagnostic (KB_DIAG_CORRUPT=1): block 0 adds one to a count, so the
                               // finalize's invariant (sum of pre-prune counts == k-mers) must fail
    uint32_t diag_alloc;       // diagnostic builds (KB_BIN_ABL): a second returning atomic in series with
                               // the prune's allocation (KB_DIAG_ALLOC; prices its round trip)
    uint32_t skew;             // diagnostic builds (KB_BIN_ABL): wave skew - 1 arrives late at every
                               // partition-loop top (KB_DIAG_SKEW; a barrier-ordering stress test)
    // Ranked bins (long lists, C3's coverage): a light bin first ranks its
    // records by call ordinal (descending, ties by record index) -- rrank[r] is
    // record r's rank inside its bin, rord[lo + k] the ordinal of rank k -- and
    // its stage holds ranks instead of ordinals.  A partition whose lists are
    // long then places every kept occurrence as one bit of its key's bitmap
    // over the bin's ranks and emits each list by walking the bitmap: reverse
    // call order (binning.c:1061-1068) with no sort and no list kernels
    uint32_t rank_mode;        // 1: rank bins of 512 .. rank_max records (KB_BIN_RANK)
    uint32_t rank_merge;       // ranked bins: long lists' bitmaps set in the id windows' stage pass (KB_BIN_RANK_MERGE)
    KB_G uint32_t* rrank;           // [R] record -> rank in its bin
    KB_G uint32_t* rord;            // [R] (bin start + rank) -> ordinal
};
constexpr int KB_PSTAT = 11;
// light pre-filtered bins (kbin_bins.hip): the per-bin sketch's cells and the
// distinct-key load it takes (the host sizes sub-bins by them)
constexpr uint32_t PFL_CELLS = 8192u * 16u;
constexpr double PFL_LOAD = 0.15;  // (h_totals[16 .. 16 + KB_PSTAT) in the stats copy)

struct ListArgs {
    const uint64_t* totals;    // totals[0] = entries
    const uint32_t* e_cnt;
    const uint64_t* e_off;
    uint32_t* ids_ord;         // call ordinals per list (scratch for long lists)
    int32_t* ids_out;
    const int32_t* read_ids;
    uint32_t id_off;
    uint32_t* long_q;          // [2 long_cap] entries with 257..4096 ids: [0, long_cap) for
                               // lists_bucket_kernel, [long_cap, 2 long_cap) passed on to lists_long_kernel
    uint64_t long_cap;
    unsigned int* long_n;      // [2] (zeroed) queue lengths
    uint32_t long_n_zeroed;    // long_n cleared by the caller already
    uint64_t lq_hint;          // grid hints from the last finalize (~0: none): queued items,
    uint64_t long_hint[2];     // long lists for lists_bucket_kernel / lists_long_kernel
    const uint64_t* lq_items;  // BinArgs::lq_items (null: every entry, chunks of 256)
    const unsigned long long* lq_n;
    uint64_t lq_cap;
};

hipError_t launch_lists(const ListArgs& a, uint64_t max_entries, hipStream_t s);
hipError_t launch_sk(const SkScanArgs& a, bool write, hipStream_t s);
// received routed records (rw words: {id | i0 << 32 | n << 48 | sig_off << 54 | rev << 60}, span words)
// -> binned records at t = off + k; ids < 0 set ST_NEG_ID in *status
hipError_t launch_sk_convert(const uint64_t* recs, uint64_t n_rec, int rw, uint64_t off, int M, int K,
                             uint64_t* pay, uint64_t* keys, uint32_t* status, unsigned long long* n_kmers,
                             hipStream_t s);
// sender: destination of every record (owner of its mmer) -> dkeys = dest << 32 | t, counts[dest]
hipError_t launch_route_dest(const uint64_t* keys, uint64_t R, uint32_t G, const uint8_t* owner_map, int M,
                             uint64_t* dkeys, unsigned long long* counts, hipStream_t s);
// sender: records in destination-sorted order -> routed record format
hipError_t launch_route_pack_binned(const uint64_t* sorted, const uint64_t* pay, uint64_t R, int rw,
                                    const int32_t* read_ids, uint32_t id_off, uint64_t* out,
                                    hipStream_t s);
uint64_t sk_blocks(uint64_t n_reads, int RW);
hipError_t launch_sk_kmers_total(const unsigned long long* part, uint64_t n, unsigned long long* out,
                                 hipStream_t s);
hipError_t launch_sk_gather(const uint64_t* keys, const uint64_t* pay, uint64_t R, uint64_t* srec,
                            hipStream_t s);
// ev_bin[2]: recorded right before and right after bin_kernel (timing), or null
// heavy: also the published bins' kernels (flat lists, partitions); without,
// launch_bins_heavy runs them later (a finalize that expected none).
// d_args: one BinArgs of device memory; the bin kernels read their arguments
// there (launch_bins writes them, stream-ordered; launch_bins_heavy reuses them)
hipError_t launch_bins(const BinArgs& a, uint64_t max_bins, int KW, hipStream_t s, hipEvent_t* ev_bin, bool heavy,
                       BinArgs* d_args);
hipError_t launch_bins_heavy(const BinArgs& a, int KW, hipStream_t s, const BinArgs* d_args);
// launch_bins_order + launch_bins_desc in one launch (bucketed path)
hipError_t launch_bins_plan(const uint32_t* bstart, const uint32_t* bcount, const uint32_t* bmmer,
                            const uint32_t* bocc, const uint64_t* totals, uint64_t max_bins, uint32_t* order,
                            uint4* desc, unsigned long long* stage_ctr, hipStream_t s);
hipError_t launch_bins_desc(const uint32_t* order, const uint32_t* bstart, const uint32_t* bcount,
                            const uint32_t* bmmer, const uint32_t* bocc, const uint64_t* totals, uint64_t max_bins,
                            uint4* desc, unsigned long long* stage_ctr, hipStream_t s);
// HyperLogLog of the k-mers of the bin-ordered records (2^12 u32 registers
// and a u64 occurrence count, zeroed here; sample > 1: the bins of 1 / sample
// of the mmers only) and its estimate (host): the cold pass's distinct keys
hipError_t launch_hll(const BinArgs& a, uint64_t R, int KW, uint32_t* regs, uint32_t sample, hipStream_t s);
double hll_estimate(const uint32_t* regs);
// resolve the binned path's kernels (kb_create: once per process and device)
hipError_t load_bin_kernels();
// this thread's kb_last_error() message (kbin_group.hip's failures)
void set_last_error(const char* msg);
// distinct / occurrences from launch_hll's registers, on the device (no host
// round trip): written to *rho (clamped to [1e-4, 1]; 0.25 with no occurrences)
hipError_t launch_hll_finish(const uint32_t* regs, float* rho, hipStream_t s);
hipError_t launch_bins_order(const uint32_t* bcount, const uint64_t* totals, uint32_t* order, uint64_t max_bins,
                             hipStream_t s);
hipError_t launch_bucket_sort(const BucketArgs& a, uint32_t NB, hipStream_t s);
uint64_t sk_bucket_salt();
uint32_t sk_hash_dest(uint32_t mmer, uint32_t G, uint64_t salt);  // host twin of dest_of
// radix path: bin descriptors from run starts of the sorted keys
hipError_t launch_bins_describe(const uint64_t* keys, const uint32_t* starts, const uint64_t* totals,
                                uint32_t* bcount, uint32_t* bmmer, uint64_t max_bins, hipStream_t s);
// received records into local bucket regions (block-aggregated reservations)
hipError_t launch_sk_convert_buckets(const uint64_t* recs, uint64_t n_rec, int rw, int spw, int M, uint32_t NB,
                                     int K, const uint32_t* bucket_map, const uint16_t* sub_map, int sub_stamp,
                                     uint64_t* regions, uint64_t cap, const uint64_t* rbase, unsigned long long* bfill,
                                     uint32_t* status, unsigned long long* n_kmers, hipStream_t s);
size_t bins_lds_bytes(uint32_t ts_log2, int KW);
#ifdef KB_BIN_PROF
void bins_prof_report(hipStream_t s);
void lists_prof_report(hipStream_t s);
#endif
hipError_t launch_digest(const uint32_t* mmer, const uint64_t* hi, const uint64_t* lo, const uint32_t* cnt,
                         const uint64_t* off, const int32_t* ids, uint64_t n_entries, unsigned long long* out,
                         hipStream_t s);
// zero up to 8 device ranges (u32 words) in one launch: a finalize's counters
// (a hipMemsetAsync each cost a launch and a host round trip)
struct ClearList {
    uint32_t* p[8];
    uint32_t words[8];
    int n;
    void add(void* q, uint64_t bytes) {
        p[n] = static_cast<uint32_t*>(q);
        words[n++] = (uint32_t)(bytes / 4);
    }
};
hipError_t launch_clear(const ClearList& l, hipStream_t s);
// totals[12] = sum of the NB bucket fills (records), totals[13] = the largest,
// totals[14] = status word misc[0]: the record pass's results in one copy;
// totals[8] += the nk per-block k-mer sums kpart (the record pass's N)
hipError_t launch_bucket_stats(const unsigned long long* bfill, uint32_t NB, const uint32_t* misc, uint64_t* totals,
                               uint64_t cap, const uint64_t* rbase, uint64_t* bbase, const unsigned long long* kpart,
                               uint64_t nk, hipStream_t s);
// report (non-null): the finalize's stats in one copy -- totals[16 ..
// 16 + KB_PSTAT) = pstat, totals[28 .. 31) = misc[0 .. 6) in pairs
hipError_t launch_bins_final(const unsigned long long* gcount, uint64_t* e_off, uint64_t* totals,
                             uint64_t max_entries, const unsigned long long* flat_n, const unsigned long long* lq_n,
                             const unsigned long long* pstat, const uint32_t* report_misc, hipStream_t s);
constexpr int KB_TOTALS = 32;  // device totals words (the report layout above)

// launch helpers implemented in kbin_kernels.hip (all asynchronous on `s`)
hipError_t launch_pack(const uint8_t* d_bases, const uint64_t* d_off, uint64_t n_reads,
                       int RW, uint64_t* d_words, uint32_t* d_lens, uint32_t* d_status,
                       hipStream_t s);
hipError_t launch_kmer_base(const uint32_t* d_lens, uint64_t n_reads, int K,
                            uint64_t* d_kmer_base, uint64_t* d_scratch, uint64_t scratch_n,
                            hipStream_t s);
uint64_t kmer_base_scratch_elems(uint64_t n_reads);
hipError_t launch_scan_insert(const ScanArgs& a, int KW, hipStream_t s);
uint64_t radix_counts_elems(uint64_t n);
uint64_t radix_scratch_elems(uint64_t n);
hipError_t launch_radix_sort(uint64_t* a, uint64_t* b, uint64_t n, int key_bits, uint32_t* counts,
                             uint64_t* scratch, uint64_t scratch_n, uint64_t** sorted,
                             hipStream_t s);
uint64_t onesweep_flag_elems(uint64_t n);
hipError_t launch_onesweep(uint64_t* a, uint64_t* b, uint64_t n, int key_bits, uint64_t* flags,
                           uint32_t* aux, uint32_t* epoch, uint64_t** sorted, hipStream_t s);
// run starts of sorted keys, a run = equal S >> key_shift
hipError_t launch_heads(const uint64_t* S, uint64_t n, uint32_t* starts, uint64_t max_runs,
                        uint64_t* scratch, uint64_t scratch_n, uint64_t* d_totals, hipStream_t s,
                        int key_shift = 32);
uint64_t runs_scratch_elems(uint64_t n, uint64_t max_runs);
hipError_t launch_runs(const uint64_t* S, uint64_t n, const uint64_t* table, int KW,
                       uint32_t keep_gt, uint32_t* starts, const int32_t* read_ids,
                       uint32_t id_off, int32_t* ids_out, uint64_t max_runs, uint32_t* e_mmer, uint64_t* e_hi, uint64_t* e_lo, uint32_t* e_cnt,
                       uint64_t* e_off, const uint64_t* first, uint64_t* e_first,
                       uint64_t* scratch, uint64_t scratch_n, uint64_t* d_totals, hipStream_t s);
hipError_t launch_route(const RouteArgs& a, bool pack, hipStream_t s);
hipError_t launch_sk_counts(const uint64_t* recs, uint64_t n_rec, int rw, uint32_t* nk, hipStream_t s);
hipError_t launch_insert_sk(const SkArgs& a, int KW, hipStream_t s);
hipError_t launch_scan_u32(uint32_t* a, uint64_t n, uint64_t* scratch, uint64_t scratch_n, hipStream_t s);
uint64_t scan_u32_scratch_elems(uint64_t n);
hipError_t launch_fill_ids(int32_t* d_ids, uint64_t n, int32_t first, hipStream_t s);
hipError_t launch_generate(uint64_t* d_words, uint32_t* d_lens, uint64_t n_reads,
                           uint32_t read_len, uint64_t genome_len, uint32_t err_ppm,
                           uint64_t seed, uint64_t read_base, hipStream_t s);
hipError_t launch_unpack(const uint64_t* d_words, const uint32_t* d_lens, uint64_t n_reads,
                         int RW, const uint64_t* d_off, uint8_t* d_bases, hipStream_t s);

}  // namespace kb
