// kbin_bins.hip -- the binned engine ("v2") for K <= 31.
//
// The reference's level-1 key is the signature mmer (binning.c:1045): every
// (mmer, kmer) entry lives in exactly one mmer bin, and prune_kmers runs per
// mmer table (binning.c:1085, 1136).  v2 uses that as the unit of locality:
//
//   sk_count / sk_write  one wavefront per read walks the sticky signature
//                        chain (as scan_insert does) and emits one record per
//                        super-k-mer (run of k-mers sharing a signature):
//                        payload {ord | i0 | n | sig_off}, sort key (mmer, t)
//   onesweep             stable sort of the keys by mmer (2 passes at M=7)
//   heads                bin boundaries
//   bin_kernel           ONE WORKGROUP PER BIN: an LDS open-addressed table
//                        keyed by the k-mer alone (the mmer is the bin -- this
//                        is the per-mmer bucket of the north star), counts by
//                        LDS atomics, prune, CSR allocation, read-id placement
//                        and per-key reverse-call-order lists, all LDS/L2-local.
//                        A bin whose keys overflow the LDS table is split by
//                        k-mer hash into sub-partitions, recursively.
//
// Nothing in the hot loops touches HBM at random except the read-word gathers
// (L2/MALL-resident packed reads) and the output writes.
#include <algorithm>
#include <cmath>
#include <cstdio>

#include <hip/hip_ext.h>

#define KB_BINS_TU  // (kbin_internal.h: BinArgs pointers are global in this file's device code)
#include "kbin_internal.h"
#include "kbin_device.h"

namespace kb {

// ---------------------------------------------------------------------------
// phase A: super-k-mer extraction
// ---------------------------------------------------------------------------
// One segment of the sticky chain per call: leftmost strict argmax of the
// complement-canonical mmer score over [lo, lo + K - M]  (binning.c:922-988).
DEV void segment_at(const uint64_t* sw, int lo, int lane, int W, int M, uint32_t maskM,
                    uint32_t halfM, int& sig, uint32_t& canon) {
    const int d = (lane - lo) & 63;
    uint32_t key = 0;
    if (d < W) {
        const int p = lo + d;
        const uint32_t s = (uint32_t)(window64(sw, p) >> (64 - 2 * M));
        const uint32_t c = s >= halfM ? s : maskM - s;
        key = (c << 16) | (0xFFFFu - (uint32_t)p);
    }
    key = wave_max_u32(key);
    sig = rfl((int)(0xFFFFu - (key & 0xFFFFu)));
    canon = (uint32_t)rfl((int)(key >> 16));
}

// QK (K < 2M): the reference's per-k-mer signature state, binning.c:922-1021.
// The incremental branch (992-1021: j runs K-M .. M-1) is live: it appends
// bases to a score it never trims, in int arithmetic that wraps, so the
// signature can move to the k-mer's last M bases and is_rev follow the
// polluted scores.  One lane walks its read k-mer by k-mer with that state;
// a record is a run of k-mers with one signature position (`next`).
struct QWalk {
    int32_t s = 0, r = 0, m = 0;  // score, rev_score, max_score
    bool rev = false;
    int sig = -1, i = -1;         // signature position, last k-mer stepped
    DEV uint32_t code(const uint64_t* sw, int p, int M, uint32_t maskM) const {
        return (uint32_t)(window64(sw, p) >> (64 - 2 * M)) & maskM;
    }
    DEV void step(const uint64_t* sw, int k, int K, int M, uint32_t maskM) {
        if (k > sig) {  // a fresh window (binning.c:922-989): leftmost strict argmax
            uint32_t sm = code(sw, k, M, maskM);
            int32_t sc = (int32_t)sm, rv = (int32_t)(maskM - sm);
            m = sc > rv ? sc : rv;
            rev = !(sc > rv);
            sig = k;
            for (int p = k + 1; p <= k + K - M; p++) {
                sm = code(sw, p, M, maskM);
                sc = (int32_t)sm;
                rv = (int32_t)(maskM - sm);
                if ((sc > rv ? sc : rv) > m) {
                    m = sc > rv ? sc : rv;
                    rev = !(sc > rv);
                    sig = p;
                }
            }
            s = sc;
            r = rv;
        } else {  // the incremental branch (binning.c:992-1021)
            for (int j = K - M; j < M; j++) {
                const uint32_t v = (uint32_t)(window64(sw, k + j) >> 62);
                s = (int32_t)((uint32_t)s * 4u + v);
                r = (int32_t)((uint32_t)r * 4u + 3u - v);
            }
            if ((s > r ? s : r) > m) {
                m = s > r ? s : r;
                rev = !(s > r);
                sig = k + K - M;
            }
        }
        i = k;
    }
    // the record starting at k-mer lo: its signature and complement flag, and
    // the first k-mer of the next record
    DEV void next(const uint64_t* sw, int lo, int nK, int K, int M, uint32_t maskM, int& rsig, bool& rrev,
                  int& e) {
        if (i < lo) step(sw, lo, K, M, maskM);
        rsig = sig;
        rrev = rev;
        e = lo + 1;
        while (e < nK) {
            step(sw, e, K, M, maskM);
            if (sig != rsig) break;
            e++;
        }
    }
};

constexpr uint64_t OWNER_SALT = 0x5851F42D4C957F2Dull;   // rank of a mmer (= owner_of(), kbin_kernels.hip)
constexpr uint64_t BUCKET_SALT = 0x2545F4914F6CDD1Dull;  // bucket of a mmer inside one rank (independent)
constexpr uint64_t PART_SALT = 0x9E3779B97F4A7C15ull;    // pass of a mmer (kb_set_partition; independent)
uint64_t sk_bucket_salt() { return BUCKET_SALT; }

DEV uint32_t dest_of(uint32_t mmer, uint32_t G, uint64_t salt) {
    return (uint32_t)((mix64((uint64_t)mmer + salt) >> 32) % G);
}
uint32_t sk_hash_dest(uint32_t mmer, uint32_t G, uint64_t salt) {
    uint64_t x = (uint64_t)mmer + salt;  // mix64 (kbin_device.h), host side
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return (uint32_t)((x >> 32) % G);
}

// CPU-callable check of the guard above (tests/test_abi.py): the first
// destination of a depth-0 record of code `canon` on a bucketed pass with map
// `map` over NB buckets -- the map's bucket for a canonical code, the hash
// route for any other (never map[canon - half] with canon < half)
extern "C" uint32_t kb_internal_map_dest(const uint32_t* map, uint32_t canon, int M, uint32_t NB) {
    if (!map || !bm_has_entry(canon, M)) return sk_hash_dest(canon, NB, BUCKET_SALT);
    return map[canon - (1u << (2 * M - 1))] & 1023u;
}
DEV uint32_t owner_of_mmer(uint32_t mmer, uint32_t G) { return dest_of(mmer, G, OWNER_SALT); }
// a pass keeps the super-k-mers of its own mmer partition
DEV bool in_part(uint32_t mmer, uint32_t part, uint32_t part_n) {
    return part_n <= 1 || dest_of(mmer, part_n, PART_SALT) == part;
}

template <bool WRITE, bool QK = false>
__global__ __launch_bounds__(256) void sk_kernel(SkScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int RW = A.RW, K = A.K, M = A.M;
    const int W = K - M + 1;
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    const uint32_t halfM = 1u << (2 * M - 1);
    uint64_t* sw = smem + wid * (RW + 2);  // two zero words: span windows never leave the read
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    uint64_t kmers = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * 4 + wid; r < A.n_reads; r += nwaves) {
        const int L = rfl((int)A.lens[r]);
        const int nK = L - K + 1;
        uint32_t nseg = 0;
        if (nK > 0) {
            wave_sync();
            for (int w = lane; w < RW + 2; w += 64) sw[w] = w < RW ? A.words[r * RW + w] : 0ull;
            wave_sync();
            const uint64_t rbase = WRITE ? A.rec_base[r] : 0;
            const uint64_t ordv = (uint64_t)(A.ord_base + (uint32_t)r);
            int lo = 0;
            QWalk qw;  // (QK: lane 0's walk, its records broadcast to the wave)
            while (lo < nK) {
                int sig, nlo;
                uint32_t canon;
                bool qrev = false;
                if (QK) {
                    int rs = 0, e = 0;
                    bool rv = false;
                    if (lane == 0) qw.next(sw, lo, nK, K, M, maskM, rs, rv, e);
                    sig = __shfl(rs, 0, 64);
                    nlo = __shfl(e, 0, 64);
                    qrev = __shfl((int)rv, 0, 64) != 0;
                    const uint32_t sm = qw.code(sw, sig, M, maskM);
                    canon = qrev ? maskM - sm : sm;  // the bin's mmer code (not canonical)
                } else {
                    segment_at(sw, lo, lane, W, M, maskM, halfM, sig, canon);
                    nlo = sig + 1;
                }
                if (!in_part(canon, A.part, A.part_n)) {  // another pass's super-k-mer
                    lo = nlo;
                    continue;
                }
                const int n = QK ? nlo - lo : min(sig, nK - 1) - lo + 1;
                kmers += (uint64_t)n;
                if (WRITE && lane == 0) {
                    // one super-k-mer: k-mers lo..lo+n-1 share the signature at
                    // sig (binning.c:1004-1040 with the sticky window).  Span =
                    // bases lo .. lo+n+K-2 (<= 56 for K <= 31).
                    const uint64_t t = rbase + nseg;
                    const uint32_t sm = (uint32_t)(window64(sw, sig) >> (64 - 2 * M));
                    // complement wins (binning.c:1029-1040)
                    const uint64_t rev = QK ? (qrev ? 1ull : 0ull) : (sm < halfM ? 1ull : 0ull);
                    A.pay[3 * t + 0] = ordv | ((uint64_t)n << 32) | ((uint64_t)(sig - lo) << 38) | (rev << 44) |
                                       ((uint64_t)lo << 45);
                    A.pay[3 * t + 1] = window64(sw, lo);
                    A.pay[3 * t + 2] = window64(sw, lo + 32);
                    A.keys[t] = ((uint64_t)canon << 38) | ((uint64_t)(63 - n) << 32) | (uint32_t)t;
                }
                nseg++;
                lo = nlo;
            }
        }
        if (!WRITE && lane == 0) A.seg_count[r] = nseg;
    }
    if (!WRITE) {
        __shared__ uint64_t sh[4];
        const uint64_t tot = block_sum256((uint64_t)(lane == 0 ? kmers : 0), sh);
        if (threadIdx.x == 0) A.n_kmers[blockIdx.x] = tot;
    }
}

// map a call ordinal to the caller's read id
DEV int32_t id_of(uint32_t ord, const int32_t* read_ids, uint32_t id_off) {
    return read_ids ? read_ids[ord] : (int32_t)(ord + id_off);
}


// one record into a destination region: the binned layout (ordinal) or the
// routed one (read id), see SkScanArgs; then rw - 1 span words from base lo
// (n + K - 1 <= 2K - M bases: 2 words for K <= 31, 4 for K <= 63)
DEV void put_record(const SkScanArgs& A, uint64_t* o, uint32_t ord, uint64_t lo, uint64_t n, uint64_t so,
                    uint64_t rev, const uint64_t* sw, uint32_t sub = 0) {
    if (A.binned_fmt) {
        o[0] = (uint64_t)ord | (n << 32) | (so << 38) | (rev << 44) | (lo << 45);
    } else {
        const uint32_t id = (uint32_t)id_of(ord, A.read_ids, A.id_off);
        o[0] = (uint64_t)id | (lo << 32) | (n << 48) | (so << 54) | (rev << ROUTED_REV_BIT);
    }
    for (int w = 1; w < A.rw; w++) {
        uint64_t x = window64(sw, (int)lo + 32 * (w - 1));
        if (A.sub_stamp && w + 1 == A.rw) x = (x & ~SUB_MASK) | sub;  // (a bucket record's sub-bin, sub_room)
        o[w] = x;
    }
}

// The pieces of one record bound for destination regions: its owner rank or
// local bucket, or -- a split mmer's record -- its context sub-bin's bucket,
// cut in two (the first ne k-mers, the edge, then the rest) when its first
// k-mers lie in the edge.  row: the read's LDS row (the context bases).
// Returns the number of pieces; d[] their regions.
DEV uint32_t record_pieces(const SkScanArgs& A, uint32_t canon, int lo, int n, int so, bool rev,
                           const uint64_t* row, uint32_t (&d)[2], uint32_t (&sub)[2], int& ne) {
    ne = 0;
    sub[0] = sub[1] = 0;
    if (!A.bucket_map || !bm_has_entry(canon, A.M)) {
        d[0] = A.owner_map && bm_has_entry(canon, A.M) ? (uint32_t)A.owner_map[canon - (1u << (2 * A.M - 1))]
                                                       : dest_of(canon, A.G, A.dest_salt);
        return 1;
    }
    const uint32_t me = A.bucket_map[canon - (1u << (2 * A.M - 1))];
    const uint32_t b = bm_depth(me);
    if (!b) {
        d[0] = me & 1023u;
        return 1;
    }
    const uint64_t w = window64(row, lo + so + A.M);  // the read's bases after the signature
    const int e = sub_edge(so, n, A.K, A.M, b);
    if (e > 0 && e < n) {
        ne = e;
        sub[1] = sub_ctx(so - e, A.K, A.M, b, w, rev);
        d[0] = bm_bucket(me, A.sub_map, 0u);
        d[1] = bm_bucket(me, A.sub_map, sub[1]);
        return 2;
    }
    sub[0] = sub_ctx(so, A.K, A.M, b, w, rev);
    d[0] = bm_bucket(me, A.sub_map, sub[0]);
    return 1;
}

// The record pass's count loop plans each staged record once -- its pieces'
// destinations from the map entry me (bucket_map[canon - 2^(2M-1)], loaded by
// the caller) -- and caches the plan in the staged entry, so the placement
// loop repeats no map lookups.  Staged entry bits: lo 0..15 (< 512 for the
// thread kernel's reads), n 16..21, so 22..27, rev 28, row 29..37, canon
// 38..63; planned: canon -> d0 | d1 << 10 | ne << 20 | (pieces - 1) << 25, and
// the sub-bin depth b in bits 9..11.
DEV uint64_t record_plan(const SkScanArgs& A, uint64_t e, uint32_t me, const uint64_t* row) {
    const uint32_t canon = (uint32_t)(e >> 38);
    const int lo = (int)(e & 0x1FFu), n = (int)((e >> 16) & 63u), so = (int)((e >> 22) & 63u);
    const bool rev = ((e >> 28) & 1u) != 0;
    uint32_t d0 = 0, d1 = 0, b = 0, two = 0;
    int ne = 0;
    if (!A.bucket_map || !bm_has_entry(canon, A.M)) {  // (me: not loaded for such a code)
        d0 = A.owner_map && bm_has_entry(canon, A.M) ? (uint32_t)A.owner_map[canon - (1u << (2 * A.M - 1))]
                                                     : dest_of(canon, A.G, A.dest_salt);
    } else if (!(b = bm_depth(me))) {
        d0 = me & 1023u;
    } else {
        const uint64_t w = window64(row, lo + so + A.M);  // the read's bases after the signature
        const int ec = sub_edge(so, n, A.K, A.M, b);
        if (ec > 0 && ec < n) {
            ne = ec;
            two = 1;
            d0 = bm_bucket(me, A.sub_map, 0u);
            d1 = bm_bucket(me, A.sub_map, sub_ctx(so - ec, A.K, A.M, b, w, rev));
        } else {
            d0 = bm_bucket(me, A.sub_map, sub_ctx(so, A.K, A.M, b, w, rev));
        }
    }
    const uint64_t pk = (uint64_t)d0 | ((uint64_t)d1 << 10) | ((uint64_t)ne << 20) | ((uint64_t)two << 25);
    return (e & 0x3FFFFF01FFull) | ((uint64_t)b << 9) | (pk << 38);
}

// Add one record to a packed 16-bit LDS destination count (two per word) and
// return the count before it, aggregated over the wave: lanes bound for the
// same destination share one atomic (the lowest lane's) and take their
// offsets from the ballot.  With few destinations (ranks) every lane of a wave
// would otherwise hit the same word and the LDS would serialise 64 returning
// atomics per instruction (1.97 ms vs 0.27 ms for the pass at one rank).
DEV uint32_t wave_dest_add(uint32_t* cnt2, uint32_t d) {
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t off = 0;
    bool pending = true;
    for (;;) {
        const uint64_t rem = __ballot(pending);
        if (!rem) break;
        const int leader = __builtin_ctzll(rem);
        const uint32_t ld = (uint32_t)__shfl((int)d, leader, 64);
        const bool mine = pending && d == ld;
        const uint64_t m = __ballot(mine);
        uint32_t b = 0;
        if (lane == leader) {
            const uint32_t sh = 16u * (ld & 1u);
            b = (atomicAdd(&cnt2[ld >> 1], (uint32_t)__popcll(m) << sh) >> sh) & 0xFFFFu;
        }
        b = (uint32_t)__shfl((int)b, leader, 64);
        if (mine) {
            off = b + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            pending = false;
        }
    }
    return off;
}

// LDS row of one read in sk_thread_kernel: the read's words, then zero words
// so that every span window (up to 4 words past the first base) stays inside
__device__ __host__ inline int sk_row_words(int RW, int rw) { return RW + (rw > 3 ? rw - 1 : 2); }

// Thread-per-read variant for short reads (RW <= SK_THREAD_RW): a block
// stages SKT reads in LDS rows and each lane walks its own read's sticky
// chain serially.  The wave-per-read kernel above keeps 64 lanes busy on a
// window of only K-M+1 positions; one lane per read does the same argmax
// with no cross-lane reduction and no idle lanes.  The window of mmer scores
// is walked with a 2-bit shift per position (two LDS reads per segment).
// The write pass stages each record as one u64 in LDS and the block then
// writes its (contiguous) record range with coalesced stores.
constexpr int SK_THREAD_RW = 16;
// staged records per block (8 B each): 256 reads of 150 bp make ~2.5 K; a
// block past it stores the rest directly.  With the per-destination arrays
// (16-bit counts, two per word) and the read rows the block fits four to a CU.
constexpr int SKT = 512;              // reads (lanes) per block
constexpr uint32_t SK_STAGE = 4992;   // (two blocks per CU)
static_assert(SKT <= 512, "a staged record keeps its row in 9 bits");
constexpr uint32_t SK_MAX_DEST = 1024;  // destination regions (ranks or buckets)

#ifdef KB_BIN_PROF
// record pass phases (thread 0's clock at the block's barriers, summed over
// blocks): row loads, walk, per-destination counts + reservations, placement
__device__ unsigned long long g_sk_prof[8];
#define SKPROF(ph)                                        \
    do {                                                  \
        if (tid == 0) {                                   \
            const unsigned long long t1_ = clock64();     \
            atomicAdd(&g_sk_prof[ph], t1_ - skt_);        \
            skt_ = t1_;                                   \
        }                                                 \
    } while (0)
#else
#define SKPROF(ph) do {} while (0)
#endif
// a value the compiler must keep in a VGPR and cannot see through
DEV uint32_t vreg(uint32_t v) {
    asm("" : "+v"(v));
    return v;
}

// QK (K < 2M): the reference's incremental branch is live (binning.c:992-1021:
// j runs K-M .. M-1, appending bases to a score it never trims, in int
// arithmetic that wraps).  Each lane then walks its read k-mer by k-mer with
// the reference's own state (score, rev_score, max_score, is_rev, signature),
// and a record is a run of k-mers with one signature position -- its so, rev
// and mmer are whatever that state says, not the window's leftmost argmax
template <bool WRITE, bool QK = false>
__global__ __launch_bounds__(SKT) void sk_thread_kernel(SkScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const int RW = A.RW, K = A.K, M = A.M;
    const int W = K - M + 1;  // <= 57 (K <= 63): mmer starts lo..lo+W-1 end inside one 64-base window pair
    const int RS = sk_row_words(RW, A.rw);  // row stride: zero words past the read
    const int sh = 64 - 2 * M;
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    const uint32_t halfM = 1u << (2 * M - 1);
    const bool one_word = K <= 31 && M <= 12;  // (scores < 2^24 keep 8 bits for the offset)
    const uint32_t tid = threadIdx.x;
    uint64_t* stg = smem + SKT * RS;  // WRITE: [SK_STAGE] {lo, n, so, rev, row, canon}
    __shared__ uint32_t span_end;
    __shared__ unsigned long long s_base;
    __shared__ uint32_t dcnt2[SK_MAX_DEST / 2];  // per-destination counts, 16 bits each (< SK_STAGE)
    __shared__ uint32_t dbase[SK_MAX_DEST];  // reserved slot in the region (< region_cap < 2^32)
    const bool route = WRITE && A.regions;          // records to destination regions, any order
    const bool alloc = WRITE && (A.rec_ctr || route);  // records placed by block allocation
    const bool rounds = alloc && !(route && A.G > 64);  // see the walk below
    uint64_t kmers = 0;
#ifdef KB_BIN_PROF
    unsigned long long skt_ = clock64();
#endif
    for (uint64_t r0 = (uint64_t)blockIdx.x * SKT; r0 < A.n_reads; r0 += (uint64_t)gridDim.x * SKT) {
        const uint32_t nrows = (uint32_t)min<uint64_t>(SKT, A.n_reads - r0);
        __syncthreads();
        {
            // (the block's reads into LDS rows, eight loads in flight per lane)
            const uint32_t nw = nrows * (uint32_t)RW;
            for (uint32_t i0 = tid; i0 < nw; i0 += 8u * SKT) {
                uint64_t v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const uint32_t i = i0 + (uint32_t)u * SKT;
                    v[u] = i < nw ? A.words[r0 * RW + i] : 0ull;
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const uint32_t i = i0 + (uint32_t)u * SKT;
                    if (i >= nw) break;
                    const uint32_t row = i / (uint32_t)RW, col = i - row * (uint32_t)RW;
                    smem[row * RS + col] = v[u];
                }
            }
        }
        if (tid < nrows)
            for (int w = RW; w < RS; w++) smem[tid * RS + w] = 0;
        if (tid == 0) span_end = 0;
        __syncthreads();
        SKPROF(0);
        const uint64_t bfirst = WRITE && !alloc ? A.rec_base[r0] : 0;
        // Block allocation onto few counters (ranks, or the one record counter)
        // runs in rounds: a walk whose record finds the stage full stops there
        // and resumes after the block has written the stage out.  (Writing such
        // records one by one took a global atomic per record on a few hot
        // counters -- 256 reads of 150 bp average ~2.5 K records, so about half
        // the blocks overflowed: 1.97 ms at one rank.)  With 1024 local buckets
        // the per-record atomics spread out and are cheaper than a round.
        const uint64_t r = r0 + tid;
        const uint64_t* sw = smem + tid * RS;
        const int nK = tid < nrows ? (int)A.lens[r] - K + 1 : 0;
        const uint64_t rbase = WRITE && !alloc && tid < nrows ? A.rec_base[r] : 0;
        uint32_t nseg = 0;
        int lo = 0;
        // (QK) the reference's walk state (QWalk), and the record it closed
        // (kept across a stage-full round: the walk does not repeat)
        QWalk qw;
        int q_lo = -1, q_e = 0, q_rsig = 0;
        bool q_rrev = false;
        for (;;) {
            while (lo < nK) {
                // leftmost strict argmax of the canonical score over the window
                int best = -1, sig = lo;
                uint32_t bsm = 0;
                int nlo = 0;  // the next record's first k-mer
                if (QK) {
                    if (q_lo != lo) {  // (a stage-full round keeps the record it closed)
                        qw.next(sw, lo, nK, K, M, maskM, q_rsig, q_rrev, q_e);
                        q_lo = lo;
                    }
                    sig = q_rsig;
                    const uint32_t sm = qw.code(sw, sig, M, maskM);
                    best = (int)(q_rrev ? maskM - sm : sm);  // the bin's mmer code
                    bsm = q_rrev ? 0u : halfM;               // (rev below: bsm < halfM)
                    nlo = q_e;
                } else if (one_word) {
                    // K <= 31: the window's W mmers all lie in the 64-bit word at
                    // lo, so each score is one shift of it (no shifting chain),
                    // and the argmax is a max over (score << 8 | 255 - offset):
                    // larger score first, then the leftmost position.  In
                    // 32-bit halves: position i's mmer sits at bit sh - 2i,
                    // inside the high half for i < 17 - M, across both for
                    // i < 16, in the low half after -- one bit-field extract
                    // (two across), and both orientations' keys in one max3
                    // (the complement's key is the forward key ^ maskM << 8)
                    const uint64_t x = window64(sw, lo);
                    const uint32_t xh = (uint32_t)(x >> 32), xl = (uint32_t)x;
                    // (loop constants held in VGPRs: a VOP3 reads one SGPR on gfx9)
                    const uint32_t xc = vreg(maskM << 8), w2 = vreg(2u * (uint32_t)M);
                    const int e1 = min(W, 17 - M), e2 = min(W, 16);
                    uint32_t bk = 0;
                    const auto hi_at = [&](int p) {
                        const uint32_t k =
                            vreg((__builtin_amdgcn_ubfe(xh, (uint32_t)(sh - 32 - 2 * p), w2) << 8) | (uint32_t)(255 - p));
                        bk = max(max(bk, k), k ^ xc);
                    };
                    const auto mid_at = [&](int p) {
                        const uint32_t k = vreg(((__builtin_amdgcn_alignbit(xh, xl, (uint32_t)(sh - 2 * p)) & maskM) << 8) |
                                                (uint32_t)(255 - p));
                        bk = max(max(bk, k), k ^ xc);
                    };
                    const auto lo_at = [&](int p) {
                        const uint32_t k =
                            vreg((__builtin_amdgcn_ubfe(xl, (uint32_t)(sh - 2 * p), w2) << 8) | (uint32_t)(255 - p));
                        bk = max(max(bk, k), k ^ xc);
                    };
                    // (unrolled by hand: the loop bounds are uniform but not constant)
                    int p = 0;
                    for (; p + 2 <= e1; p += 2) hi_at(p), hi_at(p + 1);
                    if (p < e1) hi_at(p++);
                    for (; p + 2 <= e2; p += 2) mid_at(p), mid_at(p + 1);
                    if (p < e2) mid_at(p++);
                    for (; p + 3 <= W; p += 3) lo_at(p), lo_at(p + 1), lo_at(p + 2);
                    for (; p < W; p++) lo_at(p);
                    const int i = 255 - (int)(bk & 255u);
                    sig = lo + i;
                    best = (int)(bk >> 8);
                    bsm = (uint32_t)(x >> (sh - 2 * i)) & maskM;
                } else {
                    uint64_t x = window64(sw, lo), y = window64(sw, lo + 32);
                    for (int p = lo; p < lo + W; p++) {
                        const uint32_t sm = (uint32_t)(x >> sh);
                        const int c = (int)(sm >= halfM ? sm : maskM - sm);
                        if (c > best) {
                            best = c;
                            sig = p;
                            bsm = sm;
                        }
                        x = (x << 2) | (y >> 62);
                        y <<= 2;
                    }
                }
                if (!QK) nlo = sig + 1;
                const uint64_t n = QK ? (uint64_t)(nlo - lo) : (uint64_t)(min(sig, nK - 1) - lo + 1);
                if (!in_part((uint32_t)best, A.part, A.part_n)) {  // another pass's super-k-mer
                    lo = nlo;
                    continue;
                }
                if (WRITE) {
                    const uint64_t rev = bsm < halfM ? 1ull : 0ull;  // complement wins (binning.c:1029-1040)
                    const uint64_t e = (uint64_t)lo | (n << 16) | ((uint64_t)(sig - lo) << 22) | (rev << 28) |
                                       ((uint64_t)tid << 29) | ((uint64_t)(uint32_t)best << 38);
                    // one stage slot per record: one atomic per wave (the lanes
                    // still walking take consecutive slots) -- 512 lanes' atomics
                    // on the one LDS word serialised every segment round
                    uint64_t loc;
                    if (alloc) {
                        const uint64_t am = __ballot(1);
                        const int lead = __builtin_ctzll(am);
                        uint32_t wb = 0;
                        if ((int)(tid & 63u) == lead) wb = atomicAdd(&span_end, (uint32_t)__popcll(am));
                        wb = (uint32_t)__shfl((int)wb, lead, 64);
                        loc = (uint64_t)wb + __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
                    } else {
                        loc = rbase + nseg - bfirst;
                    }
                    if (loc < SK_STAGE) {
                        stg[loc] = e;
                    } else if (rounds) {
                        break;  // stage full: resume at this record in the next round
                    } else if (route) {  // many destinations: each piece its own slot
                        uint32_t d[2], sub[2];
                        int ne;
                        const uint32_t np_ = record_pieces(A, (uint32_t)best, lo, (int)n, sig - lo, rev != 0, sw, d, sub, ne);
                        for (uint32_t q = 0; q < np_; q++) {
                            const int cut = q ? ne : 0;
                            const uint64_t pn = np_ == 2 && q == 0 ? (uint64_t)ne : n - (uint64_t)cut;
                            const uint64_t i = atomicAdd(&A.dest_ctr[d[q]], 1ull);
                            if (i < region_room(A.region_base, A.region_cap, d[q]))
                                put_record(A, A.regions + (region_off(A.region_base, A.region_cap, d[q]) + i) * (uint64_t)A.rw,
                                           A.ord_base + (uint32_t)r, (uint64_t)(lo + cut), pn,
                                           (uint64_t)(sig - lo - cut), rev, sw, sub[q]);
                        }
                    }
                    if (loc >= SK_STAGE && !route && !alloc) {  // ordered records beyond the staging area: direct (scattered) stores
                        const uint64_t t = rbase + nseg;
                        A.pay[3 * t + 0] = (uint64_t)(A.ord_base + (uint32_t)r) | (n << 32) |
                                           ((uint64_t)(sig - lo) << 38) | (rev << 44) | ((uint64_t)lo << 45);
                        A.pay[3 * t + 1] = window64(sw, lo);
                        A.pay[3 * t + 2] = window64(sw, lo + 32);
                        A.keys[t] = ((uint64_t)(uint32_t)best << 38) | ((63ull - n) << 32) | (uint32_t)t;
                    }
                }
                kmers += n;
                nseg++;
                lo = nlo;
            }
            if (!WRITE && tid < nrows) A.seg_count[r] = nseg;
            if (WRITE && !alloc && nseg)
                atomicMax(&span_end, (uint32_t)min<uint64_t>(rbase + nseg - bfirst, SK_STAGE));
            if (!WRITE) break;
            __syncthreads();
            SKPROF(1);
            const uint32_t span = min(span_end, SK_STAGE);
            if (route) {
                // per destination: count, reserve a range, place (LDS cursors)
                for (uint32_t d = tid; d < (A.G + 1) / 2; d += SKT) dcnt2[d] = 0;
                __syncthreads();
                const bool agg = A.G <= 64;  // ranks, not local buckets: aggregate per wave
                const uint32_t half = 1u << (2 * M - 1);
                // two records per trip: both map loads in flight together
                for (uint32_t i0 = tid; i0 < span; i0 += 2 * SKT) {
                    const uint32_t i1 = i0 + SKT;
                    const bool v1 = i1 < span;
                    const uint64_t e0 = stg[i0], e1 = v1 ? stg[i1] : e0;
                    uint32_t me0 = 0, me1 = 0;
                    if (A.bucket_map) {  // (codes below half: no entry, record_plan hashes them)
                        const uint32_t c0 = (uint32_t)(e0 >> 38), c1 = (uint32_t)(e1 >> 38);
                        me0 = c0 >= half ? A.bucket_map[c0 - half] : 0u;
                        me1 = c1 >= half ? A.bucket_map[c1 - half] : 0u;
                    }
                    const uint64_t p0 = record_plan(A, e0, me0, smem + ((e0 >> 29) & 0x1FFu) * RS);
                    const uint64_t p1 = record_plan(A, e1, me1, smem + ((e1 >> 29) & 0x1FFu) * RS);
                    stg[i0] = p0;
                    if (v1) stg[i1] = p1;
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        const uint64_t pl = u ? p1 : p0;
                        if (u && !v1) break;
                        const uint32_t np_ = 1u + (uint32_t)((pl >> 63) & 1u);
                        for (uint32_t q = 0; q < np_; q++) {
                            const uint32_t dq = (uint32_t)(pl >> (38 + 10 * q)) & 1023u;
                            if (agg)
                                wave_dest_add(dcnt2, dq);
                            else
                                atomicAdd(&dcnt2[dq >> 1], 1u << (16 * (dq & 1)));
                        }
                    }
                }
                __syncthreads();
                for (uint32_t d = tid; d < A.G; d += SKT) {
                    const uint32_t nd = (dcnt2[d >> 1] >> (16 * (d & 1))) & 0xFFFFu;
                    dbase[d] = nd ? (uint32_t)min<unsigned long long>(
                                        atomicAdd(&A.dest_ctr[d], (unsigned long long)nd), 0xFFFFFFFFull)
                                  : 0u;
                }
                __syncthreads();
                for (uint32_t d = tid; d < (A.G + 1) / 2; d += SKT) dcnt2[d] = 0;
                __syncthreads();
                SKPROF(2);
                for (uint32_t i = tid; i < span; i += SKT) {
                    const uint64_t e = stg[i];  // (planned)
                    const uint32_t row = (uint32_t)((e >> 29) & 0x1FFu);
                    const int lo = (int)(e & 0x1FFu), n = (int)((e >> 16) & 63u), so = (int)((e >> 22) & 63u);
                    const bool rev = ((e >> 28) & 1u) != 0;
                    const uint32_t b = (uint32_t)((e >> 9) & 7u), np_ = 1u + (uint32_t)((e >> 63) & 1u);
                    const int ne = (int)((e >> 58) & 31u);
                    const uint64_t* rw_ = smem + row * RS;
                    // the pieces' sub-bins (the stamp), from the read's bases in LDS
                    uint32_t sub[2] = {0u, 0u};
                    if (A.sub_stamp && b) {
                        const uint64_t w = window64(rw_, lo + so + M);
                        if (np_ == 2) sub[1] = sub_ctx(so - ne, K, M, b, w, rev);
                        else sub[0] = sub_ctx(so, K, M, b, w, rev);
                    }
                    for (uint32_t q = 0; q < np_; q++) {
                        const uint32_t dq = (uint32_t)(e >> (38 + 10 * q)) & 1023u;
                        const uint64_t slot =
                            (uint64_t)dbase[dq] +
                            (agg ? wave_dest_add(dcnt2, dq)
                                 : ((atomicAdd(&dcnt2[dq >> 1], 1u << (16 * (dq & 1))) >> (16 * (dq & 1))) & 0xFFFFu));
                        if (slot >= region_room(A.region_base, A.region_cap, dq)) continue;  // counted: the caller retries bigger
                        const int cut = q ? ne : 0;
                        const int pn = np_ == 2 && q == 0 ? ne : n - cut;
                        put_record(A, A.regions + (region_off(A.region_base, A.region_cap, dq) + slot) * (uint64_t)A.rw,
                                   A.ord_base + (uint32_t)(r0 + row), (uint64_t)(lo + cut), (uint64_t)pn,
                                   (uint64_t)(so - cut), rev ? 1u : 0u, rw_, sub[q]);
                    }
                }
            } else {
                if (alloc) {  // the block's staged records get one contiguous range
                    if (tid == 0) s_base = span ? atomicAdd(A.rec_ctr, (unsigned long long)span) : 0ull;
                    __syncthreads();
                }
                const uint64_t tbase = alloc ? (uint64_t)s_base : bfirst;
                for (uint32_t i = tid; i < span; i += SKT) {
                    const uint64_t e = stg[i];
                    const uint32_t elo = (uint32_t)(e & 0xFFFFu), row = (uint32_t)((e >> 29) & 0x1FFu);
                    const uint64_t en = (e >> 16) & 63u, so = (e >> 22) & 63u, rev = (e >> 28) & 1u;
                    const uint64_t* rw_ = smem + row * RS;
                    const uint64_t t = tbase + i;
                    A.pay[3 * t + 0] = (uint64_t)(A.ord_base + (uint32_t)(r0 + row)) | (en << 32) | (so << 38) |
                                       (rev << 44) | ((uint64_t)elo << 45);
                    A.pay[3 * t + 1] = window64(rw_, (int)elo);
                    A.pay[3 * t + 2] = window64(rw_, (int)elo + 32);
                    A.keys[t] = ((e >> 38) << 38) | ((63ull - en) << 32) | (uint32_t)t;
                }
            }
            // another round while a walk stopped at the full stage
#ifdef KB_BIN_PROF
            __syncthreads();
            SKPROF(3);
#endif
            if (!rounds || !__syncthreads_or(lo < nK)) break;
            if (tid == 0) span_end = 0;
            __syncthreads();
        }
    }
    if (!WRITE || (alloc && (!route || A.binned_fmt))) {  // per-block k-mer sums (sk_kmers_total_kernel)
        __shared__ unsigned long long shs;
        if (tid == 0) shs = 0;
        __syncthreads();
        uint64_t w = kmers;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) w += (uint64_t)__shfl_xor((long long)w, off, 64);
        if ((tid & 63u) == 0 && w) atomicAdd(&shs, (unsigned long long)w);
        __syncthreads();
        if (tid == 0) A.n_kmers[blockIdx.x] = shs;
    }
}

uint64_t sk_blocks(uint64_t n_reads, int RW) {
    if (!n_reads) return 0;
    if (RW <= SK_THREAD_RW) return std::min<uint64_t>((n_reads + SKT - 1) / SKT, 8192);
    return std::min<uint64_t>((n_reads + 3) / 4, 4096);
}

__global__ void sk_kmers_total_kernel(const unsigned long long* part, uint64_t n, unsigned long long* out) {
    __shared__ uint64_t sh[4];
    uint64_t v = 0;
    for (uint64_t i = threadIdx.x; i < n; i += 256) v += part[i];
    v = block_sum256(v, sh);
    if (threadIdx.x == 0) *out += v;
}

hipError_t launch_sk_kmers_total(const unsigned long long* part, uint64_t n, unsigned long long* out,
                                 hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(sk_kmers_total_kernel, dim3(1), dim3(256), 0, s, part, n, out);
    return hipGetLastError();
}

hipError_t launch_sk(const SkScanArgs& a, bool write, hipStream_t s) {
    if (!a.n_reads) return hipSuccess;
    const uint64_t blocks = sk_blocks(a.n_reads, a.RW);
    if (a.RW <= SK_THREAD_RW) {
        const size_t lds = (size_t)SKT * sk_row_words(a.RW, a.rw) * sizeof(uint64_t) +
                           (write ? SK_STAGE * sizeof(uint64_t) : 0);
        if (a.K < 2 * a.M) {  // (QK: the reference's incremental branch is live)
            if (write)
                hipLaunchKernelGGL((sk_thread_kernel<true, true>), dim3((unsigned)blocks), dim3(SKT), lds, s, a);
            else
                hipLaunchKernelGGL((sk_thread_kernel<false, true>), dim3((unsigned)blocks), dim3(SKT), lds, s, a);
        } else if (write) {
            hipLaunchKernelGGL(sk_thread_kernel<true>, dim3((unsigned)blocks), dim3(SKT), lds, s, a);
        } else {
            hipLaunchKernelGGL(sk_thread_kernel<false>, dim3((unsigned)blocks), dim3(SKT), lds, s, a);
        }
        return hipGetLastError();
    }
    const size_t lds = (size_t)4 * (a.RW + 2) * sizeof(uint64_t);
    if (a.K < 2 * a.M) {  // (QK: a long read's walk on one lane of its wave)
        if (write)
            hipLaunchKernelGGL((sk_kernel<true, true>), dim3((unsigned)blocks), dim3(256), lds, s, a);
        else
            hipLaunchKernelGGL((sk_kernel<false, true>), dim3((unsigned)blocks), dim3(256), lds, s, a);
    } else if (write) {
        hipLaunchKernelGGL(sk_kernel<true>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    } else {
        hipLaunchKernelGGL(sk_kernel<false>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    }
    return hipGetLastError();
}

// records into bin order, structure of arrays (the bin kernel streams them)
__global__ __launch_bounds__(256) void sk_gather_kernel(const uint64_t* __restrict__ keys,
                                                        const uint64_t* __restrict__ pay, uint64_t R,
                                                        uint64_t* __restrict__ srec) {
    for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k < R; k += (uint64_t)gridDim.x * 256) {
        const uint64_t t = (uint32_t)keys[k];
        const uint64_t hd = pay[3 * t], w0 = pay[3 * t + 1];
        reinterpret_cast<uint4*>(srec)[k] = make_uint4((uint32_t)hd, (uint32_t)(hd >> 32), (uint32_t)w0,
                                                        (uint32_t)(w0 >> 32));  // (header, word 0) pairs
        srec[2 * R + k] = pay[3 * t + 2];
    }
}

hipError_t launch_sk_gather(const uint64_t* keys, const uint64_t* pay, uint64_t R, uint64_t* srec,
                            hipStream_t s) {
    if (!R) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((R + 255) / 256, 8192);
    hipLaunchKernelGGL(sk_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, s, keys, pay, R, srec);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// routing (one process per GPU): the sender's records go to
// owner(mmer) in the routed record format of route_kernel (kbin_kernels.hip)
// -- header {id | i0 << 32 | n << 48 | sig_off << 54 | rev << 60}, then the
// span words (rev: kbin_internal.h ROUTED_REV_BIT) --
// destination-major, read order within a destination; the receiver turns
// them back into binned records.
// ---------------------------------------------------------------------------


__global__ __launch_bounds__(256) void route_dest_kernel(const uint64_t* __restrict__ keys, uint64_t R,
                                                         uint32_t G, const uint8_t* __restrict__ owner_map, int M,
                                                         uint64_t* __restrict__ dkeys,
                                                         unsigned long long* __restrict__ counts) {
    __shared__ uint32_t hist[64];
    if (threadIdx.x < 64) hist[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < R; t += (uint64_t)gridDim.x * 256) {
        const uint32_t mm = (uint32_t)(keys[t] >> 38);
        const uint32_t d = owner_map && bm_has_entry(mm, M) ? (uint32_t)owner_map[mm - (1u << (2 * M - 1))]
                                                            : owner_of_mmer(mm, G);
        dkeys[t] = ((uint64_t)d << 32) | (uint32_t)t;
        atomicAdd(&hist[d], 1u);
    }
    __syncthreads();
    if (threadIdx.x < G && hist[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)hist[threadIdx.x]);
}

hipError_t launch_route_dest(const uint64_t* keys, uint64_t R, uint32_t G, const uint8_t* owner_map, int M,
                             uint64_t* dkeys,
                             unsigned long long* counts, hipStream_t s) {
    if (!R) return hipSuccess;
    if (G < 1 || G > 64) return hipErrorInvalidValue;
    const uint64_t blocks = std::min<uint64_t>((R + 255) / 256, 2048);
    hipLaunchKernelGGL(route_dest_kernel, dim3((unsigned)blocks), dim3(256), 0, s, keys, R, G, owner_map, M, dkeys, counts);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void route_pack_binned_kernel(const uint64_t* __restrict__ sorted,
                                                                const uint64_t* __restrict__ pay, uint64_t R,
                                                                int rw, const int32_t* __restrict__ read_ids,
                                                                uint32_t id_off, uint64_t* __restrict__ out) {
    for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k < R; k += (uint64_t)gridDim.x * 256) {
        const uint64_t t = (uint32_t)sorted[k];
        const uint64_t hd = pay[3 * t];
        const uint32_t id = (uint32_t)id_of((uint32_t)hd, read_ids, id_off);
        const uint64_t n = (hd >> 32) & 63u, so = (hd >> 38) & 63u, lo = (hd >> 45) & 0xFFFFu, rev = (hd >> 44) & 1u;
        uint64_t* o = out + k * (uint64_t)rw;
        o[0] = (uint64_t)id | (lo << 32) | (n << 48) | (so << 54) | (rev << ROUTED_REV_BIT);
        o[1] = pay[3 * t + 1];
        if (rw >= 3) o[2] = pay[3 * t + 2];
        for (int w = 3; w < rw; w++) o[w] = 0;  // (K <= 31 spans fit two words)
    }
}

hipError_t launch_route_pack_binned(const uint64_t* sorted, const uint64_t* pay, uint64_t R, int rw,
                                    const int32_t* read_ids, uint32_t id_off, uint64_t* out,
                                    hipStream_t s) {
    if (!R) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((R + 255) / 256, 8192);
    hipLaunchKernelGGL(route_pack_binned_kernel, dim3((unsigned)blocks), dim3(256), 0, s, sorted, pay, R, rw,
                       read_ids, id_off, out);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void sk_convert_kernel(const uint64_t* __restrict__ recs, uint64_t n_rec,
                                                         int rw, uint64_t off, int M, int K, uint64_t* __restrict__ pay,
                                                         uint64_t* __restrict__ keys, uint32_t* status,
                                                         unsigned long long* n_kmers) {
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    bool neg = false;
    uint64_t kmers = 0;
    for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k < n_rec; k += (uint64_t)gridDim.x * 256) {
        const uint64_t* r = recs + k * (uint64_t)rw;
        const uint64_t h = r[0];
        const uint64_t w0 = r[1], w1 = rw >= 3 ? r[2] : 0ull;
        const uint32_t id = (uint32_t)h;
        const uint64_t lo = (h >> 32) & 0xFFFFu, n = (h >> 48) & 63u, so = (h >> 54) & 63u;
        const uint32_t sm = (uint32_t)(span_window(w0, w1, 0ull, 0ull, (int)so) >> (64 - 2 * M));
        const bool rev = routed_rev(h, sm, K, M);  // complement wins (binning.c:1029-1040)
        const uint32_t canon = rev ? maskM - sm : sm;
        neg |= (int32_t)id < 0;
        const uint64_t t = off + k;
        pay[3 * t + 0] = (uint64_t)id | (n << 32) | (so << 38) | ((uint64_t)rev << 44) | (lo << 45);
        pay[3 * t + 1] = w0;
        pay[3 * t + 2] = w1;
        keys[t] = ((uint64_t)canon << 38) | ((63ull - n) << 32) | (uint32_t)t;
        kmers += n;
    }
    if (neg) atomicOr(status, ST_NEG_ID);
    __shared__ uint64_t sh[4];
    kmers = block_sum256(kmers, sh);
    if (threadIdx.x == 0 && kmers) atomicAdd(n_kmers, (unsigned long long)kmers);
}

hipError_t launch_sk_convert(const uint64_t* recs, uint64_t n_rec, int rw, uint64_t off, int M, int K,
                             uint64_t* pay, uint64_t* keys, uint32_t* status, unsigned long long* n_kmers,
                             hipStream_t s) {
    if (!n_rec) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((n_rec + 255) / 256, 8192);
    hipLaunchKernelGGL(sk_convert_kernel, dim3((unsigned)blocks), dim3(256), 0, s, recs, n_rec, rw, off, M, K, pay,
                       keys, status, n_kmers);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// phase B: one workgroup per mmer bin
// ---------------------------------------------------------------------------
#ifdef KB_BIN_PROF
// per-phase cycle accounting (tid 0, between barriers): a diagnostic build only
constexpr int PROF_N = 37;
__device__ unsigned long long g_bin_prof[PROF_N];
#define PROF_MARK(ph)                                              \
    do {                                                           \
        if (tid == 0) {                                            \
            const unsigned long long _t = clock64();               \
            pacc[ph] += _t - pt;                                   \
            pt = _t;                                               \
        }                                                          \
    } while (0)
#define PROF_CNT(i, v) do { if (tid == 0) pacc[i] += (v); } while (0)
#define PROF_PARAMS , unsigned long long *pacc, unsigned long long &pt
#define PROF_ARGS , pacc, pt
#else
#define PROF_PARAMS
#define PROF_ARGS
#define PROF_MARK(ph) do {} while (0)
#define PROF_CNT(i, v) do {} while (0)
#endif

#ifdef KB_BIN_PROF
#define KB_BIN_ABL  // (diagnostic builds: KB_BIN_ABLATE switches parts of bin_kernel off)
#endif
#ifndef KB_BIN_THREADS
#define KB_BIN_THREADS 1024
#endif
constexpr int BIN_THREADS = KB_BIN_THREADS;
static_assert((BIN_THREADS & (BIN_THREADS - 1)) == 0 && BIN_THREADS >= 256 && BIN_THREADS <= 1024,
              "bin_kernel's LDS carve and strides assume a power-of-two workgroup (768 faulted, r06)");
#ifndef KB_WIN_LOADS
#define KB_WIN_LOADS 4  // stage loads in flight per thread in the id windows (8: more spills, measured slower)
#endif  // (A/B builds: -DKB_BIN_THREADS=512 with KB_BIN_TS_LOG2=12; powers of two only -- 768 faults)
constexpr int BIN_STACK = 32;

DEV uint64_t lds_load_u64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct alignas(16) BinShared {
    uint32_t n_keys, overflow, cur_p, cur_l, item, n_stage, part0;
    // the partition stack's depth, one word per partition parity: a partition
    // (re)starts its stack without a barrier after the waves read the last
    // one's empty stack, so it must not write the word a lagging wave is
    // about to read (bin_body; round 4's KB_EDEVICE at r4f6)
    uint32_t spq[2];
    uint32_t n_single;  // pre-filter: keys seen once in this partition
    uint32_t maxc;      // the partition's longest kept list (the LDS id windows)
    uint32_t sumc;      // the partition's occurrences counted in its table (the finalize's invariant)
    uint32_t rk_min, rk_max, dup;  // ranked bins: ordinal range; a bitmap bit set twice
    uint32_t ts;        // LDS table slots of the next partition (<= the carved TS)
    unsigned long long wkey;  // LDS id windows: cursor << 32 | entry << 16 | scan index of the next window's start
    unsigned long long e0, i0, stage_base;
    uint32_t flat_idx, fa, fb, l0;
    uint32_t stack_p[BIN_STACK], stack_l[BIN_STACK];
    uint64_t red[BIN_THREADS / 64];
    unsigned long long dummy[64];  // zero: the claim target of lanes with nothing to claim
#ifdef KB_BIN_PROF
    // (diagnostic builds) the phase accumulators and the last stamp, in LDS:
    // kept in private memory (scratch) each stamp's update waited out the
    // wave's outstanding global stores, charging their drain to the phase
    unsigned long long prof[PROF_N + 1];
#endif
};
static_assert(sizeof(BinShared) % 16 == 0, "LDS carve must stay 16-B aligned (guide G17)");

// block-wide exclusive scan of two u32 quantities packed in a u64 (each lane's
// value < 2^32, totals < 2^32)
DEV void lds_barrier();
DEV uint64_t block_excl_scan_u64(uint64_t v, uint64_t* red, uint64_t& total, bool lds_only = false) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t inc = wave_incl_scan(v, lane);
    if (lane == 63) red[wid] = inc;
    if (lds_only) lds_barrier();
    else __syncthreads();
    uint64_t wp = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BIN_THREADS / 64; w++) {
        const uint64_t x = red[w];
        if (w < wid) wp += x;
        tot += x;
    }
    if (lds_only) lds_barrier();
    else __syncthreads();
    total = tot;
    return wp + inc - v;
}

constexpr int BIN_WAVES = BIN_THREADS / 64;
// per-wave k-mer ring: flushes of 128 k-mers (2 per lane) for one-word keys,
// 64 (1 per lane) for two-word keys, whose table and ring take twice the LDS
template <int KW>
constexpr uint32_t bin_q() { return KW == 1 ? 256u : 128u; }

DEV uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// partition of a k-mer inside its bin (independent of the table hash)
DEV uint32_t part_of(uint64_t code) { return (uint32_t)((code * 0x9E3779B97F4A7C15ull) >> 40); }

// ---- the bin table's key of a k-mer (the mmer is implied by the bin)
//   KW = 1 (K <= 31): a = 2K-bit code + 1 (0 = empty slot)
//   KW = 2 (K <= 63): the 2K-bit code split at bit 63 as in the table engine
//                     (kbin_internal.h): a = (code >> 63) + 1 claims the slot,
//                     b = (code & (2^63 - 1)) | PUB is published after it
template <int KW>
struct TKey;
template <>
struct TKey<1> {
    uint64_t a;
    // the table bucket (low bits): the top bits of one 32-bit multiplicative
    // hash of the folded code, bit-reversed -- 4 instructions where a full
    // 64-bit mix took ~15 (bucket overflow measured the same on genome k-mers:
    // 6.3 % vs 6.1 % of the keys past their home bucket at 60 % fill)
    DEV uint32_t hash() const { return __builtin_bitreverse32(((uint32_t)a ^ (uint32_t)(a >> 32)) * 0x85EBCA6Bu); }
    DEV uint32_t part() const { return part_of(a - 1ull); }
    DEV void code(uint64_t& hi, uint64_t& lo) const {
        hi = 0;
        lo = a - 1ull;
    }
};
template <>
struct TKey<2> {
    uint64_t a, b;
    DEV uint64_t h64() const { return mix64(a ^ (b * 0xD6E8FEB86659FD93ull)); }
    DEV uint32_t hash() const { return (uint32_t)h64(); }
    DEV uint32_t part() const { return (uint32_t)(h64() >> 40); }
    DEV void code(uint64_t& hi, uint64_t& lo) const {
        hi = (a - 1ull) >> 1;
        lo = ((a - 1ull) << 63) | (b & ~PUB);
    }
};

// a record's span bases in registers, advanced one base per k-mer
template <int KW>
struct Span;
// Bin-ordered records (bucket_kernel, sk_gather_kernel): (header, span word
// 0) pairs at hdr[2r], hdr[2r + 1] -- one 16-B access -- then span word 1
// (K <= 31: w1[r]) or (word 1, word 2) pairs at w1[2r], w1[2r + 1] and word 3
// at w3[r] (K <= 63).  (Three 8-B SoA arrays made bucket_kernel's placement a
// scattered store per word: 0.145 of its 0.23 ms at C2.)
DEV uint64_t rec_hdr(const BinArgs& A, uint64_t r) { return A.hdr[2 * r]; }
DEV uint64_t u64_of(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }
template <>
struct Span<1> {
    uint64_t w, x;
    DEV void load(const BinArgs& A, uint32_t r) {
        w = A.hdr[2 * (uint64_t)r + 1];
        x = A.w1[r];
    }
    // the header and the span together: one 16-B load and one 8-B load
    DEV void load_rec(const BinArgs& A, uint32_t r, uint64_t& hd) {
        const uint4 q = reinterpret_cast<const uint4*>(A.hdr)[r];
        hd = u64_of(q.x, q.y);
        w = u64_of(q.z, q.w);
        x = A.w1[r];
    }
    DEV uint64_t word0() const { return w; }
    DEV uint64_t word1() const { return x; }
    // fl = all ones when the complement wins (binning.c:1029-1040), else 0
    DEV TKey<1> key(int K, uint64_t fl) const { return TKey<1>{((w ^ fl) >> (64 - 2 * K)) + 1ull}; }
    DEV void step() {
        w = (w << 2) | (x >> 62);
        x <<= 2;
    }
    DEV void advance(uint32_t s) {  // s steps at once (s < 32: W = K - M + 1 <= 31)
        if (s) {
            w = (w << (2u * s)) | (x >> (64u - 2u * s));
            x <<= 2u * s;
        }
    }
};
template <>
struct Span<2> {
    uint64_t s0, s1, s2, s3;
    DEV void load(const BinArgs& A, uint32_t r) {
        s0 = A.hdr[2 * (uint64_t)r + 1];
        const uint4 p = reinterpret_cast<const uint4*>(A.w1)[r];
        s1 = u64_of(p.x, p.y);
        s2 = u64_of(p.z, p.w);
        s3 = A.w3[r];
    }
    DEV void load_rec(const BinArgs& A, uint32_t r, uint64_t& hd) {
        const uint4 q = reinterpret_cast<const uint4*>(A.hdr)[r];
        const uint4 p = reinterpret_cast<const uint4*>(A.w1)[r];
        hd = u64_of(q.x, q.y);
        s0 = u64_of(q.z, q.w);
        s1 = u64_of(p.x, p.y);
        s2 = u64_of(p.z, p.w);
        s3 = A.w3[r];
    }
    DEV uint64_t word0() const { return s0; }
    DEV uint64_t word1() const { return s1; }
    // complement without reversal (binning.c:1029-1040) = every code bit
    // flipped: fl = all ones when the complement wins, else 0
    DEV TKey<2> key(int K, uint64_t fl) const {
        const int kh = K - 32;  // bases above the low 64-bit word (0..31)
        const uint64_t hi = kh ? (s0 ^ fl) >> (64 - 2 * kh) : 0ull;
        const uint64_t lo = (kh ? (s0 << (2 * kh)) | (s1 >> (64 - 2 * kh)) : s0) ^ fl;
        return TKey<2>{((hi << 1) | (lo >> 63)) + 1ull, lo | PUB};
    }
    DEV void step() {
        s0 = (s0 << 2) | (s1 >> 62);
        s1 = (s1 << 2) | (s2 >> 62);
        s2 = (s2 << 2) | (s3 >> 62);
        s3 <<= 2;
    }
    DEV void advance(uint32_t s) {
        for (uint32_t i = 0; i < s; i++) step();
    }
};

// ---- the bin's LDS table: claim words (a), for KW = 2 the published low
// words (b), and a u32 count (then cursor) per slot.  Slots come in buckets
// of four (32 B of claim words): a probe reads a whole bucket at once and
// compares four keys, so a wavefront's 64 lookups rarely need a second
// dependent LDS round trip (linear probing one slot at a time left the
// wave waiting on its longest chain).  Buckets fill in slot order and slots
// never empty again, so a bucket with an empty slot ends every probe sequence.
template <int KW>
struct BinTable {
    uint64_t* ca;
    uint64_t* cb;
    // the key's slot in bucket bk, -1 (absent: the bucket has an empty slot),
    // -2 (not here, bucket full), -3 (a-match whose low word is unpublished)
    DEV int in_bucket(uint32_t bk, const TKey<KW>& k, int& empty) const {
        uint64_t w[4];
#pragma unroll
        for (int j = 0; j < 4; j++) w[j] = lds_load_u64(&ca[bk * 4u + j]);
        return match(bk, w, k, empty);
    }
    // the bucket's four claim words with plain 16-B loads: straight-line code
    // only (the probe pair of a flush), where nothing can hoist them out of a
    // retry loop; they may race a concurrent claim, which match() then treats
    // as absent (the claim that follows fails and takes the full path)
    DEV void load_bucket(uint32_t bk, uint64_t (&w)[4]) const {
        const uint4* q = reinterpret_cast<const uint4*>(ca + bk * 4u);
        const uint4 x = q[0], y = q[1];
        w[0] = (uint64_t)x.x | ((uint64_t)x.y << 32);
        w[1] = (uint64_t)x.z | ((uint64_t)x.w << 32);
        w[2] = (uint64_t)y.x | ((uint64_t)y.y << 32);
        w[3] = (uint64_t)y.z | ((uint64_t)y.w << 32);
    }
    DEV int match(uint32_t bk, const uint64_t (&w)[4], const TKey<KW>& k, int& empty) const {
        const uint32_t s0 = bk * 4u;
        empty = -1;
#pragma unroll
        for (int j = 3; j >= 0; j--)
            if (w[j] == 0) empty = j;
        int hit = -1;
#pragma unroll
        for (int j = 3; j >= 0; j--)
            if (w[j] == k.a) hit = j;
        if (hit >= 0) {
            if constexpr (KW == 1) {
                return (int)s0 + hit;
            } else {
                // (two-word keys: an a-match is rare; check the low words of all a-matches)
                bool pend = false;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (w[j] != k.a) continue;
                    const uint64_t x = lds_load_u64(&cb[s0 + j]);
                    if (x == k.b) return (int)s0 + j;
                    if (x == 0) pend = true;
                }
                if (pend) return -3;
            }
        }
        return empty >= 0 ? -1 : -2;
    }
    // find-or-insert; -2 past the key limit, -1 table full
    DEV int insert(uint32_t bmask, const TKey<KW>& k, uint32_t h, uint32_t* n_keys, uint32_t limit) const {
        uint32_t bk = h & bmask;
        // (at most 64 buckets: a table filled past its limit -- the sweep is
        // redone split anyway -- would otherwise walk every bucket per new key)
        for (uint32_t probe = 0; probe <= bmask && probe < 64u;) {
            int empty;
            const int r = in_bucket(bk, k, empty);
            if (r >= 0) return r;
            if (r == -3) continue;  // claimed, low word not yet published: re-read
            if (r == -2) {          // full bucket: the next one
                bk = (bk + 1) & bmask;
                probe++;
                continue;
            }
            const uint32_t sl = bk * 4u + (uint32_t)empty;
            const uint64_t old = atomicCAS((unsigned long long*)&ca[sl], 0ull, (unsigned long long)k.a);
            if (old == 0) {
                if constexpr (KW == 2)
                    __hip_atomic_store(&cb[sl], k.b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (atomicAdd(n_keys, 1u) >= limit) return -2;
                return (int)sl;
            }
            if constexpr (KW == 1)
                if (old == k.a) return (int)sl;
            // another key (or ours, two-word: its low word decides) took the
            // slot: re-read the bucket
        }
        return -1;
    }
};

// Light pre-filtered bins (two-word keys): a bin whose keys seen twice or more
// fit under the flat depth stays light.  A 2-bit sketch of all its k-mers,
// built once per bin in LDS of its own (past the rings: the two-word carve
// leaves room), screens the sweeps: a k-mer whose cell was hit once is the
// only occurrence of its key -- count 1 <= cutoff, counted as one distinct key,
// never inserted or staged.  Exact, as for the flat bins' sketch.
constexpr uint32_t PFL_WORDS = PFL_CELLS / 16u;  // 32 KiB: 131072 two-bit cells
// (PFL_LOAD, kbin_internal.h: at most this many distinct keys per cell)
DEV uint32_t sk_cell(const TKey<1>& k, uint32_t cells);
DEV uint32_t sk_cell(const TKey<2>& k, uint32_t cells);

// Expand the k-mers of the bin's records that fall in partition (p, l) and
// hand them to f.  Records are the bin's super-k-mers, streamed from the
// bin-ordered SoA arrays, one record per lane, the next chunk's loads issued
// before the current chunk is expanded.  Matching k-mers are compacted into a
// per-wave LDS ring; every Q/2 of them f(k0, o0, s0, k1, o1, s1, v1) runs with
// up to two k-mers per lane (independent LDS chains interleave), s =
// block-unique index from *ctr (0 .. k-mers of the partition - 1).  The
// partition filter is one multiply (KW = 1); the table hash is computed by f
// on compacted k-mers.
//   Offset range [olo, ohi) (offset partitions; [0, 64) = every offset): only
// the k-mers j whose minimizer sits at offset so - j inside the k-mer, a
// contiguous run [ja, jb) of each record.
//   psk (light pre-filtered bins): k-mers whose sketch cell was hit once are
// singles -- not handed to f, counted into *nsingle
template <int KW, typename F>
DEV void for_each_kmer(const BinArgs& A, uint32_t lo, uint32_t hi, uint32_t p, uint32_t l, uint32_t olo,
                       uint32_t ohi, uint64_t* qa, uint64_t* qb, uint32_t* qo, uint16_t* qp, uint32_t* ctr, F&& f,
                       const uint32_t* psk = nullptr, uint32_t* nsingle = nullptr, const uint32_t* rk = nullptr) {
    constexpr uint32_t Q = bin_q<KW>(), FL = Q / 2;
    const int K = A.K;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t pmask = (1u << l) - 1u;
    const bool ranged = ohi - olo < 64u;
    const bool track = A.e_first != nullptr;  // k-mer positions only for KB_TRACK_FIRST
    const bool ringfree = A.ringfree != 0;
    uint32_t head = 0, fill = 0;  // wave-uniform ring state
    uint32_t singles = 0;         // (psk) this lane's singles
    auto ring = [&](uint32_t i) {
        if constexpr (KW == 1) return TKey<1>{qa[i]};
        else return TKey<2>{qa[i], qb[i]};
    };
    auto flush = [&](uint32_t cnt) {  // cnt <= FL entries from head
        wave_sync();
        // the stage reservation and every ring read go out together: one LDS
        // round trip (LDS returns in order) before the probes
        const uint32_t i0 = (head + lane) & (Q - 1), i1 = (head + 64 + lane) & (Q - 1);
        const bool v0 = (uint32_t)lane < cnt, v1 = FL > 64 && (uint32_t)lane + 64 < cnt;
        const TKey<KW> k0 = ring(i0), k1 = ring(i1);
        const uint32_t o0 = qo[i0], o1 = qo[i1];
        const uint16_t p0 = track ? qp[i0] : (uint16_t)0, p1 = track ? qp[i1] : (uint16_t)0;
        uint32_t b = 0;
#ifdef KB_BIN_ABL
        if (A.ablate == 8) {  // flushes without their stage reservation
            f(k0, o0, p0, lane, v0, k1, o1, p1, 64 + lane, v1);
            head = (head + cnt) & (Q - 1);
            fill -= cnt;
            wave_sync();
            return;
        }
        if (A.ablate == 9) {  // no flush work at all: the ring writes alone
            head = (head + cnt) & (Q - 1);
            fill -= cnt;
            return;
        }
#endif
        if (lane == 0) b = atomicAdd(ctr, cnt);
        b = (uint32_t)rfl((int)b);
        f(k0, o0, p0, b + lane, v0, k1, o1, p1, b + 64 + lane, v1);
        head = (head + cnt) & (Q - 1);
        fill -= cnt;
        wave_sync();
    };
    uint32_t base = lo + wid * 64;
    uint64_t nhd = 0;
    uint32_t nrk = 0;  // (rk) the record's rank in its bin, staged instead of its ordinal
#ifdef KB_BIN_ABL
    uint64_t abl_acc = 0;
#endif
    Span<KW> nsp{};
    if (base + lane < hi) {
        nsp.load_rec(A, base + lane, nhd);
        if (rk) nrk = rk[base + lane];
    }
    for (; base < hi; base += BIN_THREADS) {
        const uint64_t hd = nhd;
        const uint32_t crk = nrk;
        Span<KW> sp = nsp;
        const uint32_t nxt = base + BIN_THREADS + lane;
        nhd = 0;
        if (nxt < hi) {  // prefetch the next chunk
            nsp.load_rec(A, nxt, nhd);
            if (rk) nrk = rk[nxt];
        }
        const int n = (int)((hd >> 32) & 63u);
        const uint32_t ord = rk ? crk : (uint32_t)hd;
        const uint32_t rlo = (uint32_t)((hd >> 45) & 0xFFFFu);  // the record's first k-mer in its read
        const uint64_t fl = 0ull - ((hd >> 44) & 1ull);        // complement wins: flip every bit
        // records of a bin are sorted longest first: lane 0 holds the chunk's max
        int nmax = rfl(n);
        if (__ballot(n > nmax)) nmax = rfl((int)wave_max_u32((uint32_t)n));
#ifdef KB_BIN_ABL
        if (A.ablate == 7) {  // the record loads alone
            abl_acc ^= hd ^ sp.key(K, fl).a;
            continue;
        }
        if (A.ablate == 6) {  // the k-mer windows without the ring
            for (int j = 0; j < nmax; j++) {
                const TKey<KW> key = sp.key(K, fl);
                sp.step();
                if (j < n) abl_acc ^= key.a;
            }
            continue;
        }
#endif
        // offset range: this lane's k-mers [ja, ja + nl)
        const int so = (int)((hd >> 38) & 63u);
        int ja = 0, nl = n;
        if (ranged) {
            ja = max(0, so - (int)ohi + 1);
            nl = max(0, min(n, so - (int)olo + 1) - ja);
        }
        if (KW == 1 && l == 0 && ringfree) {
            // an unpartitioned bin (or an offset range of one): every k-mer
            // of the lane's run is taken, so the lanes hand their own
            // records' k-mers j, j + 1 straight to f (the ballots keep the
            // stage stores contiguous) -- no ring writes and reads; the
            // chunk's stage range is reserved once
            const uint32_t tot = (uint32_t)rfl((int)wave_sum_u32((uint32_t)nl));
            uint32_t cb = 0;
            if (lane == 0 && tot) cb = atomicAdd(ctr, tot);
            cb = (uint32_t)rfl((int)cb);
            int jmax = nmax;
            if (ranged) {
                sp.advance((uint32_t)ja);
                jmax = (int)rfl((int)wave_max_u32((uint32_t)nl));
            }
            for (int j = 0; j < jmax; j += 2) {
                const TKey<KW> k0 = sp.key(K, fl);
                sp.step();
                const TKey<KW> k1 = sp.key(K, fl);
                sp.step();
                const bool v0 = j < nl, v1 = j + 1 < nl;
                const uint64_t m0 = __ballot(v0), m1 = __ballot(v1);
                const uint32_t s0 = cb + lanes_below(m0);
                cb += (uint32_t)__popcll(m0);
                const uint32_t s1 = cb + lanes_below(m1);
                cb += (uint32_t)__popcll(m1);
                const uint32_t pj = rlo + (uint32_t)(ja + j);
                f(k0, ord, (uint16_t)pj, s0, v0, k1, ord, (uint16_t)(pj + 1u), s1, v1);
            }
            continue;
        }
        // U k-mer positions per trip (one fill update and flush check): the
        // ring holds FL - 1 + 64 U entries, so U = (Q - FL) / 64
        constexpr int U = (int)((Q - FL) / 64u);
        for (int j = 0; j < nmax; j += U) {
            TKey<KW> key[U];
            bool take[U];
            uint64_t m[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                key[u] = sp.key(K, fl);
                sp.step();
                take[u] = (uint32_t)(j + u - ja) < (uint32_t)nl && (l == 0 || (key[u].part() & pmask) == p);
                if (KW == 2 && psk && take[u]) {
                    const uint32_t q = sk_cell(key[u], PFL_WORDS * 16u);
                    if (!((psk[q >> 4] >> (2u * (q & 15u) + 1u)) & 1u)) {
                        take[u] = false;
                        singles++;
                    }
                }
                m[u] = __ballot(take[u]);
            }
            uint32_t f0 = fill;
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (take[u]) {
                    const uint32_t pos = (head + f0 + lanes_below(m[u])) & (Q - 1);
                    qa[pos] = key[u].a;
                    if constexpr (KW == 2) qb[pos] = key[u].b;
                    qo[pos] = ord;
                    if (track) qp[pos] = (uint16_t)(rlo + (uint32_t)(j + u));
                }
                f0 += (uint32_t)__popcll(m[u]);
            }
            fill = f0;
            if (fill >= FL) flush(FL);
        }
    }
    if (fill) flush(fill);
    if (KW == 2 && psk) {
        const uint32_t ws = wave_sum_u32(singles);
        if (lane == 0 && ws) atomicAdd(nsingle, ws);
    }
#ifdef KB_BIN_ABL
    if (abl_acc == 0x123456789ull) qo[0] = 1u;  // (keeps the ablated work alive)
#endif
}

// Every k-mer of the bin's records, once, to g(key, ordinal, position) on
// its own lane (no ring, no filter): the two expansions of a heavy bin.
template <int KW, int NT = BIN_THREADS, typename G>
DEV void expand_bin(const BinArgs& A, uint32_t lo, uint32_t hi, G&& g) {
    const int K = A.K;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // (the next record's loads are issued before this one is expanded)
    uint32_t base = lo + wid * 64;
    uint64_t nhd = 0;
    Span<KW> nsp{};
    if (base + lane < hi) {
        nsp.load_rec(A, base + lane, nhd);
    }
    for (; base < hi; base += NT) {
        const uint64_t hd = nhd;
        Span<KW> sp = nsp;
        const uint32_t nxt = base + NT + lane;
        nhd = 0;
        if (nxt < hi) {
            nsp.load_rec(A, nxt, nhd);
        }
        const int n = (int)((hd >> 32) & 63u);
        const uint32_t ord = (uint32_t)hd;
        const uint32_t rlo = (uint32_t)((hd >> 45) & 0xFFFFu);
        const uint64_t fl = 0ull - ((hd >> 44) & 1ull);
        for (int j = 0; j < n; j++) {
            g(sp.key(K, fl), ord, (uint32_t)(rlo + (uint32_t)j));
            sp.step();
        }
    }
}

// heavy bins' flat k-mer lists: KW words per occurrence
template <int KW>
DEV TKey<KW> kst_load(const uint64_t* kst, uint32_t i) {
    if constexpr (KW == 1) return TKey<1>{kst[i]};
    else return TKey<2>{kst[2 * (uint64_t)i], kst[2 * (uint64_t)i + 1]};
}
template <int KW>
DEV void kst_store(uint64_t* kst, uint32_t i, const TKey<KW>& k) {
    if constexpr (KW == 1) {
        kst[i] = k.a;
    } else {
        kst[2 * (uint64_t)i] = k.a;
        kst[2 * (uint64_t)i + 1] = k.b;
    }
}

// Heavy bins (more distinct keys than several LDS tables hold): rather than
// re-expanding every record once per hash partition, the bin is expanded
// twice -- count per partition, then scatter (table key, position, ordinal)
// into flat per-partition lists -- and each partition is then swept from its
// list.  Up to FLAT_MAX partitions; deeper splits filter the flat lists.
constexpr uint32_t FLAT_LOG2 = 14;
constexpr uint32_t FLAT_MAX = 1u << FLAT_LOG2;  // (a 64-KiB LDS histogram in the build kernels)
static_assert(FLAT_MAX == KB_FLAT_MAX, "host and device agree on the flat list count");
constexpr int FB_THREADS = 256;        // the build kernels' blocks
constexpr uint32_t FB_CHUNK = 1024;    // records per build item
constexpr uint32_t FSL_NP = 2048;      // flat_scatter_lds_kernel: most partitions of the bins it writes
constexpr uint32_t SPLIT_BIT = 0x100u;     // flat_l0: a split bin's partitions (no flat lists)
constexpr uint32_t PRUNED = 0x80000000u;  // cursor of a pruned (or empty) slot in sweep 2
constexpr uint32_t PF_BIT = 0x200u;        // flat_l0: a heavy bin sized for the singleton pre-filter
constexpr uint32_t FSL_BIT = 0x400u;       // flat_l0: its lists written by flat_scatter_lds_kernel
constexpr uint32_t OSPLIT_BIT = 0x800u;    // flat_l0: a split bin partitioned by minimizer offset (bin_body)
constexpr double PF_LOAD = 0.06;           // sketch load (distinct keys / cells) the partition depth aims at

// the pre-filter's sketch cell of a key (independent of the table hash, whose
// bucket comes from the low bits, and of the partition bits)
DEV uint32_t sk_cell(const TKey<1>& k, uint32_t cells) {
    return (uint32_t)(((mix64(k.a - 1ull) >> 32) * (uint64_t)cells) >> 32);
}
DEV uint32_t sk_cell(const TKey<2>& k, uint32_t cells) {
    return (uint32_t)((((k.h64() >> 8) & 0xFFFFFFFFull) * (uint64_t)cells) >> 32);
}
constexpr uint64_t M48 = (1ull << 48) - 1ull;

// workgroup barrier ordering LDS accesses only (no wait for outstanding global
// stores); the memory clobber keeps the compiler from moving memory ops across
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// bin_kernel's barriers that order LDS only (table, cursors, windows, shared
// scalars): __syncthreads also waits for every outstanding global store of the
// workgroup (the stage, the window's read ids, the entries), so a phase that
// only needs the LDS would wait out the store latency of the one before.  The
// barriers that publish global data to other waves stay full: before the id
// windows read the stage and the entries back, and on an overflow redo (whose
// stage stores must land before the redo rewrites the same slots)
DEV void bar_lds(const BinArgs& A) {
    if (A.ldsbar) lds_barrier();
    else __syncthreads();
}

// ---- ranked bins (see bin_ranks, bitmap_lists)
#ifndef KB_RANK_MIN
#define KB_RANK_MIN 512
#endif
constexpr uint32_t RANK_MIN = KB_RANK_MIN;  // fewer records: lists short, nothing to gain (A/B builds: -DKB_RANK_MIN)
constexpr uint32_t RANK_TILE = 2048;  // ranks whose ordinals are staged in LDS at once (emission)
constexpr uint32_t RANK_TILE_WORDS = 64u * 33u;  // the tile in LDS: lane l's 32 ranks at 33 l (no bank conflicts)
constexpr uint32_t RANK_GROUPS = 8;   // most passes over the stage (entries whose bitmaps fit at once)
#ifndef KB_RANK_LONG
#define KB_RANK_LONG 64
#endif
constexpr uint32_t RANK_LONG = KB_RANK_LONG;  // ranked bins: lists longer than this take the bitmaps (A/B builds: -DKB_RANK_LONG)
constexpr uint32_t LONGB = 0x40000000u;  // cnt of a ranked bin's kept long list: LONGB | cursor (< PRUNED)
DEV bool is_long_slot(uint32_t c) { return (c & (LONGB | PRUNED)) == LONGB; }

// LDS path of one partition, after its prune: the kept occurrences' ordinals
// go to an LDS window at their list positions (cursor atomics on cnt), each
// list is put in reverse call order there (binning.c:1065-1068 prepends:
// descending call ordinal) -- lists <= 32 in one lane's registers, 33..256 by
// one wavefront -- and the window is written to ids_out as read ids with
// coalesced stores: no scattered HBM stores, no lists_kernel pass.  Lists
// > 256 leave their ordinals in ids_ord and a one-entry item for the list
// kernels.  The partition's entries [e0, e0 + n_ent) are read back densely
// from e_cnt / e_off (this block wrote them: L2).  Not inlined: its sorting
// registers stay out of the sweeps' allocation.
DEV void sort_lists_lane(uint32_t* p, uint32_t n);
// words past a list window that sort_lists_lane may read (never write): the
// end of bin_kernel's LDS carve and lists_kernel's window are padded by it
constexpr uint32_t LIST_READ_PAD = 32;
template <int R>
DEV void wave_sort_desc(uint32_t* p, uint32_t n, int lane);

// (so, ss: the split stage of a light bin -- ordinals and slots -- or null:
// the 8-B stage entries; RK with so and no ss: a ranked bin's packed 4-B
// stage, slot + 1 << 16 | rank)
// (RK, rord_bin: a ranked bin's stage holds ranks; its ordinal is
// rord_bin[rank]; only the kept short lists' occurrences are mapped.  bmw:
// the long lists' bitmaps (bmW words each, past win_cap) -- their slots hold
// LONGB | long entry, and the first window's stage pass sets their bits)
template <int KW, bool RK = false>
DEV void lds_lists(const BinArgs& A, BinShared& S, uint32_t* cnt, uint32_t TS, uint32_t* win, uint32_t win_cap,
                   uint32_t ns, unsigned long long e0, unsigned long long i0, uint32_t n_ent, uint32_t n_ids,
                   const uint64_t* stage, const uint32_t* so, const uint16_t* ss, uint32_t e_mine,
                   const uint32_t* rord_bin, uint32_t* bmw, uint32_t bmW PROF_PARAMS) {
    const uint32_t tid = threadIdx.x;
    const int lane = (int)(tid & 63u);
    const uint32_t per = TS / BIN_THREADS;
    const uint32_t cap = win_cap - 3u;  // (a window starts at its ids' 16-B phase)
#ifdef KB_BIN_ABL
    if (A.ablate == 2 || A.ablate == 3 || A.ablate >= 5) return;  // no id windows (2, 5+: nothing staged)
#endif
    // Windows: runs of whole lists.  The prune scan hands out entries and ids
    // in scan order (thread t, then its k-th slot t + 1024 k), so a window is
    // a range [slo, shi) of that order, an entry range [elo, ehi) and an id
    // range [wlo, whi) at once; each window re-reads the
    // partition's stage (MALL-resident: written moments ago) instead of
    // re-expanding the records (every list <= win_cap - 3 ids: the caller checked)
    uint32_t wlo = 0, elo = 0, slo = 0;
    while (wlo < n_ids) {  // uniform
        uint32_t whi = n_ids, ehi = n_ent, shi = TS;
        const unsigned long long g0 = i0 + wlo;
        // id wlo sits at win[sh]: window and ids_out share their 16-B phase
        const uint32_t sh = (uint32_t)(g0 & 3u);
        uint32_t* const wv = win + sh;
        if (n_ids - wlo > cap) {
            // the window ends where the list holding id wlo + win_cap starts:
            // the kept slot with the largest cursor <= that position (earlier
            // windows' cursors have reached their list ends, <= wlo)
            const uint32_t X = wlo + cap;
            if (tid == 0) S.wkey = 0;
            bar_lds(A);
            unsigned long long best = 0;
            uint32_t e = e_mine;
            for (uint32_t k = 0; k < per; k++) {
                const uint32_t i = tid + k * BIN_THREADS, c = cnt[i];
                if (c >= PRUNED || (RK && bmw && (c & LONGB))) continue;  // (pruned, or a bitmap list)
                if (c <= X) best = ((unsigned long long)c << 32) | ((unsigned long long)e << 16) | (tid * per + k);
                e++;
            }
            if (best) atomicMax(&S.wkey, best);
            bar_lds(A);
            const unsigned long long w = S.wkey;
            whi = (uint32_t)(w >> 32);
            ehi = (uint32_t)(w >> 16) & 0xFFFFu;
            shi = (uint32_t)w & 0xFFFFu;
        }
        // ---- this window's occurrences into LDS at their list positions
        // (the claim words and rings are dead); WL stage loads in flight
        PROF_CNT(26, ns);
        PROF_CNT(29, 1);
        constexpr int WL = KB_WIN_LOADS;
        // (a ranked bin's packed stage has a copy of the pass of its own: the
        // layout test inside the unrolled loads cost C3 20 % of this phase)
        auto place = [&](auto&& ld) {
        for (uint32_t i0s = tid; i0s < ns; i0s += (uint32_t)WL * BIN_THREADS) {
            uint32_t vo[WL], vs[WL];  // ordinal, slot + 1 (0: a pre-filtered single, or nothing)
#pragma unroll
            for (int u = 0; u < WL; u++) ld(i0s + (uint32_t)u * BIN_THREADS, vo[u], vs[u]);
            if constexpr (RK) {
                if (rord_bin) {
                    // only kept short lists of this window gather their ordinal;
                    // a bitmap list's occurrence sets its rank's bit (first window)
#pragma unroll
                    for (int u = 0; u < WL; u++) {
                        if (!vs[u]) continue;
                        const uint32_t ls = vs[u] - 1u, c = cnt[ls];
                        const uint32_t o = (ls & (BIN_THREADS - 1u)) * per + ls / BIN_THREADS;
                        if (bmw && is_long_slot(c)) {
                            if (wlo == 0)
                                __hip_atomic_fetch_or(&bmw[(c & ~LONGB) * bmW + (vo[u] >> 5)], 1u << (vo[u] & 31u),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            vs[u] = 0;
                        } else if (c >= PRUNED || o - slo >= shi - slo) {
                            vs[u] = 0;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < WL; u++)
                        if (vs[u]) vo[u] = rord_bin[vo[u]];
                }
            }
#pragma unroll
            for (int u = 0; u < WL; u++) {
                if (!vs[u]) continue;
                const uint32_t ls = vs[u] - 1u;
                const uint32_t o = (ls & (BIN_THREADS - 1u)) * per + ls / BIN_THREADS;  // (scan order)
                if (o - slo >= shi - slo) continue;  // another window's list
                const uint32_t pos = atomicAdd(&cnt[ls], 1u);
                if (pos < PRUNED) wv[pos - wlo] = vo[u] + 1u;  // ordinal + 1 (0 pads the sorts)
            }
        }
        };
        auto ld_any = [&](uint32_t i, uint32_t& o, uint32_t& sl) {
            if (so) {
                o = i < ns ? so[i] : 0u;
                sl = i < ns ? (uint32_t)ss[i] : 0u;
            } else {
                const uint64_t x = i < ns ? stage[i] : 0ull;
                o = (uint32_t)x;
                sl = (uint32_t)(x >> 48);
            }
        };
        if (RK && so && !ss) {  // a ranked bin's packed stage: slot + 1 << 16 | rank
            place([&](uint32_t i, uint32_t& o, uint32_t& sl) {
                const uint32_t x = i < ns ? so[i] : 0u;
                o = x & 0xFFFFu;
                sl = x >> 16;
            });
        } else {
            // (the unranked kernel keeps the layout test inside the loads:
            // separate copies measured C2 bin_kernel 1.233 -> 1.328 ms)
            place(ld_any);
        }
        bar_lds(A);
        PROF_MARK(4);
        // ---- every list in place: a wave takes 64 entries at a time
        for (uint32_t eb = elo + (tid & ~63u); eb < ehi; eb += BIN_THREADS) {
            const uint32_t e = eb + (uint32_t)lane;
            const uint32_t c = e < ehi ? A.e_cnt[e0 + e] : 0u;
            const uint32_t st_me = e < ehi ? (uint32_t)(A.e_off[e0 + e] - i0) - wlo : 0u;
#ifdef KB_BIN_ABL
            if (A.ablate == 4) continue;  // windows without their sorts
#endif
            sort_lists_lane(wv + st_me, c);
            uint64_t m = __ballot(c > 32u);
            while (m) {
                const int src = __builtin_ctzll(m);
                m &= m - 1ull;
                const uint32_t n = (uint32_t)__shfl((int)c, src, 64);
                const uint32_t st = (uint32_t)__shfl((int)st_me, src, 64);
                wave_sync();
                if (n <= 64) wave_sort_desc<1>(wv + st, n, lane);
                else if (n <= 128) wave_sort_desc<2>(wv + st, n, lane);
                else if (n <= 256) wave_sort_desc<4>(wv + st, n, lane);
                else {  // the list kernels order it from ids_ord (one-entry item)
                    for (uint32_t j = (uint32_t)lane; j < n; j += 64) A.ids_ord[g0 + st + j] = wv[st + j] - 1u;
                    if (lane == 0) {
                        const unsigned long long q = atomicAdd(A.lq_n, 1ull);
                        if (q < A.lq_cap) A.lq_items[q] = ((e0 + eb + (uint32_t)src) << 16) | 1ull;
                    }
                }
                wave_sync();
            }
        }
        bar_lds(A);
        PROF_MARK(5);
        // ---- the window as read ids, 16-B stores where aligned
        const uint32_t nw = whi - wlo;
        const uint32_t head = min((4u - sh) & 3u, nw);
        if (tid < head) A.ids_out[g0 + tid] = id_of(wv[tid] - 1u, A.read_ids, A.id_off);
        const uint32_t body = (nw - head) / 4u;
        int4* dst4 = reinterpret_cast<int4*>(A.ids_out + g0 + head);
        for (uint32_t g = tid; g < body; g += BIN_THREADS) {
            const uint4 x = *reinterpret_cast<const uint4*>(wv + head + 4u * g);
            dst4[g] = make_int4(id_of(x.x - 1u, A.read_ids, A.id_off), id_of(x.y - 1u, A.read_ids, A.id_off),
                                id_of(x.z - 1u, A.read_ids, A.id_off), id_of(x.w - 1u, A.read_ids, A.id_off));
        }
        for (uint32_t j = head + 4u * body + tid; j < nw; j += BIN_THREADS)
            A.ids_out[g0 + j] = id_of(wv[j] - 1u, A.read_ids, A.id_off);
        bar_lds(A);  // (the window is the next window's, then the next partition's table)
        PROF_MARK(6);
        wlo = whi;
        elo = ehi;
        slo = shi;
    }
}

// ---- ranked bins (long lists): records ranked by call ordinal, lists
// emitted from per-key bitmaps over the ranks (BinArgs::rank_mode)

// rank of every record of the bin [lo, hi) by descending call ordinal (ties
// by record index): bucket the ordinals by a shift of their distance from the
// largest (nbk buckets, a power of two near R / 4: a few records each, the
// read ordinals being spread evenly), scatter the record indices by bucket,
// and count each record's predecessors inside its bucket (a few compares).
// rrank[r] = rank of record r, rord[lo + k] = ordinal of rank k.  lds: nbk +
// R ordinals + R 16-bit indices, everything past BinShared (the table and
// rings are not live yet)
DEV void bin_ranks(const uint64_t* __restrict__ hdr, uint32_t* __restrict__ rrank, uint32_t* __restrict__ rord,
                   BinShared& S, uint32_t lo, uint32_t hi, uint32_t nbk_log2, uint32_t* lds PROF_PARAMS) {
    const uint32_t tid = threadIdx.x, R = hi - lo, nbk = 1u << nbk_log2;
    uint32_t* hist = lds;         // [nbk] counts, then bucket ends
    uint32_t* ordv = lds + nbk;   // [R] ordinal of record index i
    uint16_t* pidx = reinterpret_cast<uint16_t*>(ordv + R);  // [R] record indices by bucket
    if (tid == 0) {
        S.rk_min = 0xFFFFFFFFu;
        S.rk_max = 0;
    }
    for (uint32_t i = tid; i < nbk; i += BIN_THREADS) hist[i] = 0;
    uint32_t mn = 0xFFFFFFFFu, mx = 0;
    for (uint32_t i0 = tid; i0 < R; i0 += 4u * BIN_THREADS) {  // (four header loads in flight)
        uint32_t o[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + (uint32_t)u * BIN_THREADS;
            o[u] = i < R ? (uint32_t)hdr[2 * (uint64_t)(lo + i)] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + (uint32_t)u * BIN_THREADS;
            if (i >= R) continue;
            ordv[i] = o[u];
            mn = min(mn, o[u]);
            mx = max(mx, o[u]);
        }
    }
    mn = ~wave_max_u32(~mn);
    mx = wave_max_u32(mx);
    __syncthreads();
    if ((tid & 63u) == 0) {
        atomicMin(&S.rk_min, mn);
        atomicMax(&S.rk_max, mx);
    }
    __syncthreads();
    PROF_MARK(22);
    // (the shift leaves at least half of the buckets in use; no division)
    const uint32_t omax = S.rk_max, d = omax - S.rk_min;
    const uint32_t lg = d ? 32u - (uint32_t)__clz((int)d) : 0u;  // bits of the largest distance
    const uint32_t sh = lg > nbk_log2 ? lg - nbk_log2 : 0u;
    auto bucket = [&](uint32_t o) { return (omax - o) >> sh; };
    for (uint32_t i = tid; i < R; i += BIN_THREADS) atomicAdd(&hist[bucket(ordv[i])], 1u);
    __syncthreads();
    PROF_MARK(23);
    // exclusive scan: each thread its run of nbk / BIN_THREADS counters
    // (nbk >= BIN_THREADS), then one block scan of the runs
    {
        const uint32_t run = nbk / BIN_THREADS, c0 = tid * run;
        uint32_t sum = 0;
        for (uint32_t k = 0; k < run; k++) sum += hist[c0 + k];
        uint64_t tot;
        uint32_t at = (uint32_t)block_excl_scan_u64(sum, S.red, tot);
        for (uint32_t k = 0; k < run; k++) {
            const uint32_t h = hist[c0 + k];
            hist[c0 + k] = at;  // cursor (then the bucket's end)
            at += h;
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < R; i += BIN_THREADS) pidx[atomicAdd(&hist[bucket(ordv[i])], 1u)] = (uint16_t)i;
    __syncthreads();
    PROF_MARK(24);
    for (uint32_t i = tid; i < R; i += BIN_THREADS) {
        const uint32_t o = ordv[i], b = bucket(o);
        const uint32_t b0 = b ? hist[b - 1] : 0u, b1 = hist[b];
        uint32_t rank = b0;
        for (uint32_t q = b0; q < b1; q++) {
            const uint32_t j = pidx[q], oj = ordv[j];
            rank += (oj > o || (oj == o && j < i)) ? 1u : 0u;
        }
        rrank[lo + i] = rank;
        rord[lo + rank] = o;
    }
#ifdef KB_BIN_PROF
    lds_barrier();
    PROF_MARK(16);
#endif
    __syncthreads();  // (the ranks go out to HBM before sweep 1 reads them; the LDS is the table's next)
    PROF_MARK(25);
}

// long slot -> LONGB | long-entry index (the prune's scan order); offs[e] =
// its list start (relative to i0)
DEV void bm_remap(uint32_t* cnt, uint32_t per, uint32_t e_mine, uint32_t* offs) {
    uint32_t e = e_mine;
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t i = threadIdx.x + k * BIN_THREADS, c = cnt[i];
        if (is_long_slot(c)) {
            offs[e] = c & ~LONGB;
            cnt[i] = LONGB | e++;
        }
    }
}

// every bitmap of the group [g0, g1) holds exactly its key's count of bits
// (one per occurrence); else (a bit set twice: the same record holding the
// key twice) the long slots get their cursors back and the result is false
DEV bool bm_check(const uint64_t* __restrict__ e_off, const uint32_t* __restrict__ e_cnt, BinShared& S,
                  uint32_t* cnt, uint32_t per, unsigned long long e0, unsigned long long i0, uint32_t e_base,
                  uint32_t e_mine, uint32_t g0, uint32_t g1, const uint32_t* bm, uint32_t W) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    for (uint32_t e = g0 + wid; e < g1; e += BIN_WAVES) {
        uint32_t pc = 0;
        for (uint32_t w = lane; w < W; w += 64u) pc += (uint32_t)__popc(bm[(e - g0) * W + w]);
        pc = wave_sum_u32(pc);
        if (lane == 0 && pc != e_cnt[e0 + e_base + e]) S.dup = 1;
    }
    __syncthreads();
    if (!S.dup) return true;  // (uniform)
    uint32_t e = e_mine;  // back to the cursors (every long list restarts; its ids are rewritten)
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t i = tid + k * BIN_THREADS;
        if (is_long_slot(cnt[i])) cnt[i] = LONGB | (uint32_t)(e_off[e0 + e_base + e++] - i0);
    }
    __syncthreads();
    return false;
}

// the group's lists in rank order (descending ordinal = reverse call order,
// binning.c:1061-1068): one wave per list and 2048-rank tile, one bitmap word
// (32 ranks) per lane -- a wave scan of the words' bit counts gives each lane
// its first position, then each lane writes its set bits' read ids from the
// tile (the next tile's ordinals loaded during this tile's emission)
DEV void bm_emit(int32_t* __restrict__ ids_out, const int32_t* __restrict__ read_ids, uint32_t id_off,
                 unsigned long long i0, uint32_t g0, uint32_t g1, const uint32_t* bm, uint32_t W, uint32_t* offs,
                 uint32_t* tile, uint32_t R, const uint32_t* rord_bin) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    constexpr uint32_t TPT = RANK_TILE / BIN_THREADS;
    uint32_t nx[TPT];
    auto fetch = [&](uint32_t t) {
#pragma unroll
        for (uint32_t u = 0; u < TPT; u++) {
            const uint32_t i = t + tid + u * BIN_THREADS;
            nx[u] = i < R ? rord_bin[i] : 0u;
        }
    };
    fetch(0);
    for (uint32_t t0 = 0; t0 < R; t0 += RANK_TILE) {
        const uint32_t tn = min(RANK_TILE, R - t0);
#pragma unroll
        for (uint32_t u = 0; u < TPT; u++) {
            const uint32_t i = tid + u * BIN_THREADS;
            if (i < tn) tile[(i >> 5) * 33u + (i & 31u)] = (uint32_t)id_of(nx[u], read_ids, id_off);
        }
        lds_barrier();
        if (t0 + RANK_TILE < R) fetch(t0 + RANK_TILE);
        static_assert(RANK_TILE == 64u * 32u, "one bitmap word per lane covers a tile");
        for (uint32_t e = g0 + wid; e < g1; e += BIN_WAVES) {
            const uint32_t* b = bm + (e - g0) * W;
            uint32_t run = offs[e];
            uint32_t x = lane * 32u < tn ? b[(t0 >> 5) + lane] : 0u;
            const uint32_t pc = (uint32_t)__popc(x);
            const uint32_t inc = wave_incl_scan(pc, (int)lane);
            uint32_t pos = run + inc - pc;
            while (x) {
                const uint32_t bit = (uint32_t)__builtin_ctz(x);
                x &= x - 1u;
                ids_out[i0 + pos++] = (int32_t)tile[lane * 33u + bit];
            }
            run += (uint32_t)__shfl((int)inc, 63, 64);
            if (lane == 0) offs[e] = run;
        }
        lds_barrier();  // (the tile is the next tile's)
    }
}

// A ranked partition's LONG lists (> RANK_LONG ids; their slots hold LONGB |
// cursor, their entries follow the short ones) from bitmaps: every long key
// gets a bitmap over the bin's R ranks; each staged occurrence (slot, rank)
// sets its bit, then bm_check and bm_emit.  Keys are handled in groups whose
// bitmaps fit the window area, one stage pass per group.  False: a bit set
// twice, the slots' cursors restored, the caller takes the cursor path.
template <int KW>
DEV bool bitmap_lists(const uint64_t* __restrict__ e_off, const uint32_t* __restrict__ e_cnt, int32_t* __restrict__ ids_out,
                      const int32_t* __restrict__ read_ids, uint32_t id_off, BinShared& S, uint32_t* cnt, uint32_t ts,
                      uint32_t* win, uint32_t win_cap, uint32_t ns, unsigned long long e0, unsigned long long i0,
                      uint32_t n_long, uint32_t e_base, uint32_t e_mine, const uint32_t* so, const uint16_t* ss,
                      uint32_t R, const uint32_t* rord_bin PROF_PARAMS) {
    const uint32_t tid = threadIdx.x;
    const uint32_t per = ts / BIN_THREADS, W = (R + 31u) / 32u;
    uint32_t* offs = win;                  // [n_long] next position of each list (relative to i0)
    uint32_t* tile = offs + ((n_long + 3u) & ~3u);  // [RANK_TILE_WORDS] read ids of the current ranks
    uint32_t* bm = tile + RANK_TILE_WORDS;  // [G * W] the group's bitmaps
    const uint32_t G = (win_cap - (uint32_t)(bm - win)) / W;
    bm_remap(cnt, per, e_mine, offs);
    for (uint32_t g0 = 0; g0 < n_long; g0 += G) {
        const uint32_t g1 = min(n_long, g0 + G);
        for (uint32_t i = tid; i < (g1 - g0) * W; i += BIN_THREADS) bm[i] = 0;
        if (tid == 0) S.dup = 0;
        __syncthreads();
        // (BL occurrences' stage loads in flight per thread; the bits go in
        // with non-returning atomics -- a bit set twice shows as a bitmap
        // holding fewer bits than its key's count, bm_check)
        constexpr int BL = 4;
        PROF_CNT(27, ns);
        PROF_CNT(33, 1);
        for (uint32_t j0 = tid; j0 < ns; j0 += (uint32_t)BL * BIN_THREADS) {
            uint32_t vs[BL], vr[BL];
#pragma unroll
            for (int u = 0; u < BL; u++) {
                const uint32_t i = j0 + (uint32_t)u * BIN_THREADS;
                const uint32_t x = i < ns ? so[i] : 0u;  // (packed: slot + 1 << 16 | rank)
                vs[u] = x >> 16;
                vr[u] = x & 0xFFFFu;
            }
#pragma unroll
            for (int u = 0; u < BL; u++) {
                if (!vs[u]) continue;
                const uint32_t c = cnt[vs[u] - 1u];
                if (!is_long_slot(c)) continue;
                const uint32_t e = c & ~LONGB;
                if (e < g0 || e >= g1) continue;
                __hip_atomic_fetch_or(&bm[(e - g0) * W + (vr[u] >> 5)], 1u << (vr[u] & 31u), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        PROF_MARK(18);
        if (!bm_check(e_off, e_cnt, S, cnt, per, e0, i0, e_base, e_mine, g0, g1, bm, W)) return false;
        bm_emit(ids_out, read_ids, id_off, i0, g0, g1, bm, W, offs, tile, R, rord_bin);
        PROF_MARK(19);
    }
    return true;
}

// RANKED: the variant of bin_kernel that ranks bins (BinArgs::rank_mode); the
// plain one compiles none of that code, so the sweeps' register allocation
// is not taxed by it
template <int KW, int PHASE, bool RANKED = false>
DEV void bin_body(const BinArgs& A) {
    constexpr uint32_t Q = bin_q<KW>();
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    BinShared& S = *reinterpret_cast<BinShared*>(smem);      // all LDS in one dynamic array
    const uint32_t TS = 1u << A.ts_log2;  // the carved table (buckets of four slots; a partition may use less)
    const float rho = A.rho_dev ? *A.rho_dev : A.rho;  // (cold pass: the device's HLL estimate)
    BinTable<KW> T;
    // cnt | claim words | low words | rings: after the prune everything past
    // cnt is dead, and the LDS path's id window takes it (win_cap ids)
    uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + sizeof(BinShared) / 8);  // [TS] count, then cursor
    T.ca = reinterpret_cast<uint64_t*>(cnt + TS);            // [TS] claim words (TS even: 8-B aligned)
    T.cb = KW == 2 ? T.ca + TS : nullptr;                    // [TS] published low words
    uint64_t* ring0 = T.ca + KW * TS;
    uint32_t* const win = reinterpret_cast<uint32_t*>(T.ca);
    const uint32_t win_cap = (KW * TS * 8u + (uint32_t)BIN_WAVES * Q * (8u * KW + 6u)) / 4u;
    const bool lds_ok = A.lq_items && !A.e_first;  // (first occurrences need the claim words)
    const uint32_t wq = (threadIdx.x >> 6) * Q;
    uint64_t* qa = ring0 + wq;
    uint64_t* qb = KW == 2 ? ring0 + BIN_WAVES * Q + wq : nullptr;
    uint32_t* qo = reinterpret_cast<uint32_t*>(ring0 + KW * BIN_WAVES * Q) + wq;
    uint16_t* qp = reinterpret_cast<uint16_t*>(reinterpret_cast<uint32_t*>(ring0 + KW * BIN_WAVES * Q) +
                                               BIN_WAVES * Q) + wq;
    // (two-word keys) the light pre-filter's sketch, past the rings
    uint32_t* const pfl_sk = KW == 2 ? reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(ring0) +
                                                                   (size_t)BIN_WAVES * Q * (8u * KW + 6u))
                                     : nullptr;
    const uint64_t nbins = min(A.totals[2], A.max_bins);
    const uint32_t tid = threadIdx.x;
#ifdef KB_BIN_PROF
    unsigned long long* const pacc = S.prof;
    unsigned long long& pt = S.prof[PROF_N];
    if (threadIdx.x == 0) {
        for (int i = 0; i < PROF_N; i++) pacc[i] = 0;
        pt = clock64();
    }
#endif
    if (tid < 64) S.dummy[tid] = 0;  // (the first loop barrier publishes it)
    // phase 0: block thread 0 claims the next bin one bin ahead, so the
    // claim's round trip overlaps this bin's work instead of opening the next
    unsigned long long next_item = 0;
    if (PHASE == 0 && tid == 0) next_item = atomicAdd(A.work, 1ull);

    while (true) {
        // phase 0: persistent blocks take bins from a shared counter, largest
        // first.  Phase 1: the partitions of the heavy bins phase 0 turned into
        // flat lists, any block any partition (a giant bin is no longer one
        // workgroup's serial loop)
        PROF_MARK(34);  // (the bin's tail)
        bar_lds(A);
        PROF_MARK(35);  // (the loop-top barrier)
        if (tid == 0) {
            if (PHASE == 0) {
                S.item = (uint32_t)min(next_item, 0xFFFFFFFFull);
                if (next_item < nbins) next_item = atomicAdd(A.work, 1ull);
#ifdef KB_BIN_PROF
                if (next_item == 0xFFFFFFFFFFFFull) S.dup = 1;  // (the claim's wait, measured here)
#endif
            } else {
                // items are offset-pool indices: entry e0 + p of a published
                // bin is its partition p (the bin's last entry is no item)
                S.item = 0xFFFFFFFFu;
                const unsigned long long npool = A.flat_n[1];
                for (;;) {
                    const unsigned long long it = atomicAdd(&A.flat_n[5], 1ull);
                    if (it >= npool) break;
                    const uint32_t fb0 = A.pool_bin[it];
                    if (fb0 == 0xFFFFFFFFu) continue;
                    S.item = fb0;
                    S.part0 = (uint32_t)(it - A.flat_obase[fb0]);
                    break;
                }
            }
        }
        PROF_MARK(36);  // (tid 0's claim)
        bar_lds(A);
        PROF_MARK(20);
        if (PHASE == 0 ? S.item >= nbins : S.item == 0xFFFFFFFFu) break;  // uniform
        if (PHASE == 1) {  // one flat partition of bin S.item
            const uint32_t b = S.item;
            if (tid == 0) {
                S.stage_base = A.flat_sbase[b];
                S.l0 = A.flat_l0[b];  // depth | SPLIT_BIT (split, not flat)
                S.fa = A.flat_off[A.flat_obase[b] + S.part0];
                S.fb = A.flat_off[A.flat_obase[b] + S.part0 + 1];
            }
            bar_lds(A);
        }
        // phase 0 with descriptors (bucketed path): one 32-B load per bin --
        // bin, records, mmer, occurrences and stage base, in processing order
        // (bins_desc_kernel) -- instead of the order -> descriptor -> stage
        // counter chain of dependent global round trips
        uint4 d0 = make_uint4(0u, 0u, 0u, 0u), d1 = make_uint4(0u, 0u, 0u, 0u);
        if (PHASE == 0 && A.bdesc) {
            d0 = A.bdesc[2 * (uint64_t)S.item];
            d1 = A.bdesc[2 * (uint64_t)S.item + 1];
        }
        const bool have_desc = PHASE == 0 && A.bdesc;
        const uint32_t b = have_desc ? d0.x : PHASE == 0 ? A.order[S.item] : S.item;
        const uint32_t lo = have_desc ? d0.y : A.bstart[b];
        const uint32_t hi = lo + (have_desc ? d0.z : A.bcount[b]);
        const uint32_t mmer = (have_desc ? d0.w : A.bmmer[b]) & 0xFFFFu;  // (a context sub-bin's index rides above)

        // occurrences of the bin -> first partition depth
        uint64_t occ_tot = 0;
        if (PHASE == 0 && have_desc && d1.x) {  // (0: a spread run's bin, counted below)
            occ_tot = d1.x;
            if (tid == 0) S.stage_base = (uint64_t)d1.y | ((uint64_t)d1.z << 32);
            bar_lds(A);
        } else if (PHASE == 0) {
            // the bucket ordering counted them (its length rows), else a pass
            // over the record headers
            occ_tot = A.bocc ? A.bocc[b] : 0u;
            if (!occ_tot) {
                uint64_t occ = 0;
                for (uint32_t rec = lo + tid; rec < hi; rec += BIN_THREADS)
                    occ += (rec_hdr(A, rec) >> 32) & 63u;
                (void)block_excl_scan_u64(occ, S.red, occ_tot);
            }
            // the bin's stage range (one slot per occurrence, reused per partition)
            if (tid == 0) S.stage_base = atomicAdd(A.stage_ctr, (unsigned long long)occ_tot);
            bar_lds(A);
        }
        uint64_t* stage = A.stage + S.stage_base;  // (flat: moved to each partition's list)
        PROF_MARK(21);
        PROF_CNT(11, PHASE == 0);
        PROF_CNT(0, PHASE == 0 ? (hi - lo) : 0u);  // records once per bin
        PROF_CNT(14, occ_tot);
#ifdef KB_BIN_PROF
        const unsigned long long bin_t0 = clock64();
#endif
        uint32_t l0 = 0;  // uniform: initial partition depth from the expected distinct keys
        if (PHASE == 0) {
            const double want = (double)occ_tot * rho / ((double)A.fill * TS);
            while ((double)(1u << l0) < want && l0 < 16) l0++;
        } else {
            l0 = S.l0 & 0xFFu;
        }
        // heavy bin: flat per-partition lists (the ring area holds the cursors)
        // flat: a heavy bin (l0 >= flat_l), or a multi-table bin above a fair
        // share of one block's occurrences (few, large bins: N ranks, high
        // coverage) -- its build and its partitions then spread over the chip
        bool flat = PHASE == 1 ? !(S.l0 & SPLIT_BIT)
                               : (A.flat_l && (l0 >= A.flat_l || (A.big_occ && l0 >= 1 && occ_tot > A.big_occ)));
        // a would-be flat bin of two-word keys whose keys seen twice or more
        // (the learned table keys per occurrence) fit under the flat depth, and
        // whose distinct keys load the sketch lightly, stays light: one sketch
        // sweep, then its partitions' sweeps skip the singles
        bool pfl = false;
        if (PHASE == 0 && KW == 2 && A.pf_light && flat && !(A.big_occ && occ_tot > A.big_occ)) {
            const double want_t = (double)occ_tot * A.rho_tab / ((double)A.fill * TS);
            uint32_t l1 = 0;
            while ((double)(1u << l1) < want_t && l1 < 16) l1++;
            if (l1 < A.flat_l && (double)occ_tot * rho <= PFL_LOAD * (double)(PFL_WORDS * 16u)) {
                flat = false;
                pfl = true;
                l0 = l1;
            }
        }
        // a big light bin (over a fair share of one block, or over the split
        // threshold) whose depth at the light load stays offset-partitioned is
        // split by offset range instead: phase 1 bins each range on any block,
        // every range expanding only its own k-mers (no flat lists, no
        // re-expansion)
        bool osplit = PHASE == 1 && !flat && (S.l0 & OSPLIT_BIT);
        if (PHASE == 0 && A.osplit && A.opart && A.flat_l && l0 < A.flat_l &&
            ((A.big_occ && l0 >= 1 && occ_tot > A.big_occ) || (A.split_occ && occ_tot > A.split_occ))) {
            const double want = (double)occ_tot * rho / ((double)A.fill_light * TS);
            uint32_t l1 = 0;
            while ((double)(1u << l1) < want && l1 < 16) l1++;
            while (l1 < A.opart && A.big_occ && (occ_tot >> l1) > A.big_occ) l1++;
            if (l1 <= A.opart) {
                l0 = l1 < 1 ? 1u : l1;
                flat = false;
                osplit = true;
            }
        }
        // a large light bin (more occurrences than a fair share of one CU) is
        // split: its k-mers are counted per hash partition (flat_count_kernel,
        // no probes), each partition gets its own stage range, and phase 1
        // bins the partitions on any block, each re-expanding the records with
        // the partition filter -- the light path, in parallel
        bool split = (PHASE == 1 && !flat) || osplit;
        if (PHASE == 0 && !flat && !osplit && !pfl && A.split_occ && occ_tot > A.split_occ) {
            const uint32_t lmax = A.flat_l ? A.flat_l - 1u : 3u;
            while (l0 < lmax && (occ_tot >> l0) > A.split_occ) l0++;
            split = l0 >= 1;
        }
        // pre-filtered heavy bin: partitions sized by the keys that enter the
        // table and by the sketch (both fewer than the distinct keys)
        const uint32_t sk_words = (uint32_t)BIN_WAVES * Q * (8u * KW + 6u) / 4u, sk_cells = sk_words * 16u;
        bool pfb = PHASE == 1 ? flat && (S.l0 & PF_BIT) : false;
        if (PHASE == 0 && flat && A.pf) {
            const double want_t = (double)occ_tot * A.rho_tab / ((double)A.fill * TS);
            const double want_s = (double)occ_tot * rho / (PF_LOAD * (double)sk_cells);
            const double want = want_t > want_s ? want_t : want_s;
            l0 = 0;
            while ((double)(1u << l0) < want && l0 < 16) l0++;
            pfb = true;
        }
        uint64_t* kst = A.kstage + KW * S.stage_base;
        if ((split || flat) && PHASE == 0) {
            // publish: flat_count_kernel counts the k-mers per partition (any
            // block, chunks of records), flat_scan_kernel turns the counts into
            // offsets, flat_scatter_kernel writes a flat bin's lists, and phase 1
            // bins the partitions (a heavy bin is no longer one block's serial build)
            if (flat) {  // at most FLAT_MAX lists; deeper splits filter them
                if (l0 > FLAT_LOG2) l0 = FLAT_LOG2;
            }
            const uint32_t np = 1u << l0;
            // LDS-staged list writes where a build chunk gives each partition
            // short runs (under 64 entries); longer runs coalesce by themselves
            const bool fsl = flat && A.fs_lds && np <= FSL_NP &&
                             (uint64_t)FB_CHUNK * occ_tot < (uint64_t)A.fsl_run * np * (uint64_t)(hi - lo);
            if (tid == 0) S.e0 = atomicAdd(A.flat_octr, (unsigned long long)(np + 1));  // this bin's pool range
            __syncthreads();
            for (uint32_t i = tid; i <= np; i += BIN_THREADS) {
                A.flat_off[S.e0 + i] = 0;  // counts, then offsets
                A.pool_bin[S.e0 + i] = i < np ? b : 0xFFFFFFFFu;
            }
            // the build kernels' items: chunks of FB_CHUNK records
            const uint32_t nch = (hi - lo + FB_CHUNK - 1) / FB_CHUNK;
            if (tid == 0) S.i0 = atomicAdd(&A.flat_n[2], (unsigned long long)nch);
            __syncthreads();
            for (uint32_t k = tid; k < nch; k += BIN_THREADS) A.chunk_bin[S.i0 + k] = b;
            if (tid == 0) {
                if (A.pstat) atomicAdd(&A.pstat[flat ? 0 : 1], 1ull);
                if (fsl) atomicAdd(&A.flat_n[6], 1ull);  // (LDS-staged lists)
                A.flat_obase[b] = S.e0;
                A.flat_sbase[b] = S.stage_base;
                A.flat_l0[b] = l0 | (split ? SPLIT_BIT : 0u) | (pfb ? PF_BIT : 0u) | (fsl ? FSL_BIT : 0u) |
                               (osplit ? OSPLIT_BIT : 0u);
                A.flat_chunk[b] = (uint32_t)S.i0;
                A.flat_list[atomicAdd(A.flat_n, 1ull)] = b;
            }
            PROF_MARK(7);
            continue;  // (the next kernel launch sees every store)
        }
        PROF_MARK(7);
        // Offset partitions (phase 0 light bins of depth 1..opart): partition
        // p0 takes the k-mers whose minimizer sits at an offset in
        // [ocut[l0][p0], ocut[l0][p0 + 1]) of the k-mer, a contiguous run of
        // each record, so the bin's records are expanded about once in all
        // rather than once per partition.  Exact: the offset is a function of
        // the key.  The signature at s is the leftmost strict argmax over the
        // window [i0, i0 + K - M] of the recompute that chose it
        // (binning.c:922-989), and every k-mer i it serves has i0 <= i <= s;
        // an earlier copy of the same canonical mmer string inside the
        // complemented-or-not k-mer, at q in [i, s), would be the same read
        // substring with the same canonical score inside that window, and the
        // leftmost argmax would have taken q.  So s - i is the first
        // occurrence of the key's mmer in the key's k-mer.  (A partition that
        // still overflows splits by the key hash on top of its range.)
        // Offset partitions cost no re-expansion, so light bins aim at a lower
        // table load (fill_light: fewer second probe rounds) where that depth
        // stays offset-partitioned
        if (PHASE == 0 && !flat && !split && A.opart) {
            const double want = (double)occ_tot * rho / ((double)A.fill_light * TS);
            uint32_t l1 = 0;
            while ((double)(1u << l1) < want && l1 < 16) l1++;
            if (l1 <= A.opart && l1 > l0) l0 = l1;
        }
        const bool omode = (PHASE == 0 && !flat && !split && l0 >= 1 && l0 <= A.opart) || (PHASE == 1 && osplit);
        // a light bin that fits one table takes the smallest table its keys
        // fill to the light load (context sub-bins and small mmers: less to
        // clear and to scan in the prune); one that overflows it retries on a
        // table four times larger before it splits
        uint32_t tsb = TS;
        if (PHASE == 0 && A.ts_adapt && !flat && !split && l0 == 0) {
            const double keys = (double)occ_tot * (pfl ? A.rho_tab : rho);
            tsb = (uint32_t)BIN_THREADS;
            while (tsb < TS && keys > (double)A.fill_light * tsb) tsb <<= 1;
        }
        const uint32_t p_lo = PHASE == 0 ? 0u : S.part0, p_hi = PHASE == 0 ? (1u << l0) : S.part0 + 1u;
        if constexpr (KW == 2) {
            if (pfl) {  // the bin's sketch: bit 2c seen, bit 2c+1 seen again
                for (uint32_t i = tid; i < PFL_WORDS; i += BIN_THREADS) pfl_sk[i] = 0;
                bar_lds(A);
                expand_bin<KW>(A, lo, hi, [&](const TKey<KW>& k, uint32_t, uint32_t) {
                    const uint32_t cl = sk_cell(k, PFL_WORDS * 16u);
                    const uint32_t bit = 1u << (2u * (cl & 15u));
                    if (atomicOr(&pfl_sk[cl >> 4], bit) & bit) atomicOr(&pfl_sk[cl >> 4], bit << 1);
                });
                bar_lds(A);
                if (tid == 0 && A.pstat) atomicAdd(&A.pstat[8], 1ull);
            }
        }
        // ranked bin (long lists expected): records ranked by call ordinal,
        // the stage holds ranks (see bitmap_lists)
        bool rmode = false;
        if (RANKED && PHASE == 0 && A.rank_mode && !flat && !split) {
            const uint32_t words = TS + 2u * KW * TS + (uint32_t)BIN_WAVES * Q * (8u * KW + 6u) / 4u;
            const uint32_t R = hi - lo;
            // buckets: a power of two near R / 4 (at least one per thread), as
            // many as the LDS leaves room for
            uint32_t nl = 10;
            while (nl < 13 && (2u << nl) <= R / 4u) nl++;
            while (nl > 10 && (1u << nl) + R + (R + 1u) / 2u > words) nl--;
            rmode = R >= RANK_MIN && R <= 65536u && (1u << nl) + R + (R + 1u) / 2u <= words;
            if (rmode) {
                bar_lds(A);
                PROF_MARK(7);
                bin_ranks(A.hdr, A.rrank, A.rord, S, lo, hi, nl, cnt PROF_ARGS);
                PROF_CNT(30, R);
                if (tid == 0 && A.pstat) atomicAdd(&A.pstat[9], 1ull);
            }
        }
        for (uint32_t p0 = p_lo; p0 < p_hi; p0++) {
        const uint32_t olo = omode ? A.ocut[l0][p0] : 0u, ohi = omode ? A.ocut[l0][p0 + 1] : 64u;
        // (this partition's stack depth lives in spq[p0 & 1]: a wave released
        // from the last barrier of partition p0 - 1 may still be about to read
        // that partition's empty word, spq[(p0 - 1) & 1], while tid 0 is
        // already here -- writing it would send that wave into a partition
        // loop the others have left, one barrier out of step with them for the
        // rest of the bin: lost counts and keys claimed twice.  Partition
        // p0 + 1 rewrites spq[(p0 + 1) & 1] only after p0's first zeroing
        // barrier, which every wave passes after reading the old word)
        const uint32_t pq = p0 & 1u;
        if (tid == 0) {
            S.spq[pq] = 1;
            S.stack_p[0] = omode ? 0u : p0;
            S.stack_l[0] = omode ? 0u : l0;
            S.ts = tsb;
        }
        bar_lds(A);
        // flat: this partition's list is [fa, fb) of the bin's stage range
        const uint32_t fa = flat || split ? S.fa : 0u, fb = flat ? S.fb : 0u;
        stage = A.stage + S.stage_base + fa;
        // the split stage (6 B per occurrence: ordinals, slots) without
        // first-occurrence tracking; a flat list's ordinals are in it already
        // (flat_scatter), so its sweep 1 writes the slots only
        uint32_t* const sp_ord = A.stage_ord && !A.e_first ? A.stage_ord + S.stage_base + fa : nullptr;
        uint16_t* const sp_slot = sp_ord ? A.stage_slot + S.stage_base + fa : nullptr;
        const bool sp_ord_w = !(PHASE == 1 && flat);
        // a ranked bin stages 4 B per occurrence, slot + 1 << 16 | rank (its
        // ranks and slots are 16-bit): one store in sweep 1 and one load per
        // occurrence in each later stage pass, instead of 4 + 2 B in two arrays
        // (C3: 3 G occurrences per pass written once and read 1.3 times)
        const bool pk = RANKED && rmode && sp_ord;
        const uint16_t* const sp_slot_rd = pk ? nullptr : sp_slot;
        while (true) {
            const uint32_t ts = S.ts, bmask = ts / 4 - 1, limit = ts - ts / 4;  // (uniform)
            // (the stack is stable here: every write to it is followed by a
            // barrier before the loop comes round; the pop is published after
            // the zeroing barrier, so no wave reads the depth while tid 0
            // writes it, and the empty stack leaves without zeroing a table no
            // one uses.  The next partition's start writes the other parity's
            // word: see spq)
#ifdef KB_BIN_ABL
            // (diagnostic builds: one wave arrives late at every loop top --
            // KB_DIAG_SKEW=w + 1 -- so a write-after-read across the last
            // barrier shows deterministically; the test suite runs it)
            if (A.skew && (tid >> 6) == A.skew - 1u) {
                for (int z = 0; z < 8; z++) __builtin_amdgcn_s_sleep(127);
                asm volatile("" ::: "memory");  // (the depth is read after the sleep, not hoisted above it)
            }
#endif
            const uint32_t sp0 = S.spq[pq];
            if (sp0 == 0) break;  // uniform
            if (tid == 0) {
                S.cur_p = S.stack_p[sp0 - 1u];
                S.cur_l = S.stack_l[sp0 - 1u];
                S.n_keys = 0;
                S.overflow = 0;
                S.n_stage = 0;
                S.n_single = 0;
                S.maxc = 0;
                S.sumc = 0;
            }
            for (uint32_t i = tid; i < ts; i += BIN_THREADS) {
                T.ca[i] = 0;
                if constexpr (KW == 2) T.cb[i] = 0;
                cnt[i] = 0;
            }
            uint32_t* const sk = reinterpret_cast<uint32_t*>(ring0);  // (flat partitions use no rings)
            if (PHASE == 1 && pfb)
                for (uint32_t i = tid; i < sk_words; i += BIN_THREADS) sk[i] = 0;
            bar_lds(A);
            if (tid == 0) S.spq[pq] = sp0 - 1u;
            PROF_MARK(1);
            const uint32_t P = S.cur_p, Lv = S.cur_l;
            PROF_CNT(8, 1);
            PROF_CNT(15, (PHASE == 0 || !flat) ? (hi - lo) : 0u);  // records expanded (all partitions)
            // ---- sweep 1: insert + count (binning.c:1042-1069 semantics per key)
            // each occurrence is staged as (slot, ordinal) for sweep 2
            // stage entry: (LDS slot + 1) << 48 | position in the read << 32 | call
            // ordinal (slot field 0: not in the table -- a pre-filtered single)
            auto insert2 = [&](const TKey<KW>& k0, uint32_t o0, uint16_t p0, uint32_t s0, bool v0,
                               const TKey<KW>& k1, uint32_t o1, uint16_t p1, uint32_t s1, bool v1) {
#ifdef KB_BIN_ABL
                if (A.ablate == 1 || A.ablate >= 8) return;  // expansion only
#endif
                // a partition already past its key limit is redone split: the
                // rest of its sweep does nothing (a badly overfull table made
                // every new key probe the whole table)
                if (__hip_atomic_load(&S.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ||
                    __hip_atomic_load(&S.n_keys, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > limit) {
                    if ((threadIdx.x & 63u) == 0) S.overflow = 1;
                    return;
                }
                const uint32_t h0 = k0.hash(), h1 = k1.hash();
                // home buckets of both k-mers in flight together
                int e0_, e1_;
                uint64_t w0[4], w1[4];
                T.load_bucket(h0 & bmask, w0);
                T.load_bucket(h1 & bmask, w1);
                uint32_t bk0 = h0 & bmask, bk1 = h1 & bmask;
                int l0 = T.match(bk0, w0, k0, e0_);
                int l1 = T.match(bk1, w1, k1, e1_);
                // a full home bucket without the key: its next bucket (the
                // probe order), one more straight-line round for the wave's
                // few such lanes (at 60 % fill 7 % of the keys live past their
                // home bucket, so nearly every flush has some; the loop in
                // insert() re-read the home bucket and serialised on the rest)
                {
                    const bool x0 = v0 && l0 == -2, x1 = v1 && l1 == -2;
                    if (__ballot(x0 || x1)) {  // (wave-uniform)
                        if (x0) {
                            bk0 = (bk0 + 1u) & bmask;
                            T.load_bucket(bk0, w0);
                        }
                        if (x1) {
                            bk1 = (bk1 + 1u) & bmask;
                            T.load_bucket(bk1, w1);
                        }
                        if (x0) l0 = T.match(bk0, w0, k0, e0_);
                        if (x1) l1 = T.match(bk1, w1, k1, e1_);
                    }
                }
                // a new key claims the first empty slot of its bucket right
                // away (both claims in flight together); the key count is
                // added per wave and checked against the limit after the
                // sweep.  A lost claim or two full buckets take the full insert
                // path (rare)
                const uint32_t c0 = bk0 * 4u + (uint32_t)e0_, c1 = bk1 * 4u + (uint32_t)e1_;
                // (every lane issues both claims, so they go out back to back:
                // a lane with nothing to claim compares 1 against its own
                // always-zero dummy word, which never matches)
                const bool t0 = v0 && l0 == -1, t1 = v1 && l1 == -1;
                const uint32_t ln = threadIdx.x & 63u;
                unsigned long long* a0 = t0 ? (unsigned long long*)&T.ca[c0] : &S.dummy[ln];
                unsigned long long* a1 = t1 ? (unsigned long long*)&T.ca[c1] : &S.dummy[ln];
                const uint64_t old0 = atomicCAS(a0, t0 ? 0ull : 1ull, (unsigned long long)k0.a);
                const uint64_t old1 = atomicCAS(a1, t1 ? 0ull : 1ull, (unsigned long long)k1.a);
                const bool n0 = t0 && old0 == 0, n1 = t1 && old1 == 0;
                if constexpr (KW == 2) {
                    if (n0) __hip_atomic_store(&T.cb[c0], k0.b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (n1) __hip_atomic_store(&T.cb[c1], k1.b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if (n0 || (KW == 1 && t0 && old0 == k0.a)) l0 = (int)c0;
                if (n1 || (KW == 1 && t1 && old1 == k1.a)) l1 = (int)c1;
                const uint32_t nn = (uint32_t)__popcll(__ballot(n0)) + (uint32_t)__popcll(__ballot(n1));
                if (nn && (threadIdx.x & 63u) == 0) atomicAdd(&S.n_keys, nn);
                if (v0 && l0 < 0) l0 = T.insert(bmask, k0, h0, &S.n_keys, limit);
                if (v1 && l1 < 0) l1 = T.insert(bmask, k1, h1, &S.n_keys, limit);
                if (v0) {
                    if (l0 < 0) {
                        S.overflow = 1;
                    } else {
                        atomicAdd(&cnt[l0], 1u);
#ifdef KB_BIN_ABL
                        if (A.ablate != 2)
#endif
                        if (pk) {
                            sp_ord[s0] = ((uint32_t)(l0 + 1) << 16) | o0;
                        } else if (sp_ord) {
                            if (sp_ord_w) sp_ord[s0] = o0;
                            sp_slot[s0] = (uint16_t)(l0 + 1);
                        } else {
                            stage[s0] = ((uint64_t)(l0 + 1) << 48) | ((uint64_t)p0 << 32) | o0;
                        }
                    }
                }
                if (v1) {
                    if (l1 < 0) {
                        S.overflow = 1;
                    } else {
                        atomicAdd(&cnt[l1], 1u);
#ifdef KB_BIN_ABL
                        if (A.ablate != 2)
#endif
                        if (pk) {
                            sp_ord[s1] = ((uint32_t)(l1 + 1) << 16) | o1;
                        } else if (sp_ord) {
                            if (sp_ord_w) sp_ord[s1] = o1;
                            sp_slot[s1] = (uint16_t)(l1 + 1);
                        } else {
                            stage[s1] = ((uint64_t)(l1 + 1) << 48) | ((uint64_t)p1 << 32) | o1;
                        }
                    }
                }
            };
            // (phase 0 never sweeps a flat partition: a flat bin is published
            // above -- each kernel compiles only its own paths)
            if (PHASE == 0 || !flat) {
#ifdef KB_BIN_ABL
                if (A.ablate != 5)  // 5: no sweep 1 at all (the per-bin overheads alone)
#endif
                for_each_kmer<KW>(A, lo, hi, P, Lv, olo, ohi, qa, qb, qo, qp, &S.n_stage, insert2,
                                  pfl ? pfl_sk : nullptr, &S.n_single, rmode ? A.rrank : nullptr);
            } else if constexpr (PHASE == 1) {
                // the partition's flat list, two entries per lane; a deeper split
                // (Lv > l0) filters it, entries keep their index (sweep 2 filters too)
                // (the next chunk's entries are loaded before this chunk's
                // inserts: the lists stream from HBM)
                const uint32_t nf = fb - fa, pmask = (1u << Lv) - 1u;
                const uint32_t lane = tid & 63u;
                if (pfb) {
                    // ---- sweep 0: every k-mer of the partition into the sketch
                    // (bit 2c: seen, bit 2c+1: seen again); four loads in flight
                    for (uint32_t i0 = tid; i0 < nf; i0 += 4u * BIN_THREADS) {
                        TKey<KW> kk[4];
#pragma unroll
                        for (int u = 0; u < 4; u++)
                            if (i0 + u * BIN_THREADS < nf) kk[u] = kst_load<KW>(kst, fa + i0 + u * BIN_THREADS);
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            if (i0 + u * BIN_THREADS >= nf) continue;
                            if (Lv > l0 && (kk[u].part() & pmask) != P) continue;
                            const uint32_t cl = sk_cell(kk[u], sk_cells);
                            const uint32_t bit = 1u << (2u * (cl & 15u));
                            if (atomicOr(&sk[cl >> 4], bit) & bit) atomicOr(&sk[cl >> 4], bit << 1);
                        }
                    }
                    __syncthreads();
                }
                uint32_t singles = 0;
                uint32_t c0 = (uint32_t)(tid >> 6) * 128u;
                TKey<KW> n0{}, n1{};
                uint64_t ne0 = 0, ne1 = 0;
                if (c0 + lane < nf) {
                    n0 = kst_load<KW>(kst, fa + c0 + lane);
                    ne0 = sp_ord ? (uint64_t)sp_ord[c0 + lane] : stage[c0 + lane];
                }
                if (c0 + 64u + lane < nf) {
                    n1 = kst_load<KW>(kst, fa + c0 + 64u + lane);
                    ne1 = sp_ord ? (uint64_t)sp_ord[c0 + 64u + lane] : stage[c0 + 64u + lane];
                }
                for (; c0 < nf; c0 += BIN_THREADS * 2) {
                    const uint32_t i0 = c0 + lane, i1 = c0 + 64u + lane;
                    bool v0 = i0 < nf, v1 = i1 < nf;
                    const TKey<KW> k0 = n0, k1 = n1;
                    const uint64_t e0 = ne0 & M48, e1 = ne1 & M48;
                    const uint32_t c1 = c0 + BIN_THREADS * 2;
                    if (c1 + lane < nf) {
                        n0 = kst_load<KW>(kst, fa + c1 + lane);
                        ne0 = sp_ord ? (uint64_t)sp_ord[c1 + lane] : stage[c1 + lane];
                    }
                    if (c1 + 64u + lane < nf) {
                        n1 = kst_load<KW>(kst, fa + c1 + 64u + lane);
                        ne1 = sp_ord ? (uint64_t)sp_ord[c1 + 64u + lane] : stage[c1 + 64u + lane];
                    }
                    if (Lv > l0) {
                        v0 = v0 && (k0.part() & pmask) == P;
                        v1 = v1 && (k1.part() & pmask) == P;
                    }
                    if (pfb) {  // keys seen once: counted, not inserted (their stage slot field stays 0)
                        const uint32_t q0 = sk_cell(k0, sk_cells), q1 = sk_cell(k1, sk_cells);
                        const bool s0 = v0 && !((sk[q0 >> 4] >> (2u * (q0 & 15u) + 1u)) & 1u);
                        const bool s1 = v1 && !((sk[q1 >> 4] >> (2u * (q1 & 15u) + 1u)) & 1u);
                        singles += (uint32_t)__popcll(__ballot(s0)) + (uint32_t)__popcll(__ballot(s1));
                        // after an overflow a redo may find a slot field from the
                        // parent's attempt: clear it
                        if (sp_ord) {  // (the split slots start unwritten: every single's is set)
                            if (s0) sp_slot[i0] = 0;
                            if (s1) sp_slot[i1] = 0;
                        } else if (Lv > l0) {
                            if (s0) stage[i0] = e0;
                            if (s1) stage[i1] = e1;
                        }
                        v0 = v0 && !s0;
                        v1 = v1 && !s1;
                    }
                    insert2(k0, (uint32_t)e0, (uint16_t)(e0 >> 32), i0, v0, k1, (uint32_t)e1, (uint16_t)(e1 >> 32),
                            i1, v1);
                }
                if (singles && lane == 0) atomicAdd(&S.n_single, singles);
                if (tid == 0) S.n_stage = nf;
            }
            if (A.corrupt && blockIdx.x == 0 && tid == 0)  // (diagnostic: one count + 1)
                for (uint32_t i = 0; i < ts; i++)
                    if (T.ca[i]) {
                        atomicAdd(&cnt[i], 1u);
                        break;
                    }
            bar_lds(A);
            PROF_MARK(2);
            if (S.overflow || S.n_keys > limit) {  // uniform: split this partition in two and redo both
                PROF_CNT(9, 1);
                PROF_CNT(10, omode ? 1000000u + (ohi - olo) * 1000u + Lv : 0u);  // (diagnostic: offset-range overflows)
                if (tid == 0) {
                    if (A.pstat) atomicAdd(&A.pstat[3], 1ull);
                    uint32_t& sp = S.spq[pq];
                    if (ts < TS) {  // a larger table first
                        S.ts = min(TS, ts << 2);
                        S.stack_p[sp] = P;
                        S.stack_l[sp] = Lv;
                        sp++;
                    } else if (Lv >= 20 || sp + 2 > BIN_STACK) {
                        atomicOr(A.status, ST_PROBE_LIMIT);
                    } else {
                        S.stack_p[sp] = P;
                        S.stack_l[sp] = Lv + 1;
                        S.stack_p[sp + 1] = P + (1u << Lv);
                        S.stack_l[sp + 1] = Lv + 1;
                        sp += 2;
                    }
                }
                __syncthreads();
                continue;
            }
            // ---- prune (binning.c:1094-1102) + CSR allocation.  Thread t owns
            // slots t, t + 1024, ...: a wave's reads of the table are consecutive
            // words (owning 8 adjacent slots put 16 lanes on one LDS bank)
            // (a ranked bin's lists longer than RANK_LONG get entries and ids
            // of their own after the short ones: bitmap_lists emits them)
            uint64_t mine = 0, mine_l = 0;  // (ids << 32) | entries over this thread's slots: short, long
            uint32_t allc = 0;  // every key's count, kept or not
            const uint32_t per = ts / BIN_THREADS;  // ts >= BIN_THREADS
            for (uint32_t k = 0; k < per; k++) {
                const uint32_t i = tid + k * BIN_THREADS;
                const uint32_t c = cnt[i];
                if (T.ca[i]) {
                    allc += c;
                    if (c > A.keep_gt) {
                        if (rmode && c > RANK_LONG) mine_l += ((uint64_t)c << 32) + 1ull;
                        else mine += ((uint64_t)c << 32) + 1ull;
                    }
                }
            }
            allc = wave_sum_u32(allc);
            if ((tid & 63u) == 0 && allc) atomicAdd(&S.sumc, allc);
            uint64_t tot_s, tot_l = 0, ex_l = 0;
            uint64_t ex = block_excl_scan_u64(mine, S.red, tot_s, A.ldsbar != 0);
            if (rmode) ex_l = block_excl_scan_u64(mine_l, S.red, tot_l, A.ldsbar != 0);  // (uniform)
            const uint64_t tot = tot_s + tot_l;  // (both fields < 2^32)
            if (tid == 0) {
                const uint32_t ne = (uint32_t)tot, ni = (uint32_t)(tot >> 32);
                atomicAdd(&A.gcount[2], (unsigned long long)(S.n_keys + S.n_single));  // distinct before prune
                // occurrences counted (pre-filtered singles count once each): the
                // finalize checks the sum against the pass's k-mers
                atomicAdd(&A.gcount[1], (unsigned long long)S.sumc + S.n_single);
                if (A.tab_keys) atomicAdd(A.tab_keys, (unsigned long long)S.n_keys);
                if (A.pstat) {
                    atomicAdd(&A.pstat[2], 1ull);
                    atomicMax(&A.pstat[4], (unsigned long long)(Lv + (omode ? l0 : 0u)));
                    if (S.n_single) atomicAdd(&A.pstat[5], (unsigned long long)S.n_single);
                    if (omode) atomicAdd(&A.pstat[6], 1ull);
                    if (PHASE == 1 && flat) atomicAdd(&A.pstat[7], 1ull);
                }
                // entries and ids from ONE packed counter (entries << 32 | ids; both
                // totals < 2^32): consecutive entries own consecutive id ranges,
                // so offset[e + 1] ends entry e's list (the CSR contract)
#ifdef KB_BIN_ABL
                if (A.diag_alloc) {
                    // (diagnostic: the price of this returning device-scope
                    // atomic on the partition's critical path -- a second one
                    // in series before it, results unchanged)
                    const unsigned long long d = atomicAdd(&A.gcount[2], 0ull);
                    const unsigned long long got = tot ? atomicAdd(&A.gcount[0] + (d == ~0ull ? 1 : 0),
                                                                   ((unsigned long long)ne << 32) | ni)
                                                       : 0ull;
                    S.e0 = got >> 32;
                    S.i0 = got & 0xFFFFFFFFull;
                } else
#endif
                {
                const unsigned long long got =
                    tot ? atomicAdd(&A.gcount[0], ((unsigned long long)ne << 32) | ni) : 0ull;
                S.e0 = got >> 32;
                S.i0 = got & 0xFFFFFFFFull;
                }
                if (S.e0 + ne > A.max_entries || S.i0 + ni > A.max_ids) atomicOr(A.status, ST_TABLE_FULL);
            }
            bar_lds(A);
            const unsigned long long e0 = S.e0, i0 = S.i0;
            const bool room = !(e0 + (uint32_t)tot > A.max_entries || i0 + (uint32_t)(tot >> 32) > A.max_ids);
            uint32_t mc = 0;  // (the longest kept short list: the LDS windows hold whole lists)
            {
                uint32_t e = (uint32_t)ex, off = (uint32_t)(ex >> 32);
                uint32_t el = (uint32_t)tot_s + (uint32_t)ex_l, offl = (uint32_t)(tot_s >> 32) + (uint32_t)(ex_l >> 32);
                for (uint32_t k = 0; k < per; k++) {
                    const uint32_t i = tid + k * BIN_THREADS;
                    const uint32_t c = cnt[i];
                    if (T.ca[i] && c > A.keep_gt) {
                        const bool lg = rmode && c > RANK_LONG;
                        if (!lg) mc = max(mc, c);
                        const uint32_t ee = lg ? el : e, oo = lg ? offl : off;
                        if (room) {
                            const uint64_t ge = e0 + ee;
                            TKey<KW> key;
                            key.a = T.ca[i];
                            if constexpr (KW == 2) key.b = T.cb[i];
                            uint64_t khi, klo;
                            key.code(khi, klo);
                            A.e_mmer[ge] = mmer;
                            if constexpr (KW == 2) A.e_hi[ge] = khi;  // (one-word keys: kept zero, finalize_binned)
                            A.e_lo[ge] = klo;
                            A.e_cnt[ge] = c;
                            A.e_off[ge] = i0 + oo;
                        }
                        if (A.e_first) T.ca[i] = ~0ull;  // first occurrence (min) from sweep 2 on
                        if (lg) {
                            cnt[i] = LONGB | offl;  // cursor (relative to i0) of a long list
                            el++;
                            offl += c;
                        } else {
                            cnt[i] = off;  // cursor (relative to i0)
                            e++;
                            off += c;
                        }
                    } else {
                        cnt[i] = PRUNED;
                    }
                }
            }
            if (lds_ok && mc) atomicMax(&S.maxc, mc);
            __threadfence_block();
            __syncthreads();
            PROF_MARK(3);
            if (!room) continue;
            // (read once here: a path that ends without another barrier --
            // no kept ids -- must not read them after tid 0 reset them for the
            // next partition)
            const uint32_t n_stage = S.n_stage, maxc = S.maxc;
            PROF_CNT(31, n_stage);
            const uint32_t n_ent_all = (uint32_t)tot;
            const uint32_t n_ent = (uint32_t)tot_s, n_ids = (uint32_t)(tot_s >> 32);  // the short lists
            // a ranked partition's long lists: from bitmaps over the ranks when
            // they fit the window area in at most RANK_GROUPS groups, else (or on
            // a key seen twice in one record) ordinals at their cursors and the
            // list kernels; then their slots leave the short lists' way
            const bool win_phase =
                PHASE == 0 || ((KW == 1 || (A.win_heavy & 2u)) && (A.win_heavy & 1u) && !(flat && Lv > l0));
            if (RANKED && n_ent_all > n_ent) {
                PROF_MARK(3);
                const uint32_t n_long = n_ent_all - n_ent;
                const uint32_t R = hi - lo, W = (R + 31u) / 32u;
                const uint32_t fixed = ((n_long + 3u) & ~3u) + RANK_TILE_WORDS;
                // merged: the short lists take the LDS windows and every long
                // list's bitmap sits past them, so the windows' first stage pass
                // also sets the bits (one stage pass less)
                const uint32_t tail = fixed + n_long * W;
                const bool merged = n_ent && win_phase && lds_ok && tail + maxc + 3u + 256u <= win_cap &&
                                    n_ids <= 64u * n_ent && A.rank_merge;
                bool bm_ok;
                if (merged) {
                    PROF_CNT(28, 1);
                    uint32_t* offs = win + (win_cap - tail);
                    uint32_t* tile = offs + ((n_long + 3u) & ~3u);
                    uint32_t* bm = tile + RANK_TILE_WORDS;
                    bm_remap(cnt, per, (uint32_t)ex_l, offs);
                    for (uint32_t i = tid; i < n_long * W; i += BIN_THREADS) bm[i] = 0;
                    if (tid == 0) S.dup = 0;
                    __syncthreads();
                    lds_lists<KW, RANKED>(A, S, cnt, ts, win, win_cap - tail, n_stage, e0, i0, n_ent, n_ids, stage,
                                          sp_ord, sp_slot_rd, (uint32_t)ex, A.rord + lo, bm, W PROF_ARGS);
                    __syncthreads();
                    PROF_MARK(18);
                    bm_ok = bm_check(A.e_off, A.e_cnt, S, cnt, per, e0, i0, n_ent, (uint32_t)ex_l, 0u, n_long, bm, W);
                    if (bm_ok) bm_emit(A.ids_out, A.read_ids, A.id_off, i0, 0u, n_long, bm, W, offs, tile, R, A.rord + lo);
                    PROF_MARK(19);
                    if (tid == 0 && A.pstat) atomicAdd(&A.pstat[10], 1ull);
                } else {
                    const uint32_t G = fixed + W <= win_cap ? (win_cap - fixed) / W : 0u;
                    bm_ok = G && (n_long + G - 1u) / G <= RANK_GROUPS &&
                            bitmap_lists<KW>(A.e_off, A.e_cnt, A.ids_out, A.read_ids, A.id_off, S, cnt, ts, win, win_cap,
                                             n_stage, e0, i0, n_long, n_ent, (uint32_t)ex_l, sp_ord, sp_slot_rd,
                                             R, A.rord + lo PROF_ARGS);
                }
                if (bm_ok) {
                    if (!merged && tid == 0 && A.pstat) atomicAdd(&A.pstat[10], 1ull);
                } else {
                    // ranks at their cursors, then the long lists' id range mapped
                    // to ordinals in one coalesced pass (no gather inside the
                    // atomics' dependent chain)
                    const uint32_t ns = n_stage;
                    PROF_CNT(32, ns);
                    for (uint32_t i = tid; i < ns; i += BIN_THREADS) {
                        const uint32_t x = sp_ord[i], sl = pk ? x >> 16 : sp_slot[i];
                        if (!sl || (cnt[sl - 1u] & (LONGB | PRUNED)) != LONGB) continue;
                        const uint32_t pos = atomicAdd(&cnt[sl - 1u], 1u) & ~LONGB;
                        A.ids_ord[i0 + pos] = pk ? x & 0xFFFFu : x;
                    }
                    __syncthreads();
                    const uint32_t l0i = (uint32_t)(tot_s >> 32), l1i = (uint32_t)(tot >> 32);
                    for (uint32_t k = l0i + tid; k < l1i; k += BIN_THREADS)
                        A.ids_ord[i0 + k] = A.rord[lo + A.ids_ord[i0 + k]];
                    if (A.lq_items && tid == 0) {
                        const uint32_t nit = (n_long + 255u) / 256u;
                        const unsigned long long q = atomicAdd(A.lq_n, (unsigned long long)nit);
                        for (uint32_t k = 0; k < nit; k++)
                            if (q + k < A.lq_cap)
                                A.lq_items[q + k] =
                                    ((e0 + n_ent + 256ull * k) << 16) | (uint64_t)min(256u, n_long - 256u * k);
                    }
                }
                __syncthreads();
                for (uint32_t k = 0; k < per; k++) {
                    const uint32_t i = tid + k * BIN_THREADS;
                    if ((cnt[i] & (LONGB | PRUNED)) == LONGB) cnt[i] = PRUNED;
                }
                __threadfence_block();
                __syncthreads();
                PROF_MARK(17);
                if (!n_ent || merged) continue;  // (merged: the short lists are out too)
            }
            // LDS id windows for short lists (mean <= 64 ids): light bins, and
            // the heavy bins' unfiltered partitions with one-word keys (C4
            // share 588 -> 502 ms per step); long lists (C3: 357 -> 479 ms)
            // and two-word keys (C5: 624 -> 641 ms) keep the global path
            if (win_phase && lds_ok && maxc <= win_cap - 3u && n_ids <= 64u * n_ent) {
                lds_lists<KW, RANKED>(A, S, cnt, ts, win, win_cap, n_stage, e0, i0, n_ent, n_ids, stage, sp_ord,
                                      sp_slot_rd, (uint32_t)ex, rmode ? A.rord + lo : nullptr, nullptr, 0u PROF_ARGS);
                PROF_MARK(4);
                continue;
            }
            // ---- sweep 2: drop every surviving occurrence's call ordinal in place
            {
#ifdef KB_BIN_ABL
                const uint32_t ns = A.ablate ? 0u : n_stage;
#else
                const uint32_t ns = n_stage;
#endif
                const bool filt = PHASE == 1 && flat && Lv > l0;
                const uint32_t pmask = (1u << Lv) - 1u;
                for (uint32_t i = tid; i < ns; i += BIN_THREADS) {
                    if (filt && (kst_load<KW>(kst, fa + i).part() & pmask) != P) continue;
                    uint64_t v;
                    if (pk) {
                        const uint32_t x = sp_ord[i];
                        v = ((uint64_t)(x >> 16) << 48) | (x & 0xFFFFu);
                    } else {
                        v = sp_ord ? ((uint64_t)sp_slot[i] << 48) | sp_ord[i] : stage[i];
                    }
                    if (PHASE == 1 && !(v >> 48)) continue;  // a pre-filtered single (flat partitions only)
                    const uint32_t ls = (uint32_t)(v >> 48) - 1u;
                    // one returning atomic: a pruned key's cursor starts at PRUNED and
                    // takes at most cutoff adds, so it never reaches a real position
                    const uint32_t pos = atomicAdd(&cnt[ls], 1u);
                    if (pos < PRUNED) {
                        A.ids_ord[i0 + pos] = rmode ? A.rord[lo + (uint32_t)v] : (uint32_t)v;
                        // (ordinal << 16 | position): binning.c inserts a key at its first
                        // occurrence (1045-1057); KB_TRACK_FIRST keeps it for the zhash layout
                        if (A.e_first)
                            atomicMin((unsigned long long*)&T.ca[ls],
                                      (unsigned long long)(((v & 0xFFFFFFFFull) << 16) | ((v >> 32) & 0xFFFFull)));
                    }
                }
            }
            if (A.e_first) {
                __syncthreads();
                uint32_t e = (uint32_t)ex;
                for (uint32_t k = 0; k < per; k++) {
                    const uint32_t i = tid + k * BIN_THREADS;
                    if (cnt[i] < PRUNED) A.e_first[e0 + e++] = T.ca[i];
                }
            }
            // lists are put in reverse call order by lists_kernel: queue them
            if (A.lq_items && tid == 0 && n_ent) {
                const uint32_t nit = (n_ent + 255u) / 256u;
                const unsigned long long q = atomicAdd(A.lq_n, (unsigned long long)nit);
                for (uint32_t k = 0; k < nit; k++)
                    if (q + k < A.lq_cap)
                        A.lq_items[q + k] = ((e0 + 256ull * k) << 16) | (uint64_t)min(256u, n_ent - 256u * k);
            }
            __threadfence_block();
            __syncthreads();
            PROF_MARK(4);
            __syncthreads();
            PROF_MARK(6);
        }
        }  // initial partitions
#ifdef KB_BIN_PROF
        if (tid == 0) {  // the slowest bin: cycles, and its occurrences
            const unsigned long long dt = clock64() - bin_t0;
            if (dt > pacc[13]) {
                pacc[13] = dt;
                pacc[12] = occ_tot;
            }
        }
#endif
        bar_lds(A);
    }
#ifdef KB_BIN_PROF
    if (tid == 0)
        for (int i = 0; i < PROF_N; i++) {
            if (i == 12) continue;
            if (i == 13) {  // max over blocks (and that bin's occurrences)
                if (atomicMax(&g_bin_prof[13], pacc[13]) < pacc[13]) g_bin_prof[12] = pacc[12];
            } else {
                atomicAdd(&g_bin_prof[i], pacc[i]);
            }
        }
#endif
}

// The bin kernels read their arguments from device memory (bin_args_kernel
// puts them there, stream-ordered, right before): a by-value BinArgs is
// loaded into SGPRs at entry and stays live through the whole persistent loop
// (297 SGPRs and 25 VGPRs spilled, 104 B of scratch per lane in bin_kernel<1>;
// the ranked variant 456 / 73 / 280 B); through a pointer the fields are
// loaded nearer their uses (109 / 13 / 40 B; ranked 194 / 45 / 168 B) -- with
// the pointer fields global-typed (kbin_internal.h KB_G), else every access
// through them is a FLAT instruction
__global__ __launch_bounds__(64) void bin_args_kernel(BinArgs a, BinArgs* __restrict__ dst) {
    static_assert(sizeof(BinArgs) % 8 == 0, "copied in 8-B words");
    constexpr uint32_t NW = sizeof(BinArgs) / 8;
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&a);
    for (uint32_t i = threadIdx.x; i < NW; i += 64) reinterpret_cast<uint64_t*>(dst)[i] = src[i];
}

// phase 0: every light bin, and each heavy bin's flat lists
template <int KW>
__global__ __launch_bounds__(BIN_THREADS) void bin_kernel(const BinArgs* __restrict__ A) {
    bin_body<KW, 0, false>(*A);
}

// phase 0 with ranked bins (the long-list regime)
template <int KW>
__global__ __launch_bounds__(BIN_THREADS) void bin_kernel_ranked(const BinArgs* __restrict__ A) {
    bin_body<KW, 0, true>(*A);
}

// phase 1: the heavy bins' partitions, any block any partition
template <int KW>
__global__ __launch_bounds__(BIN_THREADS) void bin_parts_kernel(const BinArgs* __restrict__ A) {
    bin_body<KW, 1>(*A);
}

// ---- the parallel build of published (heavy / split) bins.  Work items are
// (bin, chunk of FB_CHUNK records), numbered by phase 0 (chunk_bin); block i
// takes items i, i + grid, ... (near-equal items; a shared claim counter cost
// ~60 ns per serialised returning atomic, 0.13 ms for an empty launch)
DEV bool fb_claim(const BinArgs& A, bool flat_only, unsigned long long& it, uint32_t& b, uint32_t& c) {
    const unsigned long long n = A.flat_n[2];
    for (; it < n; it += gridDim.x) {
        b = A.chunk_bin[it];
        if (flat_only && (A.flat_l0[b] & SPLIT_BIT)) continue;
        c = (uint32_t)(it - A.flat_chunk[b]);
        return true;
    }
    return false;
}

// per chunk: an LDS histogram of its k-mers over the bin's partitions, added
// into the bin's counts (flat_off, zeroed by phase 0)
template <int KW>
__global__ __launch_bounds__(FB_THREADS) void flat_count_kernel(BinArgs A) {
    extern __shared__ uint32_t hist[];  // [np]
    __shared__ uint32_t s_b, s_c, s_ok;
    unsigned long long it = blockIdx.x;
    for (;; it += gridDim.x) {
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t b = 0, c = 0;
            s_ok = fb_claim(A, false, it, b, c);
            s_b = b;
            s_c = c;
        }
        __syncthreads();
        if (!s_ok) break;
        const uint32_t b = s_b, l0 = A.flat_l0[b] & 0xFFu, np = 1u << l0, pm = np - 1u;
        const uint32_t lo = A.bstart[b] + s_c * FB_CHUNK, hi = min(lo + FB_CHUNK, A.bstart[b] + A.bcount[b]);
        for (uint32_t i = threadIdx.x; i < np; i += FB_THREADS) hist[i] = 0;
        __syncthreads();
        if (A.flat_l0[b] & OSPLIT_BIT) {
            // offset ranges (np <= 16): each record adds the length of its
            // run inside every range, from its header alone
            uint32_t acc[16] = {};
            for (uint32_t r = lo + threadIdx.x; r < hi; r += FB_THREADS) {
                const uint64_t hd = rec_hdr(A, r);
                const int n = (int)((hd >> 32) & 63u), so = (int)((hd >> 38) & 63u);
#pragma unroll
                for (uint32_t q = 0; q < 16; q++) {
                    if (q >= np) break;
                    const int ja = max(0, so - (int)A.ocut[l0][q + 1] + 1), jb = min(n, so - (int)A.ocut[l0][q] + 1);
                    acc[q] += (uint32_t)max(0, jb - ja);
                }
            }
#pragma unroll
            for (uint32_t q = 0; q < 16; q++) {
                if (q >= np) break;
                const uint32_t c = wave_incl_scan(acc[q], (int)(threadIdx.x & 63));
                if ((threadIdx.x & 63) == 63 && c) atomicAdd(&hist[q], c);
            }
            __syncthreads();
            uint32_t* cnt = A.flat_off + A.flat_obase[b];
            for (uint32_t i = threadIdx.x; i < np; i += FB_THREADS)
                if (hist[i]) atomicAdd(&cnt[i], hist[i]);
            continue;
        }
        // up to 8 partitions: 8-bit counts packed in a lane's register (a lane
        // expands <= 4 records of <= 63 k-mers), added per wave -- 256 lanes
        // on 8 LDS words would serialise
        const bool packed = np <= 8;
        uint64_t pk = 0;
        expand_bin<KW, FB_THREADS>(A, lo, hi, [&](const TKey<KW>& key, uint32_t, uint32_t) {
            const uint32_t pp = key.part() & pm;
            if (packed)
                pk += 1ull << (8 * pp);
            else
                atomicAdd(&hist[pp], 1u);
        });
        if (packed)
            for (uint32_t pp = 0; pp < np; pp++) {
                const uint32_t c = wave_incl_scan((uint32_t)((pk >> (8 * pp)) & 0xFFull), (int)(threadIdx.x & 63));
                if ((threadIdx.x & 63) == 63 && c) atomicAdd(&hist[pp], c);
            }
        __syncthreads();
        uint32_t* cnt = A.flat_off + A.flat_obase[b];
        for (uint32_t i = threadIdx.x; i < np; i += FB_THREADS)
            if (hist[i]) atomicAdd(&cnt[i], hist[i]);
    }
}

// per published bin: counts -> exclusive offsets (np + 1, relative to the
// bin's stage range) and, for a flat bin, the scatter cursors
__global__ __launch_bounds__(1024) void flat_scan_kernel(BinArgs A) {
    __shared__ uint64_t red[16];
    const uint32_t nf = (uint32_t)min<unsigned long long>(*A.flat_n, A.max_bins);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t q = blockIdx.x; q < nf; q += gridDim.x) {
        const uint32_t b = A.flat_list[q];
        const uint32_t np = 1u << (A.flat_l0[b] & 0xFFu);
        uint32_t* off = A.flat_off + A.flat_obase[b];
        uint32_t* cur = A.flat_cur + A.flat_obase[b];
        const uint32_t per = (np + 1023) / 1024, i0 = threadIdx.x * per;
        uint64_t mine = 0;
        for (uint32_t k = 0; k < per; k++)
            if (i0 + k < np) mine += off[i0 + k];
        const uint64_t inc = wave_incl_scan(mine, lane);
        if (lane == 63) red[wid] = inc;
        __syncthreads();
        uint64_t run = inc - mine, tot = 0;
        for (int w = 0; w < 16; w++) {
            if (w < wid) run += red[w];
            tot += red[w];
        }
        for (uint32_t k = 0; k < per; k++) {
            if (i0 + k < np) {
                const uint32_t c = off[i0 + k];
                off[i0 + k] = (uint32_t)run;
                cur[i0 + k] = (uint32_t)run;
                run += c;
            }
        }
        if (threadIdx.x == 0) off[np] = (uint32_t)tot;
        __syncthreads();
    }
}

// per chunk of a flat bin: count per partition in LDS, reserve each
// partition's range with one global atomic, then scatter (table key,
// position << 32 | ordinal) into the lists (LDS cursors)
template <int KW>
__global__ __launch_bounds__(FB_THREADS) void flat_scatter_kernel(BinArgs A) {
    extern __shared__ uint32_t hist[];  // [np]: counts, then cursors
    __shared__ uint32_t s_b, s_c, s_ok;
    __shared__ uint32_t fb_wtot[FB_THREADS / 64][8];
    unsigned long long it = blockIdx.x;
    for (;; it += gridDim.x) {
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t b = 0, c = 0;
            s_ok = fb_claim(A, true, it, b, c);
            s_b = b;
            s_c = c;
        }
        __syncthreads();
        if (!s_ok) break;
        const uint32_t b = s_b, l0 = A.flat_l0[b] & 0xFFu, np = 1u << l0, pm = np - 1u;
        if (A.flat_l0[b] & FSL_BIT) continue;  // flat_scatter_lds_kernel's
        const uint32_t lo = A.bstart[b] + s_c * FB_CHUNK, hi = min(lo + FB_CHUNK, A.bstart[b] + A.bcount[b]);
        for (uint32_t i = threadIdx.x; i < np; i += FB_THREADS) hist[i] = 0;
        __syncthreads();
        // up to 8 partitions: packed per-lane counts (see flat_count_kernel)
        // give each wave a range per partition; the second expansion steps the
        // wave's lanes together and ranks them per partition by ballot, so
        // consecutive lanes of one partition store to consecutive entries
        const bool packed = np <= 8;
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        uint64_t pk = 0;
        expand_bin<KW, FB_THREADS>(A, lo, hi, [&](const TKey<KW>& key, uint32_t, uint32_t) {
            const uint32_t pp = key.part() & pm;
            if (packed)
                pk += 1ull << (8 * pp);
            else
                atomicAdd(&hist[pp], 1u);
        });
        if (packed) {
#pragma unroll
            for (uint32_t pp = 0; pp < 8; pp++) {
                const uint32_t c = pp < np ? (uint32_t)((pk >> (8 * pp)) & 0xFFull) : 0u;
                const uint32_t inc = wave_incl_scan(c, lane);
                if (lane == 63) fb_wtot[wid][pp] = inc;
            }
        }
        __syncthreads();
        if (packed && threadIdx.x < np) {
            uint32_t t = 0;
            for (int w = 0; w < FB_THREADS / 64; w++) t += fb_wtot[w][threadIdx.x];
            hist[threadIdx.x] = t;
        }
        __syncthreads();
        uint32_t* cur = A.flat_cur + A.flat_obase[b];
        for (uint32_t i = threadIdx.x; i < np; i += FB_THREADS)
            if (hist[i]) hist[i] = atomicAdd(&cur[i], hist[i]);
        __syncthreads();
        const uint64_t sb = A.flat_sbase[b];
        uint64_t* kst = A.kstage + KW * sb;
        uint64_t* stage = A.stage + sb;
        // (the split stage: the list's ordinals alone, bin_body writes the slots)
        uint32_t* const sord = A.stage_ord && !A.e_first ? A.stage_ord + sb : nullptr;
        if (packed) {
            uint32_t wb[8];  // this wave's next entry per partition (wave-uniform)
#pragma unroll
            for (uint32_t pp = 0; pp < 8; pp++) {
                uint32_t w0 = 0;
                for (int w = 0; w < wid; w++) w0 += fb_wtot[w][pp];
                wb[pp] = pp < np ? hist[pp] + w0 : 0u;
            }
            const uint64_t lt = (1ull << lane) - 1ull;
            const int K = A.K;
            uint32_t base = lo + (uint32_t)wid * 64u;
            uint64_t nhd = 0;
            Span<KW> nsp{};
            if (base + (uint32_t)lane < hi) {
                nsp.load_rec(A, base + lane, nhd);
            }
            for (; base < hi; base += FB_THREADS) {  // (next record's loads first)
                const uint64_t hd = nhd;
                Span<KW> sp = nsp;
                const uint32_t nxt = base + FB_THREADS + (uint32_t)lane;
                nhd = 0;
                if (nxt < hi) {
                    nsp.load_rec(A, nxt, nhd);
                }
                const int n = (int)((hd >> 32) & 63u);
                const uint32_t ord = (uint32_t)hd;
                const uint32_t rlo = (uint32_t)((hd >> 45) & 0xFFFFu);
                const uint64_t fl = 0ull - ((hd >> 44) & 1ull);
                const int nmax = (int)wave_max_u32((uint32_t)n);
                for (int j = 0; j < nmax; j++) {
                    const TKey<KW> key = sp.key(K, fl);
                    sp.step();
                    const uint32_t pp = j < n ? key.part() & pm : 0xFFu;
                    uint32_t i = 0;
#pragma unroll
                    for (uint32_t q = 0; q < 8; q++) {
                        const uint64_t m = __ballot(pp == q);
                        if (pp == q) i = wb[q] + (uint32_t)__popcll(m & lt);
                        wb[q] += (uint32_t)__popcll(m);
                    }
                    if (j < n) {
                        kst_store<KW>(kst, i, key);
                        if (sord) sord[i] = ord;
                        else stage[i] = ((uint64_t)(rlo + (uint32_t)j) << 32) | ord;
                    }
                }
            }
        } else {
            expand_bin<KW, FB_THREADS>(A, lo, hi, [&](const TKey<KW>& key, uint32_t ord, uint32_t pos) {
                const uint32_t i = atomicAdd(&hist[key.part() & pm], 1u);
                kst_store<KW>(kst, i, key);
                if (sord) sord[i] = ord;
                else stage[i] = ((uint64_t)pos << 32) | ord;
            });
        }
    }
}

// Heavy bins whose build chunks give each partition short runs (fewer than 64
// entries; up to 2048 partitions): the chunk's entries are staged in
// LDS sorted by partition and written out with consecutive lanes on
// consecutive entries of one partition's range, so a store instruction covers
// whole runs of lines.  (Scattered straight to HBM, the ~40 entries a chunk
// gives each of a few hundred partitions left lines partly written: the PMC
// passes counted 3.7x the list bytes written at C4, 2.8x at C5.)  A chunk is
// cut into segments of at most FSL_E entries (record k-mer counts come from
// the headers); per segment: count per partition (expansion 1), reserve each
// partition's range with one global atomic and place the partitions in LDS
// (scan), stage key, value and partition (expansion 2), copy out.
constexpr int FSL_THREADS = 1024;
template <int KW>
constexpr uint32_t fsl_entries() { return KW == 1 ? 7168u : 4864u; }
template <int KW>
constexpr size_t fsl_lds_bytes() {
    return (size_t)fsl_entries<KW>() * (8u * KW + 8u + 2u) + 3u * FSL_NP * sizeof(uint32_t) + 64;
}

template <int KW>
__global__ __launch_bounds__(FSL_THREADS) void flat_scatter_lds_kernel(BinArgs A) {
    constexpr uint32_t E = fsl_entries<KW>();
    extern __shared__ __attribute__((aligned(16))) uint64_t fsm[];
    uint64_t* const skey = fsm;                                        // [KW E]
    uint64_t* const sval = skey + KW * E;                              // [E]
    uint32_t* const cnt = reinterpret_cast<uint32_t*>(sval + E);       // [FSL_NP] counts, then cursors
    uint32_t* const loff = cnt + FSL_NP;                               // [FSL_NP] first staged entry
    uint32_t* const gbase = loff + FSL_NP;                             // [FSL_NP] first list entry
    uint16_t* const spart = reinterpret_cast<uint16_t*>(gbase + FSL_NP);  // [E]
    __shared__ uint32_t s_b, s_c, s_ok, s_seg, s_tot;
    __shared__ uint32_t red[FSL_THREADS / 64];
    if (!A.flat_n[6]) return;  // no bin with that many partitions this time
    const uint32_t tid = threadIdx.x;
    const int lane = (int)(tid & 63u), wid = (int)(tid >> 6);
    unsigned long long it = blockIdx.x;
    for (;; it += gridDim.x) {
        __syncthreads();
        if (tid == 0) {
            uint32_t b = 0, c = 0;
            s_ok = fb_claim(A, true, it, b, c);
            s_b = b;
            s_c = c;
        }
        __syncthreads();
        if (!s_ok) break;
        const uint32_t b = s_b, l0 = A.flat_l0[b] & 0xFFu, np = 1u << l0, pm = np - 1u;
        if (!(A.flat_l0[b] & FSL_BIT)) continue;  // (flat_scatter_kernel's)
        const uint32_t c_lo = A.bstart[b] + s_c * FB_CHUNK, c_hi = min(c_lo + FB_CHUNK, A.bstart[b] + A.bcount[b]);
        uint32_t* cur = A.flat_cur + A.flat_obase[b];
        const uint64_t sb = A.flat_sbase[b];
        uint64_t* kst = A.kstage + KW * sb;
        uint64_t* stage = A.stage + sb;
        // (the split stage: the list's ordinals alone, bin_body writes the slots)
        uint32_t* const sord = A.stage_ord && !A.e_first ? A.stage_ord + sb : nullptr;
        for (uint32_t lo = c_lo; lo < c_hi;) {
            // ---- this segment: the longest record run from lo within E entries
            {
                const uint32_t r = lo + tid;
                const uint32_t n = r < c_hi ? (uint32_t)((rec_hdr(A, r) >> 32) & 63u) : 0u;
                const uint32_t inc = wave_incl_scan(n, lane);
                if (lane == 63) red[wid] = inc;
                __syncthreads();
                uint32_t before = 0;
                for (int w = 0; w < wid; w++) before += red[w];
                const uint32_t incl = before + inc;
                // records [lo, lo + k) fit when their inclusive sum <= E: count them
                const uint64_t fit = __ballot(r < c_hi && incl <= E);
                if (tid == 0) s_seg = 0;
                __syncthreads();
                if (lane == 0 && fit) atomicAdd(&s_seg, (uint32_t)__popcll(fit));
                __syncthreads();
            }
            const uint32_t hi = lo + max(1u, s_seg);  // (one record always fits: n <= 63 < E)
            for (uint32_t i = tid; i < np; i += FSL_THREADS) cnt[i] = 0;
            __syncthreads();
            expand_bin<KW, FSL_THREADS>(A, lo, hi, [&](const TKey<KW>& key, uint32_t, uint32_t) {
                atomicAdd(&cnt[key.part() & pm], 1u);
            });
            __syncthreads();
            // ---- partitions: global range (one atomic each), staged offsets (scan)
            {
                constexpr uint32_t PER = FSL_NP / FSL_THREADS;
                uint32_t c[PER], sum = 0;
#pragma unroll
                for (uint32_t k = 0; k < PER; k++) {
                    const uint32_t p = tid * PER + k;
                    c[k] = p < np ? cnt[p] : 0u;
                    sum += c[k];
                }
                const uint32_t inc = wave_incl_scan(sum, lane);
                __syncthreads();
                if (lane == 63) red[wid] = inc;
                __syncthreads();
                uint32_t run = inc - sum;
                for (int w = 0; w < wid; w++) run += red[w];
#pragma unroll
                for (uint32_t k = 0; k < PER; k++) {
                    const uint32_t p = tid * PER + k;
                    if (p < np) {
                        loff[p] = run;
                        cnt[p] = run;  // cursor
                        if (c[k]) gbase[p] = atomicAdd(&cur[p], c[k]);
                        run += c[k];
                    }
                }
                if (tid == FSL_THREADS - 1) s_tot = run;
            }
            __syncthreads();
            expand_bin<KW, FSL_THREADS>(A, lo, hi, [&](const TKey<KW>& key, uint32_t ord, uint32_t pos) {
                const uint32_t p = key.part() & pm;
                const uint32_t i = atomicAdd(&cnt[p], 1u);
                if constexpr (KW == 1) {
                    skey[i] = key.a;
                } else {
                    skey[2 * i] = key.a;
                    skey[2 * i + 1] = key.b;
                }
                sval[i] = ((uint64_t)pos << 32) | ord;
                spart[i] = (uint16_t)p;
            });
            __syncthreads();
            // ---- copy out: consecutive staged entries of one partition go to
            // consecutive list entries
            const uint32_t tot = s_tot;
            for (uint32_t i = tid; i < tot; i += FSL_THREADS) {
                const uint32_t p = spart[i];
                const uint32_t g = gbase[p] + (i - loff[p]);
                if constexpr (KW == 1) {
                    kst[g] = skey[i];
                } else {
                    kst[2 * (uint64_t)g] = skey[2 * i];
                    kst[2 * (uint64_t)g + 1] = skey[2 * i + 1];
                }
                if (sord) sord[g] = (uint32_t)sval[i];
                else stage[g] = sval[i];
            }
            lo = hi;
        }
    }
}

#ifdef KB_BIN_PROF
void bins_prof_report(hipStream_t s) {
    unsigned long long h[PROF_N];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bin_prof), sizeof(h));
    {
        unsigned long long g[8];
        (void)hipMemcpyFromSymbol(g, HIP_SYMBOL(g_sk_prof), sizeof(g));
        fprintf(stderr, "[sk_prof] rows=%llu walk=%llu counts=%llu place=%llu\n", g[0], g[1], g[2], g[3]);
        unsigned long long z8[8] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sk_prof), z8, sizeof(z8));
    }
    static const char* nm[PROF_N] = {"bin records", "zero", "sweep1", "prune/entries", "sweep2/win place", "win sort", "win ids out", "flat",
                                 "partitions", "overflows", "omode-ovf(1e6*n+1e3*width+Lv)", "bins", "slowest-bin-occ", "slowest-bin-cycles",
                                 "occ", "records expanded", "rank", "long bitmaps", "bitmap set", "bitmap emit", "bin claim", "bin desc", "rank loads", "rank hist", "rank scatter", "rank stores",
                                 "win stage reads", "bm stage reads", "merged parts", "windows", "ranked records", "stage writes",
                                 "rank-fallback stage reads", "bm groups", "bin tail", "loop-top barrier", "claim wait"};
    fprintf(stderr, "[bin_prof]");
    for (int i = 0; i < PROF_N; i++)
        if (h[i]) fprintf(stderr, " %s=%llu", nm[i], h[i]);
    fprintf(stderr, "\n");
    unsigned long long z[PROF_N] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bin_prof), z, sizeof(z));
}
#endif

// ---------------------------------------------------------------------------
// phase C: every list into reverse call order (binning.c:1061-1068 prepends,
// so a list reads newest call first = descending ordinal), ordinals -> ids.
// A block takes 256 consecutive entries: lists of <= 32 ids are sorted in the
// registers of one lane, 33..256 by one wavefront in LDS, longer ones by the
// whole block (LDS bitonic up to LIST_CAP, else chunks + merge passes).
// ---------------------------------------------------------------------------
constexpr int LIST_THREADS = 256;
constexpr uint32_t LIST_CAP = 4096;   // longest list sorted in LDS in one piece (power of two)
constexpr uint32_t LIST_SPAN = 7168;  // ids staged in LDS at once (28 KiB: 5 blocks per CU)
constexpr uint32_t LIST_WIN = LIST_SPAN - 256 - 8;  // window of list starts: + one list <= 256, + alignment
constexpr uint32_t WAVE_LIST_MAX = 4096;  // longest list one wavefront sorts in its registers (64 x 64)

// descending bitonic sort of Pw (power of two) values in LDS by a group of G
// lanes (G = 64: one wavefront, wave barriers; else the block)
template <int G>
DEV void bitonic_desc(uint32_t* a, uint32_t Pw, uint32_t r) {
    for (uint32_t kk = 2; kk <= Pw; kk <<= 1) {
        for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
            for (uint32_t i = r; i < Pw; i += G) {
                const uint32_t l2 = i ^ jj;
                if (l2 > i) {
                    const uint32_t x = a[i], y = a[l2];
                    const bool desc = (i & kk) == 0;
                    if (desc ? (x < y) : (x > y)) {
                        a[i] = y;
                        a[l2] = x;
                    }
                }
            }
            if (G == 64) wave_sync();
            else __syncthreads();
        }
    }
}

// up to 256 values sorted descending by one wavefront, in registers: element
// i = r * 64 + lane lives in v[r]; partners across lanes meet by xor-shuffle,
// partners 64 or 128 apart are in the same lane.  In place in LDS.
// Bitonic sort, descending, of R*64 values held by one wavefront in
// registers, striped (value i = v[i / 64] of lane i % 64): partner distances
// below 64 are lane shuffles, 64 and up are register pairs.  No LDS, no
// barriers -- a wavefront sorts a list of up to 64 R ids on its own.
template <int R>
DEV void wave_bitonic(uint32_t (&v)[R], int lane) {
#pragma unroll
    for (int kk = 2; kk <= R * 64; kk <<= 1) {
#pragma unroll
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            if (jj >= 64) {
                const int rj = jj >> 6;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int r2 = r ^ rj;
                    if (r2 > r) {
                        const uint32_t i = (uint32_t)(r * 64 + lane);
                        const bool desc = (i & kk) == 0;
                        const uint32_t x = v[r], y = v[r2];
                        const uint32_t hi = x > y ? x : y, lo = x > y ? y : x;
                        v[r] = desc ? hi : lo;
                        v[r2] = desc ? lo : hi;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const uint32_t i = (uint32_t)(r * 64 + lane);
                    const uint32_t y = (uint32_t)__shfl_xor((int)v[r], jj, 64);
                    const bool lower = (lane & jj) == 0;
                    const bool desc = (i & kk) == 0;
                    const uint32_t hi = v[r] > y ? v[r] : y, lo = v[r] > y ? y : v[r];
                    v[r] = (lower == desc) ? hi : lo;
                }
            }
        }
    }
}

// The same network for long lists with the stage loops left rolled: the
// register-pair stages are unrolled per distance (RJ), so the code and the
// register file stay at O(R), not O(R log^2 R).
template <int R, int RJ>
DEV void reg_stage(uint32_t (&v)[R], int lane, uint32_t kk) {
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int r2 = r ^ RJ;
        if (r2 > r) {
            const bool desc = ((uint32_t)(r * 64 + lane) & kk) == 0;
            const uint32_t x = v[r], y = v[r2];
            const uint32_t hi = x > y ? x : y, lo = x > y ? y : x;
            v[r] = desc ? hi : lo;
            v[r2] = desc ? lo : hi;
        }
    }
}

template <int R>
DEV void wave_bitonic_rolled(uint32_t (&v)[R], int lane) {
    for (uint32_t kk = 2; kk <= R * 64; kk <<= 1) {
        for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
            if (jj >= 64) {
                switch (jj >> 6) {
                    case 1: if constexpr (R > 1) reg_stage<R, 1>(v, lane, kk); break;
                    case 2: if constexpr (R > 2) reg_stage<R, 2>(v, lane, kk); break;
                    case 4: if constexpr (R > 4) reg_stage<R, 4>(v, lane, kk); break;
                    case 8: if constexpr (R > 8) reg_stage<R, 8>(v, lane, kk); break;
                    case 16: if constexpr (R > 16) reg_stage<R, 16>(v, lane, kk); break;
                    case 32: if constexpr (R > 32) reg_stage<R, 32>(v, lane, kk); break;
                    default: break;
                }
            } else {
                const bool lower = (lane & jj) == 0;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const uint32_t y = (uint32_t)__shfl_xor((int)v[r], (int)jj, 64);
                    const bool desc = ((uint32_t)(r * 64 + lane) & kk) == 0;
                    const uint32_t hi = v[r] > y ? v[r] : y, lo = v[r] > y ? y : v[r];
                    v[r] = (lower == desc) ? hi : lo;
                }
            }
        }
    }
}

template <int R>
DEV void wave_sort_list_long(const uint32_t* __restrict__ src, int32_t* __restrict__ dst, uint32_t n, int lane,
                             const int32_t* read_ids, uint32_t id_off) {
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t i = (uint32_t)(r * 64 + lane);
        v[r] = i < n ? src[i] + 1u : 0u;
    }
    wave_bitonic_rolled<R>(v, lane);
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t i = (uint32_t)(r * 64 + lane);
        if (i < n) dst[i] = id_of(v[r] - 1u, read_ids, id_off);
    }
}

// n <= 64 R values (ordinal + 1) in LDS, sorted descending in place
template <int R>
DEV void wave_sort_desc(uint32_t* p, uint32_t n, int lane) {
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t i = (uint32_t)(r * 64 + lane);
        v[r] = i < n ? p[i] : 0u;
    }
    wave_bitonic<R>(v, lane);
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t i = (uint32_t)(r * 64 + lane);
        if (i < n) p[i] = v[r];
    }
}

// one list of n <= 64 R call ordinals from HBM to its ids, reverse call order
template <int R>
DEV void wave_sort_list(const uint32_t* __restrict__ src, int32_t* __restrict__ dst, uint32_t n, int lane,
                        const int32_t* read_ids, uint32_t id_off) {
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t i = (uint32_t)(r * 64 + lane);
        v[r] = i < n ? src[i] + 1u : 0u;
    }
    wave_bitonic<R>(v, lane);
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t i = (uint32_t)(r * 64 + lane);
        if (i < n) dst[i] = id_of(v[r] - 1u, read_ids, id_off);
    }
}

// up to 32 values (ordinal + 1) sorted descending in one lane's registers, in place
// Batcher's odd-even merge network on NP = 2^k inputs, descending (the larger
// of every pair to the lower index), keeping only the comparators whose upper
// index is < N: a list of n <= N ids padded with zeros (below every id + 1)
// keeps its pads in place, so the pruned network sorts it.  NP = 32: 191
// comparators (the bitonic network: 240); N = 24: 132; 16: 63; 8: 19
// (2 <= n <= N.  The loads and stores are branch-free -- a branch per
// position saved the exec mask in an SGPR pair, and in bin_kernel those were
// spilled to VGPR lanes: all N words are read (p[0 .. N) must lie inside the
// LDS allocation: both callers leave LIST_READ_PAD words after their windows)
// and the pads masked; position j >= n writes p[n - 1] instead, the stores
// going out from the last position down, so p[n - 1] ends with its own value)
template <int N, int NP>
DEV void sort_net_desc(uint32_t* p, uint32_t n) {
    uint32_t v[N];
    const uint32_t last = n - 1u;
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t x = p[j];
        v[j] = (uint32_t)j < n ? x : 0u;
    }
#pragma unroll
    for (int q = 1; q < NP; q <<= 1)
#pragma unroll
        for (int k = q; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % q; j + k < NP; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; i++) {
                    const int a = i + j, b = i + j + k;
                    if (b < N && a / (2 * q) == b / (2 * q)) {
                        const uint32_t x = v[a], y = v[b < N ? b : 0];
                        v[a] = x > y ? x : y;
                        v[b < N ? b : 0] = x > y ? y : x;
                    }
                }
#pragma unroll
    for (int j = N - 1; j >= 0; j--) p[min((uint32_t)j, last)] = v[j];
}

// every lane's list of 2..32 ids (n outside that: nothing) in descending
// order in its registers, with the smallest network that holds the wave's
// longest such list (wave-uniform call)
DEV void sort_lists_lane(uint32_t* p, uint32_t n) {
    const bool me = n >= 2 && n <= 32;
    const uint32_t m = wave_max_u32(me ? n : 0u);
    if (m > 24) {
        if (me) sort_net_desc<32, 32>(p, n);
    } else if (m > 16) {
        if (me) sort_net_desc<24, 32>(p, n);
    } else if (m > 8) {
        if (me) sort_net_desc<16, 16>(p, n);
    } else if (m >= 2) {
        if (me) sort_net_desc<8, 8>(p, n);
    }
}

#ifdef KB_BIN_PROF
__device__ unsigned long long g_list_prof[8];
#define LPROF(ph)                                                  \
    do {                                                           \
        if (tid == 0) {                                            \
            const unsigned long long _t = clock64();               \
            lacc[ph] += _t - lt;                                   \
            lt = _t;                                               \
        }                                                          \
    } while (0)
#else
#define LPROF(ph) do {} while (0)
#endif

__global__ __launch_bounds__(LIST_THREADS) __attribute__((amdgpu_waves_per_eu(5, 8))) void lists_kernel(ListArgs A) {
#ifdef KB_BIN_PROF
    unsigned long long lacc[8] = {};
    unsigned long long lt = clock64();
#endif
    // staged chunks: ibuf = the chunk's ids (ordinal + 1); other chunks: buf =
    // block sort space (LIST_CAP), wave windows inside
    __shared__ uint32_t lds[LIST_SPAN + LIST_READ_PAD];  // (the pad: sort_lists_lane's reads)
    static_assert(LIST_CAP <= LIST_SPAN, "block sort space aliases the staging area");
    uint32_t* const ibuf = lds;
    uint32_t* const buf = lds;
    __shared__ uint32_t big[LIST_THREADS], mid[LIST_THREADS];
    __shared__ uint32_t n_big, n_mid, s_long, w_lo[2], w_hi[2];
    const uint32_t tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const uint64_t n_entries = A.totals[0];
    // items: the bin kernels' queue (partitions whose ids took the global
    // path, and long lists of the LDS path), else every entry in chunks of 256
    // (an entry-capacity overflow publishes no entries, bins_final_kernel: the
    // queued items' neighbours then have unwritten offsets -- no work at all,
    // the host reruns the bin phase)
    const uint64_t n_items = !n_entries ? 0ull
                             : A.lq_items ? min<uint64_t>(*A.lq_n, A.lq_cap)
                                          : (n_entries + LIST_THREADS - 1) / LIST_THREADS;
    for (uint64_t it = blockIdx.x; it < n_items; it += gridDim.x) {
        uint64_t e0;
        uint32_t ne;
        if (A.lq_items) {
            const uint64_t x = A.lq_items[it];
            e0 = x >> 16;
            ne = (uint32_t)(x & 0xFFFFu);
        } else {
            e0 = it * LIST_THREADS;
            ne = (uint32_t)min<uint64_t>(LIST_THREADS, n_entries - e0);
        }
        const uint64_t ob = A.e_off[e0], span = A.e_off[e0 + ne] - ob;
        // (barriers in the staged path order LDS only: a full __syncthreads
        // also waits for the previous window's global stores to land)
        if (tid == 0) {
            n_big = 0;
            s_long = 0;
        }
        lds_barrier();
        // this thread's entry; lists > 256 leave the staged windows: up to
        // WAVE_LIST_MAX to lists_bucket_kernel, longer ones to this block below
        const uint32_t n_me = tid < ne ? A.e_cnt[e0 + tid] : 0u;
        const uint32_t rel = tid < ne ? (uint32_t)(A.e_off[e0 + tid] - ob) : 0u;  // < 2^32 ids per finalize
        const bool short_me = tid < ne && n_me <= 256;
        if (tid < ne && !short_me) {
            if (n_me <= WAVE_LIST_MAX) A.long_q[atomicAdd(A.long_n, 1u)] = (uint32_t)(e0 + tid);
            else big[atomicAdd(&n_big, 1u)] = tid;
            s_long = 1;
        }
        lds_barrier();
        // Staged windows: the chunk's id range cut every LIST_WIN ids; a short
        // list belongs to the window its first id falls in, and a window stages
        // [first start, last end) of its lists (<= LIST_WIN + 256 ids) with
        // coalesced 16-B loads, sorts each list in LDS (<= 32: one lane's
        // registers, 33..256: one wavefront) and writes the range back with 16-B
        // stores.  (Ids of a long list inside the range are written back
        // unsorted; its own kernel rewrites them later on the stream.)
        // (the common case -- every list short, the chunk fits -- is one window)
        const bool one = !s_long && span + 8 <= LIST_SPAN;
        const uint32_t nw = one ? 1u : (uint32_t)((span + LIST_WIN - 1) / LIST_WIN);
        const uint32_t wk = rel / LIST_WIN;
        for (uint32_t k = 0; k < nw; k++) {
            const uint32_t wb = k & 1u;  // double-buffered: a lane may still read the last window's range
            if (tid == 0) {
                w_lo[wb] = one ? 0u : 0xFFFFFFFFu;
                w_hi[wb] = one ? (uint32_t)span : 0u;
                n_mid = 0;
            }
            lds_barrier();
            const bool in_w = short_me && (one || wk == k);
            if (!one) {
                if (in_w) {
                    atomicMin(&w_lo[wb], rel);
                    atomicMax(&w_hi[wb], rel + n_me);
                }
                lds_barrier();
            }
            const uint32_t lo_w = w_lo[wb], hi_w = w_hi[wb];
            if (lo_w >= hi_w) continue;  // uniform: no short list starts here
            LPROF(0);
            const uint64_t base = (ob + lo_w) & ~3ull;   // staging is 16-B aligned
            const uint32_t sh = (uint32_t)(ob + lo_w - base);  // ibuf[j] holds id base + j
            const uint32_t nv = (sh + (hi_w - lo_w) + 3) >> 2;  // uint4 groups (<= LIST_SPAN / 4)
            const uint4* src4 = reinterpret_cast<const uint4*>(A.ids_ord + base);
            uint4* ib4 = reinterpret_cast<uint4*>(ibuf);
            for (uint32_t g0 = 0; g0 < nv; g0 += 4 * LIST_THREADS) {  // 4 x 16 B in flight
                uint4 v[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t g = g0 + q * LIST_THREADS + tid;
                    if (g < nv) v[q] = src4[g];  // may read up to 3 ids past the range: same allocation
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t g = g0 + q * LIST_THREADS + tid;
                    if (g < nv) ib4[g] = make_uint4(v[q].x + 1u, v[q].y + 1u, v[q].z + 1u, v[q].w + 1u);
                }
            }
            lds_barrier();
            LPROF(1);
            sort_lists_lane(ibuf + sh + (rel - lo_w), in_w ? n_me : 0u);
            if (in_w && n_me > 32) mid[atomicAdd(&n_mid, 1u)] = tid;
            lds_barrier();
            LPROF(2);
            const uint32_t nmid = n_mid;
            for (uint32_t q = wid; q < nmid; q += LIST_THREADS / 64) {
                const uint32_t n = A.e_cnt[e0 + mid[q]];
                uint32_t* p = ibuf + sh + (uint32_t)(A.e_off[e0 + mid[q]] - ob - lo_w);
                if (n <= 64) wave_sort_desc<1>(p, n, lane);
                else if (n <= 128) wave_sort_desc<2>(p, n, lane);
                else wave_sort_desc<4>(p, n, lane);
                wave_sync();
            }
            lds_barrier();
            LPROF(3);
            {
                // full groups as 16-B stores, the partial first/last group per id
                const uint32_t end = sh + (hi_w - lo_w);  // ibuf index past the range
                int4* dst4 = reinterpret_cast<int4*>(A.ids_out + base);
                for (uint32_t g = tid; g < nv; g += LIST_THREADS) {
                    const uint32_t j0 = g * 4;
                    const uint4 v = ib4[g];
                    if (j0 >= sh && j0 + 4 <= end) {
                        dst4[g] = make_int4(id_of(v.x - 1u, A.read_ids, A.id_off), id_of(v.y - 1u, A.read_ids, A.id_off),
                                            id_of(v.z - 1u, A.read_ids, A.id_off), id_of(v.w - 1u, A.read_ids, A.id_off));
                    } else {
                        const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                        for (int q = 0; q < 4; q++)
                            if (j0 + q >= sh && j0 + q < end)
                                A.ids_out[base + j0 + q] = id_of(vv[q] - 1u, A.read_ids, A.id_off);
                    }
                }
            }
            // the staging area is reused: every lane's LDS reads must be done (they
            // fed its stores), but its global stores need not have landed -- a
            // full __syncthreads() would wait for them (vmcnt), 36 % of the kernel
            lds_barrier();
            LPROF(4);
#ifdef KB_BIN_PROF
            if (tid == 0) lacc[5]++, lacc[6] += nmid;
#endif
        }
        const uint32_t nbig = n_big;  // lists > WAVE_LIST_MAX: the whole block
        if (nbig) {  // it rewrites ids the windows wrote: let those land first
            __threadfence_block();
            __syncthreads();
        }
        for (uint32_t q = 0; q < nbig; q++) {
            const uint64_t ge = e0 + big[q];
            const uint32_t n = A.e_cnt[ge];
            const uint64_t o = A.e_off[ge];
            if (n <= WAVE_LIST_MAX) continue;  // uniform
            if (n <= (uint32_t)LIST_CAP) {
                uint32_t Pw = 64;
                while (Pw < n) Pw <<= 1;
                for (uint32_t j = tid; j < Pw; j += LIST_THREADS) buf[j] = j < n ? A.ids_ord[o + j] + 1u : 0u;
                __syncthreads();
                for (uint32_t kk = 2; kk <= Pw; kk <<= 1) {
                    for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                        for (uint32_t i = tid; i < Pw; i += LIST_THREADS) {
                            const uint32_t l2 = i ^ jj;
                            if (l2 > i) {
                                const uint32_t x = buf[i], y = buf[l2];
                                const bool desc = (i & kk) == 0;
                                if (desc ? (x < y) : (x > y)) {
                                    buf[i] = y;
                                    buf[l2] = x;
                                }
                            }
                        }
                        __syncthreads();
                    }
                }
                for (uint32_t j = tid; j < n; j += LIST_THREADS)
                    A.ids_out[o + j] = id_of(buf[j] - 1u, A.read_ids, A.id_off);
                __syncthreads();
            } else {
                // very long list: sort LDS-sized chunks, then merge passes
                // through ids_out (as scratch) and ids_ord, ordinals + 1
                const uint32_t C = (uint32_t)LIST_CAP;
                uint32_t* src = A.ids_ord + o;
                uint32_t* dst = reinterpret_cast<uint32_t*>(A.ids_out + o);
                for (uint32_t c0 = 0; c0 < n; c0 += C) {
                    const uint32_t cn = min(C, n - c0);
                    for (uint32_t j = tid; j < C; j += LIST_THREADS) buf[j] = j < cn ? src[c0 + j] + 1u : 0u;
                    __syncthreads();
                    for (uint32_t kk = 2; kk <= C; kk <<= 1) {
                        for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                            for (uint32_t i = tid; i < C; i += LIST_THREADS) {
                                const uint32_t l2 = i ^ jj;
                                if (l2 > i) {
                                    const uint32_t x = buf[i], y = buf[l2];
                                    const bool desc = (i & kk) == 0;
                                    if (desc ? (x < y) : (x > y)) {
                                        buf[i] = y;
                                        buf[l2] = x;
                                    }
                                }
                            }
                            __syncthreads();
                        }
                    }
                    for (uint32_t j = tid; j < cn; j += LIST_THREADS) dst[c0 + j] = buf[j];
                    __syncthreads();
                }
                __threadfence_block();
                __syncthreads();
                // merge runs of width wd from dst into src, alternating
                uint32_t* a = dst;
                uint32_t* bb = src;
                for (uint32_t wd = C; wd < n; wd <<= 1) {
                    for (uint32_t t = tid; t < n; t += LIST_THREADS) {
                        const uint32_t pair0 = (t / (2 * wd)) * 2 * wd;
                        const uint32_t an = min(wd, n - pair0);
                        const uint32_t b0 = pair0 + an, bn = b0 < n ? min(wd, n - b0) : 0u;
                        const uint32_t d = t - pair0;
                        uint32_t l1 = d > bn ? d - bn : 0u, h1 = min(d, an);
                        while (l1 < h1) {
                            const uint32_t i = (l1 + h1) >> 1;
                            if (a[pair0 + i] >= a[b0 + d - i - 1]) l1 = i + 1; else h1 = i;
                        }
                        const uint32_t i = l1, j = d - l1;
                        bb[t] = (i < an && (j >= bn || a[pair0 + i] >= a[b0 + j])) ? a[pair0 + i] : a[b0 + j];
                    }
                    __threadfence_block();
                    __syncthreads();
                    uint32_t* tmp = a;
                    a = bb;
                    bb = tmp;
                }
                // a holds the merged ordinals + 1; map into ids_out
                if (a == dst) {  // ids_out holds them already: map in place
                    for (uint32_t t = tid; t < n; t += LIST_THREADS)
                        A.ids_out[o + t] = id_of(dst[t] - 1u, A.read_ids, A.id_off);
                } else {
                    for (uint32_t t = tid; t < n; t += LIST_THREADS)
                        A.ids_out[o + t] = id_of(a[t] - 1u, A.read_ids, A.id_off);
                }
                __threadfence_block();
                __syncthreads();
            }
        }
        lds_barrier();  // (LDS only: big[], n_big and the staging area are reused)
    }
#ifdef KB_BIN_PROF
    if (tid == 0)
        for (int i = 0; i < 8; i++) atomicAdd(&g_list_prof[i], lacc[i]);
#endif
}

#ifdef KB_BIN_PROF
void lists_prof_report(hipStream_t s) {
    unsigned long long h[8];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_list_prof), sizeof(h));
    fprintf(stderr, "[list_prof] pre=%llu load=%llu small=%llu mid=%llu store=%llu chunks=%llu mid_lists=%llu\n",
            h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
    unsigned long long z[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_list_prof), z, sizeof(z));
}
#endif

// lists of 257..WAVE_LIST_MAX ids that lists_bucket_kernel passed on: one
// wavefront per list, a full bitonic network in its registers (kept out of the
// other list kernels, whose occupancy its 64-register lists would cap)
__global__ __launch_bounds__(256) void lists_long_kernel(ListArgs A) {
    const int lane = threadIdx.x & 63;
    const uint32_t nq = A.long_n[1];
    for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < nq; q += gridDim.x * 4) {
        const uint32_t e = A.long_q[A.long_cap + q];
        const uint32_t n = A.e_cnt[e];
        const uint64_t o = A.e_off[e];
        const uint32_t* src = A.ids_ord + o;
        int32_t* dst = A.ids_out + o;
        if (n <= 512) wave_sort_list_long<8>(src, dst, n, lane, A.read_ids, A.id_off);
        else if (n <= 1024) wave_sort_list_long<16>(src, dst, n, lane, A.read_ids, A.id_off);
        else if (n <= 2048) wave_sort_list_long<32>(src, dst, n, lane, A.read_ids, A.id_off);
        else wave_sort_list_long<64>(src, dst, n, lane, A.read_ids, A.id_off);
    }
}

// Lists of 257..WAVE_LIST_MAX ids (high coverage: every true k-mer's list
// is this long) by bucketing rather than a full sorting network.  One
// wavefront per list: min/max of its ordinals, NB order-preserving buckets
// over that range (an LDS histogram, a wave scan, an LDS scatter), then every
// lane sorts its own bucket(s) of <= 64 ids in registers and writes them
// straight to their place in the list.  About n (log2(64) + 3) wave steps
// against the network's n log2^2(n) / 2; a list with a bucket past 64 ids
// (clustered ordinals) is queued for the network (lists_long_kernel).
constexpr uint32_t LB_WAVES = 4;
constexpr uint32_t LB_SPAN = WAVE_LIST_MAX;  // ids per wave in LDS
constexpr uint32_t LB_ILP = 16;              // loads in flight per lane

// n <= 64 values in registers, sorted descending (0 pads last)
template <int W>
DEV void lane_sort_desc(uint32_t (&v)[W]) {
#pragma unroll
    for (int kk = 2; kk <= W; kk <<= 1) {
#pragma unroll
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
#pragma unroll
            for (int i = 0; i < W; i++) {
                const int l2 = i ^ jj;
                if (l2 > i) {
                    const uint32_t x = v[i], y = v[l2];
                    const bool desc = (i & kk) == 0;
                    const bool sw = desc ? (x < y) : (x > y);
                    v[i] = sw ? y : x;
                    v[l2] = sw ? x : y;
                }
            }
        }
    }
}


// one lane's bucket buf[off, off + c) sorted ascending in place (values >= 1)
template <int W>
DEV void lane_bucket_sort_asc(uint32_t* buf, uint32_t off, uint32_t c) {
    uint32_t v[W];
#pragma unroll
    for (int j = 0; j < W; j++) v[j] = (uint32_t)j < c ? buf[off + j] : 0u;
    lane_sort_desc<W>(v);  // the c values first, descending
#pragma unroll
    for (int j = 0; j < W; j++)
        if ((uint32_t)j < c) buf[off + c - 1u - (uint32_t)j] = v[j];
}

__global__ __launch_bounds__(LB_WAVES * 64) void lists_bucket_kernel(ListArgs A) {
    __shared__ uint32_t sbuf[LB_WAVES][LB_SPAN];
    __shared__ uint32_t scnt[LB_WAVES][256], scur[LB_WAVES][256];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t* buf = sbuf[wid];
    uint32_t* cnt = scnt[wid];
    uint32_t* cur = scur[wid];
    const uint32_t nq = *A.long_n;
    for (uint32_t q = blockIdx.x * LB_WAVES + wid; q < nq; q += gridDim.x * LB_WAVES) {
        const uint32_t e = A.long_q[q];
        const uint32_t n = A.e_cnt[e];
        const uint64_t o = A.e_off[e];
        const uint32_t* src = A.ids_ord + o;
        int32_t* dst = A.ids_out + o;
        // three passes over the list, each with LB_ILP loads in flight per lane
        // (one dependent load per iteration left every wave waiting on HBM)
        uint32_t mn = 0xFFFFFFFFu, mx = 0;
        for (uint32_t i0 = lane; i0 < n; i0 += 64u * LB_ILP) {
            uint32_t x[LB_ILP];
#pragma unroll
            for (uint32_t k = 0; k < LB_ILP; k++) x[k] = i0 + 64u * k < n ? src[i0 + 64u * k] : 0u;
#pragma unroll
            for (uint32_t k = 0; k < LB_ILP; k++)
                if (i0 + 64u * k < n) {
                    mn = min(mn, x[k]);
                    mx = max(mx, x[k]);
                }
        }
        mx = wave_max_u32(mx);
        mn = ~wave_max_u32(~mn);
        // about 16 ids per bucket: each lane then sorts its buckets with
        // 16- or 32-input networks (64 buckets for 4096 ids took 64-input ones)
        const uint32_t nb = n <= 1024 ? 64u : n <= 2048 ? 128u : 256u;
        // order-preserving bucket of an ordinal: floor((x - mn) * nb / range)
        const float scale = (float)nb / ((float)(mx - mn) + 1.0f);
        for (uint32_t b = lane; b < nb; b += 64) cnt[b] = 0;
        wave_sync();
        for (uint32_t i0 = lane; i0 < n; i0 += 64u * LB_ILP) {
            uint32_t x[LB_ILP];
#pragma unroll
            for (uint32_t k = 0; k < LB_ILP; k++) x[k] = i0 + 64u * k < n ? src[i0 + 64u * k] : 0u;
#pragma unroll
            for (uint32_t k = 0; k < LB_ILP; k++)
                if (i0 + 64u * k < n) atomicAdd(&cnt[min(nb - 1u, (uint32_t)((float)(x[k] - mn) * scale))], 1u);
        }
        wave_sync();
        // lane l owns the npl = nb / 64 adjacent buckets from ba = npl l, so one
        // wave scan of the per-lane totals places them all
        const uint32_t npl = nb / 64u, ba = npl * (uint32_t)lane;
        uint32_t c[4], tot = 0, big = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            c[k] = k < npl ? cnt[ba + k] : 0u;
            tot += c[k];
            big = max(big, c[k]);
        }
        big = wave_max_u32(big);
        if (big > 64) {  // clustered ordinals: the sorting network takes the list
            if (lane == 0) A.long_q[A.long_cap + atomicAdd(A.long_n + 1, 1u)] = e;
            continue;
        }
        const uint32_t base = wave_incl_scan(tot, lane) - tot;  // ascending offsets
        wave_sync();
        {
            uint32_t run = base;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++)
                if (k < npl) {
                    cur[ba + k] = run;
                    run += c[k];
                }
        }
        wave_sync();
        for (uint32_t i0 = lane; i0 < n; i0 += 64u * LB_ILP) {
            uint32_t x[LB_ILP];
#pragma unroll
            for (uint32_t k = 0; k < LB_ILP; k++) x[k] = i0 + 64u * k < n ? src[i0 + 64u * k] : 0u;
#pragma unroll
            for (uint32_t k = 0; k < LB_ILP; k++)
                if (i0 + 64u * k < n) {
                    const uint32_t b = min(nb - 1u, (uint32_t)((float)(x[k] - mn) * scale));
                    buf[atomicAdd(&cur[b], 1u)] = x[k] + 1u;
                }
        }
        wave_sync();
        // each lane sorts its buckets in place (ascending), so buf holds the
        // whole list ascending; the wave then writes it reversed -- descending,
        // binning.c:1065-1068 -- with coalesced stores (lanes writing their own
        // buckets straight to HBM touched 64 lines per store instruction)
        uint32_t a0 = base;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            if (k >= npl) break;  // (wave-uniform)
            if (big <= 16)
                lane_bucket_sort_asc<16>(buf, a0, c[k]);
            else if (big <= 32)
                lane_bucket_sort_asc<32>(buf, a0, c[k]);
            else
                lane_bucket_sort_asc<64>(buf, a0, c[k]);
            a0 += c[k];
        }
        wave_sync();
        for (uint32_t j = lane; j < n; j += 64) dst[j] = id_of(buf[n - 1u - j] - 1u, A.read_ids, A.id_off);
        wave_sync();
    }
}

hipError_t launch_lists(const ListArgs& a, uint64_t max_entries, hipStream_t s) {
    uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>(1, (max_entries + LIST_THREADS - 1) / LIST_THREADS), 16384);
    // queued items / long lists of the last finalize (~0: none seen yet) size
    // the grids: every list kernel strides over its queue
    auto grid = [](uint64_t hint, uint64_t per_block, uint64_t full) {
        if (hint == ~0ull) return full;
        return std::min<uint64_t>(full, std::max<uint64_t>(16, (hint + hint / 2 + 64) / per_block));
    };
    if (a.lq_items) blocks = grid(a.lq_hint, 1, blocks);
    if (!a.long_n_zeroed) {
        hipError_t e = hipMemsetAsync(a.long_n, 0, 2 * sizeof(unsigned int), s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(lists_kernel, dim3((unsigned)blocks), dim3(LIST_THREADS), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lists_bucket_kernel, dim3((unsigned)grid(a.long_hint[0], LB_WAVES, 4096)), dim3(LB_WAVES * 64), 0,
                       s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lists_long_kernel, dim3((unsigned)grid(a.long_hint[1], 4, 1024)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// Bin processing order: descending records (longest-processing-time first
// for the persistent blocks; a bin's cost follows its super-k-mers).  One
// block; counting sort over 8 classes per power of two (class = log2 of the
// count with 3 fractional bits), largest class first.
DEV uint32_t order_class(uint32_t c) {
    if (c < 8) return c;
    const uint32_t msb = 31u - (uint32_t)__clz(c);
    return msb * 8u + ((c >> (msb - 3u)) & 7u);  // <= 255
}

// ---------------------------------------------------------------------------
// Cold-pass density estimate.  The partition depth of a bin comes from the
// expected distinct keys per occurrence (rho), learned from the last
// finalize; a context's first finalize has none, and a wrong guess costs
// either overflow re-splits (distinct-heavy data, C5: 2.4 s instead of 0.13 s
// per pass) or far too many partitions (high coverage).  One HyperLogLog over
// every k-mer of the bin-ordered records (2^12 registers: about 1.6 % error)
// gives rho before the bins run.  Only the k-mer is hashed (its mmer follows
// from it in all but a few sticky-signature cases): an estimate, not a count.
// ---------------------------------------------------------------------------
constexpr int HLL_LOG2 = 12;
constexpr int HLL_THREADS = 256;

// Sampled (sample > 1): only the records of the canonical mmers with
// dest_of(mmer, sample, HLL_SALT) == 0 -- whole bins, since keys of different
// mmers never coincide, so distinct / occurrences of the sample estimates the
// whole ratio -- at 1 / sample of the expansion work; occ_out counts the
// sample's occurrences.
constexpr uint64_t HLL_SALT = 0xD1B54A32D192ED03ull;

template <int KW>
__global__ __launch_bounds__(HLL_THREADS) void hll_kernel(BinArgs A, uint64_t R, uint32_t* __restrict__ regs,
                                                          uint32_t sample, unsigned long long* occ_out) {
    __shared__ uint32_t reg[1 << HLL_LOG2];
    __shared__ unsigned long long s_occ;
    for (int i = threadIdx.x; i < (1 << HLL_LOG2); i += HLL_THREADS) reg[i] = 0;
    if (threadIdx.x == 0) s_occ = 0;
    __syncthreads();
    const int M = A.M;
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    uint64_t occ = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * HLL_THREADS + threadIdx.x; r < R; r += (uint64_t)gridDim.x * HLL_THREADS) {
        uint64_t hd;
        Span<KW> sp;
        sp.load_rec(A, (uint32_t)r, hd);
        const int n = (int)((hd >> 32) & 63u);
        const uint64_t fl = 0ull - ((hd >> 44) & 1ull);
        if (sample > 1) {
            const int so = (int)((hd >> 38) & 63u);
            const uint32_t sm = (uint32_t)(span_window(sp.word0(), sp.word1(), 0ull, 0ull, so) >> (64 - 2 * M));
            const uint32_t canon = ((hd >> 44) & 1u) ? maskM - sm : sm;
            if (dest_of(canon, sample, HLL_SALT) != 0) continue;
        }
        occ += (uint64_t)n;
        for (int j = 0; j < n; j++) {
            uint64_t hi, lo;
            sp.key(A.K, fl).code(hi, lo);
            sp.step();
            const uint64_t h = mix64(lo ^ mix64(hi + 0x2545F4914F6CDD1Dull));
            const uint32_t ix = (uint32_t)(h >> (64 - HLL_LOG2));
            const uint32_t rank = (uint32_t)__builtin_clzll((h << HLL_LOG2) | (1ull << (HLL_LOG2 - 1))) + 1u;
            atomicMax(&reg[ix], rank);
        }
    }
    if (occ) atomicAdd(&s_occ, (unsigned long long)occ);
    __syncthreads();
    for (int i = threadIdx.x; i < (1 << HLL_LOG2); i += HLL_THREADS)
        if (reg[i]) atomicMax(&regs[i], reg[i]);
    if (threadIdx.x == 0 && s_occ) atomicAdd(occ_out, s_occ);
}

// regs: 2^12 registers followed by a u64 occurrence count (zeroed here)
hipError_t launch_hll(const BinArgs& a, uint64_t R, int KW, uint32_t* regs, uint32_t sample, hipStream_t s) {
    hipError_t e = hipMemsetAsync(regs, 0, (sizeof(uint32_t) << HLL_LOG2) + sizeof(uint64_t), s);
    if (e != hipSuccess || !R) return e;
    int dev = 0, cus = 0;
    e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    const uint64_t want = (R + HLL_THREADS - 1) / HLL_THREADS;
    const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)std::max(1, cus) * 8));
    unsigned long long* occ = reinterpret_cast<unsigned long long*>(regs + (1 << HLL_LOG2));
    if (KW == 1) hipLaunchKernelGGL(hll_kernel<1>, dim3(blocks), dim3(HLL_THREADS), 0, s, a, R, regs, sample, occ);
    else hipLaunchKernelGGL(hll_kernel<2>, dim3(blocks), dim3(HLL_THREADS), 0, s, a, R, regs, sample, occ);
    return hipGetLastError();
}

// hll_estimate on the device: one block reduces the registers (sum of 2^-r,
// zero registers) and writes distinct / occurrences
__global__ __launch_bounds__(256) void hll_finish_kernel(const uint32_t* __restrict__ regs, float* __restrict__ rho) {
    __shared__ double s_sum[256];
    __shared__ int s_zero[256];
    double sum = 0.0;
    int zeros = 0;
    for (int i = threadIdx.x; i < (1 << HLL_LOG2); i += 256) {
        sum += ldexp(1.0, -(int)regs[i]);
        zeros += regs[i] == 0;
    }
    s_sum[threadIdx.x] = sum;
    s_zero[threadIdx.x] = zeros;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            s_sum[threadIdx.x] += s_sum[threadIdx.x + w];
            s_zero[threadIdx.x] += s_zero[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double m = (double)(1 << HLL_LOG2);
        double est = 0.7213 / (1.0 + 1.079 / m) * m * m / s_sum[0];
        if (est <= 2.5 * m && s_zero[0]) est = m * log(m / (double)s_zero[0]);  // small range: linear counting
        const unsigned long long occ = *reinterpret_cast<const unsigned long long*>(regs + (1 << HLL_LOG2));
        const double r = occ ? est / (double)occ : 0.25;
        *rho = (float)(r < 1e-4 ? 1e-4 : (r > 1.0 ? 1.0 : r));
    }
}

hipError_t launch_hll_finish(const uint32_t* regs, float* rho, hipStream_t s) {
    hipLaunchKernelGGL(hll_finish_kernel, dim3(1), dim3(256), 0, s, regs, rho);
    return hipGetLastError();
}

double hll_estimate(const uint32_t* regs) {
    const double m = (double)(1 << HLL_LOG2);
    double sum = 0.0;
    int zeros = 0;
    for (int i = 0; i < (1 << HLL_LOG2); i++) {
        sum += std::ldexp(1.0, -(int)regs[i]);
        zeros += regs[i] == 0;
    }
    const double est = 0.7213 / (1.0 + 1.079 / m) * m * m / sum;
    if (est <= 2.5 * m && zeros) return m * std::log(m / zeros);  // small range: linear counting
    return est;
}

__global__ __launch_bounds__(1024) void bins_order_kernel(const uint32_t* __restrict__ bcount,
                                                          const uint64_t* __restrict__ totals,
                                                          uint32_t* __restrict__ order, uint64_t max_bins) {
    constexpr uint32_t NC = 256;
    __shared__ uint32_t hist[NC];
    const uint32_t nbins = (uint32_t)min(totals[2], max_bins);
    for (uint32_t i = threadIdx.x; i < NC; i += 1024) hist[i] = 0;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += 1024) atomicAdd(&hist[order_class(bcount[b])], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive offsets, largest class first
        uint32_t acc = 0;
        for (int c = NC - 1; c >= 0; c--) {
            const uint32_t h = hist[c];
            hist[c] = acc;
            acc += h;
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += 1024) order[atomicAdd(&hist[order_class(bcount[b])], 1u)] = b;
}

hipError_t launch_bins_order(const uint32_t* bcount, const uint64_t* totals, uint32_t* order, uint64_t max_bins,
                             hipStream_t s) {
    hipLaunchKernelGGL(bins_order_kernel, dim3(1), dim3(1024), 0, s, bcount, totals, order, max_bins);
    return hipGetLastError();
}

// one descriptor per processing slot: {bin, first record, records, mmer},
// {occurrences, stage base lo, hi, 0}; stage bases are the exclusive prefix of
// the occurrences in processing order (each bin's range, as the stage counter
// handed them out before)
__global__ __launch_bounds__(1024) void bins_desc_kernel(const uint32_t* __restrict__ order,
                                                         const uint32_t* __restrict__ bstart,
                                                         const uint32_t* __restrict__ bcount,
                                                         const uint32_t* __restrict__ bmmer,
                                                         const uint32_t* __restrict__ bocc,
                                                         const uint64_t* __restrict__ totals, uint64_t max_bins,
                                                         uint4* __restrict__ desc, unsigned long long* stage_ctr) {
    __shared__ uint64_t red[16];
    const uint32_t nbins = (uint32_t)min(totals[2], max_bins);
    const uint32_t per = (nbins + 1023u) / 1024u, i0 = threadIdx.x * per;
    uint64_t mine = 0;
    for (uint32_t k = 0; k < per; k++)
        if (i0 + k < nbins) mine += bocc[order[i0 + k]];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t inc = wave_incl_scan(mine, lane);
    if (lane == 63) red[wid] = inc;
    __syncthreads();
    uint64_t run = inc - mine;
    for (int w = 0; w < 16; w++)
        if (w < wid) run += red[w];
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t i = i0 + k;
        if (i >= nbins) break;
        const uint32_t b = order[i];
        const uint32_t occ = bocc[b];
        desc[2 * (uint64_t)i] = make_uint4(b, bstart[b], bcount[b], bmmer[b]);
        desc[2 * (uint64_t)i + 1] = make_uint4(occ, (uint32_t)run, (uint32_t)(run >> 32), 0u);
        run += occ;
    }
    // bins without a count (spread runs: bocc 0) take their stage ranges from
    // the stage counter, after every described range
    if (threadIdx.x == 1023) *stage_ctr = run;
}

hipError_t launch_bins_desc(const uint32_t* order, const uint32_t* bstart, const uint32_t* bcount,
                            const uint32_t* bmmer, const uint32_t* bocc, const uint64_t* totals, uint64_t max_bins,
                            uint4* desc, unsigned long long* stage_ctr, hipStream_t s) {
    hipLaunchKernelGGL(bins_desc_kernel, dim3(1), dim3(1024), 0, s, order, bstart, bcount, bmmer, bocc, totals,
                       max_bins, desc, stage_ctr);
    return hipGetLastError();
}

// bins_order_kernel and bins_desc_kernel in one launch: the class histogram,
// the processing order (kept in LDS up to PLAN_LDS bins, else re-read from
// `order`), then the descriptors in rounds of 1024 processing slots (a block
// scan of the occurrences per round carries the stage base) -- coalesced
// descriptor stores and independent gathers, where bins_desc_kernel walked
// each thread's range of slots one dependent load after another
constexpr uint32_t PLAN_LDS = 8192;
__global__ __launch_bounds__(1024) void bins_plan_kernel(const uint32_t* __restrict__ bstart,
                                                         const uint32_t* __restrict__ bcount,
                                                         const uint32_t* __restrict__ bmmer,
                                                         const uint32_t* __restrict__ bocc,
                                                         const uint64_t* __restrict__ totals, uint64_t max_bins,
                                                         uint32_t* __restrict__ order, uint4* __restrict__ desc,
                                                         unsigned long long* stage_ctr) {
    constexpr uint32_t NC = 256;
    __shared__ uint32_t hist[NC];
    __shared__ uint32_t ordl[PLAN_LDS];
    __shared__ uint64_t red[16];
    const uint32_t t = threadIdx.x;
    const int lane = (int)(t & 63u), wid = (int)(t >> 6);
    const uint32_t nbins = (uint32_t)min(totals[2], max_bins);
    if (t < NC) hist[t] = 0;
    __syncthreads();
    for (uint32_t b = t; b < nbins; b += 1024) atomicAdd(&hist[order_class(bcount[b])], 1u);
    __syncthreads();
    // exclusive offsets, largest class first: thread t < 256 holds class 255 - t
    {
        const uint32_t h = t < NC ? hist[NC - 1u - t] : 0u;
        const uint64_t inc = wave_incl_scan((uint64_t)h, lane);
        if (lane == 63 && wid < 4) red[wid] = inc;
        __syncthreads();
        uint64_t wp = 0;
        for (int w = 0; w < wid && w < 4; w++) wp += red[w];
        if (t < NC) hist[NC - 1u - t] = (uint32_t)(wp + inc - h);
        __syncthreads();
    }
    const bool in_lds = nbins <= PLAN_LDS;
    for (uint32_t b = t; b < nbins; b += 1024) {
        const uint32_t pos = atomicAdd(&hist[order_class(bcount[b])], 1u);
        order[pos] = b;
        if (in_lds) ordl[pos] = b;
    }
    __threadfence_block();
    __syncthreads();
    uint64_t carry = 0;
    // (each round's four descriptor gathers are issued a round ahead: the
    // rounds' scans no longer wait for their loads one after another)
    auto gather = [&](uint32_t i, uint32_t& occ, uint4& d0) {
        const bool v = i < nbins;
        const uint32_t b = v ? (in_lds ? ordl[i] : order[i]) : 0u;
        occ = v ? bocc[b] : 0u;
        d0 = v ? make_uint4(b, bstart[b], bcount[b], bmmer[b]) : make_uint4(0u, 0u, 0u, 0u);
    };
    uint32_t occ_n = 0;
    uint4 d0_n = make_uint4(0u, 0u, 0u, 0u);
    gather(t, occ_n, d0_n);
    for (uint32_t base = 0; base < nbins; base += 1024) {
        const uint32_t i = base + t;
        const bool v = i < nbins;
        const uint32_t occ = occ_n;
        const uint4 d0 = d0_n;
        if (base + 1024 < nbins) gather(base + 1024 + t, occ_n, d0_n);
        const uint64_t inc = wave_incl_scan((uint64_t)occ, lane);
        if (lane == 63) red[wid] = inc;
        __syncthreads();
        uint64_t wp = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            if (w < wid) wp += red[w];
            tot += red[w];
        }
        const uint64_t run = carry + wp + inc - occ;
        if (v) {
            desc[2 * (uint64_t)i] = d0;
            desc[2 * (uint64_t)i + 1] = make_uint4(occ, (uint32_t)run, (uint32_t)(run >> 32), 0u);
        }
        carry += tot;
        __syncthreads();  // (red is the next round's)
    }
    // bins without a count (bocc 0) take their stage ranges from the stage
    // counter, after every described range
    if (t == 0) *stage_ctr = carry;
}

hipError_t launch_bins_plan(const uint32_t* bstart, const uint32_t* bcount, const uint32_t* bmmer,
                            const uint32_t* bocc, const uint64_t* totals, uint64_t max_bins, uint32_t* order,
                            uint4* desc, unsigned long long* stage_ctr, hipStream_t s) {
    hipLaunchKernelGGL(bins_plan_kernel, dim3(1), dim3(1024), 0, s, bstart, bcount, bmmer, bocc, totals, max_bins,
                       order, desc, stage_ctr);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void bins_describe_kernel(const uint64_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ starts,
                                                            const uint64_t* __restrict__ totals,
                                                            uint32_t* __restrict__ bcount,
                                                            uint32_t* __restrict__ bmmer, uint64_t max_bins) {
    const uint64_t nbins = min(totals[2], max_bins);
    for (uint64_t b = blockIdx.x * 256ull + threadIdx.x; b < nbins; b += (uint64_t)gridDim.x * 256) {
        bcount[b] = starts[b + 1] - starts[b];
        bmmer[b] = (uint32_t)(keys[starts[b]] >> 38);
    }
}

hipError_t launch_bins_describe(const uint64_t* keys, const uint32_t* starts, const uint64_t* totals,
                                uint32_t* bcount, uint32_t* bmmer, uint64_t max_bins, hipStream_t s) {
    const uint64_t blocks = std::min<uint64_t>((max_bins + 255) / 256, 1024);
    hipLaunchKernelGGL(bins_describe_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, s, keys,
                       starts, totals, bcount, bmmer, max_bins);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// bucket_kernel: one workgroup per local bucket.  The bucket's records (pay
// layout, contiguous) are read twice: pass 1 maps each record's mmer to a
// slot of a small LDS table and counts (slot, 63 - n); a block scan turns the
// counts into positions; pass 2 places every record (SoA) so that each bin is
// contiguous with its longest records first.  Bins are appended to the bin
// descriptors.  Replaces a global radix sort + gather: no random reads, one
// bucket per workgroup.
// ---------------------------------------------------------------------------
#ifndef KB_BK_THREADS
#define KB_BK_THREADS 1024  // (C2 1.784 -> 1.752 ms, profiles/r06/ab_bkt/)
#endif
constexpr int BK_THREADS = KB_BK_THREADS;  // (A/B builds: -DKB_BK_THREADS)
constexpr uint32_t BK_SLOTS = 256;  // mmers per bucket (a bucket with more is reported)

// a bucket's bins: key (mmer << SUB_BITS | context sub-bin) + 1 in an LDS table
DEV int bk_slot(uint32_t* keys, uint32_t bkey, bool insert) {
    const uint32_t k = bkey + 1u;
    uint32_t i = (uint32_t)((mix64((uint64_t)bkey) >> 32) & (BK_SLOTS - 1));
    for (uint32_t p = 0; p < BK_SLOTS; p++) {
        const uint32_t v = keys[i];
        if (v == k) return (int)i;
        if (v == 0) {
            if (!insert) return -1;
            const uint32_t old = atomicCAS(&keys[i], 0u, k);
            if (old == 0 || old == k) return (int)i;
        }
        i = (i + 1) & (BK_SLOTS - 1);
    }
    return -1;
}

// ROWS = k-mers per record rounded up to a power of two: n <= K - M + 1
// (<= 31 for K <= 31, <= 57 for K <= 63); row ROWS - n puts longest first.
// The bin key: canonical mmer << SUB_BITS | the piece's context sub-bin (0
// unless the map splits the mmer; the record pass cut every piece to one side)
template <int ROWS>
DEV void bk_decode(uint64_t h, uint64_t a, uint64_t b, uint64_t last, const BucketArgs& A, uint32_t& bkey,
                   uint32_t& row) {
    const int M = A.M;
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    const int so = (int)((h >> 38) & 63u);
    const uint32_t sm = (uint32_t)(span_window(a, b, 0ull, 0ull, so) >> (64 - 2 * M));
    const uint32_t canon = ((h >> 44) & 1u) ? maskM - sm : sm;
    const uint32_t sub = A.sub ? (uint32_t)(last & SUB_MASK) : 0u;  // (stamped by the record pass)
    bkey = (canon << SUB_BITS) | sub;
    row = (uint32_t)ROWS - (uint32_t)((h >> 32) & 63u);
}

// SPW span words per record (2: K <= 31, 4: K <= 63)
template <int SPW>
__global__ __launch_bounds__(BK_THREADS) void bucket_kernel(BucketArgs A) {
    constexpr uint32_t ROWS = SPW == 2 ? 32 : 64;
    __shared__ uint32_t keys[BK_SLOTS];
    __shared__ uint32_t hist[BK_SLOTS * ROWS];  // (slot, ROWS - n) counts, then cursors
    __shared__ uint64_t red[BK_THREADS / 64];
    __shared__ unsigned long long s_base, s_bin;
    __shared__ uint32_t s_full;
    __shared__ uint32_t socc[BK_SLOTS];  // occurrences (k-mers) per slot
    const uint32_t tid = threadIdx.x, bk = blockIdx.x;
    const uint64_t cnt = min<uint64_t>(A.bfill[bk], region_room(A.rbase, A.cap, bk));
    constexpr int RWD = 1 + SPW;  // record words
    const uint64_t* src = A.regions + region_off(A.rbase, A.cap, bk) * RWD;
    for (uint32_t i = tid; i < BK_SLOTS; i += BK_THREADS) keys[i] = 0;
    for (uint32_t i = tid; i < BK_SLOTS * ROWS; i += BK_THREADS) hist[i] = 0;
    if (tid == 0) s_full = 0;
    __syncthreads();
#ifndef KB_BK_U
#define KB_BK_U 12  // (records in flight: 4 -> 8 C2 1.809 -> 1.796 ms at 512 threads, profiles/r06/ab_bku/; 12 at 1024 threads, ab_bku3/)
#endif
#ifndef KB_BK_U4
#define KB_BK_U4 4  // (C5 share 491.6 -> 489.2 ms, profiles/r06/ab_rows/)
#endif
    constexpr int U = SPW == 2 ? KB_BK_U : KB_BK_U4;  // records in flight per thread (A/B builds: -DKB_BK_U, -DKB_BK_U4)
    for (uint64_t i0 = tid; i0 < cnt; i0 += U * BK_THREADS) {
        uint64_t h[U], a[U], b[U], z[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = i0 + (uint64_t)u * BK_THREADS;
            if (i < cnt) {
                h[u] = src[RWD * i];
                a[u] = src[RWD * i + 1];
                b[u] = src[RWD * i + 2];
                z[u] = SPW == 2 ? b[u] : (A.sub ? src[RWD * i + SPW] : 0ull);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (i0 + (uint64_t)u * BK_THREADS >= cnt) break;
            uint32_t bkey, row;
            bk_decode<ROWS>(h[u], a[u], b[u], z[u], A, bkey, row);
            const int sl = bk_slot(keys, bkey, true);
            if (sl < 0) s_full = 1;
            else atomicAdd(&hist[sl * ROWS + row], 1u);
        }
    }
    __syncthreads();
    if (s_full) {  // uniform
        if (tid == 0) atomicOr(A.status, ST_BUCKET_FULL);
        return;
    }
    // exclusive scan of the counters in (slot, row) order
    constexpr uint32_t PER = BK_SLOTS * ROWS / BK_THREADS;
    static_assert(ROWS % PER == 0, "a thread's counters lie in one slot");
    uint32_t loc[PER];
    uint64_t mine = 0;
    uint32_t kmers = 0;  // this thread's slot: k-mers = records x n, n = ROWS - row
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        loc[k] = hist[tid * PER + k];
        mine += loc[k];
        kmers += loc[k] * (ROWS - (tid * PER + k) % ROWS);
    }
    if (tid < BK_SLOTS) socc[tid] = 0;
    __syncthreads();
    if (kmers) atomicAdd(&socc[(tid * PER) / ROWS], kmers);
    const int lane = tid & 63, wid = tid >> 6;
    const uint64_t inc = wave_incl_scan(mine, lane);
    if (lane == 63) red[wid] = inc;
    __syncthreads();
    uint64_t wp = 0;
    for (int w = 0; w < wid; w++) wp += red[w];
    uint32_t run = (uint32_t)(wp + inc - mine);
    if (tid == 0) s_base = A.bbase[bk];  // exclusive prefix of the fills
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint32_t c = loc[k];
        hist[tid * PER + k] = run;
        run += c;
    }
    __syncthreads();
    // count non-empty slots, reserve bin descriptors (one per bin key: an
    // mmer, or one context sub-bin of a split mmer)
    // (the dense index of a slot among the non-empty ones, from the waves'
    // ballots -- a thread counting the set slots below it walked up to 255
    // LDS words in series)
    const bool has = tid < BK_SLOTS && keys[tid] != 0;
    const uint64_t hb = __ballot(has);
    __shared__ uint32_t wset[BK_SLOTS / 64];
    if (tid < BK_SLOTS && lane == 0) wset[wid] = (uint32_t)__popcll(hb);
    __syncthreads();
    uint32_t nb = 0, below = (uint32_t)__popcll(hb & ((1ull << lane) - 1ull));
#pragma unroll
    for (int w = 0; w < (int)(BK_SLOTS / 64); w++) {
        if (w < wid) below += wset[w];
        nb += wset[w];
    }
    if (tid == 0) s_bin = nb ? atomicAdd(A.bin_ctr, (unsigned long long)nb) : 0ull;
    __syncthreads();
    if (has) {
        const uint64_t bi = s_bin + below;
        const uint32_t first = hist[tid * ROWS];
        const uint32_t last = tid + 1 < BK_SLOTS ? hist[(tid + 1) * ROWS] : (uint32_t)cnt;
        if (bi < A.max_bins) {
            A.bstart[bi] = (uint32_t)s_base + first;
            A.bcount[bi] = last - first;
            // the mmer, and its context sub-bin above bit 16 (bin_kernel masks
            // it off; the host learns each sub-bin's records from it)
            A.bmmer[bi] = ((keys[tid] - 1u) >> SUB_BITS) | (((keys[tid] - 1u) & ((1u << SUB_BITS) - 1u)) << 16);
            if (A.bocc) A.bocc[bi] = socc[tid];
        }
    }
    __syncthreads();
    const uint64_t base = s_base;
#ifdef KB_BIN_ABL
    if (A.ablate == 2) return;
#endif
    for (uint64_t i0 = tid; i0 < cnt; i0 += U * BK_THREADS) {
        uint64_t h[U], a[U], b[U], c[U], d[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = i0 + (uint64_t)u * BK_THREADS;
            if (i < cnt) {
                h[u] = src[RWD * i];
                a[u] = src[RWD * i + 1];
                b[u] = src[RWD * i + 2];
                if constexpr (SPW == 4) {
                    c[u] = src[RWD * i + 3];
                    d[u] = src[RWD * i + 4];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (i0 + (uint64_t)u * BK_THREADS >= cnt) break;
            uint32_t bkey, row;
            bk_decode<ROWS>(h[u], a[u], b[u], SPW == 2 ? b[u] : d[u], A, bkey, row);
            const int sl = bk_slot(keys, bkey, false);
            const uint64_t pos = base + atomicAdd(&hist[sl * ROWS + row], 1u);
            if (A.rcap && pos >= A.rcap) continue;  // (a speculative launch's layout is too small: rerun)
#ifdef KB_BIN_ABL
            if (A.ablate == 1) {
                if (pos == ~0ull) A.hdr[0] = h[u] ^ a[u] ^ b[u];  // (keeps the loads alive)
                continue;
            }
#endif
            reinterpret_cast<uint4*>(A.hdr)[pos] = make_uint4((uint32_t)h[u], (uint32_t)(h[u] >> 32), (uint32_t)a[u],
                                                              (uint32_t)(a[u] >> 32));
            if constexpr (SPW == 2) {
                A.w1[pos] = b[u];
            } else {
                reinterpret_cast<uint4*>(A.w1)[pos] = make_uint4((uint32_t)b[u], (uint32_t)(b[u] >> 32), (uint32_t)c[u],
                                                                 (uint32_t)(c[u] >> 32));
                A.w3[pos] = d[u];
            }
        }
    }
}

// exclusive prefix of the bucket fills (clamped to the capacity) -> bbase[NB + 1]
__global__ __launch_bounds__(1024) void bucket_bases_kernel(const unsigned long long* __restrict__ bfill, uint64_t cap,
                                                          const uint64_t* __restrict__ rbase, uint32_t NB,
                                                          uint64_t* __restrict__ bbase) {
    __shared__ uint64_t red[16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t v = threadIdx.x < NB ? min<uint64_t>(bfill[threadIdx.x], region_room(rbase, cap, threadIdx.x)) : 0ull;
    const uint64_t inc = wave_incl_scan(v, lane);
    if (lane == 63) red[wid] = inc;
    __syncthreads();
    uint64_t wp = 0, tot = 0;
    for (int w = 0; w < 16; w++) {
        if (w < wid) wp += red[w];
        tot += red[w];
    }
    if (threadIdx.x < NB) bbase[threadIdx.x] = wp + inc - v;
    if (threadIdx.x == 0) bbase[NB] = tot;
}

hipError_t launch_bucket_sort(const BucketArgs& a, uint32_t NB, hipStream_t s) {
    if (!NB) return hipSuccess;
    if (NB > 1024) return hipErrorInvalidValue;
    if (!a.bases_ready)
        hipLaunchKernelGGL(bucket_bases_kernel, dim3(1), dim3(1024), 0, s, a.bfill, a.cap, a.rbase, NB, a.bbase);
    if (a.spw == 2)
        hipLaunchKernelGGL(bucket_kernel<2>, dim3(NB), dim3(BK_THREADS), 0, s, a);
    else if (a.spw == 4)
        hipLaunchKernelGGL(bucket_kernel<4>, dim3(NB), dim3(BK_THREADS), 0, s, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// The receiver's plan for PERT records of a block trip (record k0 + j * 256 +
// tid): the destination of its (last) piece, and of its edge piece when it is
// cut (ne > 0 k-mers), its pay-layout header and span words.  In phases, so
// that the record loads, then the map lookups, then the sub-bin lookups of all
// PERT records are in flight together (one record's chain of dependent global
// loads at a time left the kernel latency-bound).
template <int SPW, int PERT>
DEV void convert_plan(const uint64_t* __restrict__ recs, uint64_t n_rec, int rw, int M, uint32_t NB, int K,
                      const uint32_t* __restrict__ bucket_map, const uint16_t* __restrict__ sub_map, uint64_t k0,
                      uint32_t (&dst)[PERT], uint32_t (&dst2)[PERT], uint32_t (&ne)[PERT], uint32_t (&sub1)[PERT],
                      uint64_t (&pay0)[PERT], uint64_t (&ps)[PERT][SPW], bool& neg, uint64_t& kmers) {
    const uint32_t maskM = (1u << (2 * M)) - 1u, halfM = 1u << (2 * M - 1);
    uint32_t canon[PERT], me[PERT];
#pragma unroll
    for (int j = 0; j < PERT; j++) {
        const uint64_t k = k0 + (uint64_t)j * 256 + threadIdx.x;
        dst[j] = 0xFFFFFFFFu;
        ne[j] = 0;
        sub1[j] = 0;
        me[j] = 0;
        if (k >= n_rec) continue;
        const uint64_t* r = recs + k * (uint64_t)rw;
        pay0[j] = r[0];
#pragma unroll
        for (int w = 0; w < SPW; w++) ps[j][w] = w + 1 < rw ? r[w + 1] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < PERT; j++) {
        if (k0 + (uint64_t)j * 256 + threadIdx.x >= n_rec) continue;
        const uint64_t h = pay0[j];
        const uint32_t id = (uint32_t)h;
        const uint64_t lo = (h >> 32) & 0xFFFFu, n = (h >> 48) & 63u, so = (h >> 54) & 63u;
        // the signature (so <= 56) ends inside the first two span words
        const uint32_t sm = (uint32_t)(span_window(ps[j][0], ps[j][1], 0ull, 0ull, (int)so) >> (64 - 2 * M));
        const bool rev = routed_rev(h, sm, K, M);  // complement wins (binning.c:1029-1040)
        canon[j] = rev ? maskM - sm : sm;
        neg |= (int32_t)id < 0;
        kmers += n;
        pay0[j] = (uint64_t)id | (n << 32) | (so << 38) | ((uint64_t)rev << 44) | (lo << 45);
        dst[j] = 0;
    }
    if (bucket_map) {
#pragma unroll
        for (int j = 0; j < PERT; j++)
            // (K >= 2M: canon >= halfM by construction, the larger of a code and
            // its complement; K < 2M passes run without a map.  The guard bounds
            // the index whatever a received record says)
            if (dst[j] != 0xFFFFFFFFu) me[j] = canon[j] >= halfM ? bucket_map[canon[j] - halfM] : 0u;
#pragma unroll
        for (int j = 0; j < PERT; j++) {
            if (dst[j] == 0xFFFFFFFFu) continue;
            const uint32_t b = bm_depth(me[j]);
            if (!b) {
                dst[j] = me[j] & 1023u;
                continue;
            }
            const uint64_t h = pay0[j];
            const int n = (int)((h >> 32) & 63u), so = (int)((h >> 38) & 63u);
            const bool rev = ((h >> 44) & 1u) != 0;
            const int e = sub_edge(so, n, K, M, b);
            // the context at so + M: past the first two span words
            // when a long (K > 31) record's first k-mers are its edge
            const uint64_t wc = span_window(ps[j][0], ps[j][1], SPW > 2 ? ps[j][SPW > 2 ? 2 : 0] : 0ull,
                                            SPW > 3 ? ps[j][SPW > 3 ? 3 : 0] : 0ull, so + M);
            if (e > 0 && e < n) ne[j] = (uint32_t)e;
            sub1[j] = sub_ctx(so - (int)ne[j], K, M, b, wc, rev);
        }
#pragma unroll
        for (int j = 0; j < PERT; j++) {
            if (dst[j] == 0xFFFFFFFFu || !(me[j] & BM_SPLIT)) continue;
            const uint32_t off = me[j] & 0x0FFFFFFFu;
            dst[j] = sub_map[off + sub1[j]];
            if (ne[j]) dst2[j] = sub_map[off];
        }
    } else {
#pragma unroll
        for (int j = 0; j < PERT; j++)
            if (dst[j] != 0xFFFFFFFFu) dst[j] = dest_of(canon[j], NB, BUCKET_SALT);
    }
}

// the 1 + SPW words of one piece of a planned record: the edge piece (its
// first ne k-mers, same span start, sub-bin 0) or the (last) piece (k-mers
// ne.., span from base ne, signature ne closer, its sub-bin stamped)
template <int SPW>
DEV void convert_piece(uint64_t h, const uint64_t (&ps)[SPW], uint32_t ne, uint32_t sub1, uint64_t stamp, bool edge,
                       uint64_t (&o)[1 + SPW]) {
    if (edge) {
        o[0] = (h & ~(63ull << 32)) | ((uint64_t)ne << 32);
#pragma unroll
        for (int w = 0; w < SPW; w++) o[1 + w] = w + 1 == SPW ? ps[w] & ~stamp : ps[w];
    } else if (ne) {
        const uint64_t c = ne;
        const uint64_t n = (h >> 32) & 63u, so = (h >> 38) & 63u, lo = (h >> 45) & 0xFFFFu;
        o[0] = (h & 0xFFFFFFFFull) | ((n - c) << 32) | ((so - c) << 38) | (h & (1ull << 44)) | ((lo + c) << 45);
        const uint64_t sw[4] = {ps[0], ps[1], SPW > 2 ? ps[SPW > 2 ? 2 : 0] : 0ull, SPW > 3 ? ps[SPW > 3 ? 3 : 0] : 0ull};
#pragma unroll
        for (int w = 0; w < SPW; w++) {
            const uint64_t x = span_window(sw[0], sw[1], sw[2], sw[3], (int)c + 32 * w);
            o[1 + w] = w + 1 == SPW ? (x & ~stamp) | (sub1 & stamp) : x;
        }
    } else {
        o[0] = h;
#pragma unroll
        for (int w = 0; w < SPW; w++) o[1 + w] = w + 1 == SPW ? (ps[w] & ~stamp) | (sub1 & stamp) : ps[w];
    }
}

// received routed records -> local bucket regions (pay layout, ordinal = id,
// 1 + spw words); a block reserves one range per bucket for its 256 x 8
// records.  A split mmer's record goes to its context sub-bin's bucket, cut in
// two (edge piece first) when its first k-mers lie in the edge.
template <int SPW>
__global__ __launch_bounds__(256) void sk_convert_buckets_kernel(const uint64_t* __restrict__ recs, uint64_t n_rec,
                                                                 int rw, int M, uint32_t NB, int K,
                                                                 const uint32_t* __restrict__ bucket_map,
                                                                 const uint16_t* __restrict__ sub_map, int sub_stamp,
                                                                 uint64_t* __restrict__ regions, uint64_t cap,
                                                                 const uint64_t* __restrict__ rbase,
                                                                 unsigned long long* bfill, uint32_t* status,
                                                                 unsigned long long* n_kmers, int diag_group) {
    constexpr int PERT = 8;
#ifdef KB_BIN_ABL
    // (diagnostic builds only, KB_DIAG_CONVERT_GROUP: only the blocks of one
    // XCD group b % 8 == 0 convert their records -- the rest are dropped,
    // results wrong by design -- so a WRITE_SIZE pass can price cross-XCD
    // line sharing; ADVICE r04: never in the product library)
    if (diag_group && (blockIdx.x & 7u)) return;
#else
    (void)diag_group;
#endif
    __shared__ uint32_t cnt[SK_MAX_DEST];
    __shared__ unsigned long long base[SK_MAX_DEST];
    bool neg = false;
    uint64_t kmers = 0;
    const uint64_t stamp = sub_stamp ? SUB_MASK : 0ull;  // (a bucket record's last span word carries its sub-bin)
    for (uint64_t k0 = (uint64_t)blockIdx.x * 256 * PERT; k0 < n_rec; k0 += (uint64_t)gridDim.x * 256 * PERT) {
        for (uint32_t d = threadIdx.x; d < NB; d += 256) cnt[d] = 0;
        __syncthreads();
        uint32_t dst[PERT], dst2[PERT], ne[PERT], sub1[PERT];
        uint64_t pay0[PERT], ps[PERT][SPW];
        convert_plan<SPW, PERT>(recs, n_rec, rw, M, NB, K, bucket_map, sub_map, k0, dst, dst2, ne, sub1, pay0, ps,
                                neg, kmers);
#pragma unroll
        for (int j = 0; j < PERT; j++) {
            if (dst[j] == 0xFFFFFFFFu) continue;
            atomicAdd(&cnt[dst[j]], 1u);
            if (ne[j]) atomicAdd(&cnt[dst2[j]], 1u);
        }
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < NB; d += 256) {
            base[d] = cnt[d] ? atomicAdd(&bfill[d], (unsigned long long)cnt[d]) : 0ull;
            cnt[d] = 0;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PERT; j++) {
            if (dst[j] == 0xFFFFFFFFu) continue;
            uint64_t o[1 + SPW];
            if (ne[j]) {  // the edge piece first
                const uint64_t slot = base[dst2[j]] + atomicAdd(&cnt[dst2[j]], 1u);
                if (slot < region_room(rbase, cap, dst2[j])) {
                    convert_piece<SPW>(pay0[j], ps[j], ne[j], sub1[j], stamp, true, o);
                    uint64_t* op = regions + (region_off(rbase, cap, dst2[j]) + slot) * (1 + SPW);
#pragma unroll
                    for (int w = 0; w <= SPW; w++) op[w] = o[w];
                }
            }
            const uint64_t slot = base[dst[j]] + atomicAdd(&cnt[dst[j]], 1u);
            if (slot >= region_room(rbase, cap, dst[j])) continue;  // counted: the caller retries bigger
            convert_piece<SPW>(pay0[j], ps[j], ne[j], sub1[j], stamp, false, o);
            uint64_t* op = regions + (region_off(rbase, cap, dst[j]) + slot) * (1 + SPW);
#pragma unroll
            for (int w = 0; w <= SPW; w++) op[w] = o[w];
        }
        __syncthreads();
    }
    if (neg) atomicOr(status, ST_NEG_ID);
    __shared__ uint64_t sh[4];
    kmers = block_sum256(kmers, sh);
    if (threadIdx.x == 0 && kmers) atomicAdd(n_kmers, (unsigned long long)kmers);
}

hipError_t launch_sk_convert_buckets(const uint64_t* recs, uint64_t n_rec, int rw, int spw, int M, uint32_t NB,
                                     int K, const uint32_t* bucket_map, const uint16_t* sub_map, int sub_stamp,
                                     uint64_t* regions, uint64_t cap, const uint64_t* rbase, unsigned long long* bfill,
                                     uint32_t* status, unsigned long long* n_kmers, hipStream_t s) {
    if (!n_rec) return hipSuccess;
    if (NB < 1 || NB > SK_MAX_DEST || (spw != 2 && spw != 4)) return hipErrorInvalidValue;
#ifdef KB_BIN_ABL
    static const int diag = getenv("KB_DIAG_CONVERT_GROUP") ? atoi(getenv("KB_DIAG_CONVERT_GROUP")) : 0;
#else
    const int diag = 0;
#endif
    const uint64_t blocks = std::min<uint64_t>((n_rec + 2047) / 2048, 4096);
    if (spw == 2)
        hipLaunchKernelGGL(sk_convert_buckets_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, s, recs, n_rec, rw, M,
                           NB, K, bucket_map, sub_map, sub_stamp, regions, cap, rbase, bfill, status, n_kmers, diag);
    else
        hipLaunchKernelGGL(sk_convert_buckets_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, s, recs, n_rec, rw, M,
                           NB, K, bucket_map, sub_map, sub_stamp, regions, cap, rbase, bfill, status, n_kmers, diag);
    return hipGetLastError();
}

size_t bins_lds_bytes(uint32_t ts_log2, int KW) {
    const size_t TS = (size_t)1 << ts_log2;
    const size_t Q = KW == 1 ? bin_q<1>() : bin_q<2>();
    return sizeof(BinShared) + TS * (KW * sizeof(uint64_t) + sizeof(uint32_t)) +
           (size_t)BIN_WAVES * Q * (KW * sizeof(uint64_t) + sizeof(uint32_t) + sizeof(uint16_t)) +
           (KW == 2 ? PFL_WORDS * sizeof(uint32_t) : 0) + LIST_READ_PAD * sizeof(uint32_t);
}

// the bin kernel's blocks (every CU, as many as fit) and the per-launch split
// thresholds derived from them
template <int KW>
static hipError_t bins_grid(const BinArgs& a, uint64_t& blocks, int& cus, size_t& lds, BinArgs& a2) {
    const uint32_t TS = 1u << a.ts_log2;
    lds = bins_lds_bytes(a.ts_log2, KW);
    if (TS < (uint32_t)BIN_THREADS || lds > 160 * 1024) return hipErrorInvalidValue;  // (the prune loop)
    int dev = 0, per_cu = 0;
    cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bin_kernel<KW>, BIN_THREADS, lds);
    if (e != hipSuccess) return e;
    blocks = (uint64_t)std::max(1, cus) * std::max(1, per_cu);
    // split a light bin above 1/split_div of an even per-block share of the occurrences
    a2 = a;
    a2.split_occ = a.flat_l && a.split_div ? a.n_occ / ((uint64_t)blocks * a.split_div) + 1 : 0;
    a2.big_occ = a.flat_l && a.big_div ? a.n_occ / ((uint64_t)blocks * a.big_div) + 1 : 0;
    return hipSuccess;
}

// the published bins: counts, offsets, flat lists -- every kernel exits at
// once without any -- then their partitions, spread over every CU (grids:
// small when the last finalize published no such bin -- an empty launch then
// costs its dispatch only; every kernel strides over its work, so a surprise
// heavy bin is still binned, more slowly, once)
// (d_args: this finalize's bin arguments, put there by launch_bins_kw's
// bin_args_kernel -- bin_parts_kernel reads the same ones)
template <int KW>
static hipError_t launch_heavy_kw(const BinArgs& a, hipStream_t s, const BinArgs* d_args) {
    if (!a.flat_l) return hipSuccess;
    uint64_t blocks = 0;
    int cus = 0;
    size_t lds = 0;
    BinArgs a2;
    hipError_t e = bins_grid<KW>(a, blocks, cus, lds, a2);
    if (e != hipSuccess) return e;
    const bool few = a.heavy_hint == 0;
    const size_t fb_lds = (size_t)FLAT_MAX * sizeof(uint32_t);
    const unsigned fb_blocks = few ? 32u : (unsigned)std::max(1, cus) * 8u;
    hipLaunchKernelGGL(flat_count_kernel<KW>, dim3(fb_blocks), dim3(FB_THREADS), fb_lds, s, a2);
    hipLaunchKernelGGL(flat_scan_kernel, dim3(few ? 32u : 1024u), dim3(1024), 0, s, a2);
    hipLaunchKernelGGL(flat_scatter_kernel<KW>, dim3(fb_blocks), dim3(FB_THREADS), fb_lds, s, a2);
    if (a2.fs_lds)
        hipLaunchKernelGGL(flat_scatter_lds_kernel<KW>, dim3(few ? 32u : (unsigned)std::max(1, cus)),
                           dim3(FSL_THREADS), fsl_lds_bytes<KW>(), s, a2);
    hipLaunchKernelGGL(bin_parts_kernel<KW>, dim3(few ? 32u : (unsigned)blocks), dim3(BIN_THREADS), lds, s, d_args);
    return hipGetLastError();
}

template <int KW>
static hipError_t launch_bins_kw(const BinArgs& a, uint64_t max_bins, hipStream_t s, hipEvent_t* ev_bin, bool heavy,
                                 BinArgs* d_args) {
    uint64_t blocks = 0;
    int cus = 0;
    size_t lds = 0;
    BinArgs a2;
    hipError_t e = bins_grid<KW>(a, blocks, cus, lds, a2);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bin_args_kernel, dim3(1), dim3(64), 0, s, a2, d_args);
    // timing: the kernel's own start and stop (hipExtLaunchKernelGGL) -- an
    // event recorded on the stream before and after it idled the GPU ~6 us each
    hipExtLaunchKernelGGL(a.rank_mode ? bin_kernel_ranked<KW> : bin_kernel<KW>,
                          dim3((unsigned)std::min<uint64_t>(max_bins, blocks)), dim3(BIN_THREADS),
                          (std::uint32_t)lds, s, ev_bin ? ev_bin[0] : nullptr, ev_bin ? ev_bin[1] : nullptr, 0u,
                          (const BinArgs*)d_args);
    e = hipGetLastError();
    if (e != hipSuccess || !heavy) return e;
    return launch_heavy_kw<KW>(a, s, d_args);
}

hipError_t launch_bins(const BinArgs& a, uint64_t max_bins, int KW, hipStream_t s, hipEvent_t* ev_bin, bool heavy,
                       BinArgs* d_args) {
    if (!max_bins) return hipSuccess;
    return KW == 1 ? launch_bins_kw<1>(a, max_bins, s, ev_bin, heavy, d_args)
                   : launch_bins_kw<2>(a, max_bins, s, ev_bin, heavy, d_args);
}

hipError_t launch_bins_heavy(const BinArgs& a, int KW, hipStream_t s, const BinArgs* d_args) {
    return KW == 1 ? launch_heavy_kw<1>(a, s, d_args) : launch_heavy_kw<2>(a, s, d_args);
}

__global__ void bins_final_kernel(const unsigned long long* gcount, uint64_t* e_off, uint64_t* totals,
                                  uint64_t max_entries, const unsigned long long* flat_n,
                                  const unsigned long long* lq_n, const unsigned long long* pstat,
                                  const uint32_t* misc) {
    if (pstat)  // (the finalize's stats next to the totals: one copy, kbin_internal.h)
        for (int k = 0; k < KB_PSTAT; k++) totals[16 + k] = pstat[k];
    if (misc)
        for (int k = 0; k < 3; k++) totals[28 + k] = (uint64_t)misc[2 * k] | ((uint64_t)misc[2 * k + 1] << 32);
    // (the next finalize's grid hints: published heavy / split bins, queued list items)
    totals[12] = flat_n ? flat_n[0] : 0ull;
    totals[13] = lq_n ? *lq_n : 0ull;
    // on overflow the counters ran past the capacity (status says so) and the
    // bins past it wrote nothing, so no entry range is whole: publish none (the
    // lists kernel then has no work and the host reruns at the exact need)
    const uint64_t ne0 = gcount[0] >> 32, ni = gcount[0] & 0xFFFFFFFFull;
    const uint64_t ne = ne0 <= max_entries ? ne0 : 0;
    totals[0] = ne;
    totals[1] = ni;
    e_off[ne] = ni;
}

__global__ __launch_bounds__(1024) void clear_kernel(ClearList l) {
    for (int k = 0; k < l.n; k++)
        for (uint32_t i = threadIdx.x; i < l.words[k]; i += 1024) l.p[k][i] = 0u;
}

// After the record pass: R (records), the largest bucket and the status word
// next to N for the host's one mid-finalize copy, and the exclusive prefix of
// the bucket fills (clamped to the capacity) -> bbase[NB + 1], which the bucket
// ordering reads (one launch where a stats kernel and a bases kernel were two)
__global__ __launch_bounds__(1024) void bucket_stats_kernel(const unsigned long long* __restrict__ bfill, uint32_t NB,
                                                            const uint32_t* misc, uint64_t* totals, uint64_t cap,
                                                            const uint64_t* __restrict__ rbase,
                                                            uint64_t* __restrict__ bbase,
                                                            const unsigned long long* __restrict__ kpart, uint64_t nk) {
    __shared__ uint64_t red[16];
    __shared__ uint32_t mxw[16];
    const uint32_t t = threadIdx.x;
    const int lane = (int)(t & 63u), wid = (int)(t >> 6);
    // (the record pass's per-block k-mer sums: N, where a kernel of its own did it)
    uint64_t ks = 0;
    for (uint64_t i = t; i < nk; i += 1024) ks += kpart[i];
    const uint64_t f = t < NB ? bfill[t] : 0ull;  // (NB <= 1024)
    const uint64_t v = t < NB ? min<uint64_t>(f, region_room(rbase, cap, t)) : 0ull;
    const uint64_t inc = wave_incl_scan(v, lane);
    // fills < 2^32 (a region's capacity); a larger one is clamped for the max
    const uint32_t m = wave_max_u32((uint32_t)min<uint64_t>(f, 0xFFFFFFFFull));
    uint64_t fs = f;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        fs += (uint64_t)__shfl_xor((long long)fs, off, 64);
        ks += (uint64_t)__shfl_xor((long long)ks, off, 64);
    }
    if (lane == 63) red[wid] = inc;
    if (lane == 0) mxw[wid] = m;
    __shared__ uint64_t fsum[16], ksum[16];
    if (lane == 0) {
        fsum[wid] = fs;
        ksum[wid] = ks;
    }
    __syncthreads();
    uint64_t wp = 0, tot = 0, sum = 0, kt = 0;
    uint32_t mx = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) {
        if (w < wid) wp += red[w];
        tot += red[w];
        sum += fsum[w];
        kt += ksum[w];
        mx = max(mx, mxw[w]);
    }
    if (t < NB) bbase[t] = wp + inc - v;
    if (t == 0) {
        bbase[NB] = tot;
        totals[8] += kt;
        totals[12] = sum;
        totals[13] = mx;
        totals[14] = misc[0];
    }
}

hipError_t launch_bucket_stats(const unsigned long long* bfill, uint32_t NB, const uint32_t* misc, uint64_t* totals,
                               uint64_t cap, const uint64_t* rbase, uint64_t* bbase, const unsigned long long* kpart,
                               uint64_t nk, hipStream_t s) {
    if (NB > 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bucket_stats_kernel, dim3(1), dim3(1024), 0, s, bfill, NB, misc, totals, cap, rbase, bbase,
                       kpart, nk);
    return hipGetLastError();
}

hipError_t launch_clear(const ClearList& l, hipStream_t s) {
    if (l.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(clear_kernel, dim3(1), dim3(1024), 0, s, l);
    return hipGetLastError();
}

hipError_t launch_bins_final(const unsigned long long* gcount, uint64_t* e_off, uint64_t* totals,
                             uint64_t max_entries, const unsigned long long* flat_n, const unsigned long long* lq_n,
                             const unsigned long long* pstat, const uint32_t* report_misc, hipStream_t s) {
    hipLaunchKernelGGL(bins_final_kernel, dim3(1), dim3(1), 0, s, gcount, e_off, totals, max_entries, flat_n, lq_n,
                       pstat, report_misc);
    return hipGetLastError();
}

// The runtime resolves a kernel (and loads the code object holding it) at its
// first launch in the process: milliseconds spread over a context's first
// finalize.  kb_create resolves the binned path's kernels once per process and
// device instead (hipFuncGetAttributes), with the other one-time setup.
hipError_t load_bin_kernels() {
    const void* k[] = {
        (const void*)sk_thread_kernel<true>, (const void*)sk_thread_kernel<false>,
        (const void*)sk_kmers_total_kernel, (const void*)sk_convert_buckets_kernel<2>,
        (const void*)sk_convert_buckets_kernel<4>, (const void*)bucket_kernel<2>, (const void*)bucket_kernel<4>,
        (const void*)bucket_bases_kernel, (const void*)bucket_stats_kernel, (const void*)bins_order_kernel,
        (const void*)bins_desc_kernel, (const void*)bins_plan_kernel, (const void*)hll_kernel<1>, (const void*)hll_kernel<2>,
        (const void*)hll_finish_kernel, (const void*)bin_kernel<1>, (const void*)bin_kernel<2>,
        (const void*)bin_kernel_ranked<1>, (const void*)bin_kernel_ranked<2>,
        (const void*)flat_count_kernel<1>, (const void*)flat_count_kernel<2>, (const void*)flat_scan_kernel,
        (const void*)flat_scatter_kernel<1>, (const void*)flat_scatter_kernel<2>,
        (const void*)flat_scatter_lds_kernel<1>, (const void*)flat_scatter_lds_kernel<2>,
        (const void*)bin_parts_kernel<1>, (const void*)bin_parts_kernel<2>, (const void*)bins_final_kernel, (const void*)bin_args_kernel,
        (const void*)lists_kernel, (const void*)lists_bucket_kernel, (const void*)lists_long_kernel,
        (const void*)clear_kernel};
    for (const void* f : k) {
        hipFuncAttributes at;
        const hipError_t e = hipFuncGetAttributes(&at, f);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace kb

