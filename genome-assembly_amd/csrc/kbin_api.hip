// kbin_api.hip -- host side of the C-ABI declared in include/kbin.h.
//
// Owns device memory and the HIP stream of a context, plans the table size,
// and sequences the kernels of kbin_kernels.hip:
//   submit   : H2D (pinned staging) + pack, or adopt device-packed reads;
//              per-read k-mer offsets (device scan)
//   finalize : zero table -> scan_insert per batch (records) -> [retry
//              bigger on overflow] -> radix sort by slot -> runs/prune/CSR ->
//              emit read ids
//   export   : D2H of the CSR
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <ctime>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <queue>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/kbin.h"
#include "kbin_internal.h"

using namespace kb;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                      \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return fail(_e == hipErrorOutOfMemory ? KB_ENOMEM : KB_EDEVICE, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(_e), __FILE__, __LINE__);                \
    } while (0)

// (KB_DEBUG) host time in DevBuf allocations since the last report; per host
// thread (a multi-GPU group drives its contexts from one thread each)
static thread_local double g_alloc_ms = 0;
static double alloc_now_ms() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    uint64_t cap = 0;
    // Data-sized buffers (slack, the default) take 1/8 headroom, so passes
    // whose sizes wander by a few percent (the partitioned passes of one job,
    // records cut into sub-bins) do not free and map them afresh each pass: a
    // re-mapped allocation is cleared by the driver at roughly 20-25 GB/s (a
    // C3-sized stage regrown per pass cost seconds).  When the headroom does
    // not fit, the allocation is exact (no KB_ENOMEM from the headroom).
    // Fixed-size buffers (exact) allocate what they ask.
    hipError_t ensure(uint64_t n, bool slack = true) {
        if (n <= cap && p) return hipSuccess;
        const double t0 = alloc_now_ms();
        uint64_t want = std::max<uint64_t>(n, 1);
        if (slack) want += want / 8;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc((void**)&p, want * sizeof(T));
        if (e != hipSuccess && want > n) {  // no room for the headroom: exactly n
            (void)hipGetLastError();
            want = std::max<uint64_t>(n, 1);
            e = hipMalloc((void**)&p, want * sizeof(T));
        }
        if (e == hipSuccess) cap = want;
        else p = nullptr;
        const double dt = alloc_now_ms() - t0;
        g_alloc_ms += dt;
        static const bool dbg = getenv("KB_DEBUG") && atoi(getenv("KB_DEBUG")) != 0;
        if (dbg && want * sizeof(T) >= (64u << 20))
            fprintf(stderr, "[kb] alloc %.1f MB in %.2f ms\n", (double)(want * sizeof(T)) / 1e6, dt);
        return e;
    }
    hipError_t ensure_exact(uint64_t n) { return ensure(n, false); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// host buffer, grown on demand: page-locked (full-rate DMA both ways) up to
// PIN_MAX_BYTES, else -- or when the pinned allocation fails -- pageable
// malloc memory (hipMemcpyAsync into it then completes synchronously).  Pinning
// only affects the copy rate, never the result.
constexpr uint64_t PIN_MAX_BYTES = 8ull << 30;
template <typename T>
struct PinBuf {
    T* p = nullptr;
    uint64_t cap = 0;
    bool pinned = false;
    hipError_t ensure(uint64_t n) {
        if (n <= cap && p) return hipSuccess;
        release();
        const uint64_t want = std::max<uint64_t>(n, 1) + std::max<uint64_t>(n, 1) / 8;
        if (want * sizeof(T) <= PIN_MAX_BYTES &&
            hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocDefault) == hipSuccess) {
            pinned = true;
            cap = want;
            return hipSuccess;
        }
        (void)hipGetLastError();  // (a failed pinned allocation is not sticky)
        p = static_cast<T*>(malloc(want * sizeof(T)));
        if (!p) return hipErrorOutOfMemory;
        pinned = false;
        cap = want;
        return hipSuccess;
    }
    void release() {
        if (p) {
            if (pinned) (void)hipHostFree(p);
            else free(p);
        }
        p = nullptr;
        cap = 0;
        pinned = false;
    }
};

// Bump allocator over device chunks for the read batches of one context
// (packed words, lengths, ids, k-mer offsets): kb_reset rewinds it and keeps
// the chunks, so a streaming job submits batch after batch without a
// hipMalloc / hipFree per batch.
struct DevPool {
    struct Chunk {
        uint8_t* p;
        uint64_t cap;
    };
    std::vector<Chunk> chunks;
    size_t cur = 0;
    uint64_t off = 0;
    template <typename T>
    hipError_t alloc(uint64_t n, T** out) {
        const uint64_t bytes = (std::max<uint64_t>(n, 1) * sizeof(T) + 255) & ~255ull;
        for (; cur < chunks.size(); cur++, off = 0)
            if (off + bytes <= chunks[cur].cap) {
                *out = reinterpret_cast<T*>(chunks[cur].p + off);
                off += bytes;
                return hipSuccess;
            }
        Chunk ch{nullptr, std::max<uint64_t>(bytes, 64ull << 20)};
        hipError_t e = hipMalloc((void**)&ch.p, ch.cap);
        if (e != hipSuccess) return e;
        chunks.push_back(ch);
        cur = chunks.size() - 1;
        off = bytes;
        *out = reinterpret_cast<T*>(ch.p);
        return hipSuccess;
    }
    void reset() {
        cur = 0;
        off = 0;
    }
    void release() {
        for (auto& ch : chunks) (void)hipFree(ch.p);
        chunks.clear();
        reset();
    }
};

// Host ingest: two staging slots, each a pinned buffer and its device twin
// (bases | offsets | ids).  kb_submit fills one slot while the other's H2D
// copy and pack kernel run; `done` (recorded after the slot's pack) gates its
// reuse, two submits later.
struct IngestSlot {
    PinBuf<uint8_t> h;
    DevBuf<uint8_t> d;
    hipEvent_t done = nullptr;
    bool used = false;
};

struct Batch {
    const uint64_t* words = nullptr;  // adopted or owned
    const uint32_t* lens = nullptr;
    uint64_t* own_words = nullptr;
    uint32_t* own_lens = nullptr;
    uint64_t* kmer_base = nullptr;  // owned, n_reads+1
    int32_t* ids = nullptr;         // owned, n_reads
    uint64_t n_reads = 0;
    int RW = 0;
    uint64_t ord_base = 0;
    uint64_t occ_base = 0;
    uint64_t n_occ = 0;
    bool affine = false;              // ids = first_id + r (no ids array until needed)
    bool have_occ = false;            // kmer_base / n_occ computed (batch_offsets)
    int64_t first_id = 0;
    // multi-GPU routing
    bool superkmers = false;          // a batch of received super-k-mer records
    const uint64_t* recs = nullptr;   // (superkmers) caller's device records
    uint32_t* rec_base = nullptr;     // (superkmers) owned, per-record occurrence base
    bool routed = false;              // (reads) shipped by kb_route_pack: not scanned here
    uint32_t* route_offs = nullptr;   // (reads) owned [G][n_reads]
    std::vector<uint64_t> route_tot;  // (reads) records per destination
};

struct kb_ctx {
    kb_params p{};
    int KW = 1;
    int dev = 0;
    hipStream_t s = nullptr;
    std::vector<Batch> batches;
    uint64_t n_reads = 0, n_occ = 0;
    uint32_t route_G = 0;  // destinations of the last kb_route_plan
    bool route_binned = false;  // the plan came from the super-k-mer record pass
    uint64_t route_R = 0;
    bool route_affine = false;
    int64_t route_id_c = 0;
    DevBuf<unsigned long long> rcount;  // records per destination
    // owner ranks of the canonical mmers per (n_dest, part, part_n) (owner_map_dev):
    // host copy (the upload's source stays alive) and device table
    std::map<uint64_t, std::pair<std::vector<uint8_t>, DevBuf<uint8_t>>> owners;

    // host ingest (kb_submit): double-buffered pinned staging, pooled batches
    IngestSlot ring[2];
    int ring_next = 0;
    DevPool pool;
    uint32_t* h_alpha = nullptr;  // pinned: the pack status word after each slot's pack
    bool alpha_bad = false;       // a submitted read had a byte outside ACGT (sticky until kb_reset)
    bool ingest_unchecked = false;  // host batches whose alphabet status is not read yet

    // finalize working set
    DevBuf<uint64_t> table;
    uint64_t slots = 0, learned_slots = 0;
    DevBuf<uint64_t> occ_a, occ_b;  // occurrence records, radix ping-pong
    uint64_t* sorted = nullptr;
    DevBuf<uint64_t> os_flags;        // onesweep look-back words
    DevBuf<uint32_t> os_aux;          // histograms/bases, tickets, error word
    uint32_t os_epoch = 0;
    DevBuf<int32_t> read_ids;
    DevBuf<uint32_t> starts;
    DevBuf<uint32_t> e_mmer, e_cnt;
    DevBuf<uint64_t> e_hi, e_lo, e_off;
    const uint64_t* e_hi_zeroed = nullptr;  // e_hi is all zero (one-word keys: bin_kernel leaves it alone)
    uint64_t e_hi_zeroed_cap = 0;           // (an allocation may come back at the same address)
    DevBuf<uint64_t> first, e_first;  // KB_TRACK_FIRST
    DevBuf<int32_t> ids_out;
    DevBuf<uint64_t> scratch;
    DevBuf<uint32_t> misc;    // [0] status [1] n_distinct
    DevBuf<uint64_t> totals;  // [0] n_entries [1] n_ids [2] runs [4..6] binned counters
    // binned engine
    DevBuf<uint32_t> seg;      // super-k-mers per read -> exclusive scan
    DevBuf<uint64_t> pay;      // super-k-mer records, call order (3 words each)
    DevBuf<uint64_t> srec;     // the same, bin order, structure of arrays
    DevBuf<uint64_t> stage;    // per-occurrence (slot, ordinal) staging
    DevBuf<uint32_t> stage_ord;   // light bins: the stage as ordinals ...
    DevBuf<uint16_t> stage_slot;  // ... and LDS slots (6 B per occurrence)
    DevBuf<uint64_t> kstage;   // heavy bins: per-occurrence k-mer code + 1
    DevBuf<uint32_t> rrank, rord;  // ranked bins: record -> rank, rank -> ordinal (BinArgs::rank_mode)
    DevBuf<BinArgs> bargs;         // the bin kernels' arguments (launch_bins)
    DevBuf<uint32_t> long_q;   // entries with 257..4096 ids (lists_long_kernel)
    DevBuf<uint64_t> lq;       // list items for lists_kernel (BinArgs::lq_items); [0] the counter
    DevBuf<uint32_t> border;   // bin processing order
    DevBuf<uint4> bdesc;       // [2 max_bins] per processing slot: bin descriptor + stage base
    DevBuf<uint32_t> bcount, bmmer, bocc;  // bin descriptors (with starts); bocc: k-mers
    DevBuf<uint32_t> flat_list, flat_next, flat_l0, flat_off, flat_cur, flat_chunk, pool_bin, chunk_bin;  // heavy bins published for phase 1
    DevBuf<unsigned long long> flat_sbase, flat_obase, flat_n;  // flat_n[0] bins, [1] offset pool
    DevBuf<unsigned long long> pstat;  // [KB_PSTAT] path counters of the bin kernels (BinArgs::pstat)
    DevBuf<uint64_t> regions;  // local bucket regions (pay layout)
    DevBuf<unsigned long long> bfill;  // records per bucket
    DevBuf<uint64_t> bbase;  // [NB + 1] bucket output bases (bucket_bases_kernel)
    DevBuf<uint64_t> rbase;  // [NB + 1] exact region bases (a pass without a learned map)
    bool rexact = false;     // the regions of the last record pass use rbase
    uint64_t bucket_cap_used = 0;  // the region stride (records per bucket) the regions were written with
    DevBuf<uint64_t> kpart;    // per-block k-mer sums of the count pass
    int ocut_km = -1;          // (K << 8 | M) the offset cut table was made for
    uint8_t ocut[5][17] = {};  // offset partitions' ranges (offset_cuts)
    float rho = 0.f;           // learned distinct / occurrences
    float rho_tab = 0.f;       // learned table keys / occurrences under the singleton pre-filter
    bool pfl_regime = false;   // (sticky) a finalize ran light pre-filtered bins: sub-bins sized for the sketch
    bool rank_regime = false;  // (sticky) a finalize ranked bins (long lists): smaller sub-bins, so more get ranked
    DevBuf<uint32_t> hll;      // cold pass: HyperLogLog registers (launch_hll)
    bool bucket_failed = false;  // a bucket overflowed its mmer map: radix path from now on
    bool prior_off = false;      // a prior map overflowed a bucket: hash routing for first passes
    uint64_t n_occ_entries_hint = 0;  // entries of the last finalize (lists grid)
    uint64_t ecap_hint = 0;    // entry capacity for the next binned finalize
    uint32_t part = 0, part_n = 1;  // kb_set_partition: this pass's mmer partition
    // balanced local buckets: records per canonical mmer seen in earlier passes,
    // and one device map (mmer -> bucket) per (part, part_n) key
    std::vector<double> prior_p;   // bmap_prior's weight shape ((i + 1) / half)^(K - M) per canonical mmer
    std::vector<uint32_t> mmer_w;  // records per canonical mmer (all its sub-bins)
    std::vector<uint64_t> mmer_o;  // k-mer occurrences per canonical mmer
    std::unordered_map<uint64_t, uint32_t> sub_w;  // (mmer << 16 | sub-bin) -> records, split mmers of the last pass
    struct BucketMap {
        uint64_t key = 0;
        uint32_t nb = 0;
        bool stale = false;
        uint64_t want_max = 0;  // the largest bucket load the packing expects (records)
        uint64_t want_tot = 0;
        uint64_t cap = 0;       // region stride of this key's passes (records per bucket)
        uint32_t split = 0;     // mmers split into context sub-bins
        std::vector<uint32_t> h_map;  // host copy of map
        // a pass's descriptors waiting to rebuild this map (bmap_apply)
        bool pending = false;
        std::vector<uint32_t> p_mm, p_cnt, p_occ;
        double p_rho = 0;
        DevBuf<uint32_t> map;   // per canonical mmer (bm_* in kbin_internal.h)
        DevBuf<uint16_t> sub;   // buckets of the split mmers' sub-bins
    };
    std::vector<BucketMap> bmaps;
    uint64_t* h_totals = nullptr;
    uint32_t* h_misc = nullptr;

    // results
    bool finalized = false;
    uint64_t n_entries = 0, n_ids = 0, n_distinct = 0;
    PinBuf<uint32_t> h_mmer, h_cnt;  // pinned: kb_export's D2H at full rate
    PinBuf<uint64_t> h_hi, h_lo, h_off, h_first;
    PinBuf<int32_t> h_ids;
    PinBuf<uint32_t> h_bins;  // a pass's bin descriptors for map learning (mmer | sub, records, occurrences)
    PinBuf<uint8_t> map_stage;  // bucket map uploads (bmap_build)
    hipEvent_t map_done = nullptr;
    bool map_stage_used = false;
    // the bucket ordering launched before the mid-finalize wait (spec_bucket_phase)
    hipEvent_t ev_mid = nullptr;
    bool spec = false;
    uint64_t spec_rlay = 0, spec_bins = 0, prev_R = 0;
    bool exported = false;

    // timing
    int timing = 0;  // KB_TIMING_ALL / KB_TIMING_KERNEL (kb_set_timing)
    kb_timing tm{};
    uint32_t nbins_hint = 0;  // bins of the last binned finalize (flat-list threshold)
    // grid hints for kernels that usually have nothing to do (~0: not seen yet)
    uint64_t hint_heavy = ~0ull, hint_lq = ~0ull, hint_long[2] = {~0ull, ~0ull};
    uint64_t hint_entries = 0, hint_ids = 0;  // the last finalize's entries and ids (kb_reset keeps them)
    double t_fin = 0;  // (KB_DEBUG) host time the finalize started
    bool alpha_dirty = false;  // a pack kernel may have set the sticky alphabet status since it was cleared
    hipEvent_t ev[8] = {};
};

static int set_device(kb_ctx* c) {
    HIPCHK(hipSetDevice(c->dev));
    return KB_OK;
}

extern "C" int kb_abi_version(void) { return 3; }  // 2: kb_timing path counters; 3: ranked-bin counters, kb_group_*

extern "C" const char* kb_last_error(void) { return g_err.c_str(); }
// (kbin_group.hip: a group call's failure is this thread's last error too)
void kb::set_last_error(const char* msg) { g_err = msg; }

extern "C" void* kb_stream(kb_ctx* ctx) { return ctx ? (void*)ctx->s : nullptr; }

static uint64_t bin_budget(const kb_ctx* c, uint32_t NB);

extern "C" int kb_create(const kb_params* params, kb_ctx** out) {
    if (!params || !out) return fail(KB_EINVAL, "null argument");
    *out = nullptr;
    const kb_params& p = *params;
    if (p.M < 1 || p.M > 8)
        return fail(KB_EINVAL, "M=%d outside [1,8] (power_val, binning.c:17)", p.M);
    // (K < 2M: the reference's incremental branch, binning.c:992-1021, is
    // live -- the binned engine's record pass walks it, reads of <= 512 bp,
    // one GPU; kb_finalize and the routing calls check the rest)
    if (p.K > 63) return fail(KB_EINVAL, "K=%d > 63 unsupported", p.K);
    // (a k-mer holds its signature mmer: K >= M, binning.c:931-936 reads M bases
    // of every k-mer; the incremental walk starts at K - M >= 0)
    if (p.K < 1 || p.K < p.M) return fail(KB_EINVAL, "K=%d outside [M=%d, 63]", p.K, p.M);
    if (p.cutoff < 0) return fail(KB_EINVAL, "cutoff < 0");
    if (p.max_read_len < 1 || p.max_read_len > 65535)
        return fail(KB_EINVAL, "max_read_len=%d outside [1,65535]", p.max_read_len);
    if (p.flags & ~(KB_TRACK_FIRST | KB_ENGINE_TABLE | KB_ENGINE_BINNED)) return fail(KB_EINVAL, "unknown flags 0x%x", p.flags);
    if (p.table_slots && (p.table_slots & (p.table_slots - 1)))
        return fail(KB_EINVAL, "table_slots must be a power of two");
    kb_ctx* c = new kb_ctx();
    c->p = p;
    c->KW = p.K <= 31 ? 1 : 2;
    c->dev = p.device;
    int rc = set_device(c);
    if (rc) { delete c; return rc; }
    hipError_t e = hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; return fail(KB_EDEVICE, "hipStreamCreate: %s", hipGetErrorString(e)); }
    for (auto& ev : c->ev) {
        e = hipEventCreate(&ev);
        if (e != hipSuccess) { kb_destroy(c); return fail(KB_EDEVICE, "hipEventCreate"); }
    }
    e = hipHostMalloc((void**)&c->h_misc, 16 * sizeof(uint32_t), hipHostMallocDefault);
    if (e != hipSuccess) { kb_destroy(c); return fail(KB_ENOMEM, "hipHostMalloc"); }
    e = hipHostMalloc((void**)&c->h_totals, 32 * sizeof(uint64_t), hipHostMallocDefault);  // [16..23] path counters
    if (e != hipSuccess) { kb_destroy(c); return fail(KB_ENOMEM, "hipHostMalloc"); }
    e = hipHostMalloc((void**)&c->h_alpha, 2 * sizeof(uint32_t), hipHostMallocDefault);
    if (e != hipSuccess) { kb_destroy(c); return fail(KB_ENOMEM, "hipHostMalloc"); }
    c->h_alpha[0] = c->h_alpha[1] = 0;
    for (auto& sl : c->ring) {
        e = hipEventCreateWithFlags(&sl.done, hipEventDisableTiming);
        if (e != hipSuccess) { kb_destroy(c); return fail(KB_EDEVICE, "hipEventCreate"); }
    }
    e = hipEventCreateWithFlags(&c->map_done, hipEventDisableTiming);
    if (e != hipSuccess) { kb_destroy(c); return fail(KB_EDEVICE, "hipEventCreate"); }
    e = hipEventCreateWithFlags(&c->ev_mid, hipEventDisableTiming);
    if (e != hipSuccess) { kb_destroy(c); return fail(KB_EDEVICE, "hipEventCreate"); }
    {
        {
            const uint32_t hm = 1u << (2 * p.M - 1);
            c->prior_p.resize(hm);
            for (uint32_t i = 0; i < hm; i++) c->prior_p[i] = std::pow((double)(i + 1) / hm, p.K - p.M);
        }
        // the bucket maps' pinned staging (map upload, bin descriptors back):
        // page-locking takes milliseconds, so here rather than inside a finalize
        const uint64_t half = 1ull << (2 * p.M - 1), bins = bin_budget(c, 1024);
        if (c->map_stage.ensure(half * sizeof(uint32_t) + bins * sizeof(uint16_t)) != hipSuccess ||
            c->h_bins.ensure(3 * bins) != hipSuccess) {
            kb_destroy(c);
            return fail(KB_ENOMEM, "hipHostMalloc");
        }
        // The runtime sets up its host-to-device copy path for copies of this
        // size on first use (milliseconds, once per process and device): a
        // map-sized warm-up copy here keeps it out of the first finalize; so
        // does resolving the kernels (load_bin_kernels)
        static std::atomic<bool> warm[64] = {};  // (contexts of several devices may be created concurrently)
        if (p.device >= 0 && p.device < 64 && !warm[p.device].load(std::memory_order_acquire)) {
            DevBuf<uint8_t> t;
            const uint64_t nb = half * sizeof(uint32_t);
            if (t.ensure_exact(nb) == hipSuccess &&
                hipMemcpyAsync(t.p, c->map_stage.p, nb, hipMemcpyHostToDevice, c->s) == hipSuccess &&
                hipStreamSynchronize(c->s) == hipSuccess &&
                (getenv("KB_PRELOAD") && atoi(getenv("KB_PRELOAD")) == 0 ? true : load_bin_kernels() == hipSuccess))
                warm[p.device].store(true, std::memory_order_release);
            t.release();
        }
    }
    // (the zeroing goes up as a host-to-device copy: the context's first such
    // copy sets up the copy path, here rather than inside a first finalize)
    memset(c->h_totals, 0, 32 * sizeof(uint64_t));
    if (c->misc.ensure_exact(16) != hipSuccess || c->totals.ensure_exact(KB_TOTALS) != hipSuccess ||
        hipMemsetAsync(c->misc.p, 0, 16 * sizeof(uint32_t), c->s) != hipSuccess ||
        hipMemcpyAsync(c->totals.p, c->h_totals, KB_TOTALS * sizeof(uint64_t), hipMemcpyHostToDevice, c->s) !=
            hipSuccess ||
        hipStreamSynchronize(c->s) != hipSuccess) {
        kb_destroy(c);
        return fail(KB_ENOMEM, "device alloc");
    }
    *out = c;
    return KB_OK;
}

// (a batch's words, lengths, ids and k-mer offsets live in c->pool: rewound here)
static void free_batches(kb_ctx* c) {
    for (auto& b : c->batches) {
        if (b.rec_base) (void)hipFree(b.rec_base);
        if (b.route_offs) (void)hipFree(b.route_offs);
    }
    c->pool.reset();
    c->route_G = 0;
    c->batches.clear();
    c->n_reads = 0;
    c->n_occ = 0;
}

extern "C" void kb_destroy(kb_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->dev);
    if (c->s) (void)hipStreamSynchronize(c->s);
    free_batches(c);
    for (auto& sl : c->ring) {
        sl.h.release();
        sl.d.release();
        if (sl.done) (void)hipEventDestroy(sl.done);
    }
    c->pool.release();
    c->h_mmer.release(); c->h_cnt.release(); c->h_hi.release(); c->h_lo.release(); c->h_off.release();
    c->h_first.release(); c->h_ids.release(); c->h_bins.release(); c->map_stage.release();
    if (c->map_done) (void)hipEventDestroy(c->map_done);
    if (c->ev_mid) (void)hipEventDestroy(c->ev_mid);
    if (c->h_alpha) (void)hipHostFree(c->h_alpha);
    c->table.release(); c->occ_a.release();
    c->seg.release(); c->pay.release(); c->srec.release(); c->stage.release(); c->stage_ord.release(); c->stage_slot.release(); c->kstage.release(); c->rrank.release(); c->rord.release(); c->bargs.release(); c->long_q.release(); c->border.release(); c->bdesc.release(); c->bcount.release(); c->bmmer.release(); c->bocc.release();
    c->regions.release(); c->bfill.release(); c->bbase.release(); c->rbase.release(); c->kpart.release(); c->rcount.release();
    c->occ_b.release(); c->os_flags.release(); c->os_aux.release(); c->read_ids.release(); c->starts.release();
    c->e_mmer.release(); c->e_cnt.release(); c->e_hi.release(); c->e_hi_zeroed = nullptr;
    c->e_lo.release(); c->e_off.release(); c->ids_out.release(); c->scratch.release();
    c->misc.release(); c->totals.release(); c->first.release(); c->e_first.release();
    for (auto& m : c->bmaps) { m.map.release(); m.sub.release(); }
    for (auto& o : c->owners) o.second.second.release();
    c->flat_list.release(); c->flat_next.release(); c->flat_l0.release(); c->flat_off.release();
    c->flat_cur.release(); c->flat_chunk.release(); c->pool_bin.release(); c->chunk_bin.release();
    c->flat_sbase.release(); c->flat_obase.release(); c->flat_n.release(); c->hll.release();
    if (c->h_totals) (void)hipHostFree(c->h_totals);
    if (c->h_misc) (void)hipHostFree(c->h_misc);
    for (auto& ev : c->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
}

extern "C" int kb_reset(kb_ctx* c) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->s));
    free_batches(c);
    c->finalized = false;
    c->exported = false;
    c->bucket_failed = false;  // a new input gets the bucketed path again
    c->alpha_bad = false;
    c->ingest_unchecked = false;
    c->h_alpha[0] = c->h_alpha[1] = 0;
    for (auto& sl : c->ring) sl.used = false;
    if (c->alpha_dirty) {  // (only a pack kernel sets the sticky status word)
        HIPCHK(hipMemsetAsync(c->misc.p + 12, 0, sizeof(uint32_t), c->s));
        c->alpha_dirty = false;
    }
    c->n_entries = c->n_ids = c->n_distinct = 0;
    c->part = 0;  // back to one full pass
    c->part_n = 1;
    return KB_OK;
}

static bool binned_applies(const kb_ctx* c);

// Partitioned passes: the next finalize (or route) covers only the mmers of
// one partition.  Received records and the result are dropped; read batches
// are kept and re-armed (a shipped batch can be routed again for this pass).
extern "C" int kb_set_partition(kb_ctx* c, uint32_t part, uint32_t n_parts) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    if (n_parts == 0 || part >= n_parts) return fail(KB_EINVAL, "partition %u of %u", part, n_parts);
    if (n_parts > 1 && !binned_applies(c))
        return fail(KB_EINVAL, "partitioned passes need the binned engine (K <= 63, reads <= 512 bp)");
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->s));
    std::vector<Batch> keep;
    for (auto& b : c->batches) {
        if (b.superkmers) {
            if (b.rec_base) (void)hipFree(b.rec_base);
            continue;
        }
        b.routed = false;
        keep.push_back(b);
    }
    c->batches.swap(keep);
    c->route_G = 0;
    c->part = part;
    c->part_n = n_parts;
    c->finalized = false;
    c->exported = false;
    c->n_entries = c->n_ids = c->n_distinct = 0;
    return KB_OK;
}

// k-mer offsets of a batch (device scan) and its occurrence total (host sync)
static int batch_offsets(kb_ctx* c, Batch& b) {
    HIPCHK(c->pool.alloc(b.n_reads + 1, &b.kmer_base));
    const uint64_t need = kmer_base_scratch_elems(b.n_reads);
    HIPCHK(c->scratch.ensure(std::max<uint64_t>(need, c->scratch.cap)));
    HIPCHK(launch_kmer_base(b.lens, b.n_reads, c->p.K, b.kmer_base, c->scratch.p, c->scratch.cap, c->s));
    uint64_t tot = 0;
    HIPCHK(hipMemcpyAsync(&tot, b.kmer_base + b.n_reads, sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    b.n_occ = tot;
    b.have_occ = true;
    return KB_OK;
}

// the ids array of an affine batch, materialised only where a path needs it
static int batch_ids(kb_ctx* c, Batch& b) {
    if (b.ids || b.superkmers) return KB_OK;
    HIPCHK(c->pool.alloc(b.n_reads, &b.ids));
    HIPCHK(launch_fill_ids(b.ids, b.n_reads, (int32_t)b.first_id, c->s));
    return KB_OK;
}

// The alphabet status of the host batches packed so far: the slot snapshot
// taken after each pack (no wait) or, with sync, the device word itself.
static int ingest_check(kb_ctx* c, bool sync) {
    if (!c->alpha_bad && c->ingest_unchecked && sync) {
        HIPCHK(hipMemcpyAsync(c->h_alpha, c->misc.p + 12, sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
        c->ingest_unchecked = false;
        if (c->h_alpha[0] & ST_ALPHABET) c->alpha_bad = true;
    }
    if (c->alpha_bad)
        return fail(KB_EALPHABET, "read byte outside {A,C,G,T} in a submitted batch (see DESIGN.md: alphabet)");
    return KB_OK;
}

// binning.c:1150-1166 feeds process_read one fgets line at a time; here the
// host hands over batches.  A batch is copied into a pinned staging slot (the
// caller may reuse its buffer on return, as binning.c:1154 does), sent H2D and
// packed to 2-bit words on the context's stream, and kb_submit returns
// without waiting: the next submit fills the other slot meanwhile.  The
// alphabet check rides along (the pack kernel's sticky status word, read back
// two submits later or by kb_finalize).
static int submit_common(kb_ctx* c, const char* bases, const uint32_t* lens, uint64_t n_reads,
                         const int32_t* ids, int32_t first_id) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    if (c->finalized) return fail(KB_ESTATE, "submit after finalize (call kb_reset)");
    if (n_reads == 0) return KB_OK;
    if (!bases || !lens) return fail(KB_EINVAL, "null bases/lens");
    if (c->n_reads + n_reads > 0xFFFFFFFFull)
        return fail(KB_EOVERFLOW, "more than 2^32 reads per context");
    int rc = set_device(c);
    if (rc) return rc;
    uint32_t maxlen = 0;
    uint64_t nb = 0;
    for (uint64_t r = 0; r < n_reads; r++) {
        if (lens[r] > (uint32_t)c->p.max_read_len)
            return fail(KB_ETOOLONG, "read %llu has %u bases > max_read_len %d",
                        (unsigned long long)r, lens[r], c->p.max_read_len);
        maxlen = std::max(maxlen, lens[r]);
        nb += lens[r];
    }
    const int RW = (int)((std::max<uint32_t>(maxlen, 1) + 31) / 32);
    // slot layout: bases | offsets (u64, 8-B aligned) | ids
    const uint64_t o_off = (nb + 7) & ~7ull;
    const uint64_t o_ids = o_off + (n_reads + 1) * sizeof(uint64_t);
    const uint64_t bytes = o_ids + (ids ? n_reads * sizeof(int32_t) : 0);
    const int si = c->ring_next;
    IngestSlot& sl = c->ring[si];
    if (sl.used) {  // its last H2D + pack (two submits ago) must be done
        HIPCHK(hipEventSynchronize(sl.done));
        if (c->h_alpha[si] & ST_ALPHABET) c->alpha_bad = true;
    }
    rc = ingest_check(c, false);
    if (rc) return rc;
    HIPCHK(sl.h.ensure(bytes));
    HIPCHK(sl.d.ensure(bytes));
    memcpy(sl.h.p, bases, nb);
    uint64_t* hoff = reinterpret_cast<uint64_t*>(sl.h.p + o_off);
    hoff[0] = 0;
    for (uint64_t r = 0; r < n_reads; r++) hoff[r + 1] = hoff[r] + lens[r];
    if (ids) memcpy(sl.h.p + o_ids, ids, n_reads * sizeof(int32_t));
    HIPCHK(hipMemcpyAsync(sl.d.p, sl.h.p, bytes, hipMemcpyHostToDevice, c->s));
    Batch b;
    b.n_reads = n_reads;
    b.RW = RW;
    b.ord_base = c->n_reads;
    HIPCHK(c->pool.alloc(n_reads * (uint64_t)RW, &b.own_words));
    HIPCHK(c->pool.alloc(n_reads, &b.own_lens));
    b.words = b.own_words;
    b.lens = b.own_lens;
    c->alpha_dirty = true;
    HIPCHK(launch_pack(sl.d.p, reinterpret_cast<const uint64_t*>(sl.d.p + o_off),
                       n_reads, RW, b.own_words, b.own_lens, c->misc.p + 12, c->s));
    if (ids) {
        HIPCHK(c->pool.alloc(n_reads, &b.ids));
        HIPCHK(hipMemcpyAsync(b.ids, sl.d.p + o_ids, n_reads * sizeof(int32_t), hipMemcpyDeviceToDevice, c->s));
    } else {
        b.affine = true;
        b.first_id = first_id;
    }
    HIPCHK(hipMemcpyAsync(c->h_alpha + si, c->misc.p + 12, sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipEventRecord(sl.done, c->s));
    sl.used = true;
    c->ring_next ^= 1;
    c->ingest_unchecked = true;
    c->n_reads += n_reads;
    c->batches.push_back(b);
    return KB_OK;
}

extern "C" int kb_submit(kb_ctx* c, const char* bases, const uint32_t* lens, uint64_t n_reads,
                         int32_t first_id) {
    return submit_common(c, bases, lens, n_reads, nullptr, first_id);
}

extern "C" int kb_submit_ids(kb_ctx* c, const char* bases, const uint32_t* lens, uint64_t n_reads,
                             const int32_t* ids) {
    if (n_reads && !ids) return fail(KB_EINVAL, "null ids");
    return submit_common(c, bases, lens, n_reads, ids, 0);
}

extern "C" int kb_submit_packed_device(kb_ctx* c, const uint64_t* d_words, const uint32_t* d_lens,
                                       uint64_t n_reads, uint32_t wpr, int32_t first_id) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    if (c->finalized) return fail(KB_ESTATE, "submit after finalize (call kb_reset)");
    if (n_reads == 0) return KB_OK;
    if (!d_words || !d_lens) return fail(KB_EINVAL, "null device pointers");
    if ((uint64_t)wpr * 32 < 1 || wpr > 2048) return fail(KB_EINVAL, "words_per_read=%u", wpr);
    if ((uint64_t)wpr * 32 > (uint64_t)c->p.max_read_len + 31)
        return fail(KB_ETOOLONG, "words_per_read=%u exceeds max_read_len %d", wpr, c->p.max_read_len);
    if (c->n_reads + n_reads > 0xFFFFFFFFull)
        return fail(KB_EOVERFLOW, "more than 2^32 reads per context");
    int rc = set_device(c);
    if (rc) return rc;
    Batch b;
    b.words = d_words;
    b.lens = d_lens;
    b.n_reads = n_reads;
    b.RW = (int)wpr;
    b.ord_base = c->n_reads;
    b.affine = true;
    b.first_id = first_id;
    c->n_reads += n_reads;
    c->batches.push_back(b);
    return KB_OK;
}

static uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

extern "C" int kb_set_timing(kb_ctx* c, int enable) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    if (enable < 0 || enable > KB_TIMING_KERNEL) return fail(KB_EINVAL, "timing mode %d", enable);
    c->timing = enable;
    return KB_OK;
}

extern "C" int kb_get_timing(kb_ctx* c, kb_timing* out) {
    if (!c || !out) return fail(KB_EINVAL, "null argument");
    *out = c->tm;
    return KB_OK;
}

// phase events: every mode on the table engine; the binned engine's
// KB_TIMING_KERNEL records only the two events around bin_kernel (each event
// record leaves the GPU idle some 5 us: seven of them cost ~35 us per C2 step)
#define REC(i) \
    do {                                                                                     \
        if (c->timing == KB_TIMING_ALL || (c->timing && c->tm.engine == KB_ENG_TABLE))      \
            HIPCHK(hipEventRecord(c->ev[i], c->s));                                          \
    } while (0)

// words per routed super-k-mer record: header + span of n + K - 1 <= 2K - M bases
static int rec_words(const kb_ctx* c) { return 1 + (2 * c->p.K - c->p.M + 31) / 32; }

static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

// KB_DEBUG=1: one stderr line per host-side event of a finalize (diagnostics)
static double now_ms() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}
#define KB_DBG(...)                                             \
    do {                                                        \
        static const bool _on = env_int("KB_DEBUG", 0) != 0;    \
        if (_on) fprintf(stderr, "[kb] " __VA_ARGS__);          \
    } while (0)

// the binned engine (kbin_bins.hip) serves K <= 63 unless the table engine is
// forced (flag, or KB_ENGINE=table).  Two-word k-mers (K > 31) take only its
// bucketed record path: reads of <= 512 bp (or received super-k-mers), no
// forced radix path, and no bucket overflow so far -- elsewhere the table
// engine bins them.
static bool binned_applies(const kb_ctx* c) {
    if (c->p.flags & KB_ENGINE_TABLE) return false;
    if (!(c->p.flags & KB_ENGINE_BINNED)) {
        const char* e = getenv("KB_ENGINE");
        if (e && strcmp(e, "table") == 0) return false;
    }
    if (c->KW == 1) return true;
    if (c->bucket_failed || env_int("KB_BIN_RADIX", 0)) return false;
    for (auto& b : c->batches)
        if (!b.routed && !b.superkmers && b.RW > 16) return false;
    return true;
}

// ordinal -> read id over the unrouted read batches: one affine map (id =
// ordinal + id_c) when every batch has affine ids that agree, else read_ids
static int read_id_map(kb_ctx* c, bool& affine, int64_t& id_c) {
    affine = true;
    id_c = 0;
    bool first_b = true;
    for (auto& b : c->batches) {
        if (b.routed || b.superkmers) continue;
        const int64_t cb = b.first_id - (int64_t)b.ord_base;
        if (!b.affine || (!first_b && cb != id_c)) affine = false;
        id_c = cb;
        first_b = false;
    }
    if (affine) return KB_OK;
    HIPCHK(c->read_ids.ensure(std::max<uint64_t>(c->n_reads, 1)));
    for (auto& b : c->batches) {
        if (b.routed || b.superkmers || !b.n_reads) continue;
        if (b.ids)
            HIPCHK(hipMemcpyAsync(c->read_ids.p + b.ord_base, b.ids, b.n_reads * sizeof(int32_t),
                                  hipMemcpyDeviceToDevice, c->s));
        else
            HIPCHK(launch_fill_ids(c->read_ids.p + b.ord_base, b.n_reads, (int32_t)b.first_id, c->s));
    }
    return KB_OK;
}

static int binned_read_records(kb_ctx* c, uint64_t& R, uint64_t& N, bool ordered);

// Owner ranks.  The owner of a canonical mmer had been a hash
// of it modulo the ranks; the minimizer rule skews the mmers' loads (bmap_prior),
// so at 8 ranks the busiest rank bound 1.19x the mean k-mers on C2's reads,
// and 1.4-1.7x inside one pass of C4's and C5's partitioned legs (the pass
// keeps a hashed fifth or quarter of the mmers).  Instead every pass packs
// its own canonical mmers onto the ranks, heaviest expected load first, each
// onto the least-loaded rank (ties: the lower rank) -- LPT over bmap_prior's
// weight shape ((i + 1) / half)^(K - M), the expected signature frequency on
// uniform sequence: C2 at 8 ranks 1.019x.  A function of (K, M, ranks, part,
// part_n) only, so every rank and process computes the same table; mmers of
// other passes keep the hash (never routed in this pass).  K < 2M codes are
// not canonical (binning.c:992-1021): the hash, as before.
static void owner_table_host(int K, int M, uint32_t n_dest, uint32_t part, uint32_t part_n, uint8_t* out) {
    const uint32_t half = 1u << (2 * M - 1);
    std::vector<double> load(n_dest, 0.0);
    for (uint32_t i = half; i-- > 0;) {  // the weight grows with i: heaviest first
        const uint32_t mm = half + i;
        if (part_n > 1 && sk_hash_dest(mm, part_n, 0x9E3779B97F4A7C15ull) != part) {
            out[i] = (uint8_t)sk_hash_dest(mm, n_dest, 0x5851F42D4C957F2Dull);
            continue;
        }
        uint32_t r = 0;
        for (uint32_t d = 1; d < n_dest; d++)
            if (load[d] < load[r]) r = d;
        out[i] = (uint8_t)r;
        load[r] += std::pow((double)(i + 1) / half, K - M);
    }
}

extern "C" int kb_owner_table(int K, int M, uint32_t n_dest, uint32_t part, uint32_t n_parts, uint8_t* out) {
    if (!out) return fail(KB_EINVAL, "null argument");
    if (M < 1 || M > 8 || K < M || K > 63) return fail(KB_EINVAL, "K=%d, M=%d outside 1 <= M <= 8, M <= K <= 63", K, M);
    if (n_dest < 1 || n_dest > 64) return fail(KB_EINVAL, "n_dest=%u outside [1,64]", n_dest);
    if (n_parts < 1 || part >= n_parts) return fail(KB_EINVAL, "part %u of %u", part, n_parts);
    owner_table_host(K, M, n_dest, part, n_parts, out);
    return KB_OK;
}

// the context's owner table for n_dest ranks in its current pass, on the
// device (null for K < 2M: the hash)
static int owner_map_dev(kb_ctx* c, uint32_t n_dest, const uint8_t** out) {
    *out = nullptr;
    if (c->p.K < 2 * c->p.M) return KB_OK;
    const uint32_t pn = std::max(1u, c->part_n), pt = pn > 1 ? c->part : 0u;
    const uint64_t key = (uint64_t)n_dest | ((uint64_t)pt << 8) | ((uint64_t)pn << 36);
    const uint32_t half = 1u << (2 * c->p.M - 1);
    auto& t = c->owners[key];  // (a partitioned job's passes each keep theirs)
    if (!t.second.p) {
        t.first.resize(half);
        owner_table_host(c->p.K, c->p.M, n_dest, pt, pn, t.first.data());
        HIPCHK(t.second.ensure_exact(half));
        HIPCHK(hipMemcpyAsync(t.second.p, t.first.data(), half, hipMemcpyHostToDevice, c->s));
    }
    *out = t.second.p;
    return KB_OK;
}

// routing through the binned engine's record pass: records in read order,
// destination = owner(mmer); counts now, a stable sort by destination and
// the pack in kb_route_pack (same record format and order as route_kernel)
static int route_plan_binned(kb_ctx* c, uint32_t G, uint64_t* h_counts) {
    HIPCHK(c->totals.ensure(KB_TOTALS));
    uint64_t R = 0, N = 0;
    int rc = binned_read_records(c, R, N, true);  // routed records keep read order
    if (rc) return rc;
    rc = read_id_map(c, c->route_affine, c->route_id_c);
    if (rc) return rc;
    HIPCHK(c->rcount.ensure(64));
    HIPCHK(hipMemsetAsync(c->rcount.p, 0, 64 * sizeof(unsigned long long), c->s));
    const uint8_t* om = nullptr;
    rc = owner_map_dev(c, G, &om);
    if (rc) return rc;
    HIPCHK(launch_route_dest(c->occ_a.p, R, G, om, c->p.M, c->occ_b.p, c->rcount.p, c->s));
    std::vector<unsigned long long> cnt(G);
    HIPCHK(hipMemcpyAsync(cnt.data(), c->rcount.p, G * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    uint64_t tot = 0;
    for (uint32_t d = 0; d < G; d++) {
        h_counts[d] = cnt[d];
        tot += h_counts[d];
    }
    if (tot != R) return fail(KB_EDEVICE, "internal: routed %llu of %llu records", (unsigned long long)tot,
                              (unsigned long long)R);
    if (R > 0xFFFFFFFFull) return fail(KB_EOVERFLOW, "more than 2^32 routed records");
    c->route_binned = true;
    c->route_R = R;
    c->route_G = G;
    return KB_OK;
}

static int route_pack_binned(kb_ctx* c, uint64_t* d_send) {
    const uint64_t R = c->route_R;
    if (R && !d_send) return fail(KB_EINVAL, "null send buffer");
    int bits = 1;
    while ((1u << bits) < c->route_G) bits++;
    const uint64_t nflags = onesweep_flag_elems(R);
    if (c->os_flags.cap < nflags || c->os_epoch > (1u << 24) - 8) {
        HIPCHK(c->os_flags.ensure(nflags));
        HIPCHK(hipMemsetAsync(c->os_flags.p, 0, c->os_flags.cap * sizeof(uint64_t), c->s));
        c->os_epoch = 0;
    }
    HIPCHK(c->os_aux.ensure(4 * 256 + 8));
    uint64_t* sorted = nullptr;
    HIPCHK(launch_onesweep(c->occ_b.p, c->occ_a.p, R, bits, c->os_flags.p, c->os_aux.p, &c->os_epoch,
                           &sorted, c->s));
    HIPCHK(launch_route_pack_binned(sorted, c->pay.p, R, rec_words(c),
                                    c->route_affine ? nullptr : c->read_ids.p,
                                    (uint32_t)(c->route_affine ? c->route_id_c : 0), d_send, c->s));
    if (R) HIPCHK(hipMemcpyAsync(c->h_misc + 8, c->os_aux.p + 1028, sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
    else c->h_misc[8] = 0;
    HIPCHK(hipStreamSynchronize(c->s));
    if (c->h_misc[8]) return fail(KB_EDEVICE, "radix look-back timed out (device error word %u)", c->h_misc[8]);
    for (auto& b : c->batches)
        if (!b.superkmers) b.routed = true;
    c->route_G = 0;
    c->route_binned = false;
    return KB_OK;
}

extern "C" int kb_record_words(kb_ctx* c, uint32_t* out) {
    if (!c || !out) return fail(KB_EINVAL, "null argument");
    *out = (uint32_t)rec_words(c);
    return KB_OK;
}

extern "C" int kb_route_plan(kb_ctx* c, uint32_t n_dest, uint64_t* h_counts) {
    if (!c || !h_counts) return fail(KB_EINVAL, "null argument");
    // (K < 2M: routed records carry the complement flag, ROUTED_REV_BIT; the
    // binned engine's record pass walks the live incremental branch)
    if (c->p.K < 2 * c->p.M && !(binned_applies(c) && c->KW == 1))
        return fail(KB_EINVAL, "K=%d < 2M=%d routes through the binned engine only", c->p.K, 2 * c->p.M);
    if (n_dest < 1 || n_dest > 64) return fail(KB_EINVAL, "n_dest=%u outside [1,64]", n_dest);
    if (c->finalized) return fail(KB_ESTATE, "route after finalize (call kb_reset)");
    int rc = set_device(c);
    if (rc) return rc;
    // every host batch routed from here must be ACGT: records built from an
    // invalid read would otherwise reach the peers, whose finalize succeeds
    rc = ingest_check(c, true);
    if (rc) return rc;
    if (binned_applies(c) && c->KW == 1) return route_plan_binned(c, n_dest, h_counts);
    c->route_binned = false;
    std::vector<uint64_t> tot(n_dest, 0);
    for (auto& b : c->batches) {
        if (b.superkmers || b.routed) continue;
        const uint64_t cells = (uint64_t)n_dest * b.n_reads;
        rc = batch_ids(c, b);
        if (rc) return rc;
        if (b.route_offs) (void)hipFree(b.route_offs);
        b.route_offs = nullptr;
        HIPCHK(hipMalloc((void**)&b.route_offs, std::max<uint64_t>(cells, 1) * sizeof(uint32_t)));
        RouteArgs a{};
        a.words = b.words;
        a.lens = b.lens;
        a.ids = b.ids;
        a.n_reads = b.n_reads;
        a.offs = b.route_offs;
        a.G = n_dest;
        a.part = c->part;
        a.part_n = c->part_n;
        a.rec_words = rec_words(c);
        a.RW = b.RW;
        a.K = c->p.K;
        a.M = c->p.M;
        rc = owner_map_dev(c, n_dest, &a.owner_map);
        if (rc) return rc;
        HIPCHK(launch_route(a, false, c->s));
        // dest-major exclusive scan -> every (dest, read) slot in a dest-major buffer
        HIPCHK(c->scratch.ensure(std::max(scan_u32_scratch_elems(cells), c->scratch.cap)));
        std::vector<uint32_t> edge(n_dest + 1, 0);
        HIPCHK(launch_scan_u32(b.route_offs, cells, c->scratch.p, c->scratch.cap, c->s));
        uint64_t grand = 0;
        const uint64_t nb = scan_u32_scratch_elems(cells) - 2;
        HIPCHK(hipMemcpyAsync(&grand, c->scratch.p + nb, 8, hipMemcpyDeviceToHost, c->s));
        for (uint32_t d = 0; d < n_dest; d++)
            HIPCHK(hipMemcpyAsync(&edge[d], b.route_offs + (uint64_t)d * b.n_reads, 4,
                                  hipMemcpyDeviceToHost, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
        edge[n_dest] = (uint32_t)grand;
        b.route_tot.assign(n_dest, 0);
        for (uint32_t d = 0; d < n_dest; d++) {
            b.route_tot[d] = (uint64_t)edge[d + 1] - edge[d];
            tot[d] += b.route_tot[d];
        }
    }
    c->route_G = n_dest;
    for (uint32_t d = 0; d < n_dest; d++) h_counts[d] = tot[d];
    return KB_OK;
}

// kb_route_scatter (destinations = owner ranks) and kb_split_passes
// (destinations = kb_set_partition passes): one super-k-mer pass into
// per-destination regions, the destination a hash of the canonical mmer
static int scatter_regions(kb_ctx* c, uint32_t n_dest, uint64_t* d_regions, uint64_t region_cap,
                           uint64_t* h_counts, uint64_t salt, bool by_pass);

extern "C" int kb_route_scatter(kb_ctx* c, uint32_t n_dest, uint64_t* d_regions, uint64_t region_cap,
                                uint64_t* h_counts) {
    return scatter_regions(c, n_dest, d_regions, region_cap, h_counts, 0x5851F42D4C957F2Dull, false);
}

extern "C" int kb_split_passes(kb_ctx* c, uint32_t n_parts, uint64_t* d_regions, uint64_t region_cap,
                               uint64_t* h_counts) {
    return scatter_regions(c, n_parts, d_regions, region_cap, h_counts, 0x9E3779B97F4A7C15ull, true);
}

static int scatter_regions(kb_ctx* c, uint32_t n_dest, uint64_t* d_regions, uint64_t region_cap,
                           uint64_t* h_counts, uint64_t salt, bool by_pass) {
    if (!c || !h_counts) return fail(KB_EINVAL, "null argument");
    if (n_dest < 1 || n_dest > 64) return fail(KB_EINVAL, "n_dest=%u outside [1,64]", n_dest);
    if (by_pass && c->part_n > 1) return fail(KB_ESTATE, "kb_split_passes on a partitioned context");
    if (c->finalized) return fail(KB_ESTATE, "route after finalize (call kb_reset)");
    if (!binned_applies(c)) return fail(KB_EINVAL, "kb_route_scatter needs the binned engine (use plan/pack)");
    for (auto& b : c->batches)
        if (!b.routed && !b.superkmers && b.RW > 16)
            return fail(KB_EINVAL, "kb_route_scatter serves reads of <= 512 bp (use plan/pack)");
    if (region_cap && !d_regions) return fail(KB_EINVAL, "null regions");
    if (region_cap >= 0xFFFFFFFFull) return fail(KB_EINVAL, "region_cap must be below 2^32 records");
    int rc = set_device(c);
    if (rc) return rc;
    rc = ingest_check(c, true);  // (as kb_route_plan: nothing invalid leaves this context)
    if (rc) return rc;
    bool affine = false;
    int64_t id_c = 0;
    rc = read_id_map(c, affine, id_c);
    if (rc) return rc;
    HIPCHK(c->rcount.ensure(64));
    HIPCHK(hipMemsetAsync(c->rcount.p, 0, 64 * sizeof(unsigned long long), c->s));
    for (auto& b : c->batches) {
        if (b.routed || b.superkmers || !b.n_reads) continue;
        SkScanArgs a{};
        a.part = c->part;
        a.part_n = c->part_n;
        a.words = b.words;
        a.lens = b.lens;
        a.n_reads = b.n_reads;
        a.ord_base = (uint32_t)b.ord_base;
        a.RW = b.RW;
        a.K = c->p.K;
        a.M = c->p.M;
        a.regions = d_regions;
        a.region_cap = region_cap;
        a.dest_ctr = c->rcount.p;
        (void)by_pass;
        a.read_ids = affine ? nullptr : c->read_ids.p;
        a.id_off = (uint32_t)(affine ? id_c : 0);
        a.G = n_dest;
        a.dest_salt = salt;  // owner_of (kbin_kernels.hip), or in_part's PART_SALT (kbin_bins.hip)
        if (!by_pass) {  // ranks: the pass's owner table (passes: the partition hash)
            const int orc = owner_map_dev(c, n_dest, &a.owner_map);
            if (orc) return orc;
        }
        a.rw = rec_words(c);
        HIPCHK(launch_sk(a, true, c->s));
    }
    std::vector<unsigned long long> cnt(n_dest);
    HIPCHK(hipMemcpyAsync(cnt.data(), c->rcount.p, n_dest * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    bool over = false;
    for (uint32_t d = 0; d < n_dest; d++) {
        h_counts[d] = cnt[d];
        over |= cnt[d] > region_cap;
    }
    if (over) return fail(KB_EOVERFLOW, "a destination needs more than %llu records (see counts)",
                          (unsigned long long)region_cap);
    for (auto& b : c->batches)
        if (!b.superkmers) b.routed = true;
    return KB_OK;
}

extern "C" int kb_route_pack(kb_ctx* c, uint64_t* d_send) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    if (!c->route_G) return fail(KB_ESTATE, "kb_route_pack before kb_route_plan");
    int rc = set_device(c);
    if (rc) return rc;
    if (c->route_binned) return route_pack_binned(c, d_send);
    const uint32_t G = c->route_G;
    // destination d's records start at sum_{d'<d} total(d'); inside it, batches in order
    std::vector<uint64_t> dest_base(G, 0), seen(G, 0);
    {
        std::vector<uint64_t> tot(G, 0);
        for (auto& b : c->batches)
            if (!b.superkmers && !b.routed && b.route_offs)
                for (uint32_t d = 0; d < G; d++) tot[d] += b.route_tot[d];
        uint64_t acc = 0;
        for (uint32_t d = 0; d < G; d++) {
            dest_base[d] = acc;
            acc += tot[d];
        }
        if (acc && !d_send) return fail(KB_EINVAL, "null send buffer");
        if (acc > 0xFFFFFFFFull) return fail(KB_EOVERFLOW, "more than 2^32 routed records");
    }
    DevBuf<uint64_t> adj;
    HIPCHK(adj.ensure(G));
    for (auto& b : c->batches) {
        if (b.superkmers || b.routed || !b.route_offs) continue;
        std::vector<uint64_t> h_adj(G);
        uint64_t below = 0;  // sum_{d'<d} total_b(d'): already inside the scanned offsets
        for (uint32_t d = 0; d < G; d++) {
            h_adj[d] = dest_base[d] + seen[d] - below;
            below += b.route_tot[d];
            seen[d] += b.route_tot[d];
        }
        HIPCHK(hipMemcpyAsync(adj.p, h_adj.data(), G * 8, hipMemcpyHostToDevice, c->s));
        RouteArgs a{};
        a.words = b.words;
        a.lens = b.lens;
        a.ids = b.ids;
        a.n_reads = b.n_reads;
        a.offs = b.route_offs;
        a.adj = adj.p;
        a.out = d_send;
        a.G = G;
        a.part = c->part;  // the same records the plan counted
        a.part_n = c->part_n;
        a.rec_words = rec_words(c);
        a.RW = b.RW;
        a.K = c->p.K;
        a.M = c->p.M;
        {
            const int orc = owner_map_dev(c, G, &a.owner_map);  // (the plan's table)
            if (orc) return orc;
        }
        HIPCHK(launch_route(a, true, c->s));
        HIPCHK(hipStreamSynchronize(c->s));  // h_adj / adj reuse
        b.routed = true;
    }
    adj.release();
    c->route_G = 0;
    return KB_OK;
}

extern "C" int kb_submit_superkmers_device(kb_ctx* c, const uint64_t* d_recs, uint64_t n_rec) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    if (c->finalized) return fail(KB_ESTATE, "submit after finalize (call kb_reset)");
    if (n_rec == 0) return KB_OK;
    if (!d_recs) return fail(KB_EINVAL, "null records");
    if (n_rec > 0xFFFFFFFFull) return fail(KB_EOVERFLOW, "more than 2^32 records");
    int rc = set_device(c);
    if (rc) return rc;
    Batch b;
    b.superkmers = true;
    b.recs = d_recs;
    b.n_reads = n_rec;
    c->batches.push_back(b);  // occurrence offsets are computed by the engine that bins them
    return KB_OK;
}

// the table engine's per-record occurrence offsets of a received batch
static int sk_batch_offsets(kb_ctx* c, Batch& b) {
    HIPCHK(hipMalloc((void**)&b.rec_base, std::max<uint64_t>(b.n_reads, 1) * sizeof(uint32_t)));
    HIPCHK(launch_sk_counts(b.recs, b.n_reads, rec_words(c), b.rec_base, c->s));
    HIPCHK(c->scratch.ensure(std::max(scan_u32_scratch_elems(b.n_reads), c->scratch.cap)));
    HIPCHK(launch_scan_u32(b.rec_base, b.n_reads, c->scratch.p, c->scratch.cap, c->s));
    uint64_t tot = 0;
    const uint64_t nb = scan_u32_scratch_elems(b.n_reads) - 2;
    HIPCHK(hipMemcpyAsync(&tot, c->scratch.p + nb, 8, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    b.n_occ = tot;
    b.have_occ = true;
    return KB_OK;
}

static int log2u(uint64_t x) {
    int b = 0;
    while ((1ull << b) < x) b++;
    return b;
}

// ---------------------------------------------------------------------------
// binned engine (kbin_bins.hip): super-k-mers -> sort by mmer -> one LDS
// table per bin.  Eligible for K <= 31 reads binned here, no first-occurrence
// tracking.
// ---------------------------------------------------------------------------

// ---- phase A (reads): one record per super-k-mer of every unrouted read
// batch -- pay[3t..3t+2] and keys[t] in occ_a, t in read order; returns the
// record count R and the k-mer count N (one host sync)
static int binned_read_records(kb_ctx* c, uint64_t& R, uint64_t& N, bool ordered) {
    const int M = c->p.M;
    const uint64_t nr = c->n_reads;
    // one pass (records allocated per block, any order) when every batch takes
    // the thread-per-read kernel and the buffers sized by the k-mer bound fit
    uint64_t nb = 0;
    bool one_pass = !ordered;
    for (auto& b : c->batches) {
        if (b.routed || b.superkmers) continue;
        if (b.RW > 16) one_pass = false;
        nb += b.n_reads * (uint64_t)std::max(0, b.RW * 32 - c->p.K + 1);
    }
    if (one_pass && nb < 0xFFFFFFFFull && nb * 40 <= (32ull << 30)) {
        HIPCHK(c->pay.ensure(3 * nb + 3));
        HIPCHK(c->occ_a.ensure(nb + 4));
        HIPCHK(c->occ_b.ensure(nb + 4));  // radix ping-pong (R <= nb) and ids by ordinal
        HIPCHK(hipMemsetAsync(c->totals.p + 8, 0, 2 * sizeof(uint64_t), c->s));
        uint64_t kp = 1;
        for (auto& b : c->batches) kp = std::max(kp, sk_blocks(b.n_reads, b.RW));
        HIPCHK(c->kpart.ensure(kp));
        for (auto& b : c->batches) {
            if (b.routed || b.superkmers) continue;
            SkScanArgs a{};
            a.part = c->part;
            a.part_n = c->part_n;
            a.words = b.words;
            a.lens = b.lens;
            a.n_reads = b.n_reads;
            a.rec_ctr = reinterpret_cast<unsigned long long*>(c->totals.p + 9);
            a.n_kmers = reinterpret_cast<unsigned long long*>(c->kpart.p);
            a.pay = c->pay.p;
            a.keys = c->occ_a.p;
            a.ord_base = (uint32_t)b.ord_base;
            a.RW = b.RW;
            a.K = c->p.K;
            a.M = M;
            HIPCHK(launch_sk(a, true, c->s));
            HIPCHK(launch_sk_kmers_total(reinterpret_cast<unsigned long long*>(c->kpart.p),
                                         sk_blocks(b.n_reads, b.RW),
                                         reinterpret_cast<unsigned long long*>(c->totals.p + 8), c->s));
            c->tm.scan_insert_launches++;
        }
        HIPCHK(hipMemcpyAsync(c->h_totals + 8, c->totals.p + 8, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
        HIPCHK(hipStreamSynchronize(c->s));  // the one mid-finalize sync: R and N size the rest
        N = c->h_totals[8];
        R = c->h_totals[9];
        if (R > N || N > nb)
            return fail(KB_EDEVICE, "internal: %llu super-k-mers, %llu k-mers, bound %llu", (unsigned long long)R,
                        (unsigned long long)N, (unsigned long long)nb);
        HIPCHK(c->srec.ensure(3 * R));
        return KB_OK;
    }
    HIPCHK(c->seg.ensure(nr + 1));
    HIPCHK(hipMemsetAsync(c->seg.p, 0, (nr + 1) * sizeof(uint32_t), c->s));
    HIPCHK(c->scratch.ensure(std::max(scan_u32_scratch_elems(nr + 1), c->scratch.cap)));
    HIPCHK(hipMemsetAsync(c->totals.p + 8, 0, sizeof(uint64_t), c->s));
    {
        uint64_t kp = 1;
        for (auto& b : c->batches) kp = std::max(kp, sk_blocks(b.n_reads, b.RW));
        HIPCHK(c->kpart.ensure(kp));
    }
    for (auto& b : c->batches) {
        if (b.routed || b.superkmers) continue;
        SkScanArgs a{};
        a.part = c->part;
        a.part_n = c->part_n;
        a.words = b.words;
        a.lens = b.lens;
        a.n_reads = b.n_reads;
        a.seg_count = c->seg.p + b.ord_base;
        a.n_kmers = reinterpret_cast<unsigned long long*>(c->kpart.p);
        a.RW = b.RW;
        a.K = c->p.K;
        a.M = M;
        HIPCHK(launch_sk(a, false, c->s));
        HIPCHK(launch_sk_kmers_total(reinterpret_cast<unsigned long long*>(c->kpart.p), sk_blocks(b.n_reads, b.RW),
                                     reinterpret_cast<unsigned long long*>(c->totals.p + 8), c->s));
        c->tm.scan_insert_launches++;
    }
    HIPCHK(launch_scan_u32(c->seg.p, nr, c->scratch.p, c->scratch.cap, c->s));
    const uint64_t nbs = scan_u32_scratch_elems(nr) - 2;
    HIPCHK(hipMemcpyAsync(c->h_totals + 7, c->scratch.p + nbs, 8, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipMemcpyAsync(c->h_totals + 8, c->totals.p + 8, 8, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));  // the one mid-finalize sync: R and N size the rest
    R = nr ? c->h_totals[7] : 0;
    N = nr ? c->h_totals[8] : 0;
    if (N >= 0xFFFFFFFFull)
        return fail(KB_EOVERFLOW, "%llu k-mer occurrences in one context (limit 2^32-1)",
                    (unsigned long long)N);
    if (R > N) return fail(KB_EDEVICE, "internal: %llu super-k-mers > %llu k-mers", (unsigned long long)R,
                           (unsigned long long)N);
    HIPCHK(c->pay.ensure(3 * R));
    HIPCHK(c->srec.ensure(3 * R));
    HIPCHK(c->occ_a.ensure(std::max<uint64_t>(R, N / 2 + 4)));
    HIPCHK(c->occ_b.ensure(std::max<uint64_t>(R, N / 2 + 4))  /* ids (u32) + 16-B over-read */);
    for (auto& b : c->batches) {
        if (b.routed || b.superkmers) continue;
        SkScanArgs a{};
        a.part = c->part;
        a.part_n = c->part_n;
        a.words = b.words;
        a.lens = b.lens;
        a.n_reads = b.n_reads;
        a.rec_base = c->seg.p + b.ord_base;
        a.pay = c->pay.p;
        a.keys = c->occ_a.p;
        a.ord_base = (uint32_t)b.ord_base;
        a.RW = b.RW;
        a.K = c->p.K;
        a.M = M;
        HIPCHK(launch_sk(a, true, c->s));
        c->tm.scan_insert_launches++;
    }
    return KB_OK;
}

// ---- balanced local buckets.  A bucket's records are ordered by ONE
// workgroup (bucket_kernel), so the largest bucket sets that kernel's time.
// The minimizer rule (leftmost max of the complement-canonical score) makes
// mmer frequencies very uneven: hashed into 1024 buckets the largest holds
// ~8x the mean.  After a pass the host learns the records per mmer from the
// bin descriptors and packs the mmers of each (part, part_n) key into buckets
// longest-processing-time first; later passes route records by that map.
static uint64_t bmap_key(const kb_ctx* c) { return ((uint64_t)c->part << 32) | c->part_n; }

static kb_ctx::BucketMap* bmap_find(kb_ctx* c, uint32_t NB) {
    for (auto& m : c->bmaps)
        if (m.key == bmap_key(c) && m.nb == NB) return &m;
    return nullptr;
}

// Context sub-bins (kbin_internal.h): an mmer whose expected distinct keys
// exceed one LDS table at the light load (few mmers per rank at N GPUs, high
// coverage), or whose records exceed 1.5 buckets' fair share, is split into
// 4^b + 1 sub-bins, b the smallest depth that brings each under both.  Each
// sub-bin is then an item of its own in the packing below, placed on any
// bucket -- a light bin of its own in bin_kernel: no flat lists, no
// re-expansion per partition, finer longest-first scheduling.
static uint32_t sub_depth(const kb_ctx* c, double w, double keys, double mean) {
    int bmax = std::min<int>((int)SUB_MAX_B, std::max(0, env_int("KB_BIN_SUB", (int)SUB_MAX_B)));
    if (!sub_room(c->p.K, c->p.M, 2 * c->KW)) bmax = 0;  // (no spare span bits for the stamp)
    if (c->p.K < 2 * c->p.M) bmax = 0;  // (K < 2M: a signature is no function of its key's k-mer)
    const double ts = c->KW == 1 ? 8192.0 : 4096.0;
    // (the long-list regime: sub-bins at 40 % of a table, so that they stay under
    // the ranking's LDS limit and their long lists take the bitmaps -- C3 261 ->
    // 247 ms per step, the list kernels 26 -> 4.5 ms)
    double cap = ts * std::min(4.0, std::max(0.2, env_int("KB_BIN_SUB_FILL_PCT", c->rank_regime ? 40 : 80) / 100.0));
    // light pre-filtered bins (two-word keys, singleton-heavy): a sub-bin's
    // distinct keys only have to load the bin's sketch lightly (PFL_LOAD of
    // its PFL_CELLS); the table holds the keys seen twice
    if (c->KW == 2 && c->pfl_regime) cap = std::max(cap, PFL_LOAD * (double)PFL_CELLS);
    uint32_t b = 0;
    while ((int)b < bmax && (keys / (double)(1u << (2 * b)) > cap || w / (double)(1u << (2 * b)) > 1.5 * mean)) b++;
    return b;
}

// bins one finalize may describe: every canonical mmer once, plus the extra
// sub-bins of the split ones (bmap_build keeps within it)
static uint64_t bin_budget(const kb_ctx* c, uint32_t NB) {
    const uint64_t half = 1ull << (2 * c->p.M - 1);
    // (at most 240: a bucket orders up to BK_SLOTS = 256 bins, one per mmer plus its extra sub-bins)
    // (the light pre-filtered regime splits every heavy mmer ~64 ways: a larger budget)
    const uint64_t per_bucket =
        (uint64_t)std::min(240, std::max(0, env_int("KB_BIN_SUB_EXTRA", c->rank_regime ? 240 : c->pfl_regime ? 160 : 48)));
    return half + (sub_room(c->p.K, c->p.M, 2 * c->KW) ? per_bucket * NB : 0ull);
}

// prior: a first pass's map from the prior weights (bmap_prior) -- packed in
// one serpentine sweep over the items in their generated order (heaviest mmers
// first) instead of sorted LPT: the prior only approximates the data, and the
// pass learns the real map (0.28 of the prior's 0.44 ms at C2 was the sort and
// the heap)
static int bmap_build(kb_ctx* c, uint32_t NB, double rho, bool prior = false) {
    const double tb0 = now_ms();
    const int M = c->p.M;
    const uint32_t half = 1u << (2 * M - 1);
    struct Item {
        double w;
        uint32_t mm, sub;  // sub: ~0 for an unsplit mmer
    };
    std::vector<uint32_t> h(half);
    uint64_t tot_w = 0;
    for (uint32_t i = 0; i < half && i < c->mmer_w.size(); i++) tot_w += c->mmer_w[i];
    const double mean = std::max(1.0, (double)tot_w / NB);
    // this pass's mmers, heaviest first: the split depths are handed out in
    // that order within the bin budget
    std::vector<std::pair<double, uint32_t>> seen;
    for (uint32_t i = 0; i < half; i++) {
        h[i] = (uint32_t)sk_hash_dest(half + i, NB, sk_bucket_salt());  // unseen (or another pass's): hash
        if (c->part_n > 1 && sk_hash_dest(half + i, c->part_n, 0x9E3779B97F4A7C15ull) != c->part) continue;
        const double w = i < c->mmer_w.size() ? (double)c->mmer_w[i] : 0.0;
        // (a negligible mmer keeps its hash bucket: no packing item)
        if (w > 0 && w >= mean / 512.0) seen.push_back({w, i});
    }
    // (a prior's weights rise with the mmer score: ascending already)
    const auto desc = [](const std::pair<double, uint32_t>& a, const std::pair<double, uint32_t>& b) {
        return a.first > b.first;
    };
    if (std::is_sorted(seen.begin(), seen.end(), [&](const auto& a, const auto& b) { return desc(b, a); }))
        std::reverse(seen.begin(), seen.end());
    else if (!std::is_sorted(seen.begin(), seen.end(), desc))
        std::sort(seen.begin(), seen.end(), desc);
    uint64_t extra = bin_budget(c, NB) - half;  // sub-bins beyond one per mmer
    const kb_ctx::BucketMap* old = bmap_find(c, NB);
    std::vector<Item> items;
    std::vector<uint16_t> subs;
    uint32_t n_split = 0;
    for (const auto& sw : seen) {
        const uint32_t i = sw.second, mm = half + i;
        const double w = sw.first;
        const double occ = i < c->mmer_o.size() && c->mmer_o[i] ? (double)c->mmer_o[i] : 12.0 * w;
        uint32_t b = sub_depth(c, w, occ * rho, mean);
        while (b && sub_count(b) - 1 > extra) b--;
        if (!b) {
            items.push_back({w, mm, ~0u});
            continue;
        }
        extra -= sub_count(b) - 1;
        // sub-bin 0, the edge, holds a few percent; the contexts share the
        // rest -- or, when the last pass split this mmer as deep, as measured
        const uint32_t nsub = sub_count(b);
        const bool same = old && !old->h_map.empty() && (old->h_map[i] & BM_SPLIT) &&
                          ((old->h_map[i] >> 28) & 7u) == b;
        h[i] = BM_SPLIT | (b << 28) | (uint32_t)subs.size();
        for (uint32_t s2 = 0; s2 < nsub; s2++) {
            double ws = s2 ? w / (double)(nsub - 1) : 0.04 * w + 1.0;
            if (same) {
                auto f = c->sub_w.find(((uint64_t)mm << 16) | s2);
                ws = f != c->sub_w.end() ? (double)f->second : 1.0;
            }
            items.push_back({ws, mm, s2});
        }
        subs.resize(subs.size() + nsub, 0);
        n_split++;
    }
    const double tb1 = now_ms();
    if (!prior || env_int("KB_BIN_PRIOR_LPT", 0))
        std::sort(items.begin(), items.end(), [](const Item& a, const Item& b) { return a.w > b.w; });
    const double tb2 = now_ms();
    // longest processing time first onto the least loaded bucket; at most 248
    // bins per bucket (bucket_kernel maps 256).  A binary min-heap of packed
    // (load in 1/16 records << 11 | bucket) words: one compare per level, the
    // top replaced in place (no pop + push)
    std::vector<uint64_t> heap(NB);
    std::vector<uint32_t> nm(NB, 0);
    for (uint32_t b = 0; b < NB; b++) heap[b] = b;  // (all loads 0: already a heap)
    uint32_t hn = NB;
    auto sift = [&](uint32_t i) {
        const uint64_t v = heap[i];
        for (;;) {
            uint32_t c2 = 2 * i + 1;
            if (c2 >= hn) break;
            if (c2 + 1 < hn && heap[c2 + 1] < heap[c2]) c2++;
            if (heap[c2] >= v) break;
            heap[i] = heap[c2];
            i = c2;
        }
        heap[i] = v;
    };
    const bool serp = prior && !env_int("KB_BIN_PRIOR_LPT", 0);
    for (size_t k = 0; serp && k < items.size(); k++) {
        const Item& it = items[k];
        const uint32_t r = (uint32_t)(k / NB), q = (uint32_t)(k % NB);
        const uint32_t b = (r & 1u) ? NB - 1u - q : q;  // (at most ceil(items / NB) <= 248 per bucket)
        if (it.sub == ~0u) h[it.mm - half] = b;
        else subs[(h[it.mm - half] & 0x0FFFFFFFu) + it.sub] = (uint16_t)b;
        nm[b]++;
        heap[b] += (uint64_t)std::llround(std::min(it.w, 1e12) * 16.0) << 11;  // (loads: heap[b] >> 11)
    }
    for (const Item& it : items) {
        if (serp) break;
        while (hn > 1 && nm[heap[0] & 2047u] >= 248) {  // full: retire it
            std::swap(heap[0], heap[--hn]);  // (kept past the heap: its load still counts)
            sift(0);
        }
        const uint32_t b = (uint32_t)(heap[0] & 2047u);
        if (it.sub == ~0u) h[it.mm - half] = b;
        else subs[(h[it.mm - half] & 0x0FFFFFFFu) + it.sub] = (uint16_t)b;
        nm[b]++;
        heap[0] += (uint64_t)std::llround(std::min(it.w, 1e12) * 16.0) << 11;
        sift(0);
    }
    double want_max = 0, want_tot = 0;
    for (uint32_t i = 0; i < NB; i++) {
        const double ld = (double)(heap[i] >> 11) / 16.0;
        want_max = std::max(want_max, ld);
        want_tot += ld;
    }
    const double tb3 = now_ms();
    kb_ctx::BucketMap* m = bmap_find(c, NB);
    if (!m) {
        c->bmaps.emplace_back();
        m = &c->bmaps.back();
        m->key = bmap_key(c);
        m->nb = NB;
    }
    HIPCHK(m->map.ensure_exact(half));
    HIPCHK(m->sub.ensure(std::max<size_t>(subs.size(), 1)));
    // uploaded from the context's pinned staging (a pageable copy stages
    // through the runtime's bounce buffers: milliseconds on a context's first
    // use); the last upload must have left it
    const uint64_t need = half * sizeof(uint32_t) + subs.size() * sizeof(uint16_t);
    if (c->map_stage_used) HIPCHK(hipEventSynchronize(c->map_done));
    HIPCHK(c->map_stage.ensure(need));
    memcpy(c->map_stage.p, h.data(), half * sizeof(uint32_t));
    if (!subs.empty()) memcpy(c->map_stage.p + half * sizeof(uint32_t), subs.data(), subs.size() * sizeof(uint16_t));
    HIPCHK(hipMemcpyAsync(m->map.p, c->map_stage.p, half * sizeof(uint32_t), hipMemcpyHostToDevice, c->s));
    if (!subs.empty())
        HIPCHK(hipMemcpyAsync(m->sub.p, c->map_stage.p + half * sizeof(uint32_t), subs.size() * sizeof(uint16_t),
                              hipMemcpyHostToDevice, c->s));
    HIPCHK(hipEventRecord(c->map_done, c->s));
    c->map_stage_used = true;
    KB_DBG("bmap_build: %zu items, setup %.3f sort %.3f pack %.3f upload %.3f ms\n", items.size(), tb1 - tb0,
           tb2 - tb1, tb3 - tb2, now_ms() - tb3);
    m->h_map = std::move(h);
    m->stale = false;
    m->pending = false;
    m->split = n_split;
    m->want_max = (uint64_t)want_max + 1;
    m->want_tot = (uint64_t)want_tot + 1;
    // the region stride (records per bucket) this key's next pass writes with:
    // the largest bucket the packing expects plus a fifth (dense regions: a
    // sparse stride spreads a block's scattered record stores over more
    // pages), a larger bucket reruns the pass bigger
    // (a rebuilt map keeps the stride its key's passes have needed so far:
    // the packing's expectation runs some 10-25 % under the fullest bucket)
    m->cap = std::max<uint64_t>(m->cap, m->want_max + m->want_max / 3 + 256);
    return KB_OK;
}

// Learning a key's map from a bucketed pass: its bins' descriptors (records,
// occurrences, mmer | sub-bin << 16) give the records and occurrences per
// mmer (a split mmer's sub-bins add up) and each sub-bin's own records.  The
// descriptors ride the finalize's last copy (bmap_stage); the map itself is
// rebuilt when the key is next binned (bmap_apply), so no finalize waits on
// the packing -- a one-shot caller never pays it.
static bool bmap_wants(kb_ctx* c, uint32_t NB, uint64_t R) {
    if (!env_int("KB_BIN_BALANCE", 1) || R < (uint64_t)std::max(0, env_int("KB_BIN_BALANCE_MIN", 1 << 18)))
        return false;
    if (c->p.K < 2 * c->p.M) return false;  // (K < 2M: no map, see binned_buckets)
    const kb_ctx::BucketMap* m = bmap_find(c, NB);
    return !m || m->stale;
}

static int bmap_apply(kb_ctx* c, uint32_t NB, const uint32_t* mm, const uint32_t* cnt, const uint32_t* occ,
                      uint64_t nbins, double rho) {
    const kb_ctx::BucketMap* m = bmap_find(c, NB);
    const uint32_t half = 1u << (2 * c->p.M - 1);
    c->mmer_w.assign(half, 0);
    c->mmer_o.assign(half, 0);
    c->sub_w.clear();
    for (uint64_t b = 0; b < nbins; b++) {
        const uint32_t mmer = mm[b] & 0xFFFFu, sub = mm[b] >> 16;
        if (mmer < half || mmer >= 2 * half) continue;
        c->mmer_w[mmer - half] += std::max(cnt[b], 1u);
        c->mmer_o[mmer - half] += occ[b];
        if (m && m->split && !m->h_map.empty() && (m->h_map[mmer - half] & BM_SPLIT))
            c->sub_w[((uint64_t)mmer << 16) | sub] += std::max(cnt[b], 1u);
    }
    return bmap_build(c, NB, rho);
}

// ---- phase A, bucketed: records straight into NB local bucket regions
// (hash of the mmer); the learned capacity grows (and the pass reruns) when a
// bucket overflows.  Reads: the one-pass super-k-mer kernel in region mode;
// received: the block-aggregated converter.  Returns R and N (one sync per try).
// A context's first pass of a (part, part_n) key has no learned map.  Hashed
// into the buckets, the records would be very uneven (the minimizer rule
// makes mmer frequencies skewed: the largest hashed bucket holds ~8x the
// mean), which took a counting pass to lay the regions out exactly.  Instead
// the first pass packs the buckets by a PRIOR: on uniform sequence, a
// canonical mmer with canonical score c is a window's leftmost maximum
// (binning.c:972) about as often as all W - 1 other positions score below it,
// i.e. in proportion to ((c - 2^(2M-1)) / 2^(2M-1))^(W-1) (W = K - M + 1
// positions; each canonical score stands for two strings).  Packed by that
// weight, buckets come out as even as packed by the true counts (simulated
// at K31 M7: max/mean 1.85 either way, 6.4 hashed).  The records expected per
// read, 2 (L - K + 1) / (K - M + 2), scale it.  The prior map is marked stale,
// so the pass's own bins replace it.
static int bmap_prior(kb_ctx* c, uint32_t NB) {
    const int K = c->p.K, M = c->p.M;
    const uint32_t half = 1u << (2 * M - 1);
    double R_est = 0;
    for (auto& b : c->batches) {
        if (b.routed || !b.n_reads) continue;
        if (b.superkmers) {
            R_est += (double)b.n_reads;
        } else {
            const double L = std::min(b.RW * 32.0, (double)c->p.max_read_len);
            R_est += (double)b.n_reads * std::max(1.0, 2.0 * std::max(1.0, L - K + 1) / (K - M + 2));
        }
    }
    const bool reads_part = c->part_n > 1 && std::none_of(c->batches.begin(), c->batches.end(),
                                                          [](const Batch& b) { return b.superkmers; });
    const std::vector<double>& p = c->prior_p;  // (kb_create: the shape depends on K and M only)
    double tot = 0, mine = 0;
    for (uint32_t i = 0; i < half; i++) {
        tot += p[i];
        if (c->part_n <= 1 || sk_hash_dest(half + i, c->part_n, 0x9E3779B97F4A7C15ull) == c->part) mine += p[i];
    }
    // reads scanned for one partition emit only its records; received ones are its own
    const double R_part = reads_part ? R_est * mine / std::max(tot, 1e-300) : R_est;
    c->mmer_w.assign(half, 0);
    c->mmer_o.assign(half, 0);
    for (uint32_t i = 0; i < half; i++) {
        const double w = R_part * p[i] / std::max(mine, 1e-300);
        c->mmer_w[i] = (uint32_t)std::min(4e9, std::ceil(w));
    }
    // (no density learned yet: a typical one -- splits then follow the keys as well as the loads)
    const int rc = bmap_build(c, NB, c->rho > 0.f ? (double)c->rho : 0.1, true);
    if (rc) return rc;
    kb_ctx::BucketMap* m = bmap_find(c, NB);
    m->stale = true;  // (the pass learns the real one)
    // a prior misses real data's skew more than a learned map: a wider stride
    // (an overflowing bucket reruns the pass bigger)
    m->cap = 3 * m->want_max + 1024;
    return KB_OK;
}

// The bucket ordering and the bin plan of a bucketed pass: records in rlay
// slots (hdr pairs, then w1 / w3 at 2 rlay / 4 rlay), descriptors for
// max_bins bins.  rcap (speculative launches): records past it are not
// placed -- the layout was sized from the last pass, and the caller reruns.
static int bucket_phase(kb_ctx* c, uint32_t NB, uint64_t rlay, uint64_t max_bins, uint64_t cap, bool rexact,
                        uint64_t rcap, bool plan = true) {
    const int KW = c->KW;
    const uint64_t RWD = 1 + 2 * (uint64_t)KW;
    HIPCHK(c->starts.ensure(max_bins + 1));
    HIPCHK(c->bcount.ensure(max_bins));
    HIPCHK(c->bmmer.ensure(max_bins));
    HIPCHK(c->bocc.ensure(max_bins));
    HIPCHK(c->srec.ensure(RWD * rlay));
    BucketArgs ba{};
    ba.regions = c->regions.p;
    ba.cap = cap;
    ba.rbase = rexact ? c->rbase.p : nullptr;
    ba.bfill = c->bfill.p;
    ba.M = c->p.M;
    ba.hdr = c->srec.p;  // ((header, word 0) pairs, then word 1 / (word 1, word 2) pairs + word 3)
    ba.w1 = c->srec.p + 2 * rlay;
    ba.w3 = KW == 2 ? c->srec.p + 4 * rlay : nullptr;
    ba.spw = 2 * KW;
    HIPCHK(c->bbase.ensure(NB + 1));
    ba.bbase = c->bbase.p;
    ba.bases_ready = 1;  // (bucket_stats_kernel, after the record pass that made these regions)
    {
        // records written by a map-routed pass carry their sub-bin (zero
        // for an unsplit mmer); a hash-routed pass writes spans untouched
        kb_ctx::BucketMap* bm = bmap_find(c, NB);  // (the map the record pass used)
        ba.sub = bm && bm->split ? 1 : 0;
    }
    ba.bin_ctr = reinterpret_cast<unsigned long long*>(c->totals.p + 2);
    ba.bstart = c->starts.p;
    ba.bcount = c->bcount.p;
    ba.bmmer = c->bmmer.p;
    ba.bocc = c->bocc.p;
    ba.max_bins = max_bins;
#ifdef KB_BIN_ABL
    {   // (diagnostic: from a context's third finalize on, so the records
        // the bin kernel reads are the last pass's -- replay input only)
        static int abl_calls = 0;
        ba.ablate = abl_calls++ >= 2 ? env_int("KB_BK_ABLATE", 0) : 0;
    }
#endif
    ba.status = c->misc.p;
    ba.rcap = rcap;
    HIPCHK(launch_bucket_sort(ba, NB, c->s));
    c->tm.sort_passes = 0;
    if (!plan) return KB_OK;  // (KB_BIN_DESC=0: the caller orders the bins by count)
    HIPCHK(c->border.ensure(max_bins));
    HIPCHK(c->bdesc.ensure(2 * max_bins));
    HIPCHK(launch_bins_plan(c->starts.p, c->bcount.p, c->bmmer.p, c->bocc.p, c->totals.p, max_bins, c->border.p,
                            c->bdesc.p, reinterpret_cast<unsigned long long*>(c->totals.p + 10), c->s));
    return KB_OK;
}

static int binned_buckets(kb_ctx* c, uint32_t NB, bool received, bool zeroed, uint64_t& R, uint64_t& N) {
    const int M = c->p.M;
    c->spec = false;
    // K < 2M: a record's mmer code is the reference's complemented-or-not
    // signature, not the canonical (larger) one the bucket map is indexed by
    // (bucket_map[canon - 2^(2M-1)]): no map -- hash routing, exact regions
    const bool nomap = c->p.K < 2 * M;
    kb_ctx::BucketMap* bm = nomap ? nullptr : bmap_find(c, NB);
    if (bm && bm->pending) {  // the last pass of this key left its bins: rebuild the map from them
        const double t0 = now_ms();
        const int rc = bmap_apply(c, NB, bm->p_mm.data(), bm->p_cnt.data(), bm->p_occ.data(), bm->p_mm.size(),
                                  bm->p_rho);
        if (rc) return rc;
        bm = bmap_find(c, NB);
        KB_DBG("map rebuilt part %u/%u: %.3f ms, %u split\n", c->part, c->part_n, now_ms() - t0, bm->split);
    }
    if (!bm && !nomap && !c->prior_off && env_int("KB_BIN_PRIOR", 1) && env_int("KB_BIN_BALANCE", 1)) {
        const double t0 = now_ms();
        const int rc = bmap_prior(c, NB);
        if (rc) return rc;
        bm = bmap_find(c, NB);
        KB_DBG("prior map part %u/%u: %.3f ms (allocations %.3f), %u split, cap %llu\n", c->part, c->part_n,
               now_ms() - t0, g_alloc_ms, bm->split, (unsigned long long)bm->cap);
    }
    const uint32_t* bmap = bm ? bm->map.p : nullptr;
    const uint16_t* bsub = bm ? bm->sub.p : nullptr;
    // Without any map (KB_BIN_PRIOR=0) the records are routed by hash and the
    // buckets are uneven: a counting pass first (capacity 0: every record
    // counted, none written), then regions laid out exactly (rbase).  With a
    // map (learned, or the prior), one pass into regions of the learned
    // capacity (stride), rerun bigger on overflow.
    const bool exact = bmap == nullptr;
    HIPCHK(c->bfill.ensure(NB));
    // (every batch's per-block k-mer sums side by side: one sum at the end,
    // inside bucket_stats_kernel, where each batch launched a kernel for it)
    uint64_t kp = 1;
    for (auto& b : c->batches) kp += b.routed || b.superkmers ? 0 : sk_blocks(b.n_reads, b.RW);
    HIPCHK(c->kpart.ensure(kp));
    if (exact) HIPCHK(c->rbase.ensure(NB + 1));
    HIPCHK(c->regions.ensure(1));  // (non-null: the record kernel's region mode keys on it)
    const uint64_t RWD = 1 + 2 * (uint64_t)c->KW;
    for (int attempt = 0; attempt < 3; attempt++) {
        const bool counting = exact && attempt == 0;
        const bool use_base = exact && attempt > 0;
        const uint64_t cap = exact ? 0 : bm->cap;
        if (c->spec) HIPCHK(hipStreamSynchronize(c->s));  // (a rerun: nothing in flight reads what is regrown)
        if (attempt > 0 || !zeroed) {  // (the finalize's first clear zeroed them for attempt 0)
            ClearList cl{};
            cl.add(c->bfill.p, NB * sizeof(unsigned long long));
            cl.add(c->totals.p + 8, sizeof(uint64_t));
            cl.add(c->misc.p, sizeof(uint32_t));
            if (c->spec) cl.add(c->totals.p + 2, sizeof(uint64_t));  // (the speculative ordering's bins)
            HIPCHK(launch_clear(cl, c->s));
        }
        c->spec = false;
        if (!counting && !use_base) HIPCHK(c->regions.ensure(NB * cap * RWD));
        uint64_t koff = 0;  // (kpart entries written by this attempt's record passes)
        for (auto& b : c->batches) {
            if (b.routed || !b.n_reads) continue;
            if (received) {
                if (!b.superkmers) continue;
                HIPCHK(launch_sk_convert_buckets(b.recs, b.n_reads, rec_words(c), 2 * c->KW, M, NB, c->p.K, bmap, bsub,
                                                 bm && bm->split ? 1 : 0, c->regions.p, cap,
                                                 use_base ? c->rbase.p : nullptr, c->bfill.p, c->misc.p,
                                                 reinterpret_cast<unsigned long long*>(c->totals.p + 8), c->s));
            } else {
                if (b.superkmers) continue;
                SkScanArgs a{};
                a.part = c->part;
                a.part_n = c->part_n;
                a.words = b.words;
                a.lens = b.lens;
                a.n_reads = b.n_reads;
                a.ord_base = (uint32_t)b.ord_base;
                a.RW = b.RW;
                a.K = c->p.K;
                a.M = M;
                a.regions = c->regions.p;
                a.region_cap = cap;
                a.region_base = use_base ? c->rbase.p : nullptr;
                a.dest_ctr = c->bfill.p;
                a.G = NB;
                a.dest_salt = sk_bucket_salt();
                a.rw = (int)RWD;  // header + span words
                a.bucket_map = bmap;
                a.sub_map = bsub;
                a.sub_stamp = bm && bm->split ? 1 : 0;
                a.binned_fmt = 1;
                a.n_kmers = reinterpret_cast<unsigned long long*>(c->kpart.p) + koff;
                HIPCHK(launch_sk(a, true, c->s));
                koff += sk_blocks(b.n_reads, b.RW);
            }
            c->tm.scan_insert_launches++;
        }
        if (counting && koff)
            HIPCHK(launch_sk_kmers_total(reinterpret_cast<unsigned long long*>(c->kpart.p), koff,
                                         reinterpret_cast<unsigned long long*>(c->totals.p + 8), c->s));
        std::vector<unsigned long long> fill(counting ? NB : 0);
        uint64_t mx = 0;
        if (counting) {  // the exact layout needs every bucket's count
            HIPCHK(hipMemcpyAsync(fill.data(), c->bfill.p, NB * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                  c->s));
            HIPCHK(hipMemcpyAsync(c->h_totals + 8, c->totals.p + 8, sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_misc, c->misc.p, sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
        } else {  // R, the largest bucket and the status word folded next to N: one copy
            HIPCHK(c->bbase.ensure(NB + 1));
            HIPCHK(launch_bucket_stats(c->bfill.p, NB, c->misc.p, c->totals.p, cap, use_base ? c->rbase.p : nullptr,
                                       c->bbase.p, reinterpret_cast<unsigned long long*>(c->kpart.p), koff, c->s));
            HIPCHK(hipMemcpyAsync(c->h_totals + 8, c->totals.p + 8, 7 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
        }
        HIPCHK(hipEventRecord(c->ev_mid, c->s));
        // Speculation: the bucket ordering and the bin plan go out before the
        // host waits for R -- sized from the last pass's R with a quarter of
        // headroom -- so the GPU orders buckets while the host wakes, checks
        // and queues the bin kernel (the wait left it idle ~20 us per C2
        // step).  finalize_binned keeps the result when R fits the layout and
        // the bin count is the budget's, else reruns the phase exactly
        if (!counting && attempt == 0 && c->prev_R && c->rho > 0.f && env_int("KB_BIN_SPEC", 1) &&
            env_int("KB_BIN_DESC", 1)) {
            const uint64_t bk = bin_budget(c, NB);
            if (c->prev_R >= 2 * bk) {
                const uint64_t rl = c->prev_R + c->prev_R / 4 + 65536;
                const int rc = bucket_phase(c, NB, rl, bk, cap, use_base, rl);
                if (rc) return rc;
                c->spec = true;
                c->spec_rlay = rl;
                c->spec_bins = bk;
            }
        }
        HIPCHK(hipEventSynchronize(c->ev_mid));  // the one mid-finalize wait (two without a map): R and N size the rest
        KB_DBG("record pass attempt %d: %s cap %llu, %.3f ms since finalize (allocations %.3f ms)\n", attempt,
               counting ? "counting" : use_base ? "exact" : "stride", (unsigned long long)cap, now_ms() - c->t_fin,
               g_alloc_ms);
        if (!counting) c->h_misc[0] = (uint32_t)c->h_totals[14];
        if (c->h_misc[0] & ST_NEG_ID)
            return fail(KB_EINVAL, "routed read ids must be non-negative (they order the id lists)");
        R = 0;
        if (counting) {
            for (uint32_t d = 0; d < NB; d++) {
                R += fill[d];
                mx = std::max<uint64_t>(mx, fill[d]);
            }
        } else {
            R = c->h_totals[12];
            mx = c->h_totals[13];
        }
        N = c->h_totals[8];
        if (counting) {  // exact bases for the writing pass
            std::vector<uint64_t> base(NB + 1, 0);
            for (uint32_t d = 0; d < NB; d++) base[d + 1] = base[d] + fill[d];
            HIPCHK(c->regions.ensure(std::max<uint64_t>(R, 1) * RWD));
            HIPCHK(hipMemcpyAsync(c->rbase.p, base.data(), (NB + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->s));
            HIPCHK(hipStreamSynchronize(c->s));  // (base is a local)
            continue;
        }
        // a map that no longer fits (largest bucket > 1.5x what the packing
        // expected, scaled to this pass's records): relearn it after this pass
        if (bm && R && bm->want_tot &&
            (double)mx > 1.5 * (double)bm->want_max * (double)R / (double)bm->want_tot + 64.0) {
            KB_DBG("map stale: bucket %llu vs expected %.0f (records %llu, k-mers %llu)\n", (unsigned long long)mx,
                   (double)bm->want_max * (double)R / (double)bm->want_tot, (unsigned long long)R,
                   (unsigned long long)N);
            bm->stale = true;
        }
        if (use_base || mx <= cap) {
            c->rexact = use_base;
            c->bucket_cap_used = cap;  // the region stride of this pass (0: exact bases)
            if (!use_base && mx + mx / 16 > cap) bm->cap = mx + mx / 5 + 256;  // (close to full: next passes wider)
            if (N >= 0xFFFFFFFFull)
                return fail(KB_EOVERFLOW, "%llu k-mer occurrences in one context (limit 2^32-1)",
                            (unsigned long long)N);
            if (R > N)
                return fail(KB_EDEVICE, "internal: %llu super-k-mers > %llu k-mers", (unsigned long long)R,
                            (unsigned long long)N);
            return KB_OK;
        }
        // grow and rerun the pass; with headroom, so a later pass's slightly
        // larger bucket does not regrow (each growth maps the regions afresh)
        KB_DBG("record pass rerun: bucket %llu > cap %llu\n", (unsigned long long)mx, (unsigned long long)cap);
        bm->cap = mx + mx / 4 + 1024;
    }
    return fail(KB_EDEVICE, "internal: bucket capacity did not converge");
}

// ---- phase A (received): the routed super-k-mer records of every
// kb_submit_superkmers_device batch, converted in place of phase A; the
// record's read id is its ordinal (ids increase with the global call order)
static int binned_sk_records(kb_ctx* c, uint64_t& R, uint64_t& N) {
    R = 0;
    for (auto& b : c->batches)
        if (b.superkmers) R += b.n_reads;
    if (R > 0xFFFFFFFFull) return fail(KB_EOVERFLOW, "more than 2^32 received records");
    // N <= 63 R; buffers that scale with N are sized after the count
    HIPCHK(c->pay.ensure(3 * R));
    HIPCHK(c->srec.ensure(3 * R));
    HIPCHK(c->occ_a.ensure(std::max<uint64_t>(R, 4)));
    HIPCHK(hipMemsetAsync(c->totals.p + 8, 0, sizeof(uint64_t), c->s));
    uint64_t off = 0;
    for (auto& b : c->batches) {
        if (!b.superkmers) continue;
        HIPCHK(launch_sk_convert(b.recs, b.n_reads, rec_words(c), off, c->p.M, c->p.K, c->pay.p, c->occ_a.p,
                                 c->misc.p, reinterpret_cast<unsigned long long*>(c->totals.p + 8), c->s));
        off += b.n_reads;
        c->tm.scan_insert_launches++;
    }
    HIPCHK(hipMemcpyAsync(c->h_totals + 8, c->totals.p + 8, sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    N = c->h_totals[8];
    if (N >= 0xFFFFFFFFull)
        return fail(KB_EOVERFLOW, "%llu k-mer occurrences in one context (limit 2^32-1)",
                    (unsigned long long)N);
    HIPCHK(c->occ_b.ensure(std::max<uint64_t>(R, N / 2 + 4)));
    if (c->occ_a.cap < N / 2 + 4) {  // grow, keeping the R keys
        DevBuf<uint64_t> t;
        HIPCHK(t.ensure(std::max<uint64_t>(R, N / 2 + 4)));
        HIPCHK(hipMemcpyAsync(t.p, c->occ_a.p, R * sizeof(uint64_t), hipMemcpyDeviceToDevice, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
        c->occ_a.release();
        c->occ_a = t;
        t.p = nullptr;
        t.cap = 0;
    }
    return KB_OK;
}

// Offset partitions.  A light bin that needs 2^l tables is split by the
// minimizer's offset o inside the k-mer: o is the first occurrence of the
// (canonical) mmer string in the (complemented) k-mer, a function of the key
// (bin_body), so every key lands in exactly one range.  The ranges are chosen
// to hold equal shares of the occurrences, whose distribution over o is
// measured here once per (K, M) on seeded uniform random reads of the sticky
// signature walk (binning.c:922-989): roughly triangular, offset 0 most
// frequent (distinct keys per offset follow occurrences per offset).
static void offset_cuts(int K, int M, uint8_t (&cut)[5][17]) {
    const int W = K - M + 1, L = std::max(150, 4 * K);
    std::vector<double> h(W, 0.0);
    std::vector<uint8_t> r(L);
    std::vector<uint32_t> cs(L);
    const uint32_t full = (1u << (2 * M)) - 1u;
    uint64_t x = 0x243F6A8885A308D3ull;
    for (int read = 0; read < 400; read++) {  // (~50 K occurrences: once per context, in its first finalize)
        for (int i = 0; i < L; i++) {
            x += 0x9E3779B97F4A7C15ull;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            r[i] = (uint8_t)((z ^ (z >> 31)) & 3u);
        }
        for (int p = 0; p + M <= L; p++) {
            uint32_t s = 0;
            for (int j = 0; j < M; j++) s = s * 4u + r[p + j];
            cs[p] = std::max(s, full - s);
        }
        int sig = -1;
        for (int i = 0; i + K <= L; i++) {
            if (i > sig) {  // leftmost strict argmax (binning.c:972)
                uint32_t best = 0;
                for (int p = i; p <= i + K - M; p++)
                    if (sig < i || cs[p] > best) {
                        best = cs[p];
                        sig = p;
                    }
            }
            h[sig - i] += 1.0;
        }
    }
    double tot = 0;
    for (double v : h) tot += v;
    for (int l = 0; l <= 4; l++) {
        const int R = 1 << l;
        cut[l][0] = 0;
        double acc = 0;
        int o = 0;
        for (int rr = 1; rr < R; rr++) {
            while (o < W && acc + h[o] * 0.5 < tot * rr / R) acc += h[o++];
            // non-empty ranges where W allows
            int c = std::max(o, (int)cut[l][rr - 1] + 1);
            cut[l][rr] = (uint8_t)std::min(c, 63);
        }
        for (int rr = R; rr <= 16; rr++) cut[l][rr] = 64;
    }
}

static int finalize_binned(kb_ctx* c, int prune, bool affine, int64_t id_c, bool received) {
    const int M = c->p.M;
    c->t_fin = now_ms();
    g_alloc_ms = 0;
    c->tm.engine = KB_ENG_BINNED;
    REC(0);
    HIPCHK(c->totals.ensure(16));
    c->tm.scan_insert_launches = 0;
    c->tm.tail_reruns = 0;
    uint64_t R = 0, N = 0;
    // bucketed (default): records into local bucket regions, one workgroup
    // orders each bucket; radix: flat records, a global sort by (mmer, n)
    bool all_short = true;
    for (auto& b : c->batches)
        if (!b.routed && !b.superkmers && b.RW > 16) all_short = false;
    const bool bucketed = all_short && env_int("KB_BIN_RADIX", 0) == 0 && !c->bucket_failed;
    const int KW = c->KW, RWD = 1 + 2 * KW;  // record words: header + span words
    if (KW != 1 && !bucketed) return fail(KB_EDEVICE, "internal: two-word k-mers off the bucketed path");
    // local buckets (power of two, <= 1024): more buckets, more workgroups in flight
    uint32_t NB = 1;
    while (NB < (uint32_t)std::min(1024, std::max(64, env_int("KB_BIN_NB", 1024)))) NB <<= 1;
    // every counter of this finalize's first attempt zeroed in one launch
    HIPCHK(c->flat_n.ensure_exact(8));
    HIPCHK(c->pstat.ensure_exact(KB_PSTAT));
    {
        ClearList cl{};
        cl.add(c->totals.p, 16 * sizeof(uint64_t));
        cl.add(c->misc.p, 6 * sizeof(uint32_t));  // (status words, the list kernels' queue lengths)
        cl.add(c->flat_n.p, 8 * sizeof(unsigned long long));
        cl.add(c->pstat.p, KB_PSTAT * sizeof(unsigned long long));
        if (bucketed) {
            HIPCHK(c->bfill.ensure(NB));
            cl.add(c->bfill.p, NB * sizeof(unsigned long long));
        }
        if (c->lq.p) cl.add(c->lq.p, sizeof(uint64_t));
        HIPCHK(launch_clear(cl, c->s));
    }
    REC(1);
    int rc = bucketed ? binned_buckets(c, NB, received, true, R, N)
                      : (received ? binned_sk_records(c, R, N) : binned_read_records(c, R, N, false));
    if (rc) return rc;
    c->n_occ = N;
    REC(2);
    // bins: canonical mmers, or context sub-bins of the split ones (a fixed
    // budget: the buffers sized by it keep their size as maps change)
    // (the radix path's bins are mmer codes: canonical ones, 2^(2M-1) of them,
    // except for K < 2M signatures, which take any of the 4^M codes -- ADVICE r05)
    const uint64_t bin_keys = bucketed ? bin_budget(c, NB) : 1ull << (2 * M - (c->p.K < 2 * M ? 0 : 1));
    const uint64_t max_bins = std::max<uint64_t>(1, std::min<uint64_t>(R, bin_keys));
    const bool use_desc = bucketed && env_int("KB_BIN_DESC", 1);
    // the speculative bucket ordering (binned_buckets) stands when R fitted
    // its layout and the bin count is the budget's; otherwise it is rerun
    // exactly, after its counter is zeroed
    const bool spec_ok = use_desc && c->spec && R <= c->spec_rlay && max_bins == c->spec_bins;
    if (c->spec && !spec_ok) {
        HIPCHK(hipStreamSynchronize(c->s));  // (nothing in flight reads what is regrown)
        HIPCHK(hipMemsetAsync(c->totals.p + 2, 0, sizeof(uint64_t), c->s));
    }
    c->spec = false;
    KB_DBG("bucket ordering: %s (R %llu, layout %llu)\n", spec_ok ? "speculative, kept" : "exact",
           (unsigned long long)R, (unsigned long long)(spec_ok ? c->spec_rlay : R));
    const uint64_t rlay = spec_ok ? c->spec_rlay : R;  // (the records' layout: hdr, w1 at 2 rlay, w3 at 4 rlay)
    c->prev_R = R;
    HIPCHK(c->starts.ensure(max_bins + 1));
    HIPCHK(c->bcount.ensure(max_bins));
    HIPCHK(c->bmmer.ensure(max_bins));
    if (bucketed) HIPCHK(c->bocc.ensure(max_bins));
    HIPCHK(c->srec.ensure(RWD * rlay));
    HIPCHK(c->occ_b.ensure(std::max<uint64_t>(R, N / 2 + 4)));  // ids by ordinal (+ radix ping-pong)
    // the stage: 4-B ordinals + 2-B slots (KB_BIN_STAGE6, default), or 8-B
    // entries -- also with first-occurrence tracking, whose entries carry the
    // k-mer's position (the 8-B array is then the only one touched)
    const bool stage6 = env_int("KB_BIN_STAGE6", 1) != 0 && !(c->p.flags & KB_TRACK_FIRST);
    HIPCHK(c->stage.ensure(stage6 ? 1 : std::max<uint64_t>(N, 1)));
    if (stage6) {
        HIPCHK(c->stage_ord.ensure(std::max<uint64_t>(N, 1)));
        HIPCHK(c->stage_slot.ensure(std::max<uint64_t>(N, 1)));
    }
    // heavy bins' flat k-mer lists (touched only when a bin needs many tables)
    // Few, large bins (the last finalize had fewer than three per CU: the
    // mmer-sharded receivers of N ranks, high coverage): bins above 1/32 of a
    // block's fair share are split (their partitions re-expanded by any block)
    // up to depth 3, deeper ones take the flat lists -- both spread over the
    // chip (bins 3.67 -> 2.70 ms per pass on the 8-rank share).  Otherwise
    // flat lists from depth 3 on and no splits (many bins keep the CUs busy).
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->dev));
    const bool few_bins = c->nbins_hint && c->nbins_hint < 3u * (uint32_t)std::max(1, cus);
    // offset partitions (bin_body) make a light bin of depth 3-4 cheaper than
    // flat lists for one-word keys
    // (one-word keys only: two-word bins expand through the ring, which
    // would still walk every k-mer of the bin per range)
    // (K < 2M: no offset partitions -- their exactness needs the leftmost-argmax signature)
    const int opart = KW == 1 && c->p.K >= 2 * M ? std::min(4, std::max(0, env_int("KB_BIN_OPART", 4))) : 0;
    const uint32_t flat_l =
        (uint32_t)std::max(0, env_int("KB_BIN_FLAT_L", few_bins ? 4 : (KW == 1 && opart >= 4) ? 5 : 3));
    if (flat_l) HIPCHK(c->kstage.ensure(std::max<uint64_t>(KW * N, 1)));
    if (bucketed) {
        if (!spec_ok) {
            const int rc2 = bucket_phase(c, NB, R, max_bins, c->bucket_cap_used, c->rexact, 0, use_desc);
            if (rc2) return rc2;
        }
    } else {
        // ---- stable sort of the records by (mmer, 63 - n), bin boundaries
        const int key_bits = 2 * M + 6;
        const uint64_t nflags = onesweep_flag_elems(R);
        if (c->os_flags.cap < nflags || c->os_epoch > (1u << 24) - 8) {
            HIPCHK(c->os_flags.ensure(nflags));
            HIPCHK(hipMemsetAsync(c->os_flags.p, 0, c->os_flags.cap * sizeof(uint64_t), c->s));
            c->os_epoch = 0;
        }
        HIPCHK(c->os_aux.ensure(4 * 256 + 8));
        HIPCHK(hipMemsetAsync(c->os_aux.p + 1028, 0, sizeof(uint32_t), c->s));
        HIPCHK(launch_onesweep(c->occ_a.p, c->occ_b.p, R, key_bits, c->os_flags.p, c->os_aux.p,
                               &c->os_epoch, &c->sorted, c->s));
        c->tm.sort_passes = (uint32_t)((key_bits + 7) / 8);
        HIPCHK(c->scratch.ensure(std::max(runs_scratch_elems(R, max_bins), c->scratch.cap)));
        HIPCHK(launch_heads(c->sorted, R, c->starts.p, max_bins, c->scratch.p, c->scratch.cap,
                            c->totals.p, c->s, 38));
        HIPCHK(launch_bins_describe(c->sorted, c->starts.p, c->totals.p, c->bcount.p, c->bmmer.p, max_bins,
                                    c->s));
        HIPCHK(launch_sk_gather(c->sorted, c->pay.p, R, c->srec.p, c->s));
    }
    HIPCHK(c->border.ensure(max_bins));
    if (!use_desc)  // (bucketed: bucket_phase planned the bins from their descriptors; bocc counted by it)
        HIPCHK(launch_bins_order(c->bcount.p, c->totals.p, c->border.p, max_bins, c->s));
    float* rho_dev = nullptr;
    if (c->rho <= 0.f && N && env_int("KB_BIN_HLL", 1)) {
        // the context's first finalize: distinct keys per occurrence from one
        // HyperLogLog over the records (no learned density yet)
        BinArgs h{};
        h.hdr = c->srec.p;  // ((header, word 0) pairs, then word 1 / (word 1, word 2) pairs + word 3)
        h.w1 = c->srec.p + 2 * rlay;
        h.w3 = KW == 2 ? c->srec.p + 4 * rlay : nullptr;
        h.K = c->p.K;
        h.M = M;
        // large passes estimate from the bins of 1/8 of the mmers (whole bins:
        // the ratio of a sample of bins, 1/8 of the expansion work) -- when the
        // pass holds enough mmers for the sample to be a fair one: at least 64
        // sampled of the canonical mmers a partition expects; received records
        // (one rank's share of the mmers, unknown here) are never sampled
        const uint32_t sample_div = (uint32_t)std::max(1, env_int("KB_BIN_HLL_SAMPLE", 8));
        const uint64_t mm_expect = (1ull << (2 * M - 1)) / std::max<uint32_t>(1u, c->part_n);
        const uint32_t sample = R >= (1u << 20) && !received && mm_expect / sample_div >= 64 ? sample_div : 1u;
        // (registers, the u64 occurrence count, then the estimate: read by the
        // bin kernel from device memory -- the host never waits for it; the
        // finalize's own distinct count replaces it afterwards)
        HIPCHK(c->hll.ensure_exact(4096 + 3));
        HIPCHK(launch_hll(h, R, KW, c->hll.p, sample, c->s));
        rho_dev = reinterpret_cast<float*>(c->hll.p + 4096 + 2);
        HIPCHK(launch_hll_finish(c->hll.p, rho_dev, c->s));
        KB_DBG("hll (sample 1/%u) queued: %.3f ms since finalize\n", sample, now_ms() - c->t_fin);
    }
    REC(3);
    // ---- one workgroup per bin.  Entry capacity: learned (or N/8), rerun once
    // with the exact need when the packed counter says it was exceeded.
    HIPCHK(c->ids_out.ensure(std::max<uint64_t>(N, 1)));
    // LDS table slots: 8192 one-word keys, 4096 two-word keys (bins_lds_bytes <= 160 KiB)
    const int ts_log2 = std::min(KW == 1 ? 13 : 12, std::max(10, env_int("KB_BIN_TS_LOG2", KW == 1 ? 13 : 12)));
    uint64_t ecap = std::min<uint64_t>(N + 1, c->ecap_hint ? c->ecap_hint : N / 8 + 1024);
    if (const int forced = env_int("KB_BIN_ECAP0", 0)) ecap = (uint64_t)forced;  // tests: force the rerun
    BinArgs a{};
    const bool learn = bucketed && bmap_wants(c, NB, R);  // (before the record pass's map may be replaced)
    for (int attempt = 0;; attempt++) {
        HIPCHK(c->e_mmer.ensure(ecap));
        HIPCHK(c->e_cnt.ensure(ecap));
        HIPCHK(c->e_hi.ensure(ecap));
        if (KW == 1 && (c->e_hi_zeroed != c->e_hi.p || c->e_hi_zeroed_cap != c->e_hi.cap)) {
            // K <= 31: every key's high code word is 0; zeroed once per
            // allocation instead of 8 B per entry from bin_kernel each finalize
            HIPCHK(hipMemsetAsync(c->e_hi.p, 0, c->e_hi.cap * sizeof(uint64_t), c->s));
            c->e_hi_zeroed = c->e_hi.p;
            c->e_hi_zeroed_cap = c->e_hi.cap;
        }
        HIPCHK(c->e_lo.ensure(ecap));
        HIPCHK(c->e_off.ensure(ecap));
        if (attempt) {  // the bin kernel's counters and status start again
            HIPCHK(hipMemsetAsync(c->totals.p + 4, 0, 4 * sizeof(uint64_t), c->s));
            HIPCHK(hipMemsetAsync(c->totals.p + 10, 0, 2 * sizeof(uint64_t), c->s));
            HIPCHK(hipMemsetAsync(c->misc.p + 2, 0, sizeof(uint32_t), c->s));
            if (use_desc)  // (the stage counter starts after the described ranges)
                HIPCHK(launch_bins_desc(c->border.p, c->starts.p, c->bcount.p, c->bmmer.p, c->bocc.p, c->totals.p,
                                        max_bins, c->bdesc.p, reinterpret_cast<unsigned long long*>(c->totals.p + 10),
                                        c->s));
            REC(3);
        }
        a = BinArgs{};
        a.hdr = c->srec.p;  // ((header, word 0) pairs, then word 1 / (word 1, word 2) pairs + word 3)
        a.w1 = c->srec.p + 2 * rlay;
        a.w3 = KW == 2 ? c->srec.p + 4 * rlay : nullptr;
        a.bstart = c->starts.p;
        a.bcount = c->bcount.p;
        a.bmmer = c->bmmer.p;
        a.bocc = bucketed ? c->bocc.p : nullptr;
        a.max_bins = max_bins;
        a.stage_ctr = reinterpret_cast<unsigned long long*>(c->totals.p + 10);
        a.order = c->border.p;
        a.bdesc = use_desc ? c->bdesc.p : nullptr;
        a.work = reinterpret_cast<unsigned long long*>(c->totals.p + 7);
        a.stage = c->stage.p;
        a.stage_ord = stage6 ? c->stage_ord.p : nullptr;
        a.stage_slot = stage6 ? c->stage_slot.p : nullptr;
        a.kstage = flat_l ? c->kstage.p : nullptr;
        a.flat_l = flat_l;
        a.n_occ = N;
        a.split_div = (uint32_t)std::max(0, env_int("KB_BIN_SPLIT_DIV", few_bins ? 32 : 0));
        a.big_div = (uint32_t)std::max(0, env_int("KB_BIN_BIG_DIV", 2));
        if (flat_l) {
            HIPCHK(c->flat_list.ensure(max_bins));
            HIPCHK(c->flat_next.ensure(max_bins));
            HIPCHK(c->flat_l0.ensure(max_bins));
            HIPCHK(c->flat_sbase.ensure(max_bins));
            HIPCHK(c->flat_obase.ensure(max_bins));
            // offsets: np + 1 per heavy bin, np < 2 x (expected keys / (fill x TS)) + 1,
            // expected keys <= occurrences, fill x TS >= 0.3 x 1024
            HIPCHK(c->flat_off.ensure(N / 150 + 9 * max_bins + KB_FLAT_MAX + 1));
            HIPCHK(c->flat_cur.ensure(c->flat_off.cap));
            HIPCHK(c->flat_chunk.ensure(max_bins));
            HIPCHK(c->pool_bin.ensure(c->flat_off.cap));
            HIPCHK(c->chunk_bin.ensure(R / 1024 + max_bins + 1));
            if (attempt) HIPCHK(hipMemsetAsync(c->flat_n.p, 0, 8 * sizeof(unsigned long long), c->s));
            a.flat_list = c->flat_list.p;
            a.flat_next = c->flat_next.p;
            a.flat_l0 = c->flat_l0.p;
            a.flat_sbase = c->flat_sbase.p;
            a.flat_off = c->flat_off.p;
            a.flat_cur = c->flat_cur.p;
            a.flat_chunk = c->flat_chunk.p;
            a.pool_bin = c->pool_bin.p;
            a.chunk_bin = c->chunk_bin.p;
            a.flat_obase = c->flat_obase.p;
            a.flat_n = c->flat_n.p;
            a.flat_octr = c->flat_n.p + 1;
        }
        a.totals = c->totals.p;
        a.K = c->p.K;
        a.M = M;
        a.keep_gt = prune ? (uint32_t)c->p.cutoff : 0u;
        a.ts_log2 = (uint32_t)ts_log2;
        a.rho = c->rho > 0.f ? c->rho : 0.25f;
        a.rho_dev = rho_dev;
        a.fill = (float)std::min(0.85, std::max(0.3, env_int("KB_BIN_FILL_PCT", 60) / 100.0));
        a.ablate = env_int("KB_BIN_ABLATE", 0);
        a.ringfree = (uint32_t)(env_int("KB_BIN_RINGFREE", 1) != 0);
        a.opart = (uint32_t)opart;
        a.osplit = (uint32_t)(env_int("KB_BIN_OSPLIT", 0) != 0);
        a.fill_light = (float)std::min(0.85, std::max(0.3, env_int("KB_BIN_FILL_LIGHT_PCT", 50) / 100.0));
        if (a.opart) {
            if (c->ocut_km != (c->p.K << 8 | M)) {
                offset_cuts(c->p.K, M, c->ocut);
                c->ocut_km = c->p.K << 8 | M;
            }
            memcpy(a.ocut, c->ocut, sizeof(a.ocut));
        }
        a.heavy_hint = attempt ? ~0ull : c->hint_heavy;
        // LDS id windows in heavy-bin partitions where the last finalize's lists
        // were short on average (C4 share: 588 -> 502 ms per step; C3's lists of
        // ~2300 ids measured 342 -> 351 ms with them)
        a.win_heavy = (uint32_t)(env_int("KB_BIN_WIN_HEAVY", 1) != 0 &&
                                 (c->hint_entries == 0 || c->hint_ids <= 128 * c->hint_entries));
        // (bit 1: two-word keys too -- KB_BIN_WIN_HEAVY2; C5 share 510 -> 482 ms
        // per step: its short lists no longer wait for the list kernels, emit
        // 32 -> 0.04 ms, the bin phase +4.5 ms; round 2 had measured 624 -> 641
        // before the pre-filter, r5g29)
        if (a.win_heavy && env_int("KB_BIN_WIN_HEAVY2", 1)) a.win_heavy |= 2u;
        a.gcount = reinterpret_cast<unsigned long long*>(c->totals.p + 4);
        a.status = c->misc.p + 2;  // the bin kernel's own status word
        a.e_mmer = c->e_mmer.p;
        a.e_hi = c->e_hi.p;
        a.e_lo = c->e_lo.p;
        a.e_cnt = c->e_cnt.p;
        a.e_off = c->e_off.p;
        a.e_first = nullptr;
        if (c->p.flags & KB_TRACK_FIRST) {
            HIPCHK(c->e_first.ensure(ecap));
            a.e_first = c->e_first.p;
        }
        a.ids_ord = reinterpret_cast<uint32_t*>(bucketed || c->sorted == c->occ_a.p ? c->occ_b.p : c->occ_a.p);
        a.ids_out = c->ids_out.p;
        a.read_ids = affine ? nullptr : c->read_ids.p;
        a.id_off = (uint32_t)(affine ? id_c : 0);
        a.max_entries = ecap - 1;
        a.max_ids = N;
        // lists placed and ordered in LDS id windows by the bins (lists_kernel
        // then takes only the queued items: lists > 256 ids, partitions whose
        // ids took the global path)
        if (env_int("KB_BIN_LDS_LISTS", 1)) {
            // items <= entries (every item holds >= 1 entry): one slot per entry
            const uint64_t* lq_was = c->lq.p;
            HIPCHK(c->lq.ensure(ecap + 1));
            // (the first clear zeroed the head of the queue it saw; a queue
            // allocated since needs its own)
            if (attempt || c->lq.p != lq_was) HIPCHK(hipMemsetAsync(c->lq.p, 0, sizeof(uint64_t), c->s));
            a.lq_n = reinterpret_cast<unsigned long long*>(c->lq.p);
            a.lq_items = c->lq.p + 1;
            a.lq_cap = ecap;
        }
        a.fs_lds = (uint32_t)(env_int("KB_BIN_FSL", 1) != 0);
        a.fsl_run = (uint32_t)std::max(1, env_int("KB_BIN_FSL_RUN", 64));
        // singleton pre-filter for the heavy bins: where most distinct keys are
        // pruned singletons (high error rates, low coverage: C5), learned from
        // the last finalize; exact because a key seen once has count 1 <= cutoff
        {
            const int pf_env = env_int("KB_BIN_PF", -1);
            const bool pf_ok = prune && c->p.cutoff >= 1 && !(c->p.flags & KB_TRACK_FIRST) && flat_l;
            a.pf = pf_ok && (pf_env == 1 || (pf_env < 0 && c->rho >= 0.3f && c->rho_tab > 0.f)) ? 1u : 0u;
            a.rho_tab = c->rho_tab > 0.f ? c->rho_tab : a.rho;
            a.pf_light = a.pf && KW == 2 && env_int("KB_BIN_PF_LIGHT", 1) != 0 ? 1u : 0u;
            if (a.pf_light) c->pfl_regime = true;  // (the next maps split for the sketch)
            a.tab_keys = reinterpret_cast<unsigned long long*>(c->totals.p + 11);
        }
        if (attempt) HIPCHK(hipMemsetAsync(c->pstat.p, 0, KB_PSTAT * sizeof(unsigned long long), c->s));
        a.pstat = c->pstat.p;
        a.ldsbar = (uint32_t)(env_int("KB_BIN_LDSBAR", 1) != 0);
        a.ts_adapt = (uint32_t)(env_int("KB_BIN_TS_ADAPT", 1) != 0);
        a.corrupt = (uint32_t)(env_int("KB_DIAG_CORRUPT", 0) != 0);
        a.skew = (uint32_t)std::max(0, env_int("KB_DIAG_SKEW", 0));
        a.diag_alloc = (uint32_t)(env_int("KB_DIAG_ALLOC", 0) != 0);
        // ranked bins where lists are long (the last finalize's mean list
        // length, C3: ~2200 ids): KB_BIN_RANK=0 off, 2 always
        {
            const int rk = env_int("KB_BIN_RANK", 1);
            const bool long_lists = c->hint_entries && c->hint_ids >= 64 * c->hint_entries;
            // (the bitmaps emit the long lists outside the list kernels, which
            // then must take only the queued items: no ranking without the
            // list queue, KB_BIN_LDS_LISTS=0)
            a.rank_mode = (rk == 2 || (rk == 1 && long_lists)) && stage6 && !a.e_first && a.lq_items ? 1u : 0u;
            a.rank_merge = (uint32_t)(env_int("KB_BIN_RANK_MERGE", 1) != 0);
            if (a.rank_mode) c->rank_regime = true;  // (the next maps split finer)
            if (a.rank_mode) {
                HIPCHK(c->rrank.ensure(std::max<uint64_t>(R, 1)));
                HIPCHK(c->rord.ensure(std::max<uint64_t>(R, 1)));
                a.rrank = c->rrank.p;
                a.rord = c->rord.p;
            }
        }
        // The tail kernels -- the heavy bins' list builds and partitions, the
        // list kernels -- have work only when bin_kernel publishes a heavy bin
        // or queues a list, and cost ~4.5 us per empty launch (8 of them: 2 %
        // of a C2 step).  Where the last finalize needed none they are left
        // out, and launched after all (full grids) only if this finalize's
        // totals say bin_kernel published or queued something
        const bool defer = attempt == 0 && c->hint_heavy == 0 && c->hint_lq == 0 && a.lq_items &&
                           env_int("KB_BIN_DEFER_TAIL", 1) != 0;
        HIPCHK(c->bargs.ensure_exact(1));
        HIPCHK(launch_bins(a, max_bins, KW, c->s, c->timing ? &c->ev[6] : nullptr, !defer, c->bargs.p));
#ifdef KB_BIN_PROF
        bins_prof_report(c->s);
#endif
        // (deferred tail: nothing runs after bins_final, so it gathers the
        // finalize's stats next to the totals for one copy instead of three)
        HIPCHK(launch_bins_final(a.gcount, c->e_off.p, c->totals.p, a.max_entries, flat_l ? c->flat_n.p : nullptr,
                                 a.lq_n, defer ? c->pstat.p : nullptr, defer ? c->misc.p : nullptr, c->s));
        REC(4);
        ListArgs la{};
        la.totals = c->totals.p;
        la.e_cnt = c->e_cnt.p;
        la.e_off = c->e_off.p;
        la.ids_ord = a.ids_ord;
        la.ids_out = c->ids_out.p;
        la.read_ids = a.read_ids;
        la.id_off = a.id_off;
        la.long_cap = N / 256 + 2;  // lists of > 256 ids
        la.lq_items = a.lq_items;
        la.lq_n = a.lq_n;
        la.lq_cap = a.lq_cap;
        HIPCHK(c->long_q.ensure(2 * la.long_cap));
        la.long_q = c->long_q.p;
        la.long_n = c->misc.p + 4;
        la.long_n_zeroed = attempt == 0;  // (the finalize's first clear)
        la.lq_hint = attempt ? ~0ull : c->hint_lq;
        la.long_hint[0] = attempt ? ~0ull : c->hint_long[0];
        la.long_hint[1] = attempt ? ~0ull : c->hint_long[1];
        if (!defer) HIPCHK(launch_lists(la, c->n_occ_entries_hint ? c->n_occ_entries_hint : ecap, c->s));
#ifdef KB_BIN_PROF
        lists_prof_report(c->s);
#endif
        REC(5);
        if (defer) {
            HIPCHK(hipMemcpyAsync(c->h_totals, c->totals.p, 31 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
        } else {
            HIPCHK(hipMemcpyAsync(c->h_totals, c->totals.p, 14 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_totals + 16, c->pstat.p, KB_PSTAT * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                  c->s));
        }
        if (learn) {  // the bins' descriptors for the map (bmap_apply), in the same copy batch
            HIPCHK(c->h_bins.ensure(3 * max_bins));
            HIPCHK(hipMemcpyAsync(c->h_bins.p, c->bmmer.p, max_bins * sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_bins.p + max_bins, c->bcount.p, max_bins * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_bins.p + 2 * max_bins, c->bocc.p, max_bins * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, c->s));
        }
        if (!defer) HIPCHK(hipMemcpyAsync(c->h_misc, c->misc.p, 6 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
        if (R && !bucketed)
            HIPCHK(hipMemcpyAsync(c->h_misc + 8, c->os_aux.p + 1028, sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
        else c->h_misc[8] = 0;
        HIPCHK(hipStreamSynchronize(c->s));
        if (defer)
            for (int k = 0; k < 3; k++) {
                c->h_misc[2 * k] = (uint32_t)c->h_totals[28 + k];
                c->h_misc[2 * k + 1] = (uint32_t)(c->h_totals[28 + k] >> 32);
            }
        if (defer && (c->h_totals[12] || c->h_totals[13])) {
            // the tail after all (a heavy bin published, or lists queued):
            // full grids, then the totals again
            c->tm.tail_reruns++;
            a.heavy_hint = ~0ull;
            HIPCHK(launch_bins_heavy(a, KW, c->s, c->bargs.p));
            HIPCHK(launch_bins_final(a.gcount, c->e_off.p, c->totals.p, a.max_entries,
                                     flat_l ? c->flat_n.p : nullptr, a.lq_n, nullptr, nullptr, c->s));
            la.lq_hint = ~0ull;
            la.long_hint[0] = la.long_hint[1] = ~0ull;
            HIPCHK(launch_lists(la, c->n_occ_entries_hint ? c->n_occ_entries_hint : ecap, c->s));
            REC(5);
            HIPCHK(hipMemcpyAsync(c->h_totals, c->totals.p, 14 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_totals + 16, c->pstat.p, KB_PSTAT * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                  c->s));
            HIPCHK(hipMemcpyAsync(c->h_misc, c->misc.p, 6 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipStreamSynchronize(c->s));
        }
        if (c->h_misc[0] & ST_BUCKET_FULL) {  // a bucket held too many mmers
            c->finalized = false;
            // a learned (or prior) map packed them: forget it and rerun on the
            // hash routing (no prior for this context from now on)
            for (size_t i = 0; i < c->bmaps.size(); i++)
                if (c->bmaps[i].key == bmap_key(c) && c->bmaps[i].nb == NB) {
                    c->prior_off = true;
                    auto& m = c->bmaps[i];
                    m.map.release(); m.sub.release();
                    c->bmaps.erase(c->bmaps.begin() + (long)i);
                    return finalize_binned(c, prune, affine, id_c, received);
                }
            // the hash itself overflowed: the radix path (K <= 31) or the
            // table engine (K > 31, which has no partitioned passes)
            if (KW == 2 && c->part_n > 1)
                return fail(KB_EINVAL, "a local bucket overflowed with two-word k-mers in a partitioned "
                                       "pass (M too large for %u buckets)", NB);
            c->bucket_failed = true;  // until kb_reset
            if (KW == 1) return finalize_binned(c, prune, affine, id_c, received);
            return kb_finalize(c, prune);
        }
        const uint64_t need = (c->h_totals[4] >> 32) + 1;  // entries asked of the packed counter
        if ((c->h_misc[2] & ST_TABLE_FULL) && attempt == 0 && need > ecap) {
            ecap = need + need / 16 + 1024;
            continue;
        }
        break;
    }
    c->hint_heavy = c->h_totals[12];
    c->hint_lq = c->h_totals[13];
    c->hint_long[0] = c->h_misc[4];
    c->hint_long[1] = c->h_misc[5];
    c->hint_entries = c->h_totals[0];
    c->hint_ids = c->h_totals[1];
    const uint32_t bst = c->h_misc[2];
    if (c->h_misc[8]) return fail(KB_EDEVICE, "radix look-back timed out (device error word %u)", c->h_misc[8]);
    if (c->h_totals[3]) return fail(KB_EDEVICE, "internal: %llu bins > %llu", (unsigned long long)c->h_totals[3],
                                    (unsigned long long)max_bins);
    if (bst & ST_TABLE_FULL) return fail(KB_EDEVICE, "internal: CSR capacity exceeded");
    if (c->h_misc[0] & ST_NEG_ID)
        return fail(KB_EINVAL, "routed read ids must be non-negative (they order the id lists)");
    if (bst & ST_PROBE_LIMIT) return fail(KB_ENOMEM, "a bin exceeded the partition depth");
    // result invariants (a wrong result must not come back as KB_OK): every
    // k-mer of the pass counted exactly once before the prune, and kept
    // entries <= distinct keys <= k-mers
#ifdef KB_BIN_ABL
    static const bool abl_on = env_int("KB_BIN_ABLATE", 0) != 0;  // (phases switched off: wrong results by design)
#else
    constexpr bool abl_on = false;
#endif
    if (!abl_on && (c->h_totals[5] != N || c->h_totals[0] > c->h_totals[6] || c->h_totals[6] > N))
        return fail(KB_EDEVICE,
                    "internal: result invariant violated (counted %llu of %llu k-mers, %llu entries, %llu distinct)",
                    (unsigned long long)c->h_totals[5], (unsigned long long)N, (unsigned long long)c->h_totals[0],
                    (unsigned long long)c->h_totals[6]);
    c->n_entries = c->h_totals[0];
    c->n_ids = c->h_totals[1];
    c->n_distinct = c->h_totals[6];
    if (bucketed) {
        const double rho_now = N ? (double)c->h_totals[6] / (double)N : 0.1;
        KB_DBG("bins done: %.3f ms since finalize (allocations %.3f ms)\n", now_ms() - c->t_fin, g_alloc_ms);
        if (learn) {
            const uint64_t nb = std::min<uint64_t>(c->h_totals[2], max_bins);
            const uint32_t* hb = c->h_bins.p;
            if (const char* dp = getenv("KB_DIAG_BINS")) {  // (diagnostic: this pass's bins, appended)
                if (FILE* f = fopen(dp, "a")) {
                    for (uint64_t i = 0; i < nb; i++)
                        fprintf(f, "%u %u %u %u %u\n", c->part, hb[i] & 0xFFFFu, hb[i] >> 16, hb[max_bins + i],
                                hb[2 * max_bins + i]);
                    fclose(f);
                }
            }
            kb_ctx::BucketMap* bm0 = bmap_find(c, NB);
            if (bm0) {  // rebuilt when this key is next binned
                bm0->p_mm.assign(hb, hb + nb);
                bm0->p_cnt.assign(hb + max_bins, hb + max_bins + nb);
                bm0->p_occ.assign(hb + 2 * max_bins, hb + 2 * max_bins + nb);
                bm0->p_rho = rho_now;
                bm0->pending = true;
            } else {  // (no map at all: KB_BIN_PRIOR=0) the next pass needs one now
                const int rc2 = bmap_apply(c, NB, hb, hb + max_bins, hb + 2 * max_bins, nb, rho_now);
                if (rc2) return rc2;
            }
            KB_DBG("learn part %u/%u: %s (bins %llu, R %llu)\n", c->part, c->part_n, bm0 ? "deferred" : "built",
                   (unsigned long long)nb, (unsigned long long)R);
        }
    }
    c->n_occ_entries_hint = c->n_entries;
    c->ecap_hint = c->n_entries + c->n_entries / 4 + 1024;
    if (N) c->rho = (float)((double)c->n_distinct / (double)N);
    // keys the tables will hold under the pre-filter: measured when it ran,
    // else the kept keys plus a margin for sketch collisions and counts 2..cutoff
    if (N) c->rho_tab = a.pf ? (float)((double)c->h_totals[11] / (double)N * 1.05)
                             : std::min(c->rho, (float)((double)c->n_entries / (double)N * 1.3 + 0.01));
    if (c->timing == KB_TIMING_ALL) {
        HIPCHK(hipEventElapsedTime(&c->tm.scan_insert_ms, c->ev[1], c->ev[2]));
        HIPCHK(hipEventElapsedTime(&c->tm.sort_ms, c->ev[2], c->ev[3]));
        HIPCHK(hipEventElapsedTime(&c->tm.runs_ms, c->ev[3], c->ev[4]));
        HIPCHK(hipEventElapsedTime(&c->tm.emit_ms, c->ev[4], c->ev[5]));
        HIPCHK(hipEventElapsedTime(&c->tm.total_ms, c->ev[0], c->ev[5]));
    } else {
        c->tm.scan_insert_ms = c->tm.sort_ms = c->tm.runs_ms = c->tm.emit_ms = c->tm.total_ms = 0.f;
    }
    if (c->timing) HIPCHK(hipEventElapsedTime(&c->tm.bin_kernel_ms, c->ev[6], c->ev[7]));
    {
        const uint64_t* ps = c->h_totals + 16;  // (BinArgs::pstat)
        c->tm.heavy_bins = (uint32_t)ps[0];
        c->tm.split_bins = (uint32_t)ps[1];
        c->tm.partitions = ps[2];
        c->tm.overflow_redos = (uint32_t)ps[3];
        c->tm.max_depth = (uint32_t)ps[4];
        c->tm.prefiltered = ps[5];
        c->tm.offset_partitions = ps[6];
        c->tm.flat_partitions = ps[7];
        c->tm.light_prefilter_bins = (uint32_t)ps[8];
        c->tm.ranked_bins = (uint32_t)ps[9];
        c->tm.bitmap_partitions = (uint32_t)ps[10];
        c->tm.long_lists = c->h_misc[4];
        c->tm.clustered_lists = c->h_misc[5];
        const kb_ctx::BucketMap* bm = bucketed ? bmap_find(c, NB) : nullptr;  // (before this pass's learning)
        c->tm.split_mmers = bm ? bm->split : 0u;
    }
    c->tm.table_slots = 1ull << ts_log2;
    c->tm.n_bins = (uint32_t)c->h_totals[2];
    c->nbins_hint = c->tm.n_bins;
    c->tm.n_superkmers = R;
    c->finalized = true;
    c->exported = false;
    return KB_OK;
}

extern "C" int kb_finalize(kb_ctx* c, int prune) {
    if (!c) return fail(KB_EINVAL, "null ctx");
    if (c->finalized) return fail(KB_ESTATE, "already finalized (call kb_reset)");
    int rc = set_device(c);
    if (rc) return rc;
    rc = ingest_check(c, true);  // every host batch packed so far was ACGT
    if (rc) return rc;
    // active batches: unrouted reads, or received super-k-mers (not both)
    bool any_reads = false, any_sk = false;
    for (auto& b : c->batches) {
        if (b.routed) continue;
        (b.superkmers ? any_sk : any_reads) = true;
    }
    if (any_reads && any_sk)
        return fail(KB_ESTATE, "a context bins either its own reads or received super-k-mers");
    // (K < 2M: the record pass walks the reference's live incremental branch,
    // one lane per read -- the thread-per-read kernel, or one lane of a wave
    // per longer read -- in the binned engine)
    if (c->p.K < 2 * c->p.M && !binned_applies(c))
        return fail(KB_EINVAL, "K=%d < 2M=%d needs the binned engine", c->p.K, 2 * c->p.M);
    memset(&c->tm, 0, sizeof(c->tm));
    const int SW = c->KW == 1 ? 2 : 4;
    const bool track_first = (c->p.flags & KB_TRACK_FIRST) != 0;
    bool affine = false;
    int64_t id_c = 0;
    if (any_sk) {
        affine = false;
    } else {
        rc = read_id_map(c, affine, id_c);
        if (rc) return rc;
    }
    if (binned_applies(c)) {
        if (any_sk) return finalize_binned(c, prune, true, 0, true);  // ordinal = read id
        return finalize_binned(c, prune, affine, id_c, false);
    }
    if (c->part_n > 1) return fail(KB_EINVAL, "partitioned passes need the binned engine (K <= 63, reads <= 512 bp)");
    c->tm.engine = KB_ENG_TABLE;
    // per-read occurrence offsets (the table engine's record slots)
    uint64_t N = 0;
    for (auto& b : c->batches) {
        if (b.routed) continue;
        if (!b.have_occ) {
            rc = b.superkmers ? sk_batch_offsets(c, b) : batch_offsets(c, b);
            if (rc) return rc;
        }
        b.occ_base = N;
        N += b.n_occ;
    }
    c->n_occ = N;
    if (N >= 0xFFFFFFFFull)
        return fail(KB_EOVERFLOW, "%llu k-mer occurrences in one context (limit 2^32-1)",
                    (unsigned long long)N);
    // ---- table plan: ~0.6 load for the expected distinct keys
    uint64_t slots = c->p.table_slots;
    if (!slots) slots = c->learned_slots;
    if (!slots) slots = next_pow2(std::max<uint64_t>(4096, N / 6));
    slots = std::max<uint64_t>(slots, 1024);
    HIPCHK(c->occ_a.ensure(N));
    HIPCHK(c->occ_b.ensure(N));
    HIPCHK(c->ids_out.ensure(N));
    uint32_t status = 0, ndist = 0;
    for (int attempt = 0;; attempt++) {
        if (slots > (1ull << 32) - 1)
            return fail(KB_ENOMEM, "table would need 2^32 slots or more");
        hipError_t e = c->table.ensure(slots * SW);
        if (e != hipSuccess)
            return fail(KB_ENOMEM, "table of %llu slots: %s", (unsigned long long)slots,
                        hipGetErrorString(e));
        c->slots = slots;
        REC(0);
        HIPCHK(hipMemsetAsync(c->table.p, 0, slots * SW * sizeof(uint64_t), c->s));
        HIPCHK(hipMemsetAsync(c->misc.p, 0, 2 * sizeof(uint32_t), c->s));
        if (track_first) {
            HIPCHK(c->first.ensure(slots));
            HIPCHK(hipMemsetAsync(c->first.p, 0xFF, slots * sizeof(uint64_t), c->s));
        }
        REC(1);
        c->tm.scan_insert_launches = 0;
        for (auto& b : c->batches) {
            if (b.routed) continue;
            if (b.superkmers) {
                SkArgs a{};
                a.recs = b.recs;
                a.rec_base = b.rec_base;
                a.n_rec = b.n_reads;
                a.rec_words = rec_words(c);
                a.table = c->table.p;
                a.mask = slots - 1;
                a.occ = c->occ_a.p;
                a.occ_base = b.occ_base;
                a.n_occ_total = N;
                a.first = track_first ? c->first.p : nullptr;
                a.n_distinct = c->misc.p + 1;
                a.status = c->misc.p;
                a.max_distinct = (uint32_t)std::min<uint64_t>(slots - slots / 8, 0xFFFFFFFFull);
                a.max_probe = (uint32_t)std::min<uint64_t>(slots, 1u << 14);  // past it: rerun bigger
                a.K = c->p.K;
                a.M = c->p.M;
                HIPCHK(launch_insert_sk(a, c->KW, c->s));
                c->tm.scan_insert_launches++;
                continue;
            }
            ScanArgs a{};
            a.words = b.words;
            a.lens = b.lens;
            a.kmer_base = b.kmer_base;
            a.n_reads = b.n_reads;
            a.table = c->table.p;
            a.mask = slots - 1;
            a.occ = c->occ_a.p;
            a.occ_base = b.occ_base;
            a.n_occ_total = N;
            a.ord_base = (uint32_t)b.ord_base;
            a.first = track_first ? c->first.p : nullptr;
            a.n_distinct = c->misc.p + 1;
            a.status = c->misc.p;
            a.max_distinct = (uint32_t)std::min<uint64_t>(slots - slots / 8, 0xFFFFFFFFull);
            a.max_probe = (uint32_t)std::min<uint64_t>(slots, 1u << 14);  // past it: rerun bigger
            a.RW = b.RW;
            a.K = c->p.K;
            a.M = c->p.M;
            HIPCHK(launch_scan_insert(a, c->KW, c->s));
            c->tm.scan_insert_launches++;
        }
        REC(2);
        HIPCHK(hipMemcpyAsync(c->h_misc, c->misc.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
        status = c->h_misc[0];
        ndist = c->h_misc[1];
        if (!(status & (ST_TABLE_FULL | ST_PROBE_LIMIT))) break;
        if (attempt >= 6) return fail(KB_ENOMEM, "table retries exhausted (status %u)", status);
        slots *= 4;
    }
    c->n_distinct = ndist;
#ifdef KB_ABLATE_TABLE
    if (c->timing) HIPCHK(hipEventElapsedTime(&c->tm.scan_insert_ms, c->ev[1], c->ev[2]));
    c->n_entries = c->n_ids = 0;
    c->finalized = true;
    return KB_OK;
#endif
    // next finalize on this context: ~0.6 load for the distinct keys seen now
    if (!c->p.table_slots)
        c->learned_slots = std::max<uint64_t>(1024, next_pow2((uint64_t)ndist * 5 / 3 + 1));
    // ---- stable radix sort of the records by slot
    const int key_bits = log2u(slots);
    const uint64_t ne_cap = (uint64_t)ndist + 1;
    HIPCHK(c->scratch.ensure(std::max(runs_scratch_elems(N, ne_cap), c->scratch.cap)));
    const uint64_t nflags = onesweep_flag_elems(N);
    if (c->os_flags.cap < nflags || c->os_epoch > (1u << 24) - 8) {
        HIPCHK(c->os_flags.ensure(nflags));
        HIPCHK(hipMemsetAsync(c->os_flags.p, 0, c->os_flags.cap * sizeof(uint64_t), c->s));
        c->os_epoch = 0;
    }
    HIPCHK(c->os_aux.ensure(4 * 256 + 8));
    HIPCHK(launch_onesweep(c->occ_a.p, c->occ_b.p, N, key_bits, c->os_flags.p, c->os_aux.p,
                           &c->os_epoch, &c->sorted, c->s));
    c->tm.sort_passes = (uint32_t)((key_bits + 7) / 8);
    REC(3);
    // ---- runs -> counts -> prune -> CSR entries
    HIPCHK(c->starts.ensure(ne_cap + 1));
    HIPCHK(c->e_mmer.ensure(ne_cap));
    HIPCHK(c->e_cnt.ensure(ne_cap));
    HIPCHK(c->e_hi.ensure(ne_cap));
    c->e_hi_zeroed = nullptr;  // (the table engine writes it)
    HIPCHK(c->e_lo.ensure(ne_cap));
    HIPCHK(c->e_off.ensure(ne_cap));
    if (track_first) HIPCHK(c->e_first.ensure(ne_cap));
    const uint32_t keep_gt = prune ? (uint32_t)c->p.cutoff : 0u;
    // ids: affine fast path (id = ordinal + c for every batch) avoids the gather
    HIPCHK(launch_runs(c->sorted, N, c->table.p, c->KW, keep_gt, c->starts.p,
                       (any_sk || affine) ? nullptr : c->read_ids.p, (uint32_t)(affine ? id_c : 0),
                       c->ids_out.p, ne_cap, c->e_mmer.p, c->e_hi.p, c->e_lo.p, c->e_cnt.p,
                       c->e_off.p, track_first ? c->first.p : nullptr,
                       track_first ? c->e_first.p : nullptr, c->scratch.p, c->scratch.cap,
                       c->totals.p, c->s));
    REC(4);
    REC(5);
    HIPCHK(hipMemcpyAsync(c->h_totals, c->totals.p, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
    if (N) HIPCHK(hipMemcpyAsync(c->h_misc + 8, c->os_aux.p + 1028, sizeof(uint32_t), hipMemcpyDeviceToHost, c->s));
    else c->h_misc[8] = 0;
    HIPCHK(hipStreamSynchronize(c->s));
    if (c->h_misc[8]) return fail(KB_EDEVICE, "radix look-back timed out (device error word %u)", c->h_misc[8]);
    if (c->h_totals[3])
        return fail(KB_EDEVICE, "internal: %llu runs > %llu distinct keys", (unsigned long long)c->h_totals[3],
                    (unsigned long long)ne_cap);
    // result invariants: kept entries <= distinct keys (runs) <= k-mers, ids <= k-mers
    if (c->h_totals[0] > c->h_totals[2] || c->h_totals[2] > N || c->h_totals[1] > N)
        return fail(KB_EDEVICE, "internal: result invariant violated (%llu entries, %llu distinct, %llu ids, %llu k-mers)",
                    (unsigned long long)c->h_totals[0], (unsigned long long)c->h_totals[2],
                    (unsigned long long)c->h_totals[1], (unsigned long long)N);
    c->n_entries = c->h_totals[0];
    c->n_ids = c->h_totals[1];
    if (c->timing) {
        HIPCHK(hipEventElapsedTime(&c->tm.scan_insert_ms, c->ev[1], c->ev[2]));
        HIPCHK(hipEventElapsedTime(&c->tm.sort_ms, c->ev[2], c->ev[3]));
        HIPCHK(hipEventElapsedTime(&c->tm.runs_ms, c->ev[3], c->ev[4]));
        HIPCHK(hipEventElapsedTime(&c->tm.emit_ms, c->ev[4], c->ev[5]));
        HIPCHK(hipEventElapsedTime(&c->tm.total_ms, c->ev[0], c->ev[5]));
    }
    c->tm.table_slots = slots;
    c->finalized = true;
    c->exported = false;
    return KB_OK;
}

extern "C" int kb_digest(kb_ctx* c, uint64_t* out) {
    if (!c || !out) return fail(KB_EINVAL, "null argument");
    if (!c->finalized) return fail(KB_ESTATE, "digest before finalize");
    int rc = set_device(c);
    if (rc) return rc;
    // totals[12..13] are free after the finalize
    unsigned long long* d = reinterpret_cast<unsigned long long*>(c->totals.p + 12);
    HIPCHK(launch_digest(c->e_mmer.p, c->e_hi.p, c->e_lo.p, c->e_cnt.p, c->e_off.p, c->ids_out.p, c->n_entries, d,
                         c->s));
    HIPCHK(hipMemcpyAsync(c->h_totals + 12, d, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    out[0] = c->n_entries;
    out[1] = c->n_ids;
    out[2] = c->h_totals[12];
    out[3] = c->h_totals[13];
    return KB_OK;
}

extern "C" int kb_export_device(kb_ctx* c, kb_csr* out) {
    if (!c || !out) return fail(KB_EINVAL, "null argument");
    if (!c->finalized) return fail(KB_ESTATE, "export before finalize");
    out->n_entries = c->n_entries;
    out->n_ids = c->n_ids;
    out->n_kmers = c->n_occ;
    out->n_distinct = c->n_distinct;
    out->mmer = c->e_mmer.p;
    out->kmer_hi = c->e_hi.p;
    out->kmer_lo = c->e_lo.p;
    out->count = c->e_cnt.p;
    out->offset = c->e_off.p;
    out->ids = c->ids_out.p;
    out->first = (c->p.flags & KB_TRACK_FIRST) ? c->e_first.p : nullptr;
    return KB_OK;
}

extern "C" int kb_export(kb_ctx* c, kb_csr* out) {
    if (!c || !out) return fail(KB_EINVAL, "null argument");
    if (!c->finalized) return fail(KB_ESTATE, "export before finalize");
    int rc = set_device(c);
    if (rc) return rc;
    if (!c->exported) {
        const uint64_t n = c->n_entries;
        const bool tf = (c->p.flags & KB_TRACK_FIRST) != 0;
        HIPCHK(c->h_mmer.ensure(n));
        HIPCHK(c->h_cnt.ensure(n));
        HIPCHK(c->h_hi.ensure(n));
        HIPCHK(c->h_lo.ensure(n));
        HIPCHK(c->h_off.ensure(n + 1));
        if (tf) HIPCHK(c->h_first.ensure(n));
        HIPCHK(c->h_ids.ensure(c->n_ids));
        if (n) {
            HIPCHK(hipMemcpyAsync(c->h_mmer.p, c->e_mmer.p, n * 4, hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_cnt.p, c->e_cnt.p, n * 4, hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_hi.p, c->e_hi.p, n * 8, hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_lo.p, c->e_lo.p, n * 8, hipMemcpyDeviceToHost, c->s));
            HIPCHK(hipMemcpyAsync(c->h_off.p, c->e_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, c->s));
            if (tf)
                HIPCHK(hipMemcpyAsync(c->h_first.p, c->e_first.p, n * 8, hipMemcpyDeviceToHost, c->s));
        } else {
            c->h_off.p[0] = 0;
        }
        if (c->n_ids)
            HIPCHK(hipMemcpyAsync(c->h_ids.p, c->ids_out.p, c->n_ids * 4, hipMemcpyDeviceToHost, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
        c->exported = true;
    }
    out->n_entries = c->n_entries;
    out->n_ids = c->n_ids;
    out->n_kmers = c->n_occ;
    out->n_distinct = c->n_distinct;
    out->mmer = c->h_mmer.p;
    out->kmer_hi = c->h_hi.p;
    out->kmer_lo = c->h_lo.p;
    out->count = c->h_cnt.p;
    out->offset = c->h_off.p;
    out->ids = c->h_ids.p;
    out->first = (c->p.flags & KB_TRACK_FIRST) ? c->h_first.p : nullptr;
    return KB_OK;
}

extern "C" int kb_generate_reads_device_at(int device, uint64_t* d_words, uint32_t* d_lens,
                                           uint64_t n_reads, uint32_t read_len, uint64_t genome_len,
                                           uint32_t err_ppm, uint64_t seed, uint64_t read_base) {
    if (!d_words || !d_lens) return fail(KB_EINVAL, "null device pointers");
    if (read_len < 1 || genome_len < read_len) return fail(KB_EINVAL, "bad read_len/genome_len");
    if (err_ppm > 1000000) return fail(KB_EINVAL, "err_per_million > 1e6");
    HIPCHK(hipSetDevice(device));
    HIPCHK(launch_generate(d_words, d_lens, n_reads, read_len, genome_len, err_ppm, seed, read_base, 0));
    HIPCHK(hipStreamSynchronize(0));
    return KB_OK;
}

extern "C" int kb_generate_reads_device(int device, uint64_t* d_words, uint32_t* d_lens,
                                        uint64_t n_reads, uint32_t read_len, uint64_t genome_len,
                                        uint32_t err_ppm, uint64_t seed) {
    return kb_generate_reads_device_at(device, d_words, d_lens, n_reads, read_len, genome_len, err_ppm,
                                       seed, 0);
}

extern "C" int kb_unpack_reads_to_host(int device, const uint64_t* d_words, const uint32_t* d_lens,
                                       uint64_t n_reads, uint32_t wpr, char* h_bases,
                                       uint32_t* h_lens) {
    if (!d_words || !d_lens || !h_bases || !h_lens) return fail(KB_EINVAL, "null argument");
    HIPCHK(hipSetDevice(device));
    if (!n_reads) return KB_OK;
    HIPCHK(hipMemcpy(h_lens, d_lens, n_reads * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint64_t> off(n_reads + 1);
    off[0] = 0;
    for (uint64_t r = 0; r < n_reads; r++) off[r + 1] = off[r] + h_lens[r];
    uint64_t *d_off = nullptr;
    uint8_t* d_out = nullptr;
    HIPCHK(hipMalloc((void**)&d_off, (n_reads + 1) * 8));
    hipError_t e = hipMalloc((void**)&d_out, std::max<uint64_t>(off[n_reads], 1));
    if (e != hipSuccess) { (void)hipFree(d_off); return fail(KB_ENOMEM, "unpack alloc"); }
    e = hipMemcpy(d_off, off.data(), (n_reads + 1) * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_unpack(d_words, d_lens, n_reads, (int)wpr, d_off, d_out, 0);
    if (e == hipSuccess) e = hipMemcpy(h_bases, d_out, off[n_reads], hipMemcpyDeviceToHost);
    (void)hipFree(d_off);
    (void)hipFree(d_out);
    if (e != hipSuccess) return fail(KB_EDEVICE, "unpack: %s", hipGetErrorString(e));
    return KB_OK;
}
