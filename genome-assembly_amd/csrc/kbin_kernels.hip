// kbin_kernels.hip -- CDNA4 (gfx950) kernels of the k-mer binning engine.
//
// Hot path = the reference's process_read (binning.c:902-1076) feeding the
// two-level zhash/llist containers, plus prune_data (binning.c:1085-1144):
//
//   scan_insert   one wavefront per read: read tile staged in LDS, the
//                 complement-canonical mmer window argmax by a wave-wide max
//                 reduction, the "sticky" signature chain walked wave-uniformly,
//                 then every k-mer key inserted/counted in one open-addressed
//                 (mmer, kmer) table with device atomics.
//                 Each occurrence leaves one record (slot << 32 | call ordinal),
//                 written in descending call order.
//   radix sort    stable LSD sort of the records by slot (8-bit digits, LDS
//                 multisplit): every key becomes one run whose ordinals are
//                 already descending = the reference's prepend order.
//   runs          run boundaries -> counts -> prune (count > cutoff) ->
//                 CSR entries (stream compaction) and the surviving runs'
//                 read ids, copied coalesced.
//
// All integer work: no MFMA.  Roofline = HBM.
#include <algorithm>

#include "kbin_internal.h"
#include "kbin_device.h"

namespace kb {

// ---------------------------------------------------------------------------
// pack: ASCII reads -> 2-bit getval codes (binning.c:91-111), 32 bases/word
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t* __restrict__ bases,
                                                   const uint64_t* __restrict__ off,
                                                   uint64_t n_reads, int RW,
                                                   uint64_t* __restrict__ words,
                                                   uint32_t* __restrict__ lens,
                                                   uint32_t* __restrict__ status) {
    const uint64_t total = n_reads * (uint64_t)RW;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = g / RW;
        const int w = (int)(g - r * RW);
        const uint64_t o = off[r];
        const int len = (int)(off[r + 1] - o);
        uint64_t word = 0;
        bool bad = false;
        const int b0 = w * 32;
        for (int j = 0; j < 32; j++) {
            const int b = b0 + j;
            if (b >= len) break;
            const uint32_t c = bases[o + b];
            bad |= !(c == 'A' || c == 'C' || c == 'G' || c == 'T');
            const uint32_t x = (c >> 1) & 3u;  // A0 C1 T2 G3
            const uint32_t v = 3u - (x ^ (x >> 1));  // -> A3 C2 G1 T0
            word |= (uint64_t)v << (62 - 2 * j);
        }
        words[g] = word;
        if (w == 0) lens[r] = (uint32_t)len;
        if (bad) atomicOr(status, ST_ALPHABET);
    }
}

hipError_t launch_pack(const uint8_t* d_bases, const uint64_t* d_off, uint64_t n_reads, int RW,
                       uint64_t* d_words, uint32_t* d_lens, uint32_t* d_status, hipStream_t s) {
    const uint64_t total = n_reads * (uint64_t)RW;
    if (!total) return hipSuccess;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_bases, d_off,
                       n_reads, RW, d_words, d_lens, d_status);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// unpack (test/bench helper): packed -> ASCII via getbp (binning.c:69-88)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void unpack_kernel(const uint64_t* __restrict__ words,
                                                     const uint32_t* __restrict__ lens,
                                                     uint64_t n_reads, int RW,
                                                     const uint64_t* __restrict__ off,
                                                     uint8_t* __restrict__ out) {
    const uint64_t total = n_reads * (uint64_t)RW;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = g / RW;
        const int w = (int)(g - r * RW);
        const int len = (int)lens[r];
        const uint64_t word = words[g];
        for (int j = 0; j < 32; j++) {
            const int b = w * 32 + j;
            if (b >= len) break;
            const uint32_t v = (uint32_t)(word >> (62 - 2 * j)) & 3u;
            out[off[r] + b] = (uint8_t)(v == 0 ? 'T' : v == 1 ? 'G' : v == 2 ? 'C' : 'A');
        }
    }
}

hipError_t launch_unpack(const uint64_t* d_words, const uint32_t* d_lens, uint64_t n_reads, int RW,
                         const uint64_t* d_off, uint8_t* d_bases, hipStream_t s) {
    const uint64_t total = n_reads * (uint64_t)RW;
    if (!total) return hipSuccess;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_words, d_lens,
                       n_reads, RW, d_off, d_bases);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// synthetic reads (mirrors generate_reads.py:93-112 with a
// counter-based RNG so every run regenerates identical reads)
// ---------------------------------------------------------------------------
DEV uint64_t rng(uint64_t stream, uint64_t ctr) {
    return mix64(stream * 0x9E3779B97F4A7C15ull + ctr + 0x632BE59BD9B4E019ull);
}

__global__ __launch_bounds__(256) void generate_kernel(uint64_t* __restrict__ words,
                                                       uint32_t* __restrict__ lens,
                                                       uint64_t n_reads, uint32_t L, int RW,
                                                       uint64_t G, uint32_t err_ppm,
                                                       uint64_t seed, uint64_t read_base) {
    const uint64_t total = n_reads * (uint64_t)RW;
    const uint64_t s_genome = mix64(seed ^ 0x1111111111111111ull);
    const uint64_t s_start = mix64(seed ^ 0x2222222222222222ull);
    const uint64_t s_err = mix64(seed ^ 0x3333333333333333ull);
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = g / RW;
        const int w = (int)(g - r * RW);
        const uint64_t rg = read_base + r;  // global read index: the stream is one genome's
        const uint64_t start = rng(s_start, rg) % (G - L + 1);
        uint64_t word = 0;
        for (int j = 0; j < 32; j++) {
            const uint32_t b = (uint32_t)w * 32u + (uint32_t)j;
            if (b >= L) break;
            const uint64_t pos = start + b;
            // 32 genome bases per RNG draw
            uint32_t v = (uint32_t)(rng(s_genome, pos >> 5) >> (2 * (pos & 31))) & 3u;
            if (err_ppm) {
                const uint64_t u = rng(s_err, rg * (uint64_t)L + b);
                if ((uint32_t)(u % 1000000ull) < err_ppm)
                    v = (v + 1u + (uint32_t)((u >> 32) % 3ull)) & 3u;
            }
            word |= (uint64_t)v << (62 - 2 * j);
        }
        words[g] = word;
        if (w == 0) lens[r] = L;
    }
}

hipError_t launch_generate(uint64_t* d_words, uint32_t* d_lens, uint64_t n_reads, uint32_t read_len,
                           uint64_t genome_len, uint32_t err_ppm, uint64_t seed, uint64_t read_base,
                           hipStream_t s) {
    const int RW = (int)((read_len + 31) / 32);
    const uint64_t total = n_reads * (uint64_t)RW;
    if (!total) return hipSuccess;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(generate_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_words, d_lens,
                       n_reads, read_len, RW, genome_len, err_ppm, seed, read_base);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// generic 3-phase exclusive scan helpers (u64), 4096 items per block
// ---------------------------------------------------------------------------
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = 256 * SCAN_ITEMS;

// scan of block partials in place (exclusive), single block of 1024 threads;
// also writes the grand total to *total_out
__global__ __launch_bounds__(1024) void scan_partials_kernel(uint64_t* __restrict__ p, uint64_t n,
                                                             uint64_t* __restrict__ total_out) {
    __shared__ uint64_t sh[1024];
    const uint64_t per = (n + 1023) / 1024;
    const uint64_t lo = threadIdx.x * per;
    const uint64_t hi = lo + per < n ? lo + per : n;
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; i++) s += p[i];
    sh[threadIdx.x] = s;
    __syncthreads();
    // Hillis-Steele inclusive scan over 1024 sums
    for (int d = 1; d < 1024; d <<= 1) {
        uint64_t t = threadIdx.x >= (unsigned)d ? sh[threadIdx.x - d] : 0;
        __syncthreads();
        sh[threadIdx.x] += t;
        __syncthreads();
    }
    uint64_t run = sh[threadIdx.x] - s;
    for (uint64_t i = lo; i < hi; i++) {
        uint64_t x = p[i];
        p[i] = run;
        run += x;
    }
    if (threadIdx.x == 1023 && total_out) *total_out = sh[1023];
}

// k-mers per read = max(0, len-K+1); kmer_base = exclusive scan, [n] = total
__global__ __launch_bounds__(256) void nk_partials_kernel(const uint32_t* __restrict__ lens,
                                                          uint64_t n, int K,
                                                          uint64_t* __restrict__ part) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t r = base + j;
        if (r < n) {
            const int nk = (int)lens[r] - K + 1;
            s += nk > 0 ? (uint64_t)nk : 0;
        }
    }
    s = block_sum256(s, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void nk_apply_kernel(const uint32_t* __restrict__ lens,
                                                       uint64_t n, int K,
                                                       const uint64_t* __restrict__ part,
                                                       uint64_t* __restrict__ kmer_base) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint64_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t r = base + j;
        uint64_t x = 0;
        if (r < n) {
            const int nk = (int)lens[r] - K + 1;
            x = nk > 0 ? (uint64_t)nk : 0;
        }
        v[j] = x;
        s += x;
    }
    uint64_t tot;
    uint64_t run = block_excl_scan256(s, sh, tot) + part[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t r = base + j;
        if (r < n) kmer_base[r] = run;
        run += v[j];
    }
}

uint64_t kmer_base_scratch_elems(uint64_t n_reads) {
    return (n_reads + SCAN_TILE - 1) / SCAN_TILE + 1;
}

hipError_t launch_kmer_base(const uint32_t* d_lens, uint64_t n_reads, int K, uint64_t* d_kmer_base,
                            uint64_t* d_scratch, uint64_t scratch_n, hipStream_t s) {
    const uint64_t nb = (n_reads + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 0) return hipMemsetAsync(d_kmer_base, 0, sizeof(uint64_t), s);
    if (scratch_n < nb) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nk_partials_kernel, dim3((unsigned)nb), dim3(256), 0, s, d_lens, n_reads, K,
                       d_scratch);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, d_scratch, nb,
                       d_kmer_base + n_reads);
    hipLaunchKernelGGL(nk_apply_kernel, dim3((unsigned)nb), dim3(256), 0, s, d_lens, n_reads, K,
                       d_scratch, d_kmer_base);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// scan_insert -- the hot kernel
// ---------------------------------------------------------------------------
// Key encodings (claim word never 0 so a zeroed table is all-empty):
//   KW=1: claim = code + 1                         (code < 2^62)
//   KW=2: claim = (code >> 63) + 1, w1 = (code & (2^63-1)) | PUB   (code < 2^126)
template <int KW>
struct Key {
    static constexpr int SW = KW == 1 ? 2 : 4;  // u64 words per slot
    uint64_t a = 0, b = 0;                      // b unused when KW == 1
    DEV uint64_t hash(uint32_t tag) const {
        if constexpr (KW == 1) return mix64(a ^ ((uint64_t)tag * 0xD6E8FEB86659FD93ull));
        else return mix64(a ^ mix64(b + (uint64_t)tag * 0xD6E8FEB86659FD93ull));
    }
};


// Find-or-insert one key; returns its slot index (NONE on probe-limit failure).
// Protocol (DESIGN.md "Table protocol"): claim by 64-bit CAS of the claim word
// on an empty slot; the winner then publishes the other words with atomic
// stores, each carrying its own marker (tag = mmer+1 != 0, PUB bit).  A reader
// that finds an unpublished word re-reads it with an atomic RMW (coherent
// across the XCD L2s) and, if still unpublished, retries the same slot on its
// next loop trip -- no lane ever waits inside a branch that another lane of
// its own wave has to leave first.  Words only ever go empty -> final, so a
// stale read can only show an older state, which the CAS / RMW re-read fixes.
template <int KW>
DEV uint32_t table_insert(uint64_t* __restrict__ table, uint64_t mask, const Key<KW>& k,
                          uint32_t tag, uint32_t max_probe, bool& is_new) {
    constexpr int SW = Key<KW>::SW;
    uint64_t idx = k.hash(tag) & mask;
    uint32_t probes = 0;
    is_new = false;
    while (true) {
        uint64_t* s = table + idx * SW;
        uint32_t* tagp = reinterpret_cast<uint32_t*>(s + (SW == 2 ? 1 : 2));
        uint64_t w0 = atomic_load_u64(s);
        uint32_t t = atomic_load_u32(tagp);
        uint64_t w1 = 0;
        if constexpr (KW == 2) w1 = atomic_load_u64(s + 1);
        if (w0 == 0) {
            const uint64_t old = atomicCAS((unsigned long long*)s, 0ull, (unsigned long long)k.a);
            if (old == 0) {
                if constexpr (KW == 2)
                    __hip_atomic_store(s + 1, k.b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(tagp, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                is_new = true;
                return (uint32_t)idx;
            }
            w0 = old;
            t = 0;  // anything loaded before the CAS may predate the claim
            w1 = 0;
        }
        if (w0 == k.a) {
            bool pending = false;
            if constexpr (KW == 2) {
                if (!(w1 & PUB)) w1 = atomicOr((unsigned long long*)(s + 1), 0ull);
                if (!(w1 & PUB)) pending = true;
            }
            if (t == 0) t = atomicOr(tagp, 0u);
            if (t == 0) pending = true;
            if (pending) continue;  // claimed but not yet published: re-read next trip
            if (t == tag && (KW == 1 || w1 == k.b)) return (uint32_t)idx;
        }
        idx = (idx + 1) & mask;
        if (++probes > max_probe) return NONE;
    }
}

// One wavefront per read.  For every k-mer occurrence it emits the record
//   (slot << 32) | call_ordinal
// at position n_total-1-(global occurrence index): occurrences are written in
// DESCENDING call order, so the stable radix sort by slot that follows leaves
// each key's ordinals descending -- the reference's prepend order
// (binning.c:1061-1068) -- with no per-key sort.
template <int KW>
__global__ __launch_bounds__(256) void scan_insert_kernel(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int RW = A.RW, K = A.K, M = A.M;
    const int W = K - M + 1;                   // mmer starts per k-mer window (<= 64)
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    const uint32_t halfM = 1u << (2 * M - 1);  // s < halfM <=> first base T/G <=> complement wins
    uint64_t* sw = smem + wid * (RW + 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    uint64_t* const occ_end = A.occ + A.n_occ_total - 1 - A.occ_base;
    uint32_t local_new = 0;
    uint32_t st = 0;

    for (uint64_t r = (uint64_t)blockIdx.x * 4 + wid; r < A.n_reads; r += nwaves) {
        // a full table (or a probe past the limit) anywhere: the host reruns
        // bigger, so the rest of this attempt is wasted work -- stop now
        if (rfl((int)atomic_load_u32(A.status)) & (int)(ST_TABLE_FULL | ST_PROBE_LIMIT)) break;
        const int L = rfl((int)A.lens[r]);
        const int nK = L - K + 1;
        if (nK <= 0) continue;
        // stage the read tile in LDS (one extra zero word for window reads)
        wave_sync();
        for (int w = lane; w < RW; w += 64) sw[w] = A.words[r * RW + w];
        if (lane == 0) sw[RW] = 0;
        wave_sync();
        uint64_t* const orow = occ_end - A.kmer_base[r];
        const uint64_t ordv = (uint64_t)(A.ord_base + (uint32_t)r);

        int seg_lo = 0, seg_hi = -1;  // current sticky segment [seg_lo, seg_hi], sig = seg_hi
        for (int i0 = 0; i0 < nK; i0 += 64) {
            const int i = i0 + lane;
            int sig = 0;
            const int chunk_end = min(i0 + 63, nK - 1);
            while (true) {
                if (i >= seg_lo && i <= seg_hi) sig = seg_hi;
                if (seg_hi >= chunk_end) break;
                // fresh signature for k-mer seg_lo (binning.c:922-988):
                // leftmost strict argmax of c(p) = max(s, 4^M-1-s) over
                // p in [seg_lo, seg_lo+K-M] -- one mmer start per lane, then a
                // wave max of (c << 16 | 0xFFFF - p).
                seg_lo = seg_hi + 1;
                const int d = (lane - seg_lo) & 63;
                uint32_t key = 0;
                if (d < W) {
                    const int p = seg_lo + d;
                    const uint32_t s = (uint32_t)(window64(sw, p) >> (64 - 2 * M));
                    const uint32_t c = s >= halfM ? s : maskM - s;
                    key = (c << 16) | (0xFFFFu - (uint32_t)p);
                }
                key = wave_max_u32(key);
                seg_hi = rfl((int)(0xFFFFu - (key & 0xFFFFu)));
            }
            if (i < nK) {
                // key build + complement without reversal (binning.c:1023-1040)
                const uint32_t s = (uint32_t)(window64(sw, sig) >> (64 - 2 * M));
                const bool rev = s < halfM;
                const uint32_t mm = rev ? maskM - s : s;
                Key<KW> key;
                if constexpr (KW == 1) {
                    uint64_t code = window64(sw, i) >> (64 - 2 * K);
                    if (rev) code ^= (1ull << (2 * K)) - 1ull;
                    key.a = code + 1ull;
                } else {
                    const int kh = K - 32;  // bases in the high word (0..31)
                    uint64_t hi = kh ? (window64(sw, i) >> (64 - 2 * kh)) : 0ull;
                    uint64_t lo = window64(sw, i + kh);
                    if (rev) {
                        hi ^= kh ? ((1ull << (2 * kh)) - 1ull) : 0ull;
                        lo = ~lo;
                    }
                    // split the 2K-bit code at bit 63
                    key.a = ((hi << 1) | (lo >> 63)) + 1ull;
                    key.b = (lo & ~PUB) | PUB;
                }
                bool is_new = false;
#ifdef KB_ABLATE_TABLE  // timing experiment only: no table, slot = hash (kbin_api stops after the scan)
                const uint32_t slot = (uint32_t)(key.hash(mm + 1u) & A.mask);
#else
                const uint32_t slot = table_insert<KW>(A.table, A.mask, key, mm + 1u, A.max_probe, is_new);
#endif
                if (slot == NONE) {
                    st |= ST_PROBE_LIMIT;
                    atomicOr(A.status, ST_PROBE_LIMIT);  // now: every wave stops at its next read
                }
                local_new += is_new ? 1u : 0u;
                *(orow - i) = ((uint64_t)slot << 32) | ordv;
                if (A.first && slot != NONE)  // insertion order of the reference (KB_TRACK_FIRST)
                    atomicMin((unsigned long long*)&A.first[slot], (unsigned long long)((ordv << 16) | (uint64_t)i));
            }
        }
    }
    // distinct-key accounting: one atomic per wave
    uint32_t tot = local_new;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tot += (uint32_t)__shfl_xor((int)tot, off, 64);
    uint32_t stw = st;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) stw |= (uint32_t)__shfl_xor((int)stw, off, 64);
    if (lane == 0) {
        if (tot) {
            const uint32_t before = atomicAdd(A.n_distinct, tot);
            if ((uint64_t)before + tot > A.max_distinct) stw |= ST_TABLE_FULL;
        }
        if (stw) atomicOr(A.status, stw);
    }
}

hipError_t launch_scan_insert(const ScanArgs& a, int KW, hipStream_t s) {
    if (!a.n_reads) return hipSuccess;
    uint64_t blocks = (a.n_reads + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    const size_t lds = (size_t)4 * (a.RW + 1) * sizeof(uint64_t);
    if (KW == 1)
        hipLaunchKernelGGL(scan_insert_kernel<1>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL(scan_insert_kernel<2>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Multi-GPU routing: a read's k-mers fall into consecutive
// runs that share one signature (super-k-mers, ~10 per 150-bp read at k31/m7).
// The owner of a super-k-mer is a hash of its canonical mmer; each super-k-mer
// travels as one fixed-size record
//   w0 = ord (bits 0-31) | i0 (32-47) | n (48-53) | sig_off (54-59)
//   w1.. = bases [i0, i0 + n + K - 1) packed like the reads (first base in the MSBs)
// where ord is the read's id, i0 its first k-mer position, n its k-mer count
// and sig_off = signature position - i0.
// route_kernel<false> counts records per (destination, read), dest-major, so
// one exclusive scan gives every record its slot in a dest-major send buffer
// in read order; route_kernel<true> writes them.
// ---------------------------------------------------------------------------
DEV uint32_t owner_of(uint32_t mmer, uint32_t G) {
    return (uint32_t)((mix64((uint64_t)mmer + 0x5851F42D4C957F2Dull) >> 32) % G);
}
// kb_set_partition membership (= in_part, kbin_bins.hip: PART_SALT)
DEV bool route_in_part(uint32_t mmer, uint32_t part, uint32_t part_n) {
    return part_n <= 1 || (uint32_t)((mix64((uint64_t)mmer + 0x9E3779B97F4A7C15ull) >> 32) % part_n) == part;
}

template <bool PACK>
__global__ __launch_bounds__(256) void route_kernel(RouteArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int RW = A.RW, K = A.K, M = A.M;
    const int W = K - M + 1;
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    const uint32_t halfM = 1u << (2 * M - 1);
    uint64_t* sw = smem + wid * (RW + 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    for (uint64_t r = (uint64_t)blockIdx.x * 4 + wid; r < A.n_reads; r += nwaves) {
        const int L = rfl((int)A.lens[r]);
        const int nK = L - K + 1;
        uint32_t run = 0;  // lane d: records of read r for destination d
        if (PACK && lane < (int)A.G) run = A.offs[(uint64_t)lane * A.n_reads + r] + (uint32_t)A.adj[lane];
        if (nK > 0) {
            wave_sync();
            for (int w = lane; w < RW; w += 64) sw[w] = A.words[r * RW + w];
            if (lane == 0) sw[RW] = 0;
            wave_sync();
            const uint32_t ordv = PACK ? (uint32_t)A.ids[r] : 0u;
            int seg_lo = 0;
            while (seg_lo < nK) {
                const int d = (lane - seg_lo) & 63;
                uint32_t key = 0;
                if (d < W) {
                    const int p = seg_lo + d;
                    const uint32_t sm = (uint32_t)(window64(sw, p) >> (64 - 2 * M));
                    const uint32_t c = sm >= halfM ? sm : maskM - sm;
                    key = (c << 16) | (0xFFFFu - (uint32_t)p);
                }
                key = wave_max_u32(key);
                const int sig = rfl((int)(0xFFFFu - (key & 0xFFFFu)));
                const uint32_t c = key >> 16;
                const int n = min(sig, nK - 1) - seg_lo + 1;
                const uint32_t dest = A.owner_map ? (uint32_t)A.owner_map[c - halfM] : owner_of(c, A.G);
                // another pass's super-k-mer: neither counted nor written
                const bool mine = route_in_part(c, A.part, A.part_n);
                if (PACK && mine) {
                    const uint64_t pos = (uint64_t)(uint32_t)__shfl((int)run, (int)dest, 64);
                    uint64_t* rec = A.out + pos * (uint64_t)A.rec_words;
                    if (lane == 0) {
                        // (the complement flag, kbin_internal.h ROUTED_REV_BIT)
                        const uint64_t rev = (uint32_t)(window64(sw, sig) >> (64 - 2 * M)) < halfM ? 1ull : 0ull;
                        rec[0] = (uint64_t)ordv | ((uint64_t)seg_lo << 32) | ((uint64_t)n << 48) |
                                 ((uint64_t)(sig - seg_lo) << 54) | (rev << ROUTED_REV_BIT);
                    }
                    else if (lane < A.rec_words) {
                        const int p = seg_lo + 32 * (lane - 1);
                        rec[lane] = p < L ? window64(sw, p) : 0ull;
                    }
                }
                if (mine && lane == (int)dest) run++;
                seg_lo = sig + 1;
            }
        }
        if (!PACK && lane < (int)A.G) A.offs[(uint64_t)lane * A.n_reads + r] = run;
    }
}

hipError_t launch_route(const RouteArgs& a, bool pack, hipStream_t s) {
    if (!a.n_reads) return hipSuccess;
    uint64_t blocks = (a.n_reads + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    const size_t lds = (size_t)4 * (a.RW + 1) * sizeof(uint64_t);
    if (pack)
        hipLaunchKernelGGL(route_kernel<true>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL(route_kernel<false>, dim3((unsigned)blocks), dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_scan_u32(uint32_t* a, uint64_t n, uint64_t* scratch, uint64_t scratch_n, hipStream_t s);

// k-mers per received record -> exclusive scan gives each record's first
// occurrence index (records arrive in ascending id order: by source rank,
// then read order)
__global__ void sk_counts_kernel(const uint64_t* __restrict__ recs, uint64_t n_rec, int rw,
                                 uint32_t* __restrict__ nk) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n_rec;
         t += (uint64_t)gridDim.x * blockDim.x)
        nk[t] = (uint32_t)(recs[t * rw] >> 48) & 63u;
}

hipError_t launch_sk_counts(const uint64_t* recs, uint64_t n_rec, int rw, uint32_t* nk, hipStream_t s) {
    if (!n_rec) return hipSuccess;
    uint64_t blocks = (n_rec + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(sk_counts_kernel, dim3((unsigned)blocks), dim3(256), 0, s, recs, n_rec, rw, nk);
    return hipGetLastError();
}

// receiver: insert every k-mer of every received super-k-mer (one thread per
// record); emits the same occurrence records as scan_insert
template <int KW>
__global__ __launch_bounds__(256) void insert_sk_kernel(SkArgs A) {
    const int K = A.K, M = A.M;
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    const uint32_t halfM = 1u << (2 * M - 1);
    uint64_t* const occ_end = A.occ + A.n_occ_total - 1 - A.occ_base;
    uint32_t local_new = 0, st = 0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < A.n_rec;
         t += (uint64_t)gridDim.x * blockDim.x) {
        if (atomic_load_u32(A.status) & (ST_TABLE_FULL | ST_PROBE_LIMIT)) break;  // rerun bigger
        const uint64_t* rec = A.recs + t * A.rec_words;
        const uint64_t h = rec[0];
        const uint64_t ordv = (uint32_t)h;
        const int i0 = (int)((h >> 32) & 0xFFFFu);
        const int n = (int)((h >> 48) & 63u);
        const int so = (int)((h >> 54) & 63u);
        const uint64_t s0 = rec[1];
        const uint64_t s1 = A.rec_words > 2 ? rec[2] : 0ull;
        const uint64_t s2 = A.rec_words > 3 ? rec[3] : 0ull;
        const uint64_t s3 = A.rec_words > 4 ? rec[4] : 0ull;
        const uint32_t sm = (uint32_t)(span_window(s0, s1, s2, s3, so) >> (64 - 2 * M));
        const bool rev = sm < halfM;
        const uint32_t mm = rev ? maskM - sm : sm;
        uint64_t* const orow = occ_end - A.rec_base[t];
        for (int j = 0; j < n; j++) {
            Key<KW> key;
            if constexpr (KW == 1) {
                uint64_t code = span_window(s0, s1, s2, s3, j) >> (64 - 2 * K);
                if (rev) code ^= (1ull << (2 * K)) - 1ull;
                key.a = code + 1ull;
            } else {
                const int kh = K - 32;
                uint64_t hi = kh ? (span_window(s0, s1, s2, s3, j) >> (64 - 2 * kh)) : 0ull;
                uint64_t lo = span_window(s0, s1, s2, s3, j + kh);
                if (rev) {
                    hi ^= kh ? ((1ull << (2 * kh)) - 1ull) : 0ull;
                    lo = ~lo;
                }
                key.a = ((hi << 1) | (lo >> 63)) + 1ull;
                key.b = (lo & ~PUB) | PUB;
            }
            bool is_new;
            const uint32_t slot = table_insert<KW>(A.table, A.mask, key, mm + 1u, A.max_probe, is_new);
            if (slot == NONE) {
                st |= ST_PROBE_LIMIT;
                atomicOr(A.status, ST_PROBE_LIMIT);
            }
            local_new += is_new ? 1u : 0u;
            *(orow - j) = ((uint64_t)slot << 32) | ordv;
            if (A.first && slot != NONE)
                atomicMin((unsigned long long*)&A.first[slot],
                          (unsigned long long)((ordv << 16) | (uint64_t)(i0 + j)));
        }
    }
    const int lane = threadIdx.x & 63;
    uint32_t tot = local_new;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tot += (uint32_t)__shfl_xor((int)tot, off, 64);
    uint32_t stw = st;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) stw |= (uint32_t)__shfl_xor((int)stw, off, 64);
    if (lane == 0) {
        if (tot) {
            const uint32_t before = atomicAdd(A.n_distinct, tot);
            if ((uint64_t)before + tot > A.max_distinct) stw |= ST_TABLE_FULL;
        }
        if (stw) atomicOr(A.status, stw);
    }
}

hipError_t launch_insert_sk(const SkArgs& a, int KW, hipStream_t s) {
    if (!a.n_rec) return hipSuccess;
    uint64_t blocks = (a.n_rec + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (KW == 1)
        hipLaunchKernelGGL(insert_sk_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(insert_sk_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// LSD radix sort of the occurrence records by their slot field (bits 32..),
// 8-bit digits, stable: per pass a tile histogram, one device-wide exclusive
// scan of the (digit-major, tile-minor) counts, and a scatter that ranks each
// tile in LDS (wave multisplit by 8 ballots) and writes digit runs coalesced.
// ---------------------------------------------------------------------------
constexpr int RUN_SPAN = 8192;  // records of one 256-run round mapped in LDS
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = 256 * RS_ITEMS;  // 4096 records per block

__global__ __launch_bounds__(256) void rs_hist_kernel(const uint64_t* __restrict__ in, uint32_t n,
                                                      int shift, uint32_t* __restrict__ counts,
                                                      uint32_t n_tiles) {
    __shared__ uint32_t h[4][256];
    const int t = threadIdx.x, wid = t >> 6;
#pragma unroll
    for (int w = 0; w < 4; w++) h[w][t] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    uint32_t d[RS_ITEMS];
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const uint64_t k = base + (uint64_t)j * 256 + t;
        d[j] = k < n ? (uint32_t)(in[k] >> shift) & 255u : 256u;
    }
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++)
        if (d[j] < 256u) atomicAdd(&h[wid][d[j]], 1u);
    __syncthreads();
    counts[(uint64_t)t * n_tiles + blockIdx.x] = h[0][t] + h[1][t] + h[2][t] + h[3][t];
}

// Each wave ranks its own contiguous 1024-record chunk of the tile (16 rounds
// of 64) against wave-private digit counters -- multisplit by 8 ballots, no
// block barrier inside the rounds; tile order = (wave, round, lane), so the
// ranking is stable.  Three block barriers per tile in all.
__global__ __launch_bounds__(256) void rs_scatter_kernel(const uint64_t* __restrict__ in,
                                                         uint64_t* __restrict__ out, uint32_t n,
                                                         int shift, const uint32_t* __restrict__ offs,
                                                         uint32_t n_tiles) {
    __shared__ uint64_t buf[RS_TILE];  // 32 KiB: the tile in local digit order
    __shared__ uint32_t wcnt[4][256];  // per-wave digit counters, then per-wave digit bases
    __shared__ uint32_t lstart[256];
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t sh[4];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t tile = blockIdx.x;
    const uint64_t base = (uint64_t)tile * RS_TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)RS_TILE, (uint64_t)n - base);
    const uint32_t wbase = (uint32_t)wid * (RS_TILE / 4);
#pragma unroll
    for (int w = 0; w < 4; w++) wcnt[w][t] = 0;
    gbase[t] = offs[(uint64_t)t * n_tiles + tile];
    uint64_t v[RS_ITEMS];
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const uint32_t li = wbase + (uint32_t)j * 64u + lane;
        v[j] = li < tn ? in[base + li] : 0ull;
    }
    __syncthreads();
    // phase 1: wave-local stable ranks
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t rk[RS_ITEMS];
    uint32_t* const cw = wcnt[wid];
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const bool valid = wbase + (uint32_t)j * 64u + lane < tn;
        const uint32_t d = (uint32_t)(v[j] >> shift) & 255u;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bl = __ballot(bit);
            m &= bit ? bl : ~bl;
        }
        const uint32_t peer = (uint32_t)__popcll(m & lt);
        const uint32_t before = valid ? cw[d] : 0u;
        wave_sync();
        if (valid && peer == 0) cw[d] = before + (uint32_t)__popcll(m);
        wave_sync();
        rk[j] = before + peer;
    }
    __syncthreads();
    // phase 2: thread t = digit t: tile digit starts and per-wave bases
    const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
    uint32_t tot;
    const uint32_t ex = block_excl_scan256<uint32_t>(c0 + c1 + c2 + c3, sh, tot);
    lstart[t] = ex;
    wcnt[0][t] = ex;
    wcnt[1][t] = ex + c0;
    wcnt[2][t] = ex + c0 + c1;
    wcnt[3][t] = ex + c0 + c1 + c2;
    __syncthreads();
    // phase 3: place in LDS, then write digit runs out coalesced
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        if (wbase + (uint32_t)j * 64u + lane < tn) {
            const uint32_t d = (uint32_t)(v[j] >> shift) & 255u;
            buf[cw[d] + rk[j]] = v[j];
        }
    }
    __syncthreads();
    for (uint32_t i = t; i < tn; i += 256) {
        const uint64_t e = buf[i];
        const uint32_t d = (uint32_t)(e >> shift) & 255u;
        out[gbase[d] + (i - lstart[d])] = e;
    }
}

// ---- onesweep variant: one up-front histogram for all digits, then one
// scatter launch per digit whose tiles obtain their global digit offsets by
// decoupled look-back (tiles take tickets in launch order; each publishes its
// digit counts and then its inclusive prefix as single 8-byte words
// {epoch:24 | flag:2 | value:38}, written and polled with agent-scope atomics
// -- the value-is-the-flag hand-off of MI355X_MICROARCH.md "Valid forms").
constexpr int OS_MAX_PASSES = 4;
constexpr uint64_t OS_VAL_MASK = (1ull << 38) - 1;
constexpr uint64_t OS_AGG = 1ull << 38, OS_INC = 2ull << 38;
constexpr int OS_WIN = 16;  // look-back window (tiles per round trip)

__global__ __launch_bounds__(256) void os_hist_kernel(const uint64_t* __restrict__ in, uint32_t n,
                                                      int npass, uint32_t* __restrict__ ghist) {
    __shared__ uint32_t h[OS_MAX_PASSES][256];
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < OS_MAX_PASSES; p++) h[p][t] = 0;
    __syncthreads();
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + t; k < n; k += (uint64_t)gridDim.x * 256) {
        const uint64_t e = in[k];
        for (int p = 0; p < npass; p++) atomicAdd(&h[p][(uint32_t)(e >> (32 + 8 * p)) & 255u], 1u);
    }
    __syncthreads();
    for (int p = 0; p < npass; p++)
        if (h[p][t]) atomicAdd(&ghist[p * 256 + t], h[p][t]);
}

__global__ __launch_bounds__(256) void os_bases_kernel(uint32_t* __restrict__ ghist, int npass) {
    __shared__ uint32_t sh[4];
    for (int p = 0; p < npass; p++) {
        uint32_t tot;
        const uint32_t ex = block_excl_scan256<uint32_t>(ghist[p * 256 + threadIdx.x], sh, tot);
        ghist[p * 256 + threadIdx.x] = ex;
    }
}

__global__ __launch_bounds__(256) void os_scatter_kernel(const uint64_t* __restrict__ in,
                                                         uint64_t* __restrict__ out, uint32_t n,
                                                         int shift, const uint32_t* __restrict__ dbase,
                                                         uint64_t* __restrict__ flags,
                                                         uint32_t* __restrict__ ticket, uint32_t epoch,
                                                         uint32_t* __restrict__ err) {
    __shared__ uint64_t buf[RS_TILE];
    __shared__ uint32_t wcnt[4][256];
    __shared__ uint32_t lstart[256];
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t sh[4];
    __shared__ uint32_t s_tile;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
#pragma unroll
    for (int w = 0; w < 4; w++) wcnt[w][t] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t base = (uint64_t)tile * RS_TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)RS_TILE, (uint64_t)n - base);
    const uint32_t wbase = (uint32_t)wid * (RS_TILE / 4);
    uint64_t v[RS_ITEMS];
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const uint32_t li = wbase + (uint32_t)j * 64u + lane;
        v[j] = li < tn ? in[base + li] : 0ull;
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t rk[RS_ITEMS];
    uint32_t* const cw = wcnt[wid];
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const bool valid = wbase + (uint32_t)j * 64u + lane < tn;
        const uint32_t d = (uint32_t)(v[j] >> shift) & 255u;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bl = __ballot(bit);
            m &= bit ? bl : ~bl;
        }
        const uint32_t peer = (uint32_t)__popcll(m & lt);
        const uint32_t before = valid ? cw[d] : 0u;
        wave_sync();
        if (valid && peer == 0) cw[d] = before + (uint32_t)__popcll(m);
        wave_sync();
        rk[j] = before + peer;
    }
    __syncthreads();
    const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
    const uint32_t c = c0 + c1 + c2 + c3;
    // decoupled look-back for digit t
    const uint64_t ep = (uint64_t)epoch << 40;
    uint64_t* const fl = flags + (uint64_t)tile * 256 + t;
    uint64_t prefix = 0;
    if (tile == 0) {
        __hip_atomic_store(fl, ep | OS_INC | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_store(fl, ep | OS_AGG | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // windowed look-back: OS_WIN predecessor words per round trip
        int64_t tp = (int64_t)tile - 1;
        uint32_t spins = 0;
        while (tp >= 0) {
            uint64_t w[OS_WIN];
#pragma unroll
            for (int i = 0; i < OS_WIN; i++)
                w[i] = tp - i >= 0 ? __hip_atomic_load(flags + (uint64_t)(tp - i) * 256 + t,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : 0ull;
            int used = 0;       // words consumed from the window
            bool done = false, blocked = false;
#pragma unroll
            for (int i = 0; i < OS_WIN; i++) {
                if (!done && !blocked) {
                    if (tp - i < 0) {
                        done = true;  // cannot happen (tile 0 publishes INC), kept for safety
                    } else if ((w[i] >> 40) != epoch || !(w[i] & (OS_AGG | OS_INC))) {
                        blocked = true;
                    } else {
                        prefix += w[i] & OS_VAL_MASK;
                        used = i + 1;
                        if (w[i] & OS_INC) done = true;
                    }
                }
            }
            if (done) break;
            tp -= used;
            if (blocked) {
                if (++spins > (1u << 22)) {  // bounded: report, never hang the device
                    atomicOr(err, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __hip_atomic_store(fl, ep | OS_INC | (prefix + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    gbase[t] = dbase[t] + (uint32_t)prefix;
    uint32_t tot;
    const uint32_t ex = block_excl_scan256<uint32_t>(c, sh, tot);
    lstart[t] = ex;
    wcnt[0][t] = ex;
    wcnt[1][t] = ex + c0;
    wcnt[2][t] = ex + c0 + c1;
    wcnt[3][t] = ex + c0 + c1 + c2;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        if (wbase + (uint32_t)j * 64u + lane < tn) {
            const uint32_t d = (uint32_t)(v[j] >> shift) & 255u;
            buf[cw[d] + rk[j]] = v[j];
        }
    }
    __syncthreads();
    for (uint32_t i = t; i < tn; i += 256) {
        const uint64_t e = buf[i];
        const uint32_t d = (uint32_t)(e >> shift) & 255u;
        out[gbase[d] + (i - lstart[d])] = e;
    }
}

uint64_t onesweep_flag_elems(uint64_t n) { return 256ull * ((n + RS_TILE - 1) / RS_TILE); }

// aux: [0, 4*256) digit histograms -> bases, [1024, 1028) tickets, [1028] error
hipError_t launch_onesweep(uint64_t* a, uint64_t* b, uint64_t n, int key_bits, uint64_t* flags,
                           uint32_t* aux, uint32_t* epoch, uint64_t** sorted, hipStream_t s) {
    *sorted = a;
    if (n == 0) return hipSuccess;
    if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const int npass = (key_bits + 7) / 8;
    if (npass > OS_MAX_PASSES) return hipErrorInvalidValue;
    const uint32_t n_tiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    hipError_t e = hipMemsetAsync(aux, 0, (4 * 256 + 8) * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(os_hist_kernel, dim3(1024), dim3(256), 0, s, a, (uint32_t)n, npass, aux);
    hipLaunchKernelGGL(os_bases_kernel, dim3(1), dim3(256), 0, s, aux, npass);
    uint64_t* src = a;
    uint64_t* dst = b;
    for (int p = 0; p < npass; p++) {
        const uint32_t ep = ++*epoch;
        hipLaunchKernelGGL(os_scatter_kernel, dim3(n_tiles), dim3(256), 0, s, src, dst, (uint32_t)n,
                           32 + 8 * p, aux + p * 256, flags, aux + 1024 + p, ep, aux + 1028);
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    *sorted = src;
    return hipGetLastError();
}

// generic exclusive scan of a u32 array (values sum < 2^32), in place
__global__ __launch_bounds__(256) void scan_u32_partials_kernel(const uint32_t* __restrict__ a, uint64_t n,
                                                                uint64_t* __restrict__ part) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++)
        if (base + j < n) s += a[base + j];
    s = block_sum256(s, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void scan_u32_apply_kernel(uint32_t* __restrict__ a, uint64_t n,
                                                             const uint64_t* __restrict__ part) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++) {
        v[j] = base + j < n ? a[base + j] : 0u;
        s += v[j];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan256(s, sh, tot) + part[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++) {
        if (base + j < n) a[base + j] = (uint32_t)run;
        run += v[j];
    }
}

hipError_t launch_scan_u32(uint32_t* a, uint64_t n, uint64_t* scratch, uint64_t scratch_n, hipStream_t s) {
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (!nb) return hipSuccess;
    if (scratch_n < nb + 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(scan_u32_partials_kernel, dim3((unsigned)nb), dim3(256), 0, s, a, n, scratch);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, scratch, nb, scratch + nb);
    hipLaunchKernelGGL(scan_u32_apply_kernel, dim3((unsigned)nb), dim3(256), 0, s, a, n, scratch);
    return hipGetLastError();
}

uint64_t scan_u32_scratch_elems(uint64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 2; }

uint64_t radix_counts_elems(uint64_t n) { return 256ull * ((n + RS_TILE - 1) / RS_TILE); }

uint64_t radix_scratch_elems(uint64_t n) {
    return (radix_counts_elems(n) + SCAN_TILE - 1) / SCAN_TILE + 2;
}

hipError_t launch_radix_sort(uint64_t* a, uint64_t* b, uint64_t n, int key_bits, uint32_t* counts,
                             uint64_t* scratch, uint64_t scratch_n, uint64_t** sorted,
                             hipStream_t s) {
    *sorted = a;
    if (n == 0) return hipSuccess;
    if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t n_tiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    uint64_t* src = a;
    uint64_t* dst = b;
    for (int lo = 0; lo < key_bits; lo += 8) {
        const int shift = 32 + lo;
        hipLaunchKernelGGL(rs_hist_kernel, dim3(n_tiles), dim3(256), 0, s, src, (uint32_t)n, shift,
                           counts, n_tiles);
        hipError_t e = launch_scan_u32(counts, 256ull * n_tiles, scratch, scratch_n, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(rs_scatter_kernel, dim3(n_tiles), dim3(256), 0, s, src, dst, (uint32_t)n,
                           shift, counts, n_tiles);
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    *sorted = src;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// runs: after the sort every key is one contiguous run of records.
//   run length = list length (binning.c:1094-1100 counts the list);
//   prune keeps runs longer than the cutoff (binning.c:1102);
//   survivors become CSR entries in slot order (= hash order, like the
//   reference's bucket order, not part of the contract).
// ---------------------------------------------------------------------------
DEV uint32_t slot_of(uint64_t rec) { return (uint32_t)(rec >> 32); }

DEV uint32_t is_head(const uint64_t* __restrict__ S, uint64_t k, int sh = 32) {
    return (k == 0 || (S[k] >> sh) != (S[k - 1] >> sh)) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void heads_partials_kernel(const uint64_t* __restrict__ S, uint64_t n,
                                                             uint64_t* __restrict__ part, int key_sh) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t c = 0;
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t k = base + (uint64_t)j * 256 + threadIdx.x;
        if (k < n) c += is_head(S, k, key_sh);
    }
    c = block_sum256(c, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = c;
}

__global__ __launch_bounds__(256) void heads_write_kernel(const uint64_t* __restrict__ S, uint64_t n,
                                                          const uint64_t* __restrict__ part,
                                                          uint32_t* __restrict__ starts,
                                                          uint64_t max_runs, int key_sh) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t run = part[blockIdx.x];
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t k = base + (uint64_t)j * 256 + threadIdx.x;
        const uint32_t h = k < n ? is_head(S, k, key_sh) : 0u;
        uint64_t tot;
        const uint64_t ex = block_excl_scan256((uint64_t)h, sh, tot);
        if (h && run + ex < max_runs) starts[run + ex] = (uint32_t)k;
        run += tot;
    }
}

__global__ void runs_total_kernel(const uint64_t* __restrict__ tot_runs, uint64_t n,
                                  uint32_t* __restrict__ starts, uint64_t* __restrict__ totals,
                                  uint64_t max_runs) {
    uint64_t D = *tot_runs;
    totals[3] = 0;
    if (D > max_runs) {  // cannot happen (runs == distinct keys); never write out of bounds
        totals[3] = D;
        D = max_runs;
    }
    starts[D] = (uint32_t)n;
    totals[2] = D;
}

// per run: kept flag / kept length partials
__global__ __launch_bounds__(256) void runs_partials_kernel(const uint32_t* __restrict__ starts,
                                                            const uint64_t* __restrict__ totals,
                                                            uint32_t keep_gt, uint64_t* __restrict__ part,
                                                            uint64_t nb) {
    __shared__ uint64_t sh[4];
    const uint64_t D = totals[2];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t nk = 0, ni = 0;
    if (base < D) {
        for (int j = 0; j < SCAN_ITEMS; j++) {
            const uint64_t r = base + (uint64_t)j * 256 + threadIdx.x;
            if (r < D) {
                const uint32_t len = starts[r + 1] - starts[r];
                if (len > keep_gt) {
                    nk++;
                    ni += len;
                }
            }
        }
    }
    nk = block_sum256(nk, sh);
    ni = block_sum256(ni, sh);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = nk;
        part[nb + blockIdx.x] = ni;
    }
}

// per 256-run round: prune, write CSR entries, then the block copies the
// round's records (a contiguous span of S) into the id array -- records are
// already in descending call order inside each run (see scan_insert)
__global__ __launch_bounds__(256) void runs_write_kernel(
    const uint64_t* __restrict__ S, const uint32_t* __restrict__ starts,
    const uint64_t* __restrict__ totals, uint32_t keep_gt, const uint64_t* __restrict__ part,
    uint64_t nb, const uint64_t* __restrict__ table, int SW, const int32_t* __restrict__ read_ids,
    uint32_t id_off, int32_t* __restrict__ ids_out, uint32_t* __restrict__ e_mmer, uint64_t* __restrict__ e_hi,
    uint64_t* __restrict__ e_lo, uint32_t* __restrict__ e_cnt, uint64_t* __restrict__ e_off,
    const uint64_t* __restrict__ first, uint64_t* __restrict__ e_first) {
    __shared__ uint64_t sh[4];
    __shared__ uint32_t rs[257];   // run starts of the round (+ end)
    __shared__ uint32_t ro[256];   // id offset of each run, NONE if pruned
    __shared__ uint8_t rofk[RUN_SPAN];  // run (within the round) of each record of the span
    const uint64_t D = totals[2];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    if (base >= D) return;  // uniform per block
    uint64_t ent = part[blockIdx.x];
    uint64_t ids = part[nb + blockIdx.x];
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t r0 = base + (uint64_t)j * 256;
        if (r0 >= D) break;  // uniform
        const uint64_t r = r0 + threadIdx.x;
        uint32_t len = 0, kept = 0, st = 0;
        if (r < D) {
            st = starts[r];
            len = starts[r + 1] - st;
            kept = len > keep_gt ? 1u : 0u;
        }
        uint64_t tk, ti;
        const uint64_t pk = block_excl_scan256((uint64_t)kept, sh, tk);
        const uint64_t pi = block_excl_scan256((uint64_t)(kept ? len : 0u), sh, ti);
        const uint32_t nr = (uint32_t)min((uint64_t)256, D - r0);
        if (r < D) {
            rs[threadIdx.x] = st;
            ro[threadIdx.x] = kept ? (uint32_t)(ids + pi) : NONE;
            if (threadIdx.x == nr - 1) rs[nr] = st + len;
            if (kept) {
                const uint64_t e = ent + pk;
                const uint32_t slot = slot_of(S[st]);
                const uint64_t* s = table + (uint64_t)slot * SW;
                const uint64_t tc = s[SW == 2 ? 1 : 2];
                e_mmer[e] = (uint32_t)tc - 1u;
                if (SW == 2) {
                    e_hi[e] = 0;
                    e_lo[e] = s[0] - 1ull;
                } else {
                    const uint64_t a = s[0] - 1ull;
                    const uint64_t b = s[1] & ~PUB;
                    e_hi[e] = a >> 1;
                    e_lo[e] = (a << 63) | b;
                }
                e_cnt[e] = len;
                e_off[e] = ids + pi;
                if (first) e_first[e] = first[slot];
            }
        }
        __syncthreads();
        // copy the round's records: [rs[0], rs[nr]) -- coalesced reads/writes
        const uint32_t k_lo = rs[0], k_hi = rs[nr];
        const bool filled = k_hi - k_lo <= (uint32_t)RUN_SPAN;  // uniform
        if (filled && r < D)
            for (uint32_t k = st; k < st + len; k++) rofk[k - k_lo] = (uint8_t)threadIdx.x;
        __syncthreads();
        for (uint32_t k = k_lo + threadIdx.x; k < k_hi; k += 256) {
            uint32_t lo = 0, hi = nr;  // last run with rs[run] <= k
            if (filled) {
                lo = rofk[k - k_lo];
            } else {
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (rs[mid] <= k) lo = mid; else hi = mid;
                }
            }
            const uint32_t off = ro[lo];
            if (off != NONE) {
                const uint32_t o = (uint32_t)S[k];
                ids_out[off + (k - rs[lo])] = read_ids ? read_ids[o] : (int32_t)(o + id_off);
            }
        }
        __syncthreads();
        ent += tk;
        ids += ti;
    }
}

__global__ void entries_total_kernel(const uint64_t* __restrict__ tk, const uint64_t* __restrict__ ti,
                                     uint64_t* __restrict__ e_off, uint64_t* __restrict__ totals) {
    totals[0] = *tk;
    totals[1] = *ti;
    e_off[*tk] = *ti;
}

// run starts of a sorted record array (key = bits 32..): starts[0..D], D in d_totals[2]
hipError_t launch_heads(const uint64_t* S, uint64_t n, uint32_t* starts, uint64_t max_runs,
                        uint64_t* scratch, uint64_t scratch_n, uint64_t* d_totals, hipStream_t s,
                        int key_shift) {
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (scratch_n < nb + 1) return hipErrorInvalidValue;
    if (n == 0) return hipMemsetAsync(d_totals, 0, 4 * sizeof(uint64_t), s);
    hipLaunchKernelGGL(heads_partials_kernel, dim3((unsigned)nb), dim3(256), 0, s, S, n, scratch, key_shift);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, scratch, nb, scratch + nb);
    hipLaunchKernelGGL(heads_write_kernel, dim3((unsigned)nb), dim3(256), 0, s, S, n, scratch, starts,
                       max_runs, key_shift);
    hipLaunchKernelGGL(runs_total_kernel, dim3(1), dim3(1), 0, s, scratch + nb, n, starts, d_totals,
                       max_runs);
    return hipGetLastError();
}

hipError_t launch_runs(const uint64_t* S, uint64_t n, const uint64_t* table, int KW,
                       uint32_t keep_gt, uint32_t* starts, const int32_t* read_ids,
                       uint32_t id_off, int32_t* ids_out, uint64_t max_runs, uint32_t* e_mmer, uint64_t* e_hi, uint64_t* e_lo, uint32_t* e_cnt,
                       uint64_t* e_off, const uint64_t* first, uint64_t* e_first,
                       uint64_t* scratch, uint64_t scratch_n, uint64_t* d_totals, hipStream_t s) {
    const int SW = KW == 1 ? 2 : 4;
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    const uint64_t nbr = (max_runs + SCAN_TILE - 1) / SCAN_TILE;
    if (scratch_n < std::max(nb + 1, 2 * nbr + 2)) return hipErrorInvalidValue;
    if (n == 0) {  // (totals[3], the run-overflow word, too: the host checks it)
        hipError_t e = hipMemsetAsync(d_totals, 0, 4 * sizeof(uint64_t), s);
        if (e == hipSuccess) e = hipMemsetAsync(e_off, 0, sizeof(uint64_t), s);
        return e;
    }
    hipError_t he = launch_heads(S, n, starts, max_runs, scratch, scratch_n, d_totals, s);
    if (he != hipSuccess) return he;
    // runs -> prune -> entries (grid sized for the max possible run count;
    // blocks past the real count exit)
    hipLaunchKernelGGL(runs_partials_kernel, dim3((unsigned)nbr), dim3(256), 0, s, starts, d_totals,
                       keep_gt, scratch, nbr);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, scratch, nbr, scratch + 2 * nbr);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, scratch + nbr, nbr,
                       scratch + 2 * nbr + 1);
    hipLaunchKernelGGL(runs_write_kernel, dim3((unsigned)nbr), dim3(256), 0, s, S, starts, d_totals,
                       keep_gt, scratch, nbr, table, SW, read_ids, id_off, ids_out, e_mmer, e_hi, e_lo, e_cnt, e_off,
                       first, e_first);
    hipLaunchKernelGGL(entries_total_kernel, dim3(1), dim3(1), 0, s, scratch + 2 * nbr,
                       scratch + 2 * nbr + 1, e_off, d_totals);
    return hipGetLastError();
}

uint64_t runs_scratch_elems(uint64_t n, uint64_t max_runs) {
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    const uint64_t nbr = (max_runs + SCAN_TILE - 1) / SCAN_TILE;
    return std::max(nb + 1, 2 * nbr + 2);
}

__global__ void fill_ids_kernel(int32_t* d, uint64_t n, int32_t first) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        d[i] = first + (int32_t)i;
}

hipError_t launch_fill_ids(int32_t* d_ids, uint64_t n, int32_t first, hipStream_t s) {
    if (!n) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(fill_ids_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_ids, n, first);
    return hipGetLastError();
}

}  // namespace kb
