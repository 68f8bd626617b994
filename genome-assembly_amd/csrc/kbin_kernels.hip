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
//   compact       prune (count > cutoff) + stream compaction into a CSR.
//   place         read-id placement per surviving key (atomic cursor).
//   sort          per key, ids in reverse call order (descending ordinal),
//                 mapped to the caller's read ids.
//
// All integer work: no MFMA.  Roofline = HBM.
#include "kbin_internal.h"

namespace kb {

#define DEV __device__ __forceinline__

DEV uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

DEV int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

DEV uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

template <typename T>
DEV T wave_incl_scan(T v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// exclusive scan over a 256-thread block; sh must hold 4 elements
template <typename T>
DEV T block_excl_scan256(T v, T* sh, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T inc = wave_incl_scan(v, lane);
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    T wp = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        T x = sh[w];
        if (w < wid) wp += x;
        tot += x;
    }
    __syncthreads();
    total = tot;
    return wp + inc - v;
}

template <typename T>
DEV T block_sum256(T v, T* sh) {
    T tot;
    (void)block_excl_scan256(v, sh, tot);
    return tot;
}

// 64-bit window of the packed read starting at base p (first base in the MSBs)
DEV uint64_t window64(const uint64_t* sw, int p) {
    const int w = p >> 5, sh = (p & 31) << 1;
    uint64_t x = sw[w];
    if (sh) x = (x << sh) | (sw[w + 1] >> (64 - sh));
    return x;
}

DEV uint64_t atomic_load_u64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV uint32_t atomic_load_u32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

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
                                                       uint64_t seed) {
    const uint64_t total = n_reads * (uint64_t)RW;
    const uint64_t s_genome = mix64(seed ^ 0x1111111111111111ull);
    const uint64_t s_start = mix64(seed ^ 0x2222222222222222ull);
    const uint64_t s_err = mix64(seed ^ 0x3333333333333333ull);
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = g / RW;
        const int w = (int)(g - r * RW);
        const uint64_t start = rng(s_start, r) % (G - L + 1);
        uint64_t word = 0;
        for (int j = 0; j < 32; j++) {
            const uint32_t b = (uint32_t)w * 32u + (uint32_t)j;
            if (b >= L) break;
            const uint64_t pos = start + b;
            // 32 genome bases per RNG draw
            uint32_t v = (uint32_t)(rng(s_genome, pos >> 5) >> (2 * (pos & 31))) & 3u;
            if (err_ppm) {
                const uint64_t u = rng(s_err, r * (uint64_t)L + b);
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
                           uint64_t genome_len, uint32_t err_ppm, uint64_t seed, hipStream_t s) {
    const int RW = (int)((read_len + 31) / 32);
    const uint64_t total = n_reads * (uint64_t)RW;
    if (!total) return hipSuccess;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(generate_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_words, d_lens,
                       n_reads, read_len, RW, genome_len, err_ppm, seed);
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

// Insert one occurrence; returns the slot index (NONE on probe-limit failure).
// Protocol (DESIGN.md "Table protocol"): claim by 64-bit CAS of the claim word
// on an empty slot; the winner then publishes the other words with atomic
// stores, each carrying its own marker.  A reader that finds an unpublished
// word re-reads it with an atomic RMW (coherent across XCD L2s) and, if still
// unpublished, retries the same slot on its next loop trip -- no lane ever
// waits inside a branch another lane of its wave must leave.
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
        if (KW == 2) w1 = atomic_load_u64(s + 1);
        if (w0 == 0) {
            const uint64_t old = atomicCAS((unsigned long long*)s, 0ull, (unsigned long long)k.a);
            if (old == 0) {
                if constexpr (KW == 2) __hip_atomic_store(s + 1, k.b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(tagp, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicAdd(tagp + 1, 1u);
                is_new = true;
                return (uint32_t)idx;
            }
            w0 = old;
            t = 0;   // anything loaded before the CAS may predate the claim
            w1 = 0;
        }
        if (w0 == k.a) {
            bool pending = false;
            if (KW == 2) {
                if (!(w1 & PUB)) w1 = atomicOr((unsigned long long*)(s + 1), 0ull);
                if (!(w1 & PUB)) pending = true;
            }
            if (t == 0) t = atomicOr(tagp, 0u);
            if (t == 0) pending = true;
            if (pending) continue;  // claimed but not yet published: re-read next trip
            if (t == tag && (KW == 1 || w1 == k.b)) {
                atomicAdd(tagp + 1, 1u);
                return (uint32_t)idx;
            }
        }
        idx = (idx + 1) & mask;
        if (++probes > max_probe) return NONE;
    }
}

template <int KW>
__global__ __launch_bounds__(256) void scan_insert_kernel(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int RW = A.RW, K = A.K, M = A.M;
    const int W = K - M + 1;                          // mmer starts per k-mer window
    const uint32_t maskM = (1u << (2 * M)) - 1u;
    const uint32_t halfM = 1u << (2 * M - 1);         // s < halfM <=> first base T/G <=> complement wins
    uint64_t* sw = smem + wid * (RW + 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    uint32_t local_new = 0;
    uint32_t st = 0;

    for (uint64_t r = (uint64_t)blockIdx.x * 4 + wid; r < A.n_reads; r += nwaves) {
        const int L = rfl((int)A.lens[r]);
        const int nK = L - K + 1;
        if (nK <= 0) continue;
        // stage the read tile in LDS (one extra zero word for window reads)
        wave_sync();
        for (int w = lane; w < RW; w += 64) sw[w] = A.words[r * RW + w];
        if (lane == 0) sw[RW] = 0;
        wave_sync();
        const uint64_t obase = A.kmer_base[r];

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
                bool is_new;
                const uint32_t slot = table_insert<KW>(A.table, A.mask, key, mm + 1u, A.max_probe, is_new);
                if (slot == NONE) st |= ST_PROBE_LIMIT;
                local_new += is_new ? 1u : 0u;
                A.occ_slot[obase + i] = slot;
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
// compact: prune (binning.c:1094-1102: keep iff count > cutoff) + CSR build
// ---------------------------------------------------------------------------
// scratch layout: [0, nb) kept-count partials, [nb, 2nb) id-count partials
DEV void slot_info(const uint64_t* __restrict__ table, int SW, uint64_t slot, uint32_t keep_gt,
                   uint32_t& kept, uint32_t& cnt) {
    const uint64_t tc = table[slot * SW + (SW == 2 ? 1 : 2)];
    const uint32_t tag = (uint32_t)tc;
    cnt = (uint32_t)(tc >> 32);
    kept = (tag != 0 && cnt > keep_gt) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void compact_partials_kernel(const uint64_t* __restrict__ table,
                                                               uint64_t slots, int SW,
                                                               uint32_t keep_gt,
                                                               uint64_t* __restrict__ part,
                                                               uint64_t nb) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t nk = 0, ni = 0;
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t slot = base + (uint64_t)j * 256 + threadIdx.x;  // coalesced
        if (slot < slots) {
            uint32_t kept, cnt;
            slot_info(table, SW, slot, keep_gt, kept, cnt);
            nk += kept;
            ni += kept ? cnt : 0;
        }
    }
    nk = block_sum256(nk, sh);
    ni = block_sum256(ni, sh);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = nk;
        part[nb + blockIdx.x] = ni;
    }
}

__global__ __launch_bounds__(256) void compact_write_kernel(
    const uint64_t* __restrict__ table, uint64_t slots, int SW, int K, uint32_t keep_gt,
    const uint64_t* __restrict__ part, uint64_t nb, uint32_t* __restrict__ slot_entry,
    uint32_t* __restrict__ e_mmer, uint64_t* __restrict__ e_hi, uint64_t* __restrict__ e_lo,
    uint32_t* __restrict__ e_cnt, uint64_t* __restrict__ e_off) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t ent = part[blockIdx.x];
    uint64_t ids = part[nb + blockIdx.x];
    // process the tile in SCAN_ITEMS coalesced rounds of 256 slots
    for (int j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t slot = base + (uint64_t)j * 256 + threadIdx.x;
        uint32_t kept = 0, cnt = 0;
        if (slot < slots) slot_info(table, SW, slot, keep_gt, kept, cnt);
        uint64_t tk, ti;
        const uint64_t pk = block_excl_scan256((uint64_t)kept, sh, tk);
        const uint64_t pi = block_excl_scan256((uint64_t)(kept ? cnt : 0), sh, ti);
        if (slot < slots) {
            if (kept) {
                const uint64_t e = ent + pk;
                const uint64_t* s = table + slot * SW;
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
                e_cnt[e] = cnt;
                e_off[e] = ids + pi;
                slot_entry[slot] = (uint32_t)e;
            } else {
                slot_entry[slot] = NONE;
            }
        }
        ent += tk;
        ids += ti;
    }
    (void)K;
}

uint64_t compact_scratch_elems(uint64_t slots) {
    return 2 * ((slots + SCAN_TILE - 1) / SCAN_TILE) + 2;
}

__global__ void compact_totals_kernel(const uint64_t* __restrict__ part, uint64_t nb,
                                      const uint64_t* __restrict__ tot_k,
                                      const uint64_t* __restrict__ tot_i,
                                      uint64_t* __restrict__ e_off, uint64_t* __restrict__ totals) {
    const uint64_t nk = *tot_k, ni = *tot_i;
    totals[0] = nk;
    totals[1] = ni;
    e_off[nk] = ni;
    (void)part;
    (void)nb;
}

hipError_t launch_compact(const uint64_t* table, uint64_t slots, int KW, int K, uint32_t keep_gt,
                          uint32_t* slot_entry, uint32_t* e_mmer, uint64_t* e_hi, uint64_t* e_lo,
                          uint32_t* e_cnt, uint64_t* e_off, uint64_t* scratch, uint64_t scratch_n,
                          uint64_t* d_totals, hipStream_t s) {
    const int SW = KW == 1 ? 2 : 4;
    const uint64_t nb = (slots + SCAN_TILE - 1) / SCAN_TILE;
    if (scratch_n < 2 * nb + 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(compact_partials_kernel, dim3((unsigned)nb), dim3(256), 0, s, table, slots,
                       SW, keep_gt, scratch, nb);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, scratch, nb,
                       scratch + 2 * nb);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, scratch + nb, nb,
                       scratch + 2 * nb + 1);
    hipLaunchKernelGGL(compact_write_kernel, dim3((unsigned)nb), dim3(256), 0, s, table, slots, SW,
                       K, keep_gt, scratch, nb, slot_entry, e_mmer, e_hi, e_lo, e_cnt, e_off);
    hipLaunchKernelGGL(compact_totals_kernel, dim3(1), dim3(1), 0, s, scratch, nb,
                       scratch + 2 * nb, scratch + 2 * nb + 1, e_off, d_totals);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// place: every occurrence of a surviving key drops its read ordinal into the
// key's id range (binning.c:1056-1068 builds the same multiset by prepend)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void place_kernel(PlaceArgs A) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t k0 = wave * 64; k0 < A.n_occ; k0 += nwaves * 64) {
        // read of occurrence k0: last r with kmer_base[r] <= k0 (wave-uniform search)
        uint64_t lo = 0, hi = A.n_reads;  // answer in [lo, hi)
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (A.kmer_base[mid] <= k0) lo = mid; else hi = mid;
        }
        const uint64_t k = k0 + lane;
        if (k < A.n_occ) {
            uint64_t r = lo;
            while (A.kmer_base[r + 1] <= k) r++;
            const uint32_t slot = A.occ_slot[k];
            const uint32_t e = slot == NONE ? NONE : A.slot_entry[slot];
            if (e != NONE) {
                const uint32_t pos = atomicAdd(&A.cursor[e], 1u);
                A.ids_ord[A.e_off[e] + pos] = A.ord_base + (uint32_t)r;
            }
        }
    }
}

hipError_t launch_place(const PlaceArgs& a, hipStream_t s) {
    if (!a.n_occ) return hipSuccess;
    uint64_t blocks = (a.n_occ + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(place_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// sort: ids of each key in descending call ordinal (= prepend order,
// binning.c:1061-1068), then ordinal -> caller read id
// ---------------------------------------------------------------------------
constexpr int SMALL_N = 32;
constexpr int MED_N = 4096;  // block LDS bitonic (16 KB)

// lists: [0, n_entries) medium entry ids, [n_entries, 2 n_entries) large;
// list_counts: [0] medium count, [1] large count, [2] max large size
__global__ __launch_bounds__(256) void sort_small_kernel(const uint64_t* __restrict__ e_off,
                                                         const uint32_t* __restrict__ e_cnt,
                                                         uint64_t n_entries,
                                                         const uint32_t* __restrict__ ids_ord,
                                                         const int32_t* __restrict__ read_ids,
                                                         int32_t* __restrict__ ids_out,
                                                         uint32_t* __restrict__ lists,
                                                         uint32_t* __restrict__ list_counts) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n_entries;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t n = e_cnt[e];
        const uint64_t o = e_off[e];
        if (n > SMALL_N) {
            if (n > MED_N) {
                const uint32_t at = atomicAdd(&list_counts[1], 1u);
                lists[n_entries + at] = (uint32_t)e;
                atomicMax(&list_counts[2], n);
            } else {
                const uint32_t at = atomicAdd(&list_counts[0], 1u);
                lists[at] = (uint32_t)e;
            }
            continue;
        }
        uint32_t v[SMALL_N];
#pragma unroll
        for (int j = 0; j < SMALL_N; j++) v[j] = (uint32_t)j < n ? ids_ord[o + j] + 1u : 0u;
        // bitonic network, descending
#pragma unroll
        for (int k = 2; k <= SMALL_N; k <<= 1) {
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
                for (int i = 0; i < SMALL_N; i++) {
                    const int l = i ^ j;
                    if (l > i) {
                        const uint32_t x = v[i], y = v[l];
                        const bool desc = (i & k) == 0;
                        const bool sw = desc ? (x < y) : (x > y);
                        v[i] = sw ? y : x;
                        v[l] = sw ? x : y;
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < SMALL_N; j++)
            if ((uint32_t)j < n) ids_out[o + j] = read_ids[v[j] - 1u];
    }
}

// one block per medium entry (grid-stride over the list), LDS bitonic
__global__ __launch_bounds__(256) void sort_medium_kernel(const uint64_t* __restrict__ e_off,
                                                          const uint32_t* __restrict__ e_cnt,
                                                          const uint32_t* __restrict__ ids_ord,
                                                          const int32_t* __restrict__ read_ids,
                                                          int32_t* __restrict__ ids_out,
                                                          const uint32_t* __restrict__ lists,
                                                          const uint32_t* __restrict__ list_counts) {
    __shared__ uint32_t buf[MED_N];
    const uint32_t nmed = list_counts[0];
    for (uint32_t li = blockIdx.x; li < nmed; li += gridDim.x) {
        const uint32_t e = lists[li];
        const uint32_t n = e_cnt[e];
        const uint64_t o = e_off[e];
        uint32_t P = 64;
        while (P < n) P <<= 1;
        for (uint32_t j = threadIdx.x; j < P; j += blockDim.x)
            buf[j] = j < n ? ids_ord[o + j] + 1u : 0u;
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const uint32_t x = buf[i], y = buf[l];
                        const bool desc = (i & k) == 0;
                        if (desc ? (x < y) : (x > y)) {
                            buf[i] = y;
                            buf[l] = x;
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) ids_out[o + j] = read_ids[buf[j] - 1u];
        __syncthreads();
    }
}

// large lists (> MED_N): sort MED_N chunks in LDS into tmp (descending), then
// merge passes between tmp and ids_ord, one launch per pass.
__global__ __launch_bounds__(256) void sort_large_chunks_kernel(const uint64_t* __restrict__ e_off,
                                                                const uint32_t* __restrict__ e_cnt,
                                                                uint64_t n_entries,
                                                                const uint32_t* __restrict__ ids_ord,
                                                                uint32_t* __restrict__ tmp,
                                                                const uint32_t* __restrict__ lists,
                                                                const uint32_t* __restrict__ list_counts) {
    __shared__ uint32_t buf[MED_N];
    const uint32_t nl = list_counts[1];
    for (uint32_t li = 0; li < nl; li++) {
        const uint32_t e = lists[n_entries + li];
        const uint32_t n = e_cnt[e];
        const uint64_t o = e_off[e];
        const uint32_t nchunks = (n + MED_N - 1) / MED_N;
        for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
            const uint32_t c0 = c * MED_N;
            const uint32_t cn = min((uint32_t)MED_N, n - c0);
            for (uint32_t j = threadIdx.x; j < MED_N; j += blockDim.x)
                buf[j] = j < cn ? ids_ord[o + c0 + j] + 1u : 0u;
            __syncthreads();
            for (uint32_t k = 2; k <= (uint32_t)MED_N; k <<= 1) {
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    for (uint32_t i = threadIdx.x; i < (uint32_t)MED_N; i += blockDim.x) {
                        const uint32_t l = i ^ j;
                        if (l > i) {
                            const uint32_t x = buf[i], y = buf[l];
                            const bool desc = (i & k) == 0;
                            if (desc ? (x < y) : (x > y)) {
                                buf[i] = y;
                                buf[l] = x;
                            }
                        }
                    }
                    __syncthreads();
                }
            }
            for (uint32_t j = threadIdx.x; j < cn; j += blockDim.x) tmp[o + c0 + j] = buf[j];
            __syncthreads();
        }
    }
}

// merge runs of width w (descending, values are ordinal+1) from src into dst
__global__ __launch_bounds__(256) void merge_pass_kernel(const uint64_t* __restrict__ e_off,
                                                         const uint32_t* __restrict__ e_cnt,
                                                         uint64_t n_entries,
                                                         const uint32_t* __restrict__ src,
                                                         uint32_t* __restrict__ dst, uint32_t w,
                                                         const uint32_t* __restrict__ lists,
                                                         const uint32_t* __restrict__ list_counts) {
    const uint32_t nl = list_counts[1];
    for (uint32_t li = 0; li < nl; li++) {
        const uint32_t e = lists[n_entries + li];
        const uint32_t n = e_cnt[e];
        const uint64_t o = e_off[e];
        for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n;
             t += (uint64_t)gridDim.x * blockDim.x) {
            const uint32_t pair0 = (uint32_t)(t / (2ull * w)) * 2u * w;
            const uint32_t a0 = pair0, an = min(w, n - a0);
            const uint32_t b0 = a0 + an, bn = b0 < n ? min(w, n - b0) : 0u;
            const uint32_t d = (uint32_t)t - pair0;  // output rank within the pair
            // co-rank: find i in A, j = d - i in B with stable descending merge
            uint32_t lo = d > bn ? d - bn : 0u, hi = min(d, an);
            while (lo < hi) {
                const uint32_t i = (lo + hi) >> 1;
                const uint32_t j = d - i - 1;
                // take more from A if A[i] >= B[j]
                if (src[o + a0 + i] >= src[o + b0 + j]) lo = i + 1; else hi = i;
            }
            const uint32_t i = lo, j = d - lo;
            uint32_t v;
            if (i < an && (j >= bn || src[o + a0 + i] >= src[o + b0 + j])) v = src[o + a0 + i];
            else v = src[o + b0 + j];
            dst[o + t] = v;
        }
    }
}

__global__ __launch_bounds__(256) void large_finish_kernel(const uint64_t* __restrict__ e_off,
                                                           const uint32_t* __restrict__ e_cnt,
                                                           uint64_t n_entries,
                                                           const uint32_t* __restrict__ src,
                                                           const int32_t* __restrict__ read_ids,
                                                           int32_t* __restrict__ ids_out,
                                                           const uint32_t* __restrict__ lists,
                                                           const uint32_t* __restrict__ list_counts) {
    const uint32_t nl = list_counts[1];
    for (uint32_t li = 0; li < nl; li++) {
        const uint32_t e = lists[n_entries + li];
        const uint32_t n = e_cnt[e];
        const uint64_t o = e_off[e];
        for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n;
             t += (uint64_t)gridDim.x * blockDim.x)
            ids_out[o + t] = read_ids[src[o + t] - 1u];
    }
}

hipError_t launch_sort(const uint64_t* e_off, const uint32_t* e_cnt, uint64_t n_entries,
                       uint32_t* ids_ord, uint32_t* ids_tmp, const int32_t* read_ids,
                       int32_t* ids_out, uint32_t* lists, uint32_t* list_counts, hipStream_t s) {
    if (!n_entries) return hipSuccess;
    hipError_t err = hipMemsetAsync(list_counts, 0, 4 * sizeof(uint32_t), s);
    if (err != hipSuccess) return err;
    uint64_t blocks = (n_entries + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(sort_small_kernel, dim3((unsigned)blocks), dim3(256), 0, s, e_off, e_cnt,
                       n_entries, ids_ord, read_ids, ids_out, lists, list_counts);
    hipLaunchKernelGGL(sort_medium_kernel, dim3(2048), dim3(256), 0, s, e_off, e_cnt, ids_ord,
                       read_ids, ids_out, lists, list_counts);
    // large lists need the max size on the host to plan merge passes
    uint32_t hc[4];
    err = hipMemcpyAsync(hc, list_counts, sizeof(hc), hipMemcpyDeviceToHost, s);
    if (err != hipSuccess) return err;
    err = hipStreamSynchronize(s);
    if (err != hipSuccess) return err;
    if (hc[1] == 0) return hipGetLastError();
    hipLaunchKernelGGL(sort_large_chunks_kernel, dim3(256), dim3(256), 0, s, e_off, e_cnt, n_entries,
                       ids_ord, ids_tmp, lists, list_counts);
    uint32_t* src = ids_tmp;
    uint32_t* dst = ids_ord;
    for (uint32_t w = MED_N; w < hc[2]; w <<= 1) {
        hipLaunchKernelGGL(merge_pass_kernel, dim3(1024), dim3(256), 0, s, e_off, e_cnt, n_entries,
                           src, dst, w, lists, list_counts);
        uint32_t* t = src;
        src = dst;
        dst = t;
    }
    hipLaunchKernelGGL(large_finish_kernel, dim3(1024), dim3(256), 0, s, e_off, e_cnt, n_entries,
                       src, read_ids, ids_out, lists, list_counts);
    return hipGetLastError();
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
