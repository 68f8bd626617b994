// kbin_digest.hip -- order-independent digest of a finalized result (CSR).
//
// A result of 10^7 keys and 10^10 ids cannot be
// compared against a host dump, so full-size runs are checked through this
// digest instead: per key a term of (mmer, kmer, count) and per id a term of
// (key, position in the list, id), summed mod 2^64.  Sums do not depend on
// the entry order (hash order, unspecified) but do on every list's order, and
// they add over disjoint results: the passes of kb_set_partition or the ranks
// of a sharded job add up to the single-pass digest.  kbin.result_digest is
// the same function in numpy (tests pin one against the other).
#include <algorithm>

#include "kbin_internal.h"
#include "kbin_device.h"

namespace kb {

DEV uint64_t digest_key(uint32_t mmer, uint64_t hi, uint64_t lo) {
    return mix64(mix64(mix64((uint64_t)mmer) ^ hi) ^ lo);
}

// one wavefront per entry: lanes stride the entry's id list (coalesced)
__global__ __launch_bounds__(256) void digest_kernel(const uint32_t* __restrict__ mmer,
                                                     const uint64_t* __restrict__ hi,
                                                     const uint64_t* __restrict__ lo,
                                                     const uint32_t* __restrict__ cnt,
                                                     const uint64_t* __restrict__ off,
                                                     const int32_t* __restrict__ ids, uint64_t n_entries,
                                                     unsigned long long* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * 4;
    uint64_t dk = 0, dl = 0;
    for (uint64_t e = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); e < n_entries; e += waves) {
        const uint64_t key = digest_key(mmer[e], hi[e], lo[e]);
        const uint32_t n = cnt[e];
        if (lane == 0) dk += mix64(key ^ ((uint64_t)n << 1));
        const uint64_t o = off[e];
        for (uint32_t j = lane; j < n; j += 64)
            dl += mix64(key ^ (((uint64_t)(j + 1) << 32) | (uint32_t)ids[o + j]));
    }
    __shared__ uint64_t sh[4];
    dk = block_sum256(dk, sh);
    __syncthreads();
    dl = block_sum256(dl, sh);
    if (threadIdx.x == 0) {
        atomicAdd(&out[0], (unsigned long long)dk);
        atomicAdd(&out[1], (unsigned long long)dl);
    }
}

hipError_t launch_digest(const uint32_t* mmer, const uint64_t* hi, const uint64_t* lo, const uint32_t* cnt,
                         const uint64_t* off, const int32_t* ids, uint64_t n_entries, unsigned long long* out,
                         hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, 2 * sizeof(unsigned long long), s);
    if (e != hipSuccess || !n_entries) return e;
    const uint64_t blocks = std::min<uint64_t>((n_entries + 3) / 4, 16384);
    hipLaunchKernelGGL(digest_kernel, dim3((unsigned)blocks), dim3(256), 0, s, mmer, hi, lo, cnt, off, ids,
                       n_entries, out);
    return hipGetLastError();
}

}  // namespace kb
