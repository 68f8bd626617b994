// kbin_device.h -- device helpers shared by the kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

DEV uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
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


// 64-bit window of a record's span words (s0..s3 in registers, no scratch)
DEV uint64_t span_window(uint64_t s0, uint64_t s1, uint64_t s2, uint64_t s3, int p) {
    const int w = p >> 5, sh = (p & 31) << 1;
    const uint64_t a = w == 0 ? s0 : w == 1 ? s1 : w == 2 ? s2 : s3;
    const uint64_t b = w == 0 ? s1 : w == 1 ? s2 : w == 2 ? s3 : 0ull;
    return sh ? (a << sh) | (b >> (64 - sh)) : a;
}

}  // namespace kb
