// ubench.hip -- microbenchmarks behind DESIGN.md's table-placement decisions
// (not part of the product).  Random 16-B loads and random u32 atomics over
// footprints from L2-size to HBM-size, agent vs workgroup scope.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench.hip -o tools/ubench && tools/ubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull; x ^= x >> 31;
    return x;
}

// each thread: `iters` random 16-B loads within [0, mask] (in 16-B units)
__global__ void rand_load16(const uint4* __restrict__ t, uint64_t mask, int iters, uint64_t* sink) {
    uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t acc = 0;
    for (int i = 0; i < iters; i++) {
        uint4 v = t[mix(gid * 1000003ull + i) & mask];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345) sink[0] = acc;
}

// region-local: block b only touches region b (size mask+1 units), like a bin owned by a workgroup
__global__ void region_load16(const uint4* __restrict__ t, uint64_t rmask, int iters, uint64_t* sink) {
    uint64_t base = (uint64_t)blockIdx.x * (rmask + 1);
    uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t acc = 0;
    for (int i = 0; i < iters; i++) {
        uint4 v = t[base + (mix(gid * 1000003ull + i) & rmask)];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345) sink[0] = acc;
}

template <int SCOPE>
__global__ void rand_atomic(uint32_t* __restrict__ t, uint64_t mask, uint64_t rsize, int iters) {
    uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t base = rsize ? (uint64_t)blockIdx.x * rsize : 0;
    for (int i = 0; i < iters; i++) {
        uint64_t a = base + (mix(gid * 1000003ull + i) & mask);
        if (SCOPE == 0) __hip_atomic_fetch_add(&t[a], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_add(&t[a], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

template <int SCOPE>
__global__ void rand_atomic_ret(uint32_t* __restrict__ t, uint64_t mask, uint64_t rsize, int iters, uint64_t* sink) {
    uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t base = rsize ? (uint64_t)blockIdx.x * rsize : 0;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        uint64_t a = base + (mix(gid * 1000003ull + i) & mask);
        if (SCOPE == 0) acc += __hip_atomic_fetch_add(&t[a], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else acc += __hip_atomic_fetch_add(&t[a], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (acc == 0x12345) sink[0] = acc;
}

__global__ void stream_copy(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

int main() {
    const uint64_t BIG = 1ull << 30;  // 1 GiB
    void *buf, *buf2;
    uint64_t* sink;
    CHK(hipMalloc(&buf, BIG));
    CHK(hipMalloc(&buf2, BIG));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(buf, 1, BIG));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float ms;
    const int blocks = 4096, threads = 256, iters = 64;
    const double nops = (double)blocks * threads * iters;
    // streaming copy reference
    {
        uint64_t n = BIG / 16;
        stream_copy<<<8192, 256>>>((uint4*)buf, (uint4*)buf2, n);
        CHK(hipEventRecord(e0));
        for (int r = 0; r < 5; r++) stream_copy<<<8192, 256>>>((uint4*)buf, (uint4*)buf2, n);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("stream copy 1GiB: %.1f GB/s (read+write)\n", 5 * 2.0 * BIG / (ms * 1e-3) / 1e9);
    }
    for (uint64_t fp : {1ull << 20, 4ull << 20, 32ull << 20, 128ull << 20, 256ull << 20, 512ull << 20, 1ull << 30}) {
        uint64_t mask = fp / 16 - 1;
        rand_load16<<<blocks, threads>>>((uint4*)buf, mask, iters, sink);
        CHK(hipEventRecord(e0));
        rand_load16<<<blocks, threads>>>((uint4*)buf, mask, iters, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("random 16B loads, footprint %7.1f MiB: %6.1f G loads/s\n", fp / 1048576.0, nops / (ms * 1e-3) / 1e9);
    }
    for (uint64_t rs : {16ull << 10, 64ull << 10, 256ull << 10}) {  // bytes per block region
        uint64_t rmask = rs / 16 - 1;
        region_load16<<<blocks, threads>>>((uint4*)buf, rmask, iters, sink);
        CHK(hipEventRecord(e0));
        region_load16<<<blocks, threads>>>((uint4*)buf, rmask, iters, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("region 16B loads, %5.0f KiB per block:          %6.1f G loads/s\n", rs / 1024.0, nops / (ms * 1e-3) / 1e9);
    }
    for (int scope = 0; scope < 2; scope++) {
        for (uint64_t fp : {1ull << 20, 32ull << 20, 256ull << 20, 1ull << 30}) {
            uint64_t mask = fp / 4 - 1;
            if (scope == 0) rand_atomic<0><<<blocks, threads>>>((uint32_t*)buf, mask, 0, iters);
            else rand_atomic<1><<<blocks, threads>>>((uint32_t*)buf, mask, 0, iters);
            CHK(hipEventRecord(e0));
            if (scope == 0) rand_atomic<0><<<blocks, threads>>>((uint32_t*)buf, mask, 0, iters);
            else rand_atomic<1><<<blocks, threads>>>((uint32_t*)buf, mask, 0, iters);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
            printf("random u32 atomic add (no ret) %s, footprint %7.1f MiB: %6.1f G/s\n", scope ? "wg   " : "agent", fp / 1048576.0, nops / (ms * 1e-3) / 1e9);
        }
        for (uint64_t rs : {16ull << 10, 256ull << 10}) {
            uint64_t rmask = rs / 4 - 1;
            if (scope == 0) rand_atomic_ret<0><<<blocks, threads>>>((uint32_t*)buf, rmask, rs / 4, iters, sink);
            else rand_atomic_ret<1><<<blocks, threads>>>((uint32_t*)buf, rmask, rs / 4, iters, sink);
            CHK(hipEventRecord(e0));
            if (scope == 0) rand_atomic_ret<0><<<blocks, threads>>>((uint32_t*)buf, rmask, rs / 4, iters, sink);
            else rand_atomic_ret<1><<<blocks, threads>>>((uint32_t*)buf, rmask, rs / 4, iters, sink);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
            printf("region u32 atomic add (ret)    %s, %5.0f KiB per block:   %6.1f G/s\n", scope ? "wg   " : "agent", rs / 1024.0, nops / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
