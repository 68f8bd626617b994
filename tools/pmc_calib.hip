// pmc_calib.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950
// for the access widths the binned engine uses (not part of the product).
// MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of a 16-B/lane coalesced
// streaming read; other widths are uncalibrated -- this measures them on known
// byte counts, over 2 GiB buffers (past the 256 MiB Infinity Cache).
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -- tools/pmc_calib ; rocprofv3 --pmc WRITE_SIZE -- tools/pmc_calib
// Each kernel moves exactly BYTES bytes (printed), so counter / BYTES is the factor.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr uint64_t BYTES = 2ull << 30;

// coalesced 8 B per lane (bin_kernel: record headers/spans, stage entries)
__global__ void read8(const uint64_t* __restrict__ a, uint64_t n, uint64_t* sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        acc += a[i];
    if (acc == 0x12345) sink[0] = acc;
}

// coalesced 16 B per lane (the guide's calibrated case: FETCH_SIZE = 1/2)
__global__ void read16(const uint4* __restrict__ a, uint64_t n, uint64_t* sink) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        acc += a[i].x ^ a[i].w;
    if (acc == 0x12345) sink[0] = acc;
}

// coalesced 8 B per lane stores (stage entries, SoA records)
__global__ void write8(uint64_t* __restrict__ a, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = i;
}

// 4-B stores scattered inside 192 KiB regions, every word written once (the
// bin kernel's sweep 2 placing ordinals inside a bin's id range)
__global__ void scatter4(uint32_t* __restrict__ a, uint64_t n) {
    constexpr uint32_t R = 48 * 1024;  // words per region
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t reg = i / R, k = i % R;
        const uint32_t j = (uint32_t)((k * 40503u) % R);  // 40503 odd and coprime with R: a permutation
        a[reg * R + j] = (uint32_t)i;
    }
}

int main() {
    void* buf = nullptr;
    uint64_t* sink = nullptr;
    CHK(hipMalloc(&buf, BYTES));
    CHK(hipMalloc((void**)&sink, 64));
    CHK(hipMemset(buf, 1, BYTES));
    const dim3 g(8192), b(256);
    hipLaunchKernelGGL(read8, g, b, 0, 0, (const uint64_t*)buf, BYTES / 8, sink);
    hipLaunchKernelGGL(read16, g, b, 0, 0, (const uint4*)buf, BYTES / 16, sink);
    hipLaunchKernelGGL(write8, g, b, 0, 0, (uint64_t*)buf, BYTES / 8);
    const uint64_t nsc = BYTES / 4 / (48 * 1024) * (48 * 1024);  // whole regions only
    hipLaunchKernelGGL(scatter4, g, b, 0, 0, (uint32_t*)buf, nsc);
    CHK(hipDeviceSynchronize());
    printf("bytes: read8 read16 write8 %llu, scatter4 %llu\n", (unsigned long long)BYTES,
           (unsigned long long)(nsc * 4));
    return 0;
}
