// sortbench.hip -- calibration of the engine's record sort (not product):
// 120M (slot << 32 | ordinal) records, stable sort by bits [32, 56), our
// onesweep (kbin_kernels.hip) vs rocPRIM radix_sort_keys on the same data.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I genome-assembly_amd/csrc tools/sortbench.hip \
//         genome-assembly_amd/lib/obj/kbin_kernels.o -o tools/sortbench
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <cstdio>
#include <vector>

#include "kbin_internal.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void fill(uint64_t* a, uint64_t n, int bits) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 32;
        a[i] = ((x & ((1ull << bits) - 1)) << 32) | (uint32_t)(n - 1 - i);
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 120000000ull;
    const int bits = argc > 2 ? atoi(argv[2]) : 24;
    uint64_t *a, *b, *flags, *c;
    uint32_t* aux;
    CHK(hipMalloc(&a, n * 8));
    CHK(hipMalloc(&b, n * 8));
    CHK(hipMalloc(&c, n * 8));
    CHK(hipMalloc(&flags, kb::onesweep_flag_elems(n) * 8));
    CHK(hipMemset(flags, 0, kb::onesweep_flag_elems(n) * 8));
    CHK(hipMalloc(&aux, 4096 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    fill<<<4096, 256>>>(c, n, bits);
    uint32_t epoch = 0;
    float ms;
    for (int rep = 0; rep < 3; rep++) {
        CHK(hipMemcpy(a, c, n * 8, hipMemcpyDeviceToDevice));
        uint64_t* sorted;
        CHK(hipEventRecord(e0));
        CHK(kb::launch_onesweep(a, b, n, bits, flags, aux, &epoch, &sorted, 0));
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("kbin onesweep: %.3f ms  (%.2f G rec/s, %.0f GB/s per pass incl. hist)\n", ms, n / (ms * 1e-3) / 1e9,
               ((bits + 7) / 8 * 16.0 + 8.0) * n / (ms * 1e-3) / 1e9);
    }
    // rocPRIM
    size_t tmp = 0;
    CHK(rocprim::radix_sort_keys(nullptr, tmp, a, b, n, 32, 32 + bits));
    void* dtmp;
    CHK(hipMalloc(&dtmp, tmp));
    for (int rep = 0; rep < 3; rep++) {
        CHK(hipMemcpy(a, c, n * 8, hipMemcpyDeviceToDevice));
        CHK(hipEventRecord(e0));
        CHK(rocprim::radix_sort_keys(dtmp, tmp, a, b, n, 32, 32 + bits));
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("rocprim radix_sort_keys: %.3f ms  (%.2f G rec/s)\n", ms, n / (ms * 1e-3) / 1e9);
    }
    // check both agree
    std::vector<uint64_t> h1(n), h2(n);
    CHK(hipMemcpy(a, c, n * 8, hipMemcpyDeviceToDevice));
    uint64_t* sorted;
    CHK(kb::launch_onesweep(a, b, n, bits, flags, aux, &epoch, &sorted, 0));
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h1.data(), sorted, n * 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(a, c, n * 8, hipMemcpyDeviceToDevice));
    CHK(rocprim::radix_sort_keys(dtmp, tmp, a, b, n, 32, 32 + bits));
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h2.data(), b, n * 8, hipMemcpyDeviceToHost));
    printf("identical: %s\n", h1 == h2 ? "yes" : "NO");
    return 0;
}
