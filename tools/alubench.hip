// tools/alubench.hip -- per-instruction VALU/LDS throughput on one MI355X, to
// price the bin kernel's inner loops (64-bit shifts, 32-bit multiplies, mbcnt,
// LDS ring writes).  hipcc -O3 --offload-arch=gfx950 tools/alubench.hip -o /tmp/alubench
// Each kernel runs 8 independent chains per lane (no dependency stalls) over
// 4 waves per SIMD; the report is wave-instructions per SIMD per cycle at the
// measured clock-free rate: G wave-instructions/s across the chip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                                         \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

constexpr int IT = 4096, CH = 8;

__global__ __launch_bounds__(1024) void k_add32(uint32_t* out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c;
    for (int i = 0; i < IT; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) a[c] = a[c] + (s ^ c);
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = r;
}
__global__ __launch_bounds__(1024) void k_shl64(uint32_t* out, uint32_t s) {
    uint64_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c * 77ull;
    for (int i = 0; i < IT; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) a[c] = a[c] << (s & 7);
    uint64_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = (uint32_t)r;
}
__global__ __launch_bounds__(1024) void k_mul32(uint32_t* out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c;
    for (int i = 0; i < IT; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) a[c] = a[c] * (s | 1u);
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = r;
}
__global__ __launch_bounds__(1024) void k_mbcnt(uint32_t* out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c;
    for (int i = 0; i < IT; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) a[c] = __builtin_amdgcn_mbcnt_lo(s ^ (uint32_t)c, a[c]);
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = r;
}
__global__ __launch_bounds__(1024) void k_lds64(uint32_t* out, uint32_t s) {
    __shared__ uint64_t ring[16 * 256];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    uint64_t v = threadIdx.x;
    for (int i = 0; i < IT; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) ring[w * 256 + ((l + 64u * c + s) & 255u)] = v + c;
        v += s;
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (ring[threadIdx.x] == 0x12345) out[0] = 1;
}

int main() {
    uint32_t* d;
    CHK(hipMalloc(&d, 64));
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus;  // one 1024-thread block per CU: 4 waves per SIMD
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    struct K {
        const char* name;
        void (*f)(uint32_t*, uint32_t);
        double insts_per_op;  // wave instructions per source-level op
    } ks[] = {{"v_add_u32", k_add32, 1}, {"64-bit shift (v_lshlrev_b64)", k_shl64, 1},
              {"v_mul_lo_u32", k_mul32, 1}, {"v_mbcnt_lo", k_mbcnt, 1}, {"ds_write_b64 (ring)", k_lds64, 1}};
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(1024), 0, 0, d, 3u);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(a));
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(1024), 0, 0, d, 3u);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        const double waves = (double)blocks * 16.0, ops = waves * IT * CH * 5 * k.insts_per_op;
        const double per_simd_ns = ms * 1e6 / (ops / (cus * 4.0));
        printf("%-32s %8.1f G wave-ops/s  %.3f ns per wave-op per SIMD (%.1f cycles at 2.4 GHz)\n", k.name,
               ops / (ms * 1e6), per_simd_ns, per_simd_ns * 2.4);
    }
    return 0;
}
