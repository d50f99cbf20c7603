// Issue cost of the integer VALU forms the k = 2 kernel leans on (Philox's 32x32->64 product,
// 24-bit products, bitops, 64-bit shifts), one wave per SIMD and four, measured with
// s_memtime around an unrolled loop of 8 independent chains.  Diagnostic probe only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N_IT 4096
template <int OP>
__global__ void probe(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = seed * (threadIdx.x + 1) + i; b[i] = a[i] ^ 0x9E3779B9u; }
    const uint32_t M = 0xD2511F53u;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) {  // v_mad_u64_u32: both halves of a 32x32 product
                const uint64_t p = (uint64_t)a[i] * M + b[i];
                a[i] = (uint32_t)(p >> 32);
                b[i] = (uint32_t)p;
            } else if constexpr (OP == 1) {  // v_mul_hi_u32 alone
                a[i] = __umulhi(a[i], M) + b[i];
            } else if constexpr (OP == 2) {  // v_mul_lo_u32
                a[i] = a[i] * M + b[i];
            } else if constexpr (OP == 3) {  // v_mul_u32_u24
                a[i] = __umul24(a[i], b[i]) + 7u;
            } else if constexpr (OP == 4) {  // v_xor3 / bitop3
                a[i] = a[i] ^ b[i] ^ (a[i] >> 3);
            } else if constexpr (OP == 5) {  // v_add_u32
                a[i] = a[i] + b[i];
            }
            asm volatile("" : "+v"(a[i]), "+v"(b[i]));
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= a[i] ^ b[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char *name, int waves_per_simd) {
    const int blocks = 256 * 4 * waves_per_simd;  // one-wave blocks: ~waves_per_simd per SIMD
    uint32_t *out; uint64_t *cyc;
    hipMalloc(&out, blocks * 64 * 4); hipMalloc(&cyc, blocks * 8);
    probe<OP><<<blocks, 64>>>(out, cyc, 1u);
    hipDeviceSynchronize();
    probe<OP><<<blocks, 64>>>(out, cyc, 3u);
    hipDeviceSynchronize();
    uint64_t *h = new uint64_t[blocks];
    hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double sum = 0; for (int i = 0; i < blocks; ++i) sum += (double)h[i];
    printf("%-22s waves/SIMD %d: %.2f cycles per wave-instruction-slot (8 chains x %d it)\n", name, waves_per_simd,
           sum / blocks / (8.0 * N_IT), N_IT);
    delete[] h; hipFree(out); hipFree(cyc);
}

int main() {
    for (int w : {1, 4}) {
        run<0>("v_mad_u64_u32", w);
        run<1>("v_mul_hi_u32+add", w);
        run<2>("v_mad_u32 (lo)", w);
        run<3>("v_mul_u32_u24+add", w);
        run<4>("xor3+shift", w);
        run<5>("v_add_u32", w);
    }
    return 0;
}
