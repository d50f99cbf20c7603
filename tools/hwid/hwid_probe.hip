// Placement probe: 4096 one-wave workgroups with the k = 2 kernel's LDS footprint record
// HW_ID and XCC_ID (scalar reads) into a buffer (vector store from lane 0).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void probe(uint32_t *out, int spin) {
    extern __shared__ uint32_t sm[];
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    sm[threadIdx.x] = hw;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) {}
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc; }
}
int main() {
    const int B = 4096;
    uint32_t *d; hipMalloc(&d, B * 8);
    hipLaunchKernelGGL(probe, dim3(B), dim3(64), 9600, 0, d, 100000);  // 1 ms spin: all resident together
    std::vector<uint32_t> h(B * 2);
    hipMemcpy(h.data(), d, B * 8, hipMemcpyDeviceToHost);
    std::map<uint32_t, int> simd, cu;
    for (int b = 0; b < B; ++b) {
        uint32_t hw = h[2 * b], x = h[2 * b + 1];
        simd[((x & 7) << 12) | ((hw >> 4) & 0xfff)]++;
        cu[((x & 7) << 12) | ((hw >> 8) & 0xff)]++;
        if (b < 40) printf("block %4d hw %08x xcc %u wave %u simd %u pipe %u cu %u sh %u se %u\n", b, hw, x, hw & 15, (hw >> 4) & 3, (hw >> 6) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7);
    }
    std::map<int, int> hs, hc;
    for (auto &kv : simd) hs[kv.second]++;
    for (auto &kv : cu) hc[kv.second]++;
    printf("distinct simd keys %zu, cu keys %zu\n", simd.size(), cu.size());
    for (auto &kv : hs) printf("  %d waves: %d simd keys\n", kv.first, kv.second);
    for (auto &kv : hc) printf("  %d waves: %d cu keys\n", kv.first, kv.second);
    return 0;
}
