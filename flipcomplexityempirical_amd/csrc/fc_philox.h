// Counter-based random stream shared by the host (initial-state wait) and the kernels.
//
// Draw d of chain c: Philox4x32-10(ctr = (lo32 d, hi32 d, c, purpose), key = seed).
// purpose 0: the proposal words; 1: the geometric wait of the state created by draw d;
// 2 (d = 0): the geometric wait of the initial state.  DESIGN.md "Random stream".
#pragma once
#include <stdint.h>

#include <cmath>

#if defined(__HIPCC__) || defined(__HIP__)
#define FC_HD __host__ __device__ __forceinline__
#else
#define FC_HD inline
#endif

namespace fc {

struct Words4 {
    uint32_t x0, x1, x2, x3;
};

FC_HD Words4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
#if defined(__HIP_DEVICE_COMPILE__)
            // keep the key schedule two scalar adds per round: hoisted out of the kernels'
            // loops, its 20 round keys were held in SGPRs, spilled to VGPR lanes and reloaded
            // (v_readlane + hazard nop) in every round
            asm volatile("" : "+s"(k0), "+s"(k1));
#endif
        }
        // one v_mad_u64_u32 per product gives both halves
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);  // 3-way xor
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
#else
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
#endif
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
    }
    return Words4{c0, c1, c2, c3};
}

// 53-bit mantissa of CPython random() / numpy random_sample() from two words.
FC_HD uint64_t mant53(uint32_t a, uint32_t b) { return ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6); }

FC_HD double u53(uint32_t a, uint32_t b) { return (double)mant53(a, b) * (1.0 / 9007199254740992.0); }

// geom_wait (grid_chain_sec11.py:147-148) by numpy's legacy inversion, ceil(log(1-U)/log(1-p)) - 1,
// saturated at 2^62 where log(1-p) rounds to 0 (|B| / (N^k - 1) below 2^-53, e.g. k >= 5 on 10^4
// nodes) -- the reference's float pipeline has no defined value there.
constexpr double kWaitCap = 4611686018427387904.0;  // 2^62
FC_HD int64_t geom_from(double U, double log1mp) {
    const double q = log(1.0 - U) / log1mp;
    if (!(fabs(q) < kWaitCap)) return (int64_t)kWaitCap;
    return (int64_t)ceil(q) - 1;
}

}  // namespace fc
