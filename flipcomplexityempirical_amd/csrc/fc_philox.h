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

FC_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

FC_HD Words4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
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
