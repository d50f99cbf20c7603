// The planar run rule's ring test, shared by the kernels and the host-side check
// (tests/native/one_run_check.cpp compares it with the interval-counting statement).
//
// A node's ring holds L cells (bits 0..L-1).  nbrA marks its old-district neighbours and brk
// the ring steps that are not old-district links.  The neighbours form one run -- removing the
// node leaves its old-district neighbours connected around it (single_flip_contiguous's local
// case) -- iff at most one of the cyclic intervals [n_k, n_{k+1}) between
// consecutive neighbours (the last one wrapping: [n_last, L) U [0, n_first)) holds a break.
//
// Loop-free form: with b_min / b_max the lowest / highest break, every break lies in one
// interval iff no neighbour lies in (b_min, b_max] (they share b_min's interval) or no break
// lies in [n_first, n_last) (they are all in the wrapping interval).  The per-lane loop over
// the neighbours cost two divergent loops per slot evaluation.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define FC_RING_HD __host__ __device__ __forceinline__
#else
#define FC_RING_HD inline
#endif

namespace fc {

FC_RING_HD bool one_run(uint32_t nbrA, uint32_t brk, uint32_t full) {
    const uint32_t B = brk & full;
    if ((nbrA & (nbrA - 1u)) == 0u || B == 0u) return true;  // <= 1 neighbour, or no break
    const int bmin = __builtin_ctz(B), bmax = 31 - __builtin_clz(B);
    const int nf = __builtin_ctz(nbrA), nl = 31 - __builtin_clz(nbrA);
    const uint32_t between = ((2u << bmax) - 1u) & ~((2u << bmin) - 1u);  // (b_min, b_max]; L <= 16
    const uint32_t inner = ((1u << nl) - 1u) & ~((1u << nf) - 1u);          // [n_first, n_last)
    return (nbrA & between) == 0u || (B & inner) == 0u;
}

}  // namespace fc
