// The planar run rule's ring test and the k > 2 district-graph rule, shared by the kernels
// and the host-side checks (tests/native/one_run_check.cpp compares one_run with the
// interval-counting statement; tests/native/district_rule_lib.cpp exposes district_rule to
// tests/test_district_rule.py, which compares it with the oracle's BFS).
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

// The same verdict without the early return, for the k = 2 kernel, where the early return put
// every slot's verdict behind exec-mask branches (the k > 2 kernel keeps one_run: there this form
// costs SGPR and VGPR spills).  With B or nbrA zero the scans see the guard bits
// and the masks are meaningless, but the trivial case decides those inputs.
FC_RING_HD bool one_run_flat(uint32_t nbrA, uint32_t brk, uint32_t full) {
    const uint32_t B = brk & full;
    const bool trivial = ((nbrA & (nbrA - 1u)) == 0u) | (B == 0u);
    const int bmin = __builtin_ctz(B | 0x80000000u), bmax = 31 - __builtin_clz(B | 1u);
    const int nf = __builtin_ctz(nbrA | 0x80000000u), nl = 31 - __builtin_clz(nbrA | 1u);
    const uint32_t between = ((2u << bmax) - 1u) & ~((2u << bmin) - 1u);
    const uint32_t inner = ((1u << nl) - 1u) & ~((1u << nf) - 1u);
    return trivial | ((nbrA & between) == 0u) | ((B & inner) == 0u);
}

// District-graph contiguity rule (k > 2; every node exact, so each ring lists every cell that
// shares a face with its node and the outer face is one wedge of the outer nodes' rings).
//
// Removing v from its district A disconnects A (single_flip_contiguous [gc-0.2],
// grid_chain_sec11.py:22,340) iff two "super-gaps" of v's ring -- the stretches between
// consecutive A-runs that hold old neighbours, made of other districts' cells, irrelevant
// A-corners and (outer nodes) the outer-face wedge -- are joined through the complement of
// A: cells of districts != A under face adjacency, plus the outer face.  (=>: a complement
// path from one super-gap to another, closed through v, is a curve that separates the A-runs
// on its two sides; no A edge can cross it, since it runs through face interiors and the
// outer face.  <=: the boundary cycle around a piece cut off by v passes through v, entering
// and leaving through two super-gaps, and otherwise through the complement.)  Every district
// is connected, so the complement's components are those of the district graph without A:
// X - Y when some face holds cells of both (adj, kept incrementally from the per-chain pair
// counts), X - outer face when X has an outer-face node (bit 31).  The verdict is a few
// bitmask closures -- no search.  Exactness holds for any such graph; the oracle's BFS is
// the reference (tests/test_district_rule.py checks this function, built for the host, and a
// restatement; the GPU parity tests the kernel, per proposal, enclave states included).
template <int RMAX>
FC_RING_HD bool district_rule(const int (&adv)[RMAX], uint32_t inA, uint32_t nbr, uint32_t Ln, bool gam, int A,
                              const uint32_t *adj) {
    // ring augmented with the outer wedge (position Ln) for outer nodes
    const uint32_t Lp = Ln + (gam ? 1u : 0u);
    const uint32_t fullp = (1u << Lp) - 1u;
    inA &= (1u << Ln) - 1u;
    const uint32_t rotA = ((inA << 1) | (inA >> (Lp - 1))) & fullp;
    uint32_t st0 = inA & ~rotA;  // run starts
    const uint32_t a2 = inA | (inA << Lp);
    uint32_t relA = 0;           // A-runs holding an old neighbour
    while (st0) {
        const int s0 = __builtin_ctz(st0);
        st0 &= st0 - 1u;
        const int len = __builtin_ctz(~(a2 >> s0));
        uint32_t run = ((1u << len) - 1u) << s0;
        run = (run | (run >> Lp)) & fullp;
        if (run & nbr) relA |= run;
    }
    const uint32_t gap = fullp & ~relA;
    const uint32_t rotG = ((gap << 1) | (gap >> (Lp - 1))) & fullp;
    uint32_t gst = gap & ~rotG;  // super-gap starts
    const uint32_t g2 = gap | (gap << Lp);
    const uint32_t notA = ~(1u << A);
    uint32_t seen = 0;
    while (gst) {
        const int s0 = __builtin_ctz(gst);
        gst &= gst - 1u;
        const int len = __builtin_ctz(~(g2 >> s0));
        uint32_t run = ((1u << len) - 1u) << s0;
        run = (run | (run >> Lp)) & fullp & ~inA;
        uint32_t D = 0;          // districts of the super-gap's cells (+ the outer face)
        while (run) {
            const int i = __builtin_ctz(run);
            run &= run - 1u;
            // ring positions < Ln are cells; position Ln (outer nodes) is the outer wedge.  The
            // padded entries past Ln hold v itself (district A), so q must stay below Ln: with
            // q == Ln the wedge took A's bit and its closure swallowed adj[A]
            uint32_t di = 1u << 31;
#pragma unroll
            for (int q = 0; q < RMAX; ++q) di = (q == i && q < (int)Ln) ? (1u << adv[q]) : di;
            D |= di;
        }
        if (D & seen) return false;
        uint32_t comp = D, fr = D;  // closure in the district graph without A
        while (fr) {
            const int X = __builtin_ctz(fr);
            fr &= fr - 1u;
            const uint32_t nb = adj[X] & notA & ~comp;
            if (nb & seen) return false;
            comp |= nb;
            fr |= nb;
        }
        seen |= comp;
    }
    return true;
}

}  // namespace fc
