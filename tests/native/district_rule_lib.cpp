// Host build of the k > 2 kernel's district-graph contiguity rule (csrc/fc_ring.h
// district_rule, the exact function flip_kernel calls) for tests/test_district_rule.py, which
// compares it with the oracle's BFS restatement of single_flip_contiguous [gc-0.2]
// (grid_chain_sec11.py:22,340).  Loaded through ctypes; test infrastructure only.
#include <cstdint>

#include "fc_ring.h"

template <int RMAX>
static int call(const int32_t *adv_in, uint32_t inA, uint32_t nbr, uint32_t Ln, int32_t gam, int32_t A,
                const uint32_t *adj) {
    int adv[RMAX];
    for (int i = 0; i < RMAX; ++i) adv[i] = adv_in[i];
    return fc::district_rule<RMAX>(adv, inA, nbr, Ln, gam != 0, A, adj) ? 1 : 0;
}

extern "C" int fc_test_district_rule(int32_t ring_max, const int32_t *adv, uint32_t inA, uint32_t nbr, uint32_t Ln,
                                     int32_t gam, int32_t A, const uint32_t *adj) {
    if (ring_max == 8) return call<8>(adv, inA, nbr, Ln, gam, A, adj);
    if (ring_max == 16) return call<16>(adv, inA, nbr, Ln, gam, A, adj);
    return -1;
}
