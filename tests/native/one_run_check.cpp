// Host check of the planar run rule's loop-free ring test (csrc/fc_ring.h: one_run and its
// branch-free form one_run_flat) against its
// statement: count the cyclic intervals between consecutive old-district neighbours that hold
// a break; one run <=> at most one.  Exhaustive for rings of 1..10 cells, random beyond (the
// kernels use rings of at most 16).  Prints "checked N bad B"; exit status 1 on any mismatch.
#include <cstdint>
#include <cstdio>
#include <random>

#include "fc_ring.h"

static bool one_run_intervals(uint32_t nbrA, uint32_t brk, uint32_t full) {
    if (__builtin_popcount(nbrA) <= 1) return true;
    uint32_t cur = nbrA & (0u - nbrA), rest = nbrA & (nbrA - 1u);
    int cnt = 0;
    while (rest) {  // [n_k, n_{k+1})
        const uint32_t nx = rest & (0u - rest);
        cnt += (brk & (nx - cur)) != 0u;
        cur = nx;
        rest &= rest - 1u;
    }
    const uint32_t first = nbrA & (0u - nbrA);  // [n_last, L) U [0, n_first)
    cnt += (brk & ((full & ~(cur - 1u)) | (first - 1u))) != 0u;
    return cnt <= 1;
}

int main() {
    long n = 0, bad = 0;
    auto check = [&](int L, uint32_t M, uint32_t B) {
        const uint32_t full = (1u << L) - 1u;
        ++n;
        const bool want = one_run_intervals(M, B & full, full);
        if (fc::one_run(M, B, full) != want || fc::one_run_flat(M, B, full) != want) {
            if (bad < 8) printf("mismatch L=%d nbrA=%x brk=%x\n", L, M, B);
            ++bad;
        }
    };
    for (int L = 1; L <= 10; ++L)
        for (uint32_t M = 0; M < (1u << L); ++M)
            for (uint32_t B = 0; B < (1u << L); ++B) check(L, M, B);
    std::mt19937 g(12345);
    for (int L = 11; L <= 16; ++L)
        for (int it = 0; it < 2000000; ++it) {
            const uint32_t full = (1u << L) - 1u;
            uint32_t M = g() & full, B = g() & full;
            if (it & 1) M &= g();
            if (it & 2) B &= g() & g();
            check(L, M, B);
        }
    printf("checked %ld bad %ld\n", n, bad);
    return bad ? 1 : 0;
}
