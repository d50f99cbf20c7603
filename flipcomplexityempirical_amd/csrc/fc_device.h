// Device helpers shared by the flip-walk kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fc_internal.h"

namespace fc {
namespace dev {

// LDS operations of one wave execute in order; the fence only stops the compiler moving
// LDS accesses across it.  Full waits (wave_sync) are used where lanes hand data to each
// other through atomics (BFS).
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ void wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

#ifdef FC_PHASE_PROF
#define FC_STAMP(t) const int64_t t = (int64_t)__builtin_amdgcn_s_memtime()
// accumulators live in the chain's LDS tail (prof_acc), so profiling adds no registers
#define FC_PROF(i, x) \
    do { if (lane == 0) atomicAdd((unsigned long long *)&prof_acc[i], (unsigned long long)(int64_t)(x)); } while (0)
#else
#define FC_STAMP(t)
#define FC_PROF(i, x)
#endif

__device__ __forceinline__ uint64_t bits_below(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }
__device__ __forceinline__ uint64_t lane_range(int lo, int hi) { return bits_below(hi) & ~bits_below(lo); }

__device__ __forceinline__ int rl32(int x, int lane) { return __builtin_amdgcn_readlane(x, lane); }
__device__ __forceinline__ uint32_t rlu(uint32_t x, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)x, lane); }

__device__ __forceinline__ int count_below(uint64_t m) {  // set bits of m below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int CTRL>
__device__ __forceinline__ int dpp_mov(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}

// Inclusive prefix sum over the 64 lanes (call with the whole wave active): Hillis-Steele
// row_shr steps inside each 16-lane row, then the row totals.
__device__ __forceinline__ int wave_scan_incl(int x) {
    x += dpp_mov<0x111>(x);
    x += dpp_mov<0x112>(x);
    x += dpp_mov<0x114>(x);
    x += dpp_mov<0x118>(x);
    const int r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31),
              r2 = __builtin_amdgcn_readlane(x, 47);
    const int lane = (int)__lane_id();
    return x + (lane >= 16 ? r0 : 0) + (lane >= 32 ? r1 : 0) + (lane >= 48 ? r2 : 0);
}

__device__ __forceinline__ int kth_set_bit(uint64_t x, int k) {  // k >= 1
    for (int i = 1; i < k; ++i) x &= x - 1;
    return __builtin_ctzll(x);
}

template <int RMAX>
__device__ __forceinline__ int ring_entry(const uint32_t (&ring)[RMAX / 2], int i) {
    return (int)((ring[i >> 1] >> (16 * (i & 1))) & 0xffffu);
}

// At most one of the cyclic intervals between consecutive old-district neighbours holds a
// break (a ring step that is not an old-district link) <=> the neighbours form one run.
__device__ __forceinline__ bool one_run(uint32_t nbrA, uint32_t brk, uint32_t full) {
    if (__popc(nbrA) <= 1) return true;
    uint32_t cur = nbrA & (0u - nbrA);
    uint32_t rest = nbrA & (nbrA - 1u);
    int cnt = 0;
    while (rest) {
        const uint32_t nx = rest & (0u - rest);
        cnt += (brk & (nx - cur)) != 0u;
        cur = nx;
        rest &= rest - 1u;
    }
    const uint32_t first = nbrA & (0u - nbrA);  // wrap interval [cur, L) U [0, first)
    cnt += (brk & ((full & ~(cur - 1u)) | (first - 1u))) != 0u;
    return cnt <= 1;
}

// Wave-cooperative BFS over the old district with v removed: are all old-district
// neighbours of v (each lane < RMAX may hold one as its target) connected to `start`?
template <int RMAX>
__device__ bool wave_bfs(const NodeRec<RMAX> *__restrict__ G, const int8_t *a, uint64_t *vis, uint64_t *front,
                         uint64_t *nxt, int words, int lane, int vf, int A, int my_target, int start,
                         int64_t &levels) {
    for (int i = lane; i < words; i += kWave) {
        vis[i] = 0;
        front[i] = 0;
        nxt[i] = 0;
    }
    wave_sync();
    if (lane == 0) {
        vis[vf >> 6] |= 1ull << (vf & 63);
        vis[start >> 6] |= 1ull << (start & 63);
        front[start >> 6] |= 1ull << (start & 63);
    }
    wave_sync();
    for (;;) {
        ++levels;
        for (int i = lane; i < words; i += kWave) {
            uint64_t bits = front[i];
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                const NodeRec<RMAX> r = G[i * 64 + b];
                const uint32_t nbr = (uint32_t)(r.meta >> kMetaNbrShift) & 0xffffu;
#pragma unroll
                for (int j = 0; j < RMAX; ++j) {
                    if (!((nbr >> j) & 1u)) continue;
                    const int e = ring_entry<RMAX>(r.ring, j);
                    if (a[e] != A) continue;
                    const uint64_t bit = 1ull << (e & 63);
                    const uint64_t old = atomicOr((unsigned long long *)&vis[e >> 6], (unsigned long long)bit);
                    if (!(old & bit)) atomicOr((unsigned long long *)&nxt[e >> 6], (unsigned long long)bit);
                }
            }
        }
        wave_sync();
        const bool found = my_target < 0 || ((vis[my_target >> 6] >> (my_target & 63)) & 1ull);
        if (__all(found)) return true;
        bool any = false;
        for (int i = lane; i < words; i += kWave) {
            const uint64_t x = nxt[i];
            front[i] = x;
            nxt[i] = 0;
            any |= x != 0;
        }
        wave_sync();
        if (!__any(any)) return false;
    }
}

// per-lane status bits of the slots of one batch
constexpr uint32_t ST_VS = 1u;   // valid step
constexpr uint32_t ST_AC = 2u;   // accepted
constexpr uint32_t ST_IC = 4u;   // invalid: contiguity
constexpr uint32_t ST_IP = 8u;   // invalid: population
constexpr uint32_t ST_BD = 16u;  // contiguity resolved by BFS
constexpr uint32_t ST_BR = 32u;  // ... and its result
// per-slot predicates of the k = 2 kernel, packed beside the status bits
constexpr uint32_t LF_HIT = 1u << 8;     // proposal (boundary node)
constexpr uint32_t LF_ACC = 1u << 9;     // Metropolis test passed
constexpr uint32_t LF_SLIN = 1u << 10;   // run rule, open ring
constexpr uint32_t LF_SCYC = 1u << 11;   // run rule, ring closed through the outer face
constexpr uint32_t LF_EXACT = 1u << 12;  // the run rule decides contiguity exactly
constexpr uint32_t LF_GAM = 1u << 13;    // outer-face node
constexpr uint32_t LF_HAS = 1u << 14;    // the lane holds a slot
constexpr uint32_t LF_WROTE = 1u << 15;  // the lane holds commit marks
constexpr uint32_t LF_FRZ = 1u << 16;    // FC_CON_FIXED: the node may not flip

}  // namespace dev
}  // namespace fc
