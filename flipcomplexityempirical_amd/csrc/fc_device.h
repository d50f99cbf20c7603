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

// BFS scratch of one chain (LDS): 4-bit source labels of the visited nodes, the per-label
// merge masks, and the frontier bitmaps.  Bitmaps are strided: node u is bit (u >> lsh) of
// word (u & (W - 1)), W = 2^lsh words, so a spatially compact frontier (consecutive ids)
// spreads over the lanes instead of queueing in one lane's word.
struct BfsScratch {
    uint32_t *lab;    // [(n + 7) / 8] nibbles: 0 unvisited, 1..15 source label
    uint32_t *mm;     // [16] label i touched the labels in mm[i]
    uint64_t *front;  // [W]
    uint64_t *nxt;    // [W]
    int lab_words;    // u32 words of lab
    int lsh;          // log2 W
};

__device__ __forceinline__ uint32_t or_reduce(uint32_t x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x |= (uint32_t)__shfl_xor((int)x, off);
    return x;
}

// Multi-source wave BFS over the old district A with v removed (single_flip_contiguous
// [gc-0.2], grid_chain_sec11.py:22,340): are all old-district neighbours of v connected?
// Every neighbour (lane < RMAX holding it in my_target) starts its own labelled search;
// searches that meet are merged (16-bit component masks, one per label, in lanes 0..15).
// It answers yes once one component holds every label, and no once some component has
// no frontier left -- it is then a whole connected piece of A - v without all of them,
// which usually happens long before a single-source search would have exhausted A.
template <int RMAX>
__device__ bool wave_bfs(const NodeRec<RMAX> *__restrict__ G, const int8_t *a, const BfsScratch &S, int lane,
                         int vf, int A, int my_target, int64_t &levels) {
    const int W = 1 << S.lsh;
    const uint32_t wm = (uint32_t)W - 1u;
    for (int i = lane; i < S.lab_words; i += kWave) S.lab[i] = 0;
    for (int i = lane; i < W; i += kWave) {
        S.front[i] = 0;
        S.nxt[i] = 0;
    }
    if (lane < 16) S.mm[lane] = 0;
    wave_sync();
    const bool src = my_target >= 0;
    const uint64_t SM = __ballot(src);
    const int ns = __popcll(SM);
    if (ns <= 1) return true;
    const uint32_t lab_me = src ? (uint32_t)(count_below(SM) + 1) : 0u;  // labels 1..ns
    if (src) {
        atomicOr(&S.lab[my_target >> 3], lab_me << ((my_target & 7) * 4));
        atomicOr((unsigned long long *)&S.front[(uint32_t)my_target & wm], 1ull << (my_target >> S.lsh));
    }
    const uint32_t all = ((1u << (ns + 1)) - 1u) & ~1u;  // labels 1..ns
    uint32_t comp = lane < 16 ? (1u << lane) : 0u;      // component mask of label `lane`
    wave_sync();
    for (;;) {
        ++levels;
        uint32_t live = 0;  // labels that claimed a node at this level
        bool merged = false;
        for (int i = lane; i < W; i += kWave) {
            uint64_t bits = S.front[i];
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                const int u = (b << S.lsh) | i;
                const uint32_t la = (S.lab[u >> 3] >> ((u & 7) * 4)) & 15u;
                const NodeRec<RMAX> r = G[u];
                const uint32_t nbr = (uint32_t)(r.meta >> kMetaNbrShift) & 0xffffu;
#pragma unroll
                for (int j = 0; j < RMAX; ++j) {
                    if (!((nbr >> j) & 1u)) continue;
                    const int w = ring_entry<RMAX>(r.ring, j);
                    if (w == vf || a[w] != A) continue;
                    uint32_t *wd = &S.lab[w >> 3];
                    const int sh = (w & 7) * 4;
                    uint32_t old = *wd;
                    for (;;) {
                        const uint32_t nib = (old >> sh) & 15u;
                        if (nib) {
                            if (nib != la) {
                                atomicOr(&S.mm[la], 1u << nib);
                                merged = true;
                            }
                            break;
                        }
                        const uint32_t prev = atomicCAS(wd, old, old | (la << sh));
                        if (prev == old) {
                            atomicOr((unsigned long long *)&S.nxt[(uint32_t)w & wm], 1ull << (w >> S.lsh));
                            live |= 1u << la;
                            break;
                        }
                        old = prev;
                    }
                }
            }
        }
        wave_sync();
        if (__any(merged)) {
            // comp(i) |= labels i touched, symmetric, then transitive closure (<= 4 rounds)
            uint32_t adj = comp | (lane < 16 ? S.mm[lane] : 0u);
            uint32_t sym = adj;
#pragma unroll
            for (int j = 1; j < 16; ++j) {
                const uint32_t aj = (uint32_t)__shfl((int)adj, j);
                if (lane < 16 && ((aj >> lane) & 1u)) sym |= 1u << j;
            }
            comp = lane < 16 ? sym : 0u;
            for (int it = 0; it < 4; ++it) {
                uint32_t nx = comp;
#pragma unroll
                for (int j = 1; j < 16; ++j) {
                    const uint32_t cj = (uint32_t)__shfl((int)comp, j);
                    if ((comp >> j) & 1u) nx |= cj;
                }
                const bool ch = nx != comp;
                comp = nx;
                if (!__any(ch)) break;
            }
            if (lane < 16) S.mm[lane] = 0;
        }
        if ((((uint32_t)__shfl((int)comp, 1)) & all) == all) return true;  // one component
        live = or_reduce(live);
        // a component without a live label is closed: a piece of A - v missing some label
        const bool dead = lane >= 1 && lane <= ns && (comp & live) == 0u;
        if (__any(dead)) return false;
        bool any = false;
        for (int i = lane; i < W; i += kWave) {
            const uint64_t x = S.nxt[i];
            S.front[i] = x;
            S.nxt[i] = 0;
            any |= x != 0;
        }
        wave_sync();
        if (!__any(any)) return false;  // unreachable: some label would be dead
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
