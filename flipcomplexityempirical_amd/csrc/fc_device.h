// Device helpers shared by the flip-walk kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fc_internal.h"
#include "fc_philox.h"
#include "fc_ring.h"

namespace fc {
namespace dev {

// LDS operations of one wave execute in order; the fence only stops the compiler moving
// LDS accesses across it.  Full waits (wave_sync) are used where lanes hand data to each
// other through atomics (BFS).
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ void wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

#ifdef FC_PHASE_PROF
#ifdef FC_PHASE_SYNC  // drain outstanding memory first: each phase is charged its own latency
#define FC_STAMP(t)                                                    \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");        \
    const int64_t t = (int64_t)__builtin_amdgcn_s_memtime()
#else
#define FC_STAMP(t) const int64_t t = (int64_t)__builtin_amdgcn_s_memtime()
#endif
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
    // row totals by the row broadcasts: row_bcast:15 adds lane 15 to row 1 and lane 47 to row
    // 3 (row mask 0xa), then row_bcast:31 adds lane 31 to rows 2 and 3 (row mask 0xc); two DPP
    // adds instead of three readlanes and their selects
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return x;
}

// position of the r-th (0-based) set bit of x, r < popcount(x): five popcount halvings
__device__ __forceinline__ int select_bit64(uint64_t x, int r) {
    uint32_t y = (uint32_t)x;
    int pos = 0, c = __popc(y);
    if (r >= c) { r -= c; y = (uint32_t)(x >> 32); pos = 32; }
    c = __popc(y & 0xffffu);
    if (r >= c) { r -= c; y >>= 16; pos += 16; }
    c = __popc(y & 0xffu);
    if (r >= c) { r -= c; y >>= 8; pos += 8; }
    c = __popc(y & 0xfu);
    if (r >= c) { r -= c; y >>= 4; pos += 4; }
    c = __popc(y & 0x3u);
    if (r >= c) { r -= c; y >>= 2; pos += 2; }
    return pos + (r >= (int)(y & 1u) ? 1 : 0);
}

__device__ __forceinline__ int kth_set_bit(uint64_t x, int k) {  // k >= 1
    for (int i = 1; i < k; ++i) x &= x - 1;
    return __builtin_ctzll(x);
}

template <int RMAX>
__device__ __forceinline__ int ring_entry(const uint32_t (&ring)[RMAX / 2], int i) {
    return (int)((ring[i >> 1] >> (16 * (i & 1))) & 0xffffu);
}

using fc::one_run;  // fc_ring.h
using fc::one_run_flat;

// Chain dealing (fc_deal.hip): the chain this wave runs.  Lane 0 reads the wave's SIMD
// (HW_ID: SIMD, pipe, CU, SH, SE; XCC_ID: the XCD), takes the next arrival slot s on that
// SIMD and claims the next chain of quarter s of p.order (slowest quarter first), falling
// through to the following quarters when one is used up: the claims are a bijection of the
// launch's waves onto its chains whatever the placement.  Vector atomics only.
__device__ __forceinline__ int deal_chain(const KParams &p, int lane) {
    int cc = 0;
    if (lane == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const uint32_t key = ((xcc & 7u) << 12) | ((hw >> 4) & 0xfffu);
        const uint32_t slot = atomicAdd(&p.deal[key], 1u);
        const uint32_t C = (uint32_t)p.n_chains;
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t q = (slot + k) & 3u;
            const uint32_t lo = q * C / 4u, hi = (q + 1u) * C / 4u;
            const uint32_t i = atomicAdd(&p.deal[kDealKeys + q], 1u);
            if (lo + i < hi) {
                cc = (int)p.order[lo + i];
                break;
            }
        }
    }
    return __builtin_amdgcn_readfirstlane(__shfl(cc, 0));
}

// BFS scratch of one chain (LDS): the source label of every visited node (one byte:
// claimed nodes have exactly one writer, so plain stores), per-label merge and component
// masks, the visited bitmap, two frontier lists (ping-pong; a level's claimers append to the
// next one) and frontier bitmaps for the nodes that overflow a list.
constexpr int kBfsList = 512;
struct BfsScratch {
    uint32_t *lab;    // [lab_words] bytes: source label 0..15 of a visited node
    uint32_t *mm;     // [16] labels that label i ran into this level
    uint32_t *cm;     // [16] component mask of label i
    int32_t *lcnt;    // [2] list lengths (may exceed kBfsList: the rest is in the bitmap)
    uint16_t *list;   // [2][kBfsList] frontier lists
    uint64_t *vis;    // [W] visited
    uint64_t *front;  // [W] overflowed frontier nodes of this level
    uint64_t *nxt;    // [W] overflowed frontier nodes of the next level
    int lab_words;    // u32 words of lab
    int W;            // ceil(n / 64)
    int64_t *prof;    // FC_PHASE_PROF builds: phase accumulators (slot 15: expansion cycles)
};

__device__ __forceinline__ uint32_t or_reduce(uint32_t x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x |= (uint32_t)__shfl_xor((int)x, off);
    return x;
}

// Multi-source wave BFS over the old district A with v removed (single_flip_contiguous
// [gc-0.2], grid_chain_sec11.py:22,340): are all old-district neighbours of v connected?
// Every neighbour (lane < RMAX holding it in my_target) starts its own labelled search;
// searches that meet are merged (16-bit component masks, one per label).  It answers yes
// once one component holds every label, and no once some component has no frontier left
// -- a whole connected piece of A - v without all of them -- which usually comes long
// before a single-source search would have exhausted A.  A level's frontier is a list the
// previous level appended to (wave prefix sums), dealt out one node per lane; a node's
// expansion is branch-free over its ring slots, so its ring reads, its claims and its
// label reads each go out together.  Nodes beyond a list's capacity go to a bitmap that
// the next level expands too.
template <int RMAX>
__device__ __forceinline__ bool wave_bfs(const NodeRec<RMAX> *__restrict__ G, const int8_t *a, const BfsScratch &S,
                                         int lane, int vf, int A, int my_target, int64_t &levels) {
    const int W = S.W;
    uint8_t *const lab = (uint8_t *)S.lab;
    for (int i = lane; i < W; i += kWave) {
        S.vis[i] = 0;
        S.front[i] = 0;
        S.nxt[i] = 0;
    }
    if (lane < 16) {
        S.mm[lane] = 0;
        S.cm[lane] = 1u << lane;
    }
    const bool src = my_target >= 0;
    const uint64_t SM = __ballot(src);
    const int ns = __popcll(SM);  // <= 16 (degree <= 16)
    wave_sync();
    if (ns <= 1) return true;
    if (src) {
        const uint32_t lab_me = (uint32_t)count_below(SM);  // labels 0..ns-1
        lab[my_target] = (uint8_t)lab_me;
        atomicOr((unsigned long long *)&S.vis[my_target >> 6], 1ull << (my_target & 63));
        S.list[lab_me] = (uint16_t)my_target;
    }
    if (lane == 0) atomicOr((unsigned long long *)&S.vis[vf >> 6], 1ull << (vf & 63));
    const uint32_t all = (uint32_t)((1ull << ns) - 1ull);  // labels 0..ns-1
    uint32_t comp = lane < 16 ? (1u << lane) : 0u;        // component mask of label `lane`
    bool spill_in = false;                                 // frontier nodes wait in S.front
    int fcur = ns;                                         // list length of this level
    wave_sync();
    for (int cur = 0;; cur ^= 1) {
        ++levels;
        uint32_t live = 0;  // labels that claimed a node at this level
        bool merged = false, spill_out = false;
        uint16_t *const lcur = S.list + cur * kBfsList, *const lnxt = S.list + (cur ^ 1) * kBfsList;
        int fnext = 0;  // appended to the next list so far (wave-uniform)
        // expand u (active lanes): claim every A neighbour at once (vis bit: the first
        // claimant wins), winners write their label, then losers read the labels they ran
        // into; returns the ring slots this lane won
        auto expand = [&](int u, bool active, int (&wn)[RMAX]) -> uint32_t {
            const uint32_t la = lab[u];
            const uint32_t cla = S.cm[la & 15u];
            const NodeRec<RMAX> rr = G[u];
            const uint32_t nbr = active ? (uint32_t)(rr.meta >> kMetaNbrShift) & 0xffffu : 0u;
            uint32_t cand = 0, won = 0;
#pragma unroll
            for (int j = 0; j < RMAX; ++j) {
                wn[j] = ring_entry<RMAX>(rr.ring, j);
                cand |= (((nbr >> j) & 1u) & (uint32_t)(a[wn[j]] == A)) << j;
            }
            uint64_t old[RMAX];
#pragma unroll
            for (int j = 0; j < RMAX; ++j) {
                const uint64_t bit = ((cand >> j) & 1u) ? 1ull << (wn[j] & 63) : 0ull;
                old[j] = bit ? atomicOr((unsigned long long *)&S.vis[wn[j] >> 6], bit) : 0ull;
            }
#pragma unroll
            for (int j = 0; j < RMAX; ++j) {
                won |= (uint32_t)(((cand >> j) & 1u) && !((old[j] >> (wn[j] & 63)) & 1ull)) << j;
                if ((won >> j) & 1u) lab[wn[j]] = (uint8_t)la;
            }
            live |= won ? 1u << la : 0u;
            compiler_fence();  // every winner's label store precedes the losers' reads
            uint32_t hit = 0;
#pragma unroll
            for (int j = 0; j < RMAX; ++j) {
                const bool lose = ((cand & ~won) >> j & 1u) && wn[j] != vf;
                const uint32_t lj = lose ? lab[wn[j]] & 15u : la;
                hit |= ((cla >> lj) & 1u) ? 0u : 1u << lj;
            }
            if (hit) {  // another component
                atomicOr(&S.mm[la], hit);
                merged = true;
            }
            return won;
        };
#ifdef FC_PHASE_PROF
        const int64_t t_x0 = (int64_t)__builtin_amdgcn_s_memtime();
        levels += fcur - 1;  // diagnostic build: count expanded list nodes instead of levels
#endif
        const int Fl = min(fcur, kBfsList);
        for (int q0 = 0; q0 < Fl; q0 += kWave) {  // one node per lane, wave-uniform trip count
            const int q = q0 + lane;
            const bool active = q < Fl;
            int wn[RMAX];
            const uint32_t won = expand(active ? (int)lcur[q] : vf, active, wn);
            const int nw = __popc(won);
            const int incl = wave_scan_incl(nw);
            int pos = fnext + incl - nw;
            fnext += __builtin_amdgcn_readlane(incl, kWave - 1);
#pragma unroll
            for (int j = 0; j < RMAX; ++j) {
                if (!((won >> j) & 1u)) continue;
                if (pos < kBfsList) {
                    lnxt[pos] = (uint16_t)wn[j];
                } else {
                    atomicOr((unsigned long long *)&S.nxt[wn[j] >> 6], 1ull << (wn[j] & 63));
                    spill_out = true;
                }
                ++pos;
            }
        }
        if (spill_in) {  // the overflow of the previous level, from its bitmap (rare)
            if (lane == 0) S.lcnt[0] = fnext;
            wave_sync();
            for (int i = lane; i < W; i += kWave) {
                uint64_t bits = S.front[i];
                while (bits) {
                    const int b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    int wn[RMAX];
                    const uint32_t won = expand(i * 64 + b, true, wn);
                    int pos = won ? atomicAdd(&S.lcnt[0], __popc(won)) : 0;
#pragma unroll
                    for (int j = 0; j < RMAX; ++j) {
                        if (!((won >> j) & 1u)) continue;
                        if (pos < kBfsList) {
                            lnxt[pos] = (uint16_t)wn[j];
                        } else {
                            atomicOr((unsigned long long *)&S.nxt[wn[j] >> 6], 1ull << (wn[j] & 63));
                            spill_out = true;
                        }
                        ++pos;
                    }
                }
            }
            wave_sync();
            fnext = S.lcnt[0];
        }
        wave_sync();
#ifdef FC_PHASE_PROF
        if (lane == 0 && S.prof)
            atomicAdd((unsigned long long *)&S.prof[15],
                      (unsigned long long)((int64_t)__builtin_amdgcn_s_memtime() - t_x0));
#endif
        if (__any(merged)) {
            // comp(i) |= labels i touched, symmetric, then transitive closure (<= 4 rounds)
            const uint32_t adj = comp | (lane < 16 ? S.mm[lane] : 0u);
            uint32_t sym = adj;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t aj = (uint32_t)__shfl((int)adj, j);
                if (lane < 16 && ((aj >> lane) & 1u)) sym |= 1u << j;
            }
            comp = lane < 16 ? sym : 0u;
            for (int it = 0; it < 4; ++it) {
                uint32_t nx = comp;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t cj = (uint32_t)__shfl((int)comp, j);
                    if ((comp >> j) & 1u) nx |= cj;
                }
                const bool ch = nx != comp;
                comp = nx;
                if (!__any(ch)) break;
            }
            if (lane < 16) {
                S.mm[lane] = 0;
                S.cm[lane] = comp;
            }
        }
        if ((((uint32_t)__shfl((int)comp, 0)) & all) == all) return true;  // one component
        live = or_reduce(live);
        // a component without a live label is closed: a piece of A - v missing some label
        const bool dead = lane < ns && (comp & live) == 0u;
        if (__any(dead)) return false;
        const bool so = __any(spill_out);
        if (spill_in || so) {
            for (int i = lane; i < W; i += kWave) {
                S.front[i] = S.nxt[i];
                S.nxt[i] = 0;
            }
        }
        spill_in = so;
        fcur = fnext;
        wave_sync();
    }
}

// Workgroup-cooperative form of the multi-source search, for large graphs whose chain has a
// workgroup to itself (one chain per workgroup; SURVEY §5 "one workgroup per chain with a
// cooperative LDS BFS").  Every thread of the workgroup expands frontier nodes; the chain's
// wave issues the search and the other waves wait for it at a barrier (coop_helper_loop).
//
// A node's label byte (label + 1; 0 = unvisited, 0xff = the removed node v) is claimed with
// one LDS compare-and-swap on its dword, so the claim and the label are one atomic step and a
// losing thread reads the winner's label from the swap's result, whatever wave won.  Appends
// go to the next level's list through an LDS counter (overflow to a bitmap); merges and live
// labels collect in LDS masks; after a barrier the chain's wave closes the component masks
// and decides (connected / disconnected / go on), and a second barrier publishes it.
// Control words (ctl, 32 ints): 0 cmd, 1 vf, 2 A, 3 ns, 4 decision, 5 live, 6 merged,
// 7 spill_out, 8 spill_in, 9-10 list lengths, 16-31 source nodes.
enum : int { kCtlCmd = 0, kCtlVf, kCtlA, kCtlNs, kCtlDec, kCtlLive, kCtlMerged, kCtlSpillOut, kCtlSpillIn,
             kCtlLen0, kCtlLen1, kCtlSrc = 16 };

__device__ __forceinline__ void block_sync() { __syncthreads(); }

template <int RMAX>
__device__ bool coop_bfs(const NodeRec<RMAX> *__restrict__ G, const int8_t *a, const BfsScratch &S,
                         int32_t *ctl, int tid, int nthr, int64_t &levels) {
    // every value that steers a barrier is made wave-uniform (readfirstlane), so the compiler
    // never executes a barrier on a masked path
    const int W = S.W;
    const int vf = __builtin_amdgcn_readfirstlane(ctl[kCtlVf]), A = __builtin_amdgcn_readfirstlane(ctl[kCtlA]),
              ns = __builtin_amdgcn_readfirstlane(ctl[kCtlNs]);
    uint8_t *const lab = (uint8_t *)S.lab;
    for (int i = tid; i < S.lab_words; i += nthr) S.lab[i] = 0;
    for (int i = tid; i < W; i += nthr) {
        S.front[i] = 0;
        S.nxt[i] = 0;
    }
    if (tid < 16) {
        S.mm[tid] = 0;
        S.cm[tid] = 1u << tid;
    }
    block_sync();
    if (tid < ns) {
        const int x = ctl[kCtlSrc + tid];
        lab[x] = (uint8_t)(tid + 1);
        S.list[tid] = (uint16_t)x;
    }
    if (tid == 0) {
        lab[vf] = 0xff;
        ctl[kCtlLen0] = ns;
        ctl[kCtlLen1] = 0;
        ctl[kCtlLive] = 0;
        ctl[kCtlMerged] = 0;
        ctl[kCtlSpillOut] = 0;
        ctl[kCtlSpillIn] = 0;
    }
    block_sync();
    const uint32_t all = (uint32_t)((1ull << ns) - 1ull);
    for (int cur = 0;; cur ^= 1) {
        if (tid == 0) ++levels;
        const int fcur = __builtin_amdgcn_readfirstlane(ctl[kCtlLen0 + cur]);
        const bool spill_in = __builtin_amdgcn_readfirstlane(ctl[kCtlSpillIn]) != 0;
        uint16_t *const lcur = S.list + cur * kBfsList, *const lnxt = S.list + (cur ^ 1) * kBfsList;
        uint32_t live = 0;
        bool merged = false, spill = false;
        auto expand = [&](int u) {
            const uint32_t la = (uint32_t)lab[u] - 1u;  // this node's label
            const uint32_t cla = S.cm[la & 15u];
            const NodeRec<RMAX> rr = G[u];
            const uint32_t nbr = (uint32_t)(rr.meta >> kMetaNbrShift) & 0xffffu;
            uint32_t hit = 0;
#pragma unroll
            for (int j = 0; j < RMAX; ++j) {
                if (!((nbr >> j) & 1u)) continue;
                const int w = ring_entry<RMAX>(rr.ring, j);
                if (w == vf || a[w] != A) continue;
                uint32_t *wd = S.lab + (w >> 2);
                const int sh = 8 * (w & 3);
                uint32_t old = *wd, other = 0;
                for (;;) {
                    other = (old >> sh) & 0xffu;
                    if (other) break;
                    const uint32_t prev = atomicCAS(wd, old, old | ((la + 1u) << sh));
                    if (prev == old) break;
                    old = prev;
                }
                if (!other) {  // won: w joins the next level
                    live |= 1u << la;
                    const int pos = atomicAdd(&ctl[kCtlLen0 + (cur ^ 1)], 1);
                    if (pos < kBfsList) {
                        lnxt[pos] = (uint16_t)w;
                    } else {
                        atomicOr((unsigned long long *)&S.nxt[w >> 6], 1ull << (w & 63));
                        spill = true;
                    }
                } else if (other != 0xffu && !((cla >> (other - 1u)) & 1u)) {
                    hit |= 1u << (other - 1u);  // ran into another component
                }
            }
            if (hit) {
                atomicOr(&S.mm[la], hit);
                merged = true;
            }
        };
        const int Fl = min(fcur, kBfsList);
        for (int q = tid; q < Fl; q += nthr) expand((int)lcur[q]);
        if (spill_in) {
            for (int i = tid; i < W; i += nthr) {
                uint64_t bits = S.front[i];
                while (bits) {
                    const int b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    expand(i * 64 + b);
                }
            }
        }
        if (live) atomicOr((uint32_t *)&ctl[kCtlLive], live);
        if (merged) atomicOr(&ctl[kCtlMerged], 1);
        if (spill) atomicOr(&ctl[kCtlSpillOut], 1);
        block_sync();
        if (tid < kWave) {  // the first wave decides
            const int lane = tid;
            uint32_t comp = lane < 16 ? S.cm[lane] : 0u;
            if (ctl[kCtlMerged]) {
                const uint32_t adj = comp | (lane < 16 ? S.mm[lane] : 0u);
                uint32_t sym = adj;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t aj = (uint32_t)__shfl((int)adj, j);
                    if (lane < 16 && ((aj >> lane) & 1u)) sym |= 1u << j;
                }
                comp = lane < 16 ? sym : 0u;
                for (int it = 0; it < 4; ++it) {
                    uint32_t nx = comp;
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const uint32_t cj = (uint32_t)__shfl((int)comp, j);
                        if ((comp >> j) & 1u) nx |= cj;
                    }
                    const bool ch = nx != comp;
                    comp = nx;
                    if (!__any(ch)) break;
                }
                if (lane < 16) {
                    S.mm[lane] = 0;
                    S.cm[lane] = comp;
                }
            }
            const uint32_t lv = (uint32_t)ctl[kCtlLive];
            int dec = 0;
            if ((((uint32_t)__shfl((int)comp, 0)) & all) == all) dec = 1;                  // one component
            else if (__any(lane < ns && (comp & lv) == 0u)) dec = 2;                        // a closed piece
            wave_sync();
            if (lane == 0) {
                ctl[kCtlDec] = dec;
                ctl[kCtlSpillIn] = ctl[kCtlSpillOut];
                ctl[kCtlSpillOut] = 0;
                ctl[kCtlLive] = 0;
                ctl[kCtlMerged] = 0;
                ctl[kCtlLen0 + cur] = 0;  // this level's list is refilled two levels on
            }
        }
        block_sync();
        const int dec = __builtin_amdgcn_readfirstlane(ctl[kCtlDec]);
        if (dec) return dec == 1;
        if (__builtin_amdgcn_readfirstlane(ctl[kCtlSpillIn])) {  // the next level expands the overflow bitmap too
            for (int i = tid; i < W; i += nthr) {
                S.front[i] = S.nxt[i];
                S.nxt[i] = 0;
            }
            block_sync();
        }
    }
}

// The helper waves of a cooperative chain: wait for a search command, take part, repeat
// until the chain's wave sends the exit command (ctl[kCtlCmd] = 0).
template <int RMAX>
__device__ void coop_helper_loop(const NodeRec<RMAX> *__restrict__ G, const int8_t *a, const BfsScratch &S,
                                 int32_t *ctl, int tid, int nthr) {
    int64_t dummy = 0;
    for (;;) {
        block_sync();
        if (__builtin_amdgcn_readfirstlane(ctl[kCtlCmd]) == 0) return;
        (void)coop_bfs<RMAX>(G, a, S, ctl, tid, nthr, dummy);
    }
}

// Register-light single-source form for the k = 2 kernel, where the planar rule decides
// every node of the reference's lattices and the search is the rare fallback: are all
// old-district neighbours (lanes < RMAX hold them in my_target) reached from `start`?
template <int RMAX>
__device__ bool wave_bfs_single(const NodeRec<RMAX> *__restrict__ G, const int8_t *a, const BfsScratch &S,
                                int lane, int vf, int A, int my_target, int start, int64_t &levels) {
    const int W = S.W;
    for (int i = lane; i < W; i += kWave) {
        S.vis[i] = 0;
        S.front[i] = 0;
        S.nxt[i] = 0;
    }
    wave_sync();
    if (lane == 0) {
        S.vis[vf >> 6] |= 1ull << (vf & 63);
        S.vis[start >> 6] |= 1ull << (start & 63);
        S.front[start >> 6] |= 1ull << (start & 63);
    }
    wave_sync();
    for (;;) {
        ++levels;
        for (int i = lane; i < W; i += kWave) {
            uint64_t bits = S.front[i];
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
                    const uint64_t old = atomicOr((unsigned long long *)&S.vis[e >> 6], (unsigned long long)bit);
                    if (!(old & bit)) atomicOr((unsigned long long *)&S.nxt[e >> 6], (unsigned long long)bit);
                }
            }
        }
        wave_sync();
        const bool found = my_target < 0 || ((S.vis[my_target >> 6] >> (my_target & 63)) & 1ull);
        if (__all(found)) return true;
        bool any = false;
        for (int i = lane; i < W; i += kWave) {
            const uint64_t x = S.nxt[i];
            S.front[i] = x;
            S.nxt[i] = 0;
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

// The queued waits' inversion (geom_wait, grid_chain_sec11.py:147-148), out of line: inlined
// into a flip kernel, the f64 log's polynomial constants were hoisted out of the batch loop into
// VGPRs that the whole loop then carried (and spilled); the call runs once per queue drain.
__device__ __attribute__((noinline)) inline int64_t geom_wait_of(uint32_t x0, uint32_t x1, double log1mp) {
    return geom_from(u53(x0, x1), log1mp);
}

}  // namespace dev
}  // namespace fc
