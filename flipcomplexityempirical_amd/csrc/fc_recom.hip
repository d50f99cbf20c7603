// ReCom tree proposal for gfx950: the step the reference builds beside its flip chain
// (grid_chain_sec11.py:328-335, partial(recom, pop_col="population",
// pop_target=ideal_population, epsilon=0.05, node_repeats=1)) under gerrychain 0.2's
// MarkovChain loop [gc-0.2] (Validator re-draws, cut_accept-style acceptance).
//
// One chain per wavefront; the chain's assignment and the spanning-tree working set live
// in LDS.  A proposal:
//   1. picks a cut edge (k-th cut edge in edge-id order: per-lane edge chunks + a wave scan)
//      and merges its two districts M;
//   2. draws a random spanning tree of M: edge weights splitmix64(key + e) >> 32, maximum
//      spanning tree by Boruvka (per-component best edge by LDS atomicMax on
//      weight << 32 | ~e, hooking, pointer jumping);
//   3. roots it at the k-th node of tree degree > 1, orders it by a level-synchronous BFS
//      over the tree and sums subtree populations level by level from the leaves;
//   4. picks the k-th balanced cut (|pop(subtree) - pop_target| < epsilon * pop_target),
//      trying new roots / trees while there is none (node_repeats roots per tree);
//   5. relabels subtree(child) -> parts[0], the rest of M -> parts[1], evaluates the
//      population Validator and the cut_accept test, and applies the accepted state.
// The canonical random stream (recomref.h) makes the trajectory bit-identical to the CPU
// restatement in oracle/recomref.c.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <type_traits>

#include "fc_device.h"
#include "fc_internal.h"
#include "fc_philox.h"

namespace fc {

using namespace dev;

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t mulhi64(uint64_t r, uint64_t n) { return __umul64hi(r, n); }

__device__ __forceinline__ uint32_t word4(const uint4 &w, int t) { return t == 0 ? w.x : t == 1 ? w.y : t == 2 ? w.z : w.w; }

__device__ __forceinline__ int64_t wave_sum64(int64_t x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor((long long)x, off);
    return x;
}

// Index of the k-th set flag over items [0, count) split into per-lane contiguous chunks:
// `flag(i)` is evaluated twice per item of the owning lane (count, then locate).
template <typename F>
__device__ int kth_item(int count, int lane, uint64_t k, F flag, int &total) {
    const int chunk = (count + kWave - 1) / kWave;
    const int lo = min(count, lane * chunk), hi = min(count, lo + chunk);
    int c = 0;
    for (int i = lo; i < hi; ++i) c += flag(i) ? 1 : 0;
    const int incl = wave_scan_incl(c);
    total = __builtin_amdgcn_readlane(incl, kWave - 1);
    const int excl = incl - c;
    int found = -1;
    if ((uint64_t)excl <= k && k < (uint64_t)incl) {
        int r = (int)(k - (uint64_t)excl);
        for (int i = lo; i < hi; ++i)
            if (flag(i)) {
                if (r == 0) { found = i; break; }
                --r;
            }
    }
    const uint64_t own = __ballot(found >= 0);
    return own ? __builtin_amdgcn_readlane(found, __builtin_ctzll(own)) : -1;
}

#ifndef FC_RECOM_SCAN_U
#define FC_RECOM_SCAN_U 2
#endif
#ifndef FC_RECOM_JUMP_U
#define FC_RECOM_JUMP_U 4
#endif
constexpr int kScanU8 = FC_RECOM_SCAN_U;  // Boruvka scan: nodes per lane in flight (RMAX = 8; 2 for 16)
constexpr int kJumpU = FC_RECOM_JUMP_U;  // pointer jumping: nodes per lane in flight

template <int RMAX>
__global__ __launch_bounds__(256) void recom_kernel(RecomParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = (int)(threadIdx.x & 63u);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int c = (int)blockIdx.x * (int)(blockDim.x >> 6) + wv;
    if (c >= p.n_chains) return;
    const int n = p.n, E = p.n_edges;
    const int npad = (n + 15) & ~15;
    unsigned char *base = smem + (size_t)wv * p.chain_lds_bytes;
    // LDS layout (recom_lds_bytes: 14 B per node for RMAX = 8, 15 for 16; the kernel is
    // latency-bound, so the chains a CU holds set its rate):
    //   [0, 8 npad)   Boruvka keys; then the tree's CSR [0, 6 npad) and the BFS parents
    //                 [6 npad, 8 npad); then subtree populations [0, 4 npad) (sign bit: subset mark)
    //   comp          component; then level starts
    //   order         hook targets; then BFS order
    //   tadj          tree edges (bit k: neighbour row entry k)
    //   a             assignment
    using TAdj = typename std::conditional<RMAX == 8, uint8_t, uint16_t>::type;
    uint64_t *best = (uint64_t *)base;
    int32_t *spop = (int32_t *)best;
    int16_t *par = (int16_t *)(base + 6 * (size_t)npad);
    int16_t *comp = (int16_t *)(best + npad);
    int16_t *order = comp + npad;
    TAdj *tadj = (TAdj *)(order + npad);
    int8_t *a = (int8_t *)(tadj + npad);
    // tree-edge bits by 32-bit LDS atomics on the word holding the node's entry
    auto tadj_or = [&](int x, uint32_t bits) {
        constexpr int kPer = 4 / (int)sizeof(TAdj);
        atomicOr((uint32_t *)tadj + x / kPer, bits << (8 * (int)sizeof(TAdj) * (x % kPer)));
    };
    const NodeRec<RMAX> *__restrict__ G = (const NodeRec<RMAX> *)p.graph;
    constexpr int kScanU = RMAX == 8 ? kScanU8 : 2;
    const uint4 *__restrict__ NB = (const uint4 *)p.nbe;  // neighbour rows, nq vectors each
    const int nq = p.nb_d >> 2;

    {
        const uint4 *ga = (const uint4 *)(p.assign + (size_t)c * npad);
        for (int i = lane; i < npad / 16; i += kWave) ((uint4 *)a)[i] = ga[i];
    }
    ChainScalars *scp = p.sc + c;
    uint64_t draw = scp->draw;
    const uint64_t draw_cap = draw + (uint64_t)p.max_draws;
    int64_t steps = scp->steps, proposals = scp->proposals, accepted = scp->accepted, inv_pop = scp->inv_pop;
    int64_t sum_cut = scp->sum_cut, sum_nb = scp->sum_nb, attempts_tot = scp->bfs_calls, trees_tot = scp->bfs_levels;
    int64_t trace_len = scp->trace_len;
    int cut = scp->cut, nb = scp->nb;
    const int pop_lo = scp->pop_lo, pop_hi = scp->pop_hi;  // this chain's bounds (chain_pop_bounds)
    int stuck = 0;
    const uint32_t gid = p.chain_id_offset + (uint32_t)c;
    const bool trace_on = p.trace && c < p.trace_chains;
    int64_t rem = p.n_steps;
#ifdef FC_PHASE_PROF
    // phase cycles (diagnostic build; tools/prof_recom_report.py): 0 loop, 1 edge + popM,
    // 2 spanning trees, 3 Boruvka scans, 4 hooks, 5 pointer jumps, 6 root choice, 7 BFS order,
    // 8 subtree sums, 9 cut choice, 10 subset marks, 11 step 5; counts: 12 Boruvka rounds,
    // 13 BFS levels, 14 trees, 15 pointer-jump passes, 16 proposals, 17 attempts
    int64_t *prof_acc = (int64_t *)(base + p.chain_lds_bytes - kProfSlots * 8);
    if (lane < kProfSlots) prof_acc[lane] = 0;
#endif
    wave_sync();
    FC_STAMP(t_loop0);

    while (rem > 0) {
        if (draw >= draw_cap) {
            stuck = 1;
            break;
        }
        const uint64_t d = draw++;
        FC_STAMP(t_s0);
        FC_PROF(16, 1);
        const Words4 w = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), gid, 0u, p.seed_lo, p.seed_hi);
        // ---- 1. recom: edge = random.choice(tuple(partition["cut_edges"])) ----------------
        int tot = 0;
        const int e_sel = kth_item(E, lane, mulhi64(((uint64_t)w.x3 << 32) | w.x0, (uint64_t)cut),
                                   [&](int e) { return a[p.eu[e]] != a[p.ev[e]]; }, tot);
        const int d0 = a[p.eu[e_sel]], d1 = a[p.ev[e_sel]];
        auto inM = [&](int x) { return a[x] == d0 || a[x] == d1; };
        int64_t pm = 0;
        for (int x = lane; x < n; x += kWave) pm += inM(x) ? G[x].pop : 0;
        const int64_t popM = wave_sum64(pm);
        ++proposals;
        FC_STAMP(t_s1);
        FC_PROF(1, t_s1 - t_s0);
        // ---- 2-4. bipartition_tree ----------------------------------------------------
        int tree = -1, root = -1, child = -1, attempts = 0;
        int64_t p0 = 0;  // subtree(child)'s population
        for (int t = 0; t < p.max_attempts; ++t) {
            ++attempts;
            FC_PROF(17, 1);
            if (t / p.node_repeats != tree) {
                tree = t / p.node_repeats;
                ++trees_tot;
                FC_STAMP(t_tr0);
                FC_PROF(14, 1);
                const Words4 kw = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), gid, 0x80000000u | (uint32_t)tree,
                                                p.seed_lo, p.seed_hi);
                const uint64_t key = ((uint64_t)kw.x1 << 32) | kw.x0;
                // Boruvka maximum spanning tree of M (weights with edge-id tie break).  A root's
                // hook target goes to the high half of its key word (the low half, ~edge id, still
                // tells a mutual hook); order[] holds the active nodes -- those with a neighbour in
                // another component at the last scan (components only merge, so a node without one
                // never has one again), kept in node order
                auto tgt = [&](int x) -> int { return ((const int32_t *)best)[2 * x + 1]; };
                auto set_tgt = [&](int x, int r) { ((int32_t *)best)[2 * x + 1] = r; };
                int m_act = 0;
                for (int x0 = 0; x0 < npad; x0 += kWave) {
                    const int x = x0 + lane;
                    const bool in = x < n && inM(x);
                    if (x < npad) {  // (npad is a multiple of 16 only)
                        comp[x] = in ? (int16_t)x : (int16_t)-1;
                        tadj[x] = 0;
                    }
                    const int incl = wave_scan_incl(in ? 1 : 0);
                    if (in) order[m_act + incl - 1] = (int16_t)x;
                    m_act += __builtin_amdgcn_readlane(incl, kWave - 1);
                }
                wave_sync();
                for (;;) {
                    FC_STAMP(t_b0);
                    FC_PROF(12, 1);
                    for (int x = lane; x < n; x += kWave) best[x] = 0;
                    wave_sync();
                    // kScanU active nodes per lane at a time: their neighbour rows (nb_d / 4
                    // vector loads: ids and edge ids) and the neighbours' components, every read
                    // issued before the first use; the keys are then formed by selects, without a
                    // branch per neighbour (a row holds the neighbours only: a ring's other cells
                    // cost no weight); the nodes still active are written back in order
                    int m_next = 0;
                    for (int i0 = 0; i0 < m_act; i0 += kScanU * kWave) {
                        int xs[kScanU], cxs[kScanU];
                        uint4 nw[kScanU][RMAX / 4];
#pragma unroll
                        for (int u = 0; u < kScanU; ++u) {
                            const int i = i0 + u * kWave + lane;
                            xs[u] = i < m_act ? (int)order[i] : -1;
                        }
#pragma unroll
                        for (int u = 0; u < kScanU; ++u) {
                            const int xc = xs[u] >= 0 ? xs[u] : 0;
                            cxs[u] = xs[u] >= 0 ? (int)comp[xc] : -1;
#pragma unroll
                            for (int q = 0; q < RMAX / 4; ++q)
                                nw[u][q] = q < nq ? NB[(size_t)xc * nq + q] : make_uint4(~0u, ~0u, ~0u, ~0u);
                        }
                        int cyv[kScanU][RMAX];
#pragma unroll
                        for (int u = 0; u < kScanU; ++u)
#pragma unroll
                            for (int j = 0; j < RMAX; ++j) {
                                const uint32_t nb = word4(nw[u][j >> 2], j & 3) & 0xffffu;
                                cyv[u][j] = nb != 0xffffu ? (int)comp[nb] : -1;
                            }
#pragma unroll
                        for (int u = 0; u < kScanU; ++u)
#pragma unroll
                            for (int j = 0; j < RMAX; ++j) asm volatile("" : "+v"(cyv[u][j]));
#pragma unroll
                        for (int u = 0; u < kScanU; ++u) {
                            const int cx = cxs[u];
                            uint64_t bk = 0;
                            bool any = false;
#pragma unroll
                            for (int q = 0; q < RMAX / 4; ++q) {
                                if (q >= nq) break;
#pragma unroll
                                for (int t4 = 0; t4 < 4; ++t4) {
                                    const int j = 4 * q + t4;
                                    const uint32_t e = word4(nw[u][q], t4) >> 16;
                                    const bool use = cx >= 0 && cyv[u][j] >= 0 && cyv[u][j] != cx;
                                    any |= use;
                                    const uint64_t kk = ((splitmix64(key + (uint64_t)e) >> 32) << 32) | (0xffffffffu - e);
                                    bk = (use && kk > bk) ? kk : bk;
                                }
                            }
                            if (bk) atomicMax((unsigned long long *)&best[cx], (unsigned long long)bk);
                            // (positions <= the entries this iteration read: in-place is safe)
                            const int incl = wave_scan_incl(any ? 1 : 0);
                            if (any) order[m_next + incl - 1] = (int16_t)xs[u];
                            m_next += __builtin_amdgcn_readlane(incl, kWave - 1);
                        }
                    }
                    m_act = m_next;
                    wave_sync();
                    FC_STAMP(t_b1);
                    FC_PROF(3, t_b1 - t_b0);
                    bool hooked = false;
                    for (int x0 = lane; x0 < n; x0 += kJumpU * kWave) {  // kJumpU roots' reads in flight
                        bool rt[kJumpU];
                        uint64_t bxs[kJumpU];
                        int es[kJumpU], us[kJumpU], vs[kJumpU];
                        uint32_t kss[kJumpU];
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) {
                            const int x = x0 + u * kWave;
                            rt[u] = x < n && comp[x] == x;
                        }
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) bxs[u] = rt[u] ? best[x0 + u * kWave] : 0ull;
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) {
                            es[u] = bxs[u] ? (int)(0xffffffffu - (uint32_t)bxs[u]) : 0;
                            us[u] = p.eu[es[u]];
                            vs[u] = p.ev[es[u]];
                            kss[u] = p.eslot[es[u]];
                        }
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) {
                            if (!rt[u]) continue;
                            const int x = x0 + u * kWave;
                            if (bxs[u] == 0) {  // no edge out (M's last component)
                                set_tgt(x, x);
                                continue;
                            }
                            const int other = comp[us[u]] == x ? comp[vs[u]] : comp[us[u]];
                            // hook (both roots chose this edge: the smaller id stays a root)
                            set_tgt(x, ((uint32_t)best[other] == (uint32_t)bxs[u] && x < other) ? x : other);
                            hooked = true;
                            // record the tree edge on both endpoints (the other end's index in the row)
                            tadj_or(us[u], 1u << (kss[u] & 0xffu));
                            tadj_or(vs[u], 1u << (kss[u] >> 8));
                        }
                    }
                    wave_sync();
                    FC_STAMP(t_b2);
                    FC_PROF(4, t_b2 - t_b1);
                    if (!__any(hooked)) break;
                    // the new roots: every old root follows its hook targets to the one hooked onto
                    // itself (distinct keys: the only cycles are mutual hooks, broken by id), then
                    // every node takes its old root's new root -- two passes, where pointer jumping
                    // over all nodes took about four per round
                    FC_PROF(15, 1);
                    for (int x0 = lane; x0 < n; x0 += kJumpU * kWave) {
                        bool rt[kJumpU];
                        int rs[kJumpU];
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) rt[u] = x0 + u * kWave < n && comp[x0 + u * kWave] == x0 + u * kWave;
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) rs[u] = rt[u] ? tgt(x0 + u * kWave) : 0;
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) {
                            if (!rt[u]) continue;
                            int r = rs[u];
                            for (int r2 = tgt(r); r2 != r; r2 = tgt(r)) r = r2;
                            set_tgt(x0 + u * kWave, r);
                        }
                    }
                    wave_sync();
                    for (int x0 = lane; x0 < n; x0 += kJumpU * kWave) {  // kJumpU reads in flight
                        int cxs[kJumpU], rts[kJumpU];
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) cxs[u] = x0 + u * kWave < n ? (int)comp[x0 + u * kWave] : -1;
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u) rts[u] = cxs[u] >= 0 ? tgt(cxs[u]) : -1;
#pragma unroll
                        for (int u = 0; u < kJumpU; ++u)
                            if (rts[u] != cxs[u]) comp[x0 + u * kWave] = (int16_t)rts[u];
                    }
                    wave_sync();
                    FC_STAMP(t_b3);
                    FC_PROF(5, t_b3 - t_b2);
                }
                FC_STAMP(t_tr1);
                FC_PROF(2, t_tr1 - t_tr0);
            }
            FC_STAMP(t_r0);
            const Words4 cw = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), gid, 0x40000000u | (uint32_t)t,
                                            p.seed_lo, p.seed_hi);
            // root = choice([x for x in h if h.degree(x) > 1]), ascending node id
            int nroot = 0;
            auto is_inner = [&](int x) { return inM(x) && __popc((uint32_t)tadj[x]) > 1; };
            int nr_tot = 0;
            {
                // count first (the choice multiplies by the count)
                const int chunk = (n + kWave - 1) / kWave;
                const int lo = min(n, lane * chunk), hi = min(n, lo + chunk);
                int cc = 0;
                for (int i = lo; i < hi; ++i) cc += is_inner(i) ? 1 : 0;
                nr_tot = __builtin_amdgcn_readlane(wave_scan_incl(cc), kWave - 1);
            }
            if (nr_tot == 0) continue;
            root = kth_item(n, lane, mulhi64(((uint64_t)cw.x1 << 32) | cw.x0, (uint64_t)nr_tot), is_inner, nroot);
            FC_STAMP(t_r1);
            FC_PROF(6, t_r1 - t_r0);
            // the tree's adjacency as a CSR in the Boruvka keys' space (dead until the subtree sums):
            // offsets by a wave scan of the tree degrees, neighbour ids from the ring slots
            int16_t *toff = (int16_t *)best;       // [n + 1]
            int16_t *tnb = toff + ((n + 2) & ~1);  // [2 (|M| - 1)]
            {
                int ob = 0;
                for (int x0 = 0; x0 < n; x0 += kWave) {
                    const int x = x0 + lane;
                    const int dg = x < n ? __popc((uint32_t)tadj[x]) : 0;
                    const int incl = wave_scan_incl(dg);
                    if (x < n) toff[x] = (int16_t)(ob + incl - dg);
                    ob += __builtin_amdgcn_readlane(incl, kWave - 1);
                }
                if (lane == 0) toff[n] = (int16_t)ob;
                for (int x0 = lane; x0 < n; x0 += kScanU * kWave) {
                    uint32_t tbs[kScanU];
                    int os[kScanU];
                    uint4 nw[kScanU][RMAX / 4];
#pragma unroll
                    for (int u = 0; u < kScanU; ++u) {
                        const int x = x0 + u * kWave;
                        const int xc = x < n ? x : x0;
                        tbs[u] = x < n ? (uint32_t)tadj[x] : 0u;
                        os[u] = toff[xc];
#pragma unroll
                        for (int q = 0; q < RMAX / 4; ++q)
                            nw[u][q] = q < nq ? NB[(size_t)xc * nq + q] : make_uint4(~0u, ~0u, ~0u, ~0u);
                    }
#pragma unroll
                    for (int u = 0; u < kScanU; ++u) {
                        int o = os[u];
#pragma unroll
                        for (int j = 0; j < RMAX; ++j)
                            if ((tbs[u] >> j) & 1u) tnb[o++] = (int16_t)(word4(nw[u][j >> 2], j & 3) & 0xffffu);
                    }
                }
            }
            wave_sync();
            // BFS order over the tree, a level at a time; children placed by a wave scan of the
            // child counts; level starts in comp[]
            if (lane == 0) {
                order[0] = (int16_t)root;
                par[root] = -1;
                comp[0] = 0;
                comp[1] = 1;
            }
            wave_sync();
            int L = 0;
            {
                int ls = 0, le = 1;
                while (ls < le) {
                    int nb_end = le;
                    for (int i0 = ls; i0 < le; i0 += kWave) {
                        const int i = i0 + lane;
                        int x = 0, o0 = 0, o1 = 0, px = -1;
                        if (i < le) {
                            x = order[i];
                            o0 = toff[x];
                            o1 = toff[x + 1];
                            px = par[x];
                        }
                        const int nch = o1 - o0 - (px >= 0 ? 1 : 0);
                        const int incl = wave_scan_incl(nch);
                        int pos = nb_end + incl - nch;
                        nb_end += __builtin_amdgcn_readlane(incl, kWave - 1);
                        // every child read issued at once (entries past o1 stay inside the keys'
                        // space: tnb has room for 4 npad - n - 2 >= 2 n + RMAX of them)
                        int yv[RMAX];
#pragma unroll
                        for (int j = 0; j < RMAX; ++j) yv[j] = tnb[o0 + j];
#pragma unroll
                        for (int j = 0; j < RMAX; ++j) asm volatile("" : "+v"(yv[j]));
#pragma unroll
                        for (int j = 0; j < RMAX; ++j) {
                            if (o0 + j >= o1 || yv[j] == px) continue;
                            order[pos++] = (int16_t)yv[j];
                            par[yv[j]] = (int16_t)x;
                        }
                    }
                    wave_sync();
                    ++L;
                    ls = le;
                    le = nb_end;
                    if (lane == 0) comp[L + 1] = (int16_t)le;
                }
            }
            wave_sync();
            FC_STAMP(t_r2);
            FC_PROF(7, t_r2 - t_r1);
            FC_PROF(13, L);
            // subtree populations, leaves upward
            const int nM = comp[L];
            for (int i = lane; i < nM; i += kWave) {
                const int x = order[i];
                spop[x] = G[x].pop;
            }
            wave_sync();
            for (int l = L - 1; l >= 1; --l) {
                for (int i = comp[l] + lane; i < comp[l + 1]; i += kWave) {
                    const int x = order[i];
                    atomicAdd(&spop[par[x]], spop[x]);
                }
                wave_sync();
            }
            FC_STAMP(t_r3);
            FC_PROF(8, t_r3 - t_r2);
            // cuts: |pop(subtree(x)) - ideal| < epsilon * ideal (has_ideal_population)
            auto is_cut = [&](int x) {
                return inM(x) && x != root && fabs((double)spop[x] - p.pop_target) < p.epsilon * p.pop_target;
            };
            int ncut = 0;
            {
                const int chunk = (n + kWave - 1) / kWave;
                const int lo = min(n, lane * chunk), hi = min(n, lo + chunk);
                int cc = 0;
                for (int i = lo; i < hi; ++i) cc += is_cut(i) ? 1 : 0;
                ncut = __builtin_amdgcn_readlane(wave_scan_incl(cc), kWave - 1);
            }
            if (ncut == 0) continue;
            int dummy = 0;
            child = kth_item(n, lane, mulhi64(((uint64_t)cw.x3 << 32) | cw.x2, (uint64_t)ncut), is_cut, dummy);
            FC_STAMP(t_r4);
            FC_PROF(9, t_r4 - t_r3);
            // subset = subtree(child): marks flow down the BFS levels
            p0 = spop[child];
            if (lane == 0) spop[child] |= (int32_t)0x80000000u;
            wave_sync();
            for (int l = 1; l < L; ++l) {
                for (int i = comp[l] + lane; i < comp[l + 1]; i += kWave) {
                    const int x = order[i];
                    if (spop[par[x]] < 0) spop[x] |= (int32_t)0x80000000u;
                }
                wave_sync();
            }
            FC_STAMP(t_r5);
            FC_PROF(10, t_r5 - t_r4);
            break;
        }
        attempts_tot += attempts;
        if (child < 0) {
            stuck = 1;
            break;
        }
        // ---- 5. the proposed state: subtree(child) -> parts[0], rest of M -> parts[1] --------
        FC_STAMP(t_5a);
        auto na = [&](int x) -> int { return inM(x) ? (spop[x] < 0 ? d0 : d1) : a[x]; };
        const int64_t p1 = popM - p0;
        int flags;
        if (p0 < pop_lo || p0 > pop_hi || p1 < pop_lo || p1 > pop_hi) {
            ++inv_pop;
            flags = 8;
        } else {
            ++steps;
            --rem;
            flags = 1;
            // one pass over the nodes' neighbour rows: |cut'| (every cut edge seen from both
            // ends) and |B'| (nodes with a neighbour in another district)
            int cc = 0, bb = 0;
            for (int x0 = lane; x0 < n; x0 += kJumpU * kWave) {
                uint4 nw[kJumpU][RMAX / 4];
#pragma unroll
                for (int u = 0; u < kJumpU; ++u) {
                    const int xc = x0 + u * kWave < n ? x0 + u * kWave : x0;
#pragma unroll
                    for (int q = 0; q < RMAX / 4; ++q)
                        nw[u][q] = q < nq ? NB[(size_t)xc * nq + q] : make_uint4(~0u, ~0u, ~0u, ~0u);
                }
#pragma unroll
                for (int u = 0; u < kJumpU; ++u) {
                    if (x0 + u * kWave >= n) break;
                    const int ax = na(x0 + u * kWave);
                    int dn = 0;
#pragma unroll
                    for (int j = 0; j < RMAX; ++j) {
                        const uint32_t y = word4(nw[u][j >> 2], j & 3) & 0xffffu;
                        dn += (y != 0xffffu && na((int)y) != ax) ? 1 : 0;
                    }
                    cc += dn;
                    bb += dn > 0 ? 1 : 0;
                }
            }
            const int cut_new = (int)(wave_sum64(cc) / 2);
            // cut_accept: random() < base ** (cut - cut'), table over cut - cut' in [-E, E]
            if (mant53(w.x1, w.x2) < p.accept_thresh[cut - cut_new + E]) {
                flags |= 2;
                ++accepted;
                nb = (int)wave_sum64(bb);
                wave_sync();
                for (int x = lane; x < n; x += kWave) a[x] = (int8_t)na(x);
                cut = cut_new;
            }
            sum_cut += cut;
            sum_nb += nb;
        }
        wave_sync();
        if (trace_on && lane == 0 && trace_len < p.trace_cap) {
            fc_recom_record &rr = p.trace[(size_t)c * p.trace_cap + trace_len];
            rr.draw = (int64_t)d;
            rr.edge = e_sel;
            rr.root = root;
            rr.child = child;
            rr.attempts = attempts;
            rr.flags = flags;
            rr.cut = cut;
        }
        if (trace_on) ++trace_len;
        wave_sync();
        FC_STAMP(t_5b);
        FC_PROF(11, t_5b - t_5a);
    }
    FC_STAMP(t_loop1);
    FC_PROF(0, t_loop1 - t_loop0);
#ifdef FC_PHASE_PROF
    wave_sync();
    if (lane == 0)
        for (int i = 0; i < kProfSlots; ++i) p.prof[(size_t)c * kProfSlots + i] = prof_acc[i];
#endif

    // ---- write back ---------------------------------------------------------------------
    {
        uint4 *ga = (uint4 *)(p.assign + (size_t)c * npad);
        for (int i = lane; i < npad / 16; i += kWave) ga[i] = ((const uint4 *)a)[i];
    }
    if (lane == 0) {
        scp->draw = draw;
        scp->steps = steps;
        scp->proposals = proposals;
        scp->accepted = accepted;
        scp->inv_pop = inv_pop;
        scp->sum_cut = sum_cut;
        scp->sum_nb = sum_nb;
        scp->bfs_calls = attempts_tot;
        scp->bfs_levels = trees_tot;
        scp->trace_len = trace_len;
        scp->cut = cut;
        scp->nb = nb;
        scp->stuck = stuck;
    }
}

}  // namespace

int launch_recom(const RecomParams &p, int ring_max, void *stream, char *name, size_t name_cap) {
    const int wpb = waves_per_block(p.chain_lds_bytes);
    const int blocks = (p.n_chains + wpb - 1) / wpb;
    const size_t lds = (size_t)p.chain_lds_bytes * wpb;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(blocks), block(kWave * wpb);
#define FC_LAUNCH_R(R)                                                                                       \
    do {                                                                                                     \
        if (lds > 65536)                                                                                     \
            (void)hipFuncSetAttribute((const void *)recom_kernel<R>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                      (int)lds);                                                            \
        if (name) snprintf(name, name_cap, "fc::recom_kernel<%d>", R);                                         \
        hipLaunchKernelGGL((recom_kernel<R>), grid, block, lds, s, p);                                        \
    } while (0)
    if (ring_max == 8) FC_LAUNCH_R(8);
    else if (ring_max == 16) FC_LAUNCH_R(16);
    else return (int)hipErrorInvalidValue;
#undef FC_LAUNCH_R
    return (int)hipGetLastError();
}

}  // namespace fc
