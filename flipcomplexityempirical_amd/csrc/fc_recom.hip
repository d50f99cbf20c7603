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
    uint64_t *best = (uint64_t *)base;                    // [npad] Boruvka best key; then int32 spop
    int32_t *spop = (int32_t *)best;
    uint32_t *tadj = (uint32_t *)(best + npad);          // [npad] tree slots (bits 0-15), subset mark (31)
    int16_t *comp = (int16_t *)(tadj + npad);            // [npad] component; then level starts
    int16_t *order = comp + npad;                        // [npad] hook targets; then BFS order
    int16_t *par = order + npad;                         // [npad]
    int8_t *a = (int8_t *)(par + npad);                  // [npad]
    int32_t *cnt = (int32_t *)(a + npad);                // [4] counters
    const NodeRec<RMAX> *__restrict__ G = (const NodeRec<RMAX> *)p.graph;

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
    wave_sync();

    while (rem > 0) {
        if (draw >= draw_cap) {
            stuck = 1;
            break;
        }
        const uint64_t d = draw++;
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
        // ---- 2-4. bipartition_tree ----------------------------------------------------
        int tree = -1, root = -1, child = -1, attempts = 0;
        for (int t = 0; t < p.max_attempts; ++t) {
            ++attempts;
            if (t / p.node_repeats != tree) {
                tree = t / p.node_repeats;
                ++trees_tot;
                const Words4 kw = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), gid, 0x80000000u | (uint32_t)tree,
                                                p.seed_lo, p.seed_hi);
                const uint64_t key = ((uint64_t)kw.x1 << 32) | kw.x0;
                // Boruvka maximum spanning tree of M (weights with edge-id tie break)
                for (int x = lane; x < npad; x += kWave) {
                    comp[x] = (x < n && inM(x)) ? (int16_t)x : (int16_t)-1;
                    tadj[x] = 0;
                }
                wave_sync();
                for (;;) {
                    for (int x = lane; x < n; x += kWave) best[x] = 0;
                    wave_sync();
                    for (int x = lane; x < n; x += kWave) {
                        const int cx = comp[x];
                        if (cx < 0) continue;
                        const NodeRec<RMAX> r = G[x];
                        // the node's ring edge ids (static, RMAX / 4 vector loads) and its ring
                        // cells' components, every read issued before the first use (one at a time
                        // behind each neighbour test before: a dependent L2 and LDS round trip per
                        // edge); the keys are then formed by selects, without a branch per cell
                        int4 er[RMAX / 4];
                        const int4 *rp = (const int4 *)(p.ring_eid + (size_t)x * RMAX);
#pragma unroll
                        for (int q = 0; q < RMAX / 4; ++q) er[q] = rp[q];
                        const uint32_t nbr = (uint32_t)(r.meta >> kMetaNbrShift) & 0xffffu;
                        int cyv[RMAX];
#pragma unroll
                        for (int j = 0; j < RMAX; ++j) cyv[j] = comp[ring_entry<RMAX>(r.ring, j)];
#pragma unroll
                        for (int j = 0; j < RMAX; ++j) asm volatile("" : "+v"(cyv[j]));
                        uint64_t bk = 0;
#pragma unroll
                        for (int j = 0; j < RMAX; ++j) {
                            const int4 eq = er[j >> 2];
                            const int ej = (j & 3) == 0 ? eq.x : (j & 3) == 1 ? eq.y : (j & 3) == 2 ? eq.z : eq.w;
                            const bool use = ((nbr >> j) & 1u) && cyv[j] >= 0 && cyv[j] != cx;
                            const uint32_t e = (uint32_t)ej;
                            const uint64_t kk = ((splitmix64(key + (uint64_t)e) >> 32) << 32) | (0xffffffffu - e);
                            bk = (use && kk > bk) ? kk : bk;
                        }
                        if (bk) atomicMax((unsigned long long *)&best[cx], (unsigned long long)bk);
                    }
                    wave_sync();
                    bool hooked = false;
                    for (int x = lane; x < n; x += kWave) {
                        if (comp[x] != x || best[x] == 0) continue;
                        const uint64_t bx = best[x];
                        const int e = (int)(0xffffffffu - (uint32_t)bx);
                        const int u = p.eu[e], v = p.ev[e];
                        const int other = comp[u] == x ? comp[v] : comp[u];
                        order[x] = (best[other] == bx && x < other) ? (int16_t)x : (int16_t)other;  // hook
                        hooked = true;
                        // record the tree edge on both endpoints (ring slot of the other end)
                        const NodeRec<RMAX> ru = G[u], rv = G[v];
                        uint32_t su = 0, sv = 0;
#pragma unroll
                        for (int j = 0; j < RMAX; ++j) {
                            su |= (uint32_t)(ring_entry<RMAX>(ru.ring, j) == v && ((ru.meta >> (kMetaNbrShift + j)) & 1u)) << j;
                            sv |= (uint32_t)(ring_entry<RMAX>(rv.ring, j) == u && ((rv.meta >> (kMetaNbrShift + j)) & 1u)) << j;
                        }
                        atomicOr(&tadj[u], su);
                        atomicOr(&tadj[v], sv);
                    }
                    wave_sync();
                    if (!__any(hooked)) break;
                    for (int x = lane; x < n; x += kWave)
                        if (comp[x] == x && best[x] != 0) comp[x] = order[x];
                    wave_sync();
                    for (;;) {  // pointer jumping to the new roots
                        bool ch = false;
                        for (int x = lane; x < n; x += kWave) {
                            const int cx = comp[x];
                            if (cx < 0) continue;
                            const int cc = comp[cx];
                            if (cc != cx) {
                                comp[x] = (int16_t)cc;
                                ch = true;
                            }
                        }
                        wave_sync();
                        if (!__any(ch)) break;
                    }
                }
            }
            const Words4 cw = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), gid, 0x40000000u | (uint32_t)t,
                                            p.seed_lo, p.seed_hi);
            // root = choice([x for x in h if h.degree(x) > 1]), ascending node id
            int nroot = 0;
            auto is_inner = [&](int x) { return inM(x) && __popc(tadj[x] & 0xffffu) > 1; };
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
            // BFS order over the tree; level starts in comp[]
            if (lane == 0) {
                order[0] = (int16_t)root;
                par[root] = -1;
                cnt[0] = 1;
                comp[0] = 0;
                comp[1] = 1;
            }
            wave_sync();
            int L = 0;
            for (;;) {
                const int ls = comp[L], le = comp[L + 1];
                if (ls == le) break;
                for (int i = ls + lane; i < le; i += kWave) {
                    const int x = order[i];
                    const NodeRec<RMAX> r = G[x];
                    const uint32_t tb = tadj[x] & 0xffffu;
#pragma unroll
                    for (int j = 0; j < RMAX; ++j) {
                        if (!((tb >> j) & 1u)) continue;
                        const int y = ring_entry<RMAX>(r.ring, j);
                        if (y == par[x]) continue;
                        const int pos = atomicAdd(&cnt[0], 1);
                        order[pos] = (int16_t)y;
                        par[y] = (int16_t)x;
                    }
                }
                wave_sync();
                ++L;
                if (lane == 0) comp[L + 1] = (int16_t)cnt[0];
                wave_sync();
            }
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
            // subset = subtree(child): marks flow down the BFS levels
            if (lane == 0) atomicOr(&tadj[child], 0x80000000u);
            wave_sync();
            for (int l = 1; l < L; ++l) {
                for (int i = comp[l] + lane; i < comp[l + 1]; i += kWave) {
                    const int x = order[i];
                    if (tadj[par[x]] & 0x80000000u) atomicOr(&tadj[x], 0x80000000u);
                }
                wave_sync();
            }
            break;
        }
        attempts_tot += attempts;
        if (child < 0) {
            stuck = 1;
            break;
        }
        // ---- 5. the proposed state: subtree(child) -> parts[0], rest of M -> parts[1] --------
        auto na = [&](int x) -> int { return inM(x) ? ((tadj[x] & 0x80000000u) ? d0 : d1) : a[x]; };
        int cc = 0;
        for (int e = lane; e < E; e += kWave) cc += na(p.eu[e]) != na(p.ev[e]);
        const int cut_new = (int)wave_sum64(cc);
        const int64_t p0 = spop[child], p1 = popM - p0;
        int flags;
        if (p0 < pop_lo || p0 > pop_hi || p1 < pop_lo || p1 > pop_hi) {
            ++inv_pop;
            flags = 8;
        } else {
            ++steps;
            --rem;
            flags = 1;
            // cut_accept: random() < base ** (cut - cut'), table over cut - cut' in [-E, E]
            if (mant53(w.x1, w.x2) < p.accept_thresh[cut - cut_new + E]) {
                flags |= 2;
                ++accepted;
                int bb = 0;
                for (int x = lane; x < n; x += kWave) {
                    const NodeRec<RMAX> r = G[x];
                    const uint32_t nbr = (uint32_t)(r.meta >> kMetaNbrShift) & 0xffffu;
                    const int ax = na(x);
                    int f = 0;
#pragma unroll
                    for (int j = 0; j < RMAX; ++j)
                        if ((nbr >> j) & 1u) f |= na(ring_entry<RMAX>(r.ring, j)) != ax;
                    bb += f;
                }
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
        for (int x = lane; x < npad; x += kWave) tadj[x] &= 0x7fffffffu;
        wave_sync();
    }

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
