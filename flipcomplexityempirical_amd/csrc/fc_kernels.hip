// Flip-walk kernels for gfx950 (MI355X).
//
// One chain per wavefront.  The chain's state (int8 district per node, uint8 count of
// foreign neighbours per node, its acceptance-threshold table and BFS bitmaps) lives in
// LDS; the graph (one 32/48-byte record per node: meta, population, packed int16 link ring)
// is shared by all chains and read through L1/L2.
//
// A wave advances its chain in batches of 64 consecutive draws, one per lane:
//   1. every lane evaluates its draw against the current state -- node by an exact
//      Lemire map of the Philox word, boundary membership, the local contiguity test on
//      the link ring, the population bound and the Metropolis threshold;
//   2. a wave-uniform commit loop walks the lanes in draw order exactly as the reference's
//      MarkovChain.__next__ would ([gc-0.2], used grid_chain_sec11.py:340-342,366):
//      invalid proposals are skipped, rejected valid ones are steps that re-yield the
//      state, and each accepted one is applied (a[v], populations, cut, boundary count);
//      lanes whose ring an applied flip touched are re-drawn in the next batch, so the
//      trajectory is bit-identical to a one-draw-at-a-time chain;
//   3. the per-yield driver diagnostics (grid_chain_sec11.py:366-402) are accumulated
//      lane-parallel from the committed masks.
#include <hip/hip_runtime.h>

#include "fc_internal.h"
#include "fc_philox.h"

namespace fc {

namespace {

__device__ __forceinline__ void wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint64_t bits_below(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }
__device__ __forceinline__ uint64_t lane_range(int lo, int hi) { return bits_below(hi) & ~bits_below(lo); }

__device__ __forceinline__ int rl32(int x, int lane) { return __builtin_amdgcn_readlane(x, lane); }
__device__ __forceinline__ uint32_t rlu(uint32_t x, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)x, lane); }
__device__ __forceinline__ uint64_t rl64(uint64_t x, int lane) {
    return ((uint64_t)rlu((uint32_t)(x >> 32), lane) << 32) | rlu((uint32_t)x, lane);
}

__device__ __forceinline__ int kth_set_bit(uint64_t x, int64_t k) {  // k >= 1
    for (int64_t i = 1; i < k; ++i) x &= x - 1;
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
    // wrap interval [cur, L) U [0, first)
    const uint32_t first = nbrA & (0u - nbrA);
    cnt += (brk & ((full & ~(cur - 1u)) | (first - 1u))) != 0u;
    return cnt <= 1;
}

// Wave-cooperative BFS over the old district with v removed: are all old-district
// neighbours of v (targets) connected?  Bitmaps in LDS; frontier words owned by lanes.
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
                const int u = i * 64 + b;
                const NodeRec<RMAX> r = G[u];
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

struct LaneDraw {
    int v, av, pv, delta, nA;
    uint32_t inA, nbrA, L, nbr;
    bool okdraw, isprop, exact, gam, s_lin, s_cyc, acc;
};

}  // namespace

template <int RMAX>
__global__ __launch_bounds__(256) void flip_k2_kernel(KParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = (int)(threadIdx.x & 63u);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int c = (int)blockIdx.x * kWavesPerBlock + wv;
    if (c >= p.n_chains) return;

    const int n = p.n;
    const int npad = (n + 15) & ~15;
    unsigned char *base = smem + (size_t)wv * p.chain_lds_bytes;
    int8_t *a = (int8_t *)base;
    uint8_t *fcnt = base + npad;
    uint64_t *T = (uint64_t *)(base + 2 * npad);
    uint64_t *vis = T + (2 * RMAX + 2);
    uint64_t *front = vis + p.words;
    uint64_t *nxt = front + p.words;
    const NodeRec<RMAX> *__restrict__ G = (const NodeRec<RMAX> *)p.graph;

    // ---- load the chain into LDS -------------------------------------------------------
    {
        const uint4 *ga = (const uint4 *)(p.assign + (size_t)c * npad);
        const uint4 *gf = (const uint4 *)(p.fcnt + (size_t)c * npad);
        for (int i = lane; i < npad / 16; i += kWave) {
            ((uint4 *)a)[i] = ga[i];
            ((uint4 *)fcnt)[i] = gf[i];
        }
        if (lane < 2 * RMAX + 1) T[lane] = p.thresh[(size_t)c * (2 * RMAX + 1) + lane];
    }
    ChainScalars *scp = p.sc + c;
    uint64_t draw = scp->draw;
    int64_t steps = scp->steps;
    int64_t proposals = scp->proposals, accepted = scp->accepted;
    int64_t inv_contig = scp->inv_contig, inv_pop = scp->inv_pop;
    int64_t bfs_calls = scp->bfs_calls, bfs_levels = scp->bfs_levels;
    int64_t trace_len = scp->trace_len;
    int cut = scp->cut, nb = scp->nb;
    int pops0 = scp->pops[0], pops1 = scp->pops[1];
    int ng0 = scp->ngamma[0], ng1 = scp->ngamma[1];
    int64_t wait_cur = scp->wait_cur;
    int last_flip = scp->last_flip;
    int stuck = 0;
    const int64_t target = steps + p.n_steps;
    uint64_t draw_cap = draw + (uint64_t)p.max_draws;
    if (p.tape && draw_cap > (uint64_t)p.tape_draws) draw_cap = (uint64_t)p.tape_draws;
    const uint32_t chain_gid = p.chain_id_offset + (uint32_t)c;
    const bool force_bfs = (p.flags & FC_FLAG_FORCE_BFS) != 0;
    const bool want_wait = (p.diag & FC_DIAG_WAIT) != 0;
    const bool trace_on = p.trace && c < p.trace_chains;

    // per-lane partial sums over yields, reduced once at the end
    int64_t acc_cut = 0, acc_nb = 0, acc_wait = 0, acc_cut2 = 0, acc_nb2 = 0;
    wave_sync();

    while (steps < target) {
        if (draw >= draw_cap) {
            stuck = 1;
            break;
        }
        const int avail = (int)((draw_cap - draw) < 64 ? (draw_cap - draw) : 64);
        // ---- 1. speculative evaluation: lane = draw ----------------------------------
        const uint64_t d = draw + (uint64_t)lane;
        Words4 w;
        if (p.tape) {
            const uint32_t *t = p.tape + ((size_t)c * (size_t)p.tape_draws + (lane < avail ? d : draw)) * 6;
            w = Words4{t[0], t[1], t[2], t[3]};
        } else {
            w = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), chain_gid, 0u, p.seed_lo, p.seed_hi);
        }
        LaneDraw L;
        const uint64_t m = (uint64_t)w.x0 * (uint64_t)(uint32_t)n;
        L.v = (int)(m >> 32);
        L.okdraw = ((uint32_t)m >= p.lemire_thresh) && lane < avail;
        const NodeRec<RMAX> rec = G[L.v];
        L.av = a[L.v];
        L.pv = rec.pop;
        L.L = (uint32_t)(rec.meta & kMetaLenMask);
        const uint32_t full = (L.L >= 32) ? 0xffffffffu : ((1u << L.L) - 1u);
        L.nbr = (uint32_t)(rec.meta >> kMetaNbrShift) & 0xffffu;
        const uint32_t link = (uint32_t)(rec.meta >> kMetaLinkShift) & 0xffffu;
        uint32_t inA = 0;
#pragma unroll
        for (int i = 0; i < RMAX; ++i) inA |= (uint32_t)(a[ring_entry<RMAX>(rec.ring, i)] == L.av) << i;
        inA &= full;
        L.inA = inA;
        L.nbrA = inA & L.nbr;
        L.nA = __popc(L.nbrA);
        const int nBn = rec.deg - L.nA;
        L.isprop = L.okdraw && nBn > 0;
        {
            const uint32_t rot = L.L ? (((inA >> 1) | (inA << (L.L - 1))) & full) : 0u;
            const uint32_t lk = inA & rot & link;
            L.s_lin = one_run(L.nbrA, full & ~lk, full);
            const uint32_t vlink = (L.L >= 2 && (inA & 1u) && ((inA >> (L.L - 1)) & 1u)) ? (1u << (L.L - 1)) : 0u;
            L.s_cyc = one_run(L.nbrA, full & ~(lk | vlink), full);
        }
        L.exact = (rec.meta & kMetaExact) && !force_bfs;
        L.gam = (rec.meta & kMetaGamma) != 0;
        L.delta = L.nA - nBn;
        L.acc = mant53(w.x1, w.x2) < T[L.delta + RMAX];

        // ---- 2. commit loop (wave-uniform) -------------------------------------------
        const uint64_t P = __ballot(L.isprop);
        const uint64_t ACC = __ballot(L.acc);
        uint64_t BFSDONE = 0, BFSRES = 0, ACCM = 0, VSM = 0, INVC = 0, INVP = 0;
        int end = avail, pos = 0;
        const int cut0 = cut, nb0 = nb;
        const int64_t steps0 = steps;
        const int last_flip0 = last_flip;
        const int a_last0 = last_flip0 >= 0 ? (int)a[last_flip0] : 0;
        int cut_after = cut, nb_after = nb;
        while (pos < end) {
            // per-lane status against the current populations / outer-face counts
            const bool bdone = (BFSDONE >> lane) & 1ull;
            const int other = 1 - L.av;
            const bool touch = (other == 0 ? ng0 : ng1) > 0;
            bool known, ok;
            if (L.nA == 0) {
                known = true;
                ok = false;
            } else if (bdone) {
                known = true;
                ok = (BFSRES >> lane) & 1ull;
            } else if (L.exact) {
                known = true;
                ok = (L.gam && !touch) ? L.s_cyc : L.s_lin;
            } else {
                known = L.s_lin;
                ok = L.s_lin;
            }
            const int pa = L.av == 0 ? pops0 : pops1, pb = L.av == 0 ? pops1 : pops0;
            const bool popok = (pa - L.pv >= p.pop_lo) && (pb + L.pv <= p.pop_hi);
            const uint64_t VAL = __ballot(L.isprop && known && ok && popok);
            const uint64_t UNK = __ballot(L.isprop && !known);
            const uint64_t IC = __ballot(L.isprop && known && !ok);
            const uint64_t IP = __ballot(L.isprop && known && ok && !popok);
            const uint64_t ev = ((VAL & ACC) | UNK) & lane_range(pos, end);
            const int f = ev ? __builtin_ctzll(ev) : end;
            const uint64_t seg = lane_range(pos, f);
            const int nvalid = __popcll(VAL & seg);
            if (steps + nvalid >= target) {
                const int e = kth_set_bit(VAL & seg, target - steps);
                const uint64_t s2 = lane_range(pos, e + 1);
                VSM |= VAL & s2;
                INVC |= IC & s2;
                INVP |= IP & s2;
                steps = target;
                end = e + 1;
                break;
            }
            VSM |= VAL & seg;
            INVC |= IC & seg;
            INVP |= IP & seg;
            steps += nvalid;
            pos = f;
            if (f >= end) break;
            if ((UNK >> f) & 1ull) {
                // resolve lane f by device BFS on the current state
                const int vf = rl32(L.v, f), Af = rl32(L.av, f);
                const uint32_t nbrAf = rlu(L.nbrA, f);
                int my_target = -1, start = -1;
#pragma unroll
                for (int k2 = 0; k2 < RMAX / 2; ++k2) {
                    const uint32_t wrd = rlu(rec.ring[k2], f);
                    if ((lane >> 1) == k2) my_target = (int)((wrd >> (16 * (lane & 1))) & 0xffffu);
                    const int j0 = 2 * k2, j1 = 2 * k2 + 1;
                    if (start < 0 && ((nbrAf >> j0) & 1u)) start = (int)(wrd & 0xffffu);
                    if (start < 0 && ((nbrAf >> j1) & 1u)) start = (int)(wrd >> 16);
                }
                if (!(lane < RMAX && ((nbrAf >> lane) & 1u))) my_target = -1;
                const bool res = wave_bfs<RMAX>(G, a, vis, front, nxt, p.words, lane, vf, Af, my_target, start, bfs_levels);
                ++bfs_calls;
                BFSDONE |= 1ull << f;
                if (res) BFSRES |= 1ull << f;
                continue;
            }
            // ---- accept lane f: apply the flip ---------------------------------------
            const int vf = rl32(L.v, f), Af = rl32(L.av, f), pvf = rl32(L.pv, f);
            const int df = rl32(L.delta, f), nAf = rl32(L.nA, f);
            const uint32_t inAf = rlu(L.inA, f), nbrf = rlu(L.nbr, f);
            const bool gamf = rl32((int)L.gam, f) != 0;
            int my_e = -1;
#pragma unroll
            for (int k2 = 0; k2 < RMAX / 2; ++k2) {
                const uint32_t wrd = rlu(rec.ring[k2], f);
                if ((lane >> 1) == k2) my_e = (int)((wrd >> (16 * (lane & 1))) & 0xffffu);
            }
            const bool is_nbr = lane < RMAX && ((nbrf >> lane) & 1u);
            const bool inA_l = (inAf >> lane) & 1u;
            bool enter = false, leave = false;
            if (is_nbr) {
                const int old = fcnt[my_e];
                fcnt[my_e] = (uint8_t)(old + (inA_l ? 1 : -1));
                enter = inA_l && old == 0;
                leave = !inA_l && old == 1;
            }
            const int dnb = __popcll(__ballot(enter)) - __popcll(__ballot(leave));
            if (lane == 0) {
                a[vf] = (int8_t)(1 - Af);
                fcnt[vf] = (uint8_t)nAf;
            }
            if (Af == 0) { pops0 -= pvf; pops1 += pvf; } else { pops1 -= pvf; pops0 += pvf; }
            if (gamf) { if (Af == 0) { --ng0; ++ng1; } else { --ng1; ++ng0; } }
            cut += df;
            nb += dnb;
            ++steps;
            VSM |= 1ull << f;
            ACCM |= 1ull << f;
            last_flip = vf;
            if (lane == f) { cut_after = cut; nb_after = nb; }
            wave_sync();
            // lanes whose ring contains vf were evaluated on a stale neighbourhood
            bool hit = false;
            if (L.okdraw && lane > f) {
                hit = L.v == vf;
#pragma unroll
                for (int i = 0; i < RMAX; ++i) hit |= ring_entry<RMAX>(rec.ring, i) == vf;
            }
            const uint64_t aff = __ballot(hit);
            if (aff) {
                const int fa = __builtin_ctzll(aff);
                if (fa < end) end = fa;
            }
            pos = f + 1;
            if (steps >= target) {
                end = pos;
                break;
            }
        }

        // ---- 3. lane-parallel bookkeeping of the committed batch ------------------------
        const uint64_t done_mask = bits_below(end);
        proposals += __popcll(P & done_mask);
        accepted += __popcll(ACCM);
        inv_contig += __popcll(INVC);
        inv_pop += __popcll(INVP);
        const bool is_acc = (ACCM >> lane) & 1ull;
        const uint64_t later_acc = ACCM & ~bits_below(lane + 1);
        const int next_acc = later_acc ? __builtin_ctzll(later_acc) : end;
        const int run_len = is_acc ? 1 + __popcll(VSM & lane_range(lane + 1, next_acc)) : 0;
        const int first_acc = ACCM ? __builtin_ctzll(ACCM) : end;
        const int r0 = __popcll(VSM & bits_below(first_acc));
        int64_t my_wait = 0;
        if (want_wait && is_acc) {
            Words4 g;
            if (p.tape) {
                const uint32_t *t = p.tape + ((size_t)c * (size_t)p.tape_draws + d) * 6;
                g = Words4{t[4], t[5], 0u, 0u};
            } else {
                g = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), chain_gid, 1u, p.seed_lo, p.seed_hi);
            }
            const double U = u53(g.x0, g.x1);
            my_wait = (int64_t)ceil(log(1.0 - U) / p.log1mp[nb_after]) - 1;
        }
        if (is_acc) {
            acc_cut += (int64_t)cut_after * run_len;
            acc_cut2 += (int64_t)cut_after * cut_after * run_len;
            acc_nb += (int64_t)nb_after * run_len;
            acc_nb2 += (int64_t)nb_after * nb_after * run_len;
            acc_wait += my_wait * run_len;
        }
        if (lane == 0 && r0) {
            acc_cut += (int64_t)cut0 * r0;
            acc_cut2 += (int64_t)cut0 * cut0 * r0;
            acc_nb += (int64_t)nb0 * r0;
            acc_nb2 += (int64_t)nb0 * nb0 * r0;
            acc_wait += wait_cur * r0;
        }
        const int t_acc = (int)(steps0 + __popcll(VSM & bits_below(lane + 1)));  // yield index of this lane
        if (p.diag & FC_DIAG_HIST) {
            if (is_acc) {
                atomicAdd((unsigned long long *)&p.cut_hist[(size_t)c * (p.n_edges + 1) + cut_after], (unsigned long long)run_len);
                atomicAdd((unsigned long long *)&p.nb_hist[(size_t)c * (n + 1) + nb_after], (unsigned long long)run_len);
            }
            if (lane == 0 && r0) {
                atomicAdd((unsigned long long *)&p.cut_hist[(size_t)c * (p.n_edges + 1) + cut0], (unsigned long long)r0);
                atomicAdd((unsigned long long *)&p.nb_hist[(size_t)c * (n + 1) + nb0], (unsigned long long)r0);
            }
        }
        if (p.diag & FC_DIAG_FLIPS) {
            // part.flips is stale on rejected steps: every yield of a run repeats the update
            // for the node whose flip created the state (grid_chain_sec11.py:396-400).
            int64_t *nf = p.num_flips + (size_t)c * n, *ps = p.part_sum + (size_t)c * n;
            unsigned long long *lf = (unsigned long long *)(p.last_flipped + (size_t)c * n);
            if (lane == 0 && r0 && last_flip0 >= 0) {
                const int64_t t_last = steps0 + r0;
                const int64_t old = (int64_t)atomicExch(lf + last_flip0, (unsigned long long)t_last);
                atomicAdd((unsigned long long *)(ps + last_flip0), (unsigned long long)(-(int64_t)p.labels[a_last0] * (t_last - old)));
                atomicAdd((unsigned long long *)(nf + last_flip0), (unsigned long long)r0);
            }
            __builtin_amdgcn_s_waitcnt(0);
            if (is_acc) {
                const int64_t t_last = (int64_t)t_acc + run_len - 1;
                const int64_t old = (int64_t)atomicExch(lf + L.v, (unsigned long long)t_last);
                atomicAdd((unsigned long long *)(ps + L.v), (unsigned long long)(-(int64_t)p.labels[1 - L.av] * (t_last - old)));
                atomicAdd((unsigned long long *)(nf + L.v), (unsigned long long)run_len);
            }
        }
        if ((p.diag & FC_DIAG_EDGES) && is_acc) {
            int64_t *ea = p.edge_acc + (size_t)c * p.n_edges;
            unsigned long long *es = (unsigned long long *)(p.edge_since + (size_t)c * p.n_edges);
            for (int i = 0; i < RMAX; ++i) {
                if (!((L.nbr >> i) & 1u)) continue;
                const int e = p.ring_eid[(size_t)L.v * RMAX + i];
                if ((L.inA >> i) & 1u) {
                    atomicExch(es + e, (unsigned long long)t_acc);             // becomes cut
                } else {
                    const int64_t since = (int64_t)atomicAdd(es + e, 0ull);    // becomes uncut
                    atomicAdd((unsigned long long *)(ea + e), (unsigned long long)((int64_t)t_acc - since));
                }
            }
        }
        if (trace_on) {
            const bool in_done = lane < end && L.isprop;
            const uint64_t mine = ACCM & bits_below(lane + 1);
            const int src = mine ? 63 - __builtin_clzll(mine) : 0;
            const int c_j = __shfl(cut_after, src), n_j = __shfl(nb_after, src);
            const long long w_j = __shfl((long long)my_wait, src);
            const int64_t idx = trace_len + __popcll(P & done_mask & bits_below(lane));
            if (in_done && idx < p.trace_cap) {
                fc_record &rr = p.trace[(size_t)c * p.trace_cap + idx];
                const bool valid = (VSM >> lane) & 1ull;
                rr.draw = (int64_t)d;
                rr.v = L.v;
                rr.flags = valid ? (1 | (is_acc ? 2 : 0)) : (((INVC >> lane) & 1ull) ? 4 : 8);
                rr.cut = mine ? c_j : cut0;
                rr.nb = mine ? n_j : nb0;
                rr.wait = valid ? (mine ? (int64_t)w_j : wait_cur) : 0;
            }
            trace_len += __popcll(P & done_mask);
        }
        if (ACCM) {
            const int la = 63 - __builtin_clzll(ACCM);
            wait_cur = (int64_t)__shfl((long long)my_wait, la);
        }
        draw += (uint64_t)end;
        wave_sync();
    }

    // ---- write back ---------------------------------------------------------------------
    {
        uint4 *ga = (uint4 *)(p.assign + (size_t)c * npad);
        uint4 *gf = (uint4 *)(p.fcnt + (size_t)c * npad);
        for (int i = lane; i < npad / 16; i += kWave) {
            ga[i] = ((const uint4 *)a)[i];
            gf[i] = ((const uint4 *)fcnt)[i];
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        acc_cut += __shfl_xor((long long)acc_cut, off);
        acc_nb += __shfl_xor((long long)acc_nb, off);
        acc_wait += __shfl_xor((long long)acc_wait, off);
        acc_cut2 += __shfl_xor((long long)acc_cut2, off);
        acc_nb2 += __shfl_xor((long long)acc_nb2, off);
    }
    if (lane == 0) {
        scp->draw = draw;
        scp->steps = steps;
        scp->proposals = proposals;
        scp->accepted = accepted;
        scp->inv_contig = inv_contig;
        scp->inv_pop = inv_pop;
        scp->bfs_calls = bfs_calls;
        scp->bfs_levels = bfs_levels;
        scp->trace_len = trace_len;
        scp->sum_cut += acc_cut;
        scp->sum_nb += acc_nb;
        scp->sum_wait += acc_wait;
        scp->sum_cut2 += acc_cut2;
        scp->sum_nb2 += acc_nb2;
        scp->cut = cut;
        scp->nb = nb;
        scp->pops[0] = pops0;
        scp->pops[1] = pops1;
        scp->ngamma[0] = ng0;
        scp->ngamma[1] = ng1;
        scp->wait_cur = wait_cur;
        scp->last_flip = last_flip;
        scp->stuck = stuck;
    }
}

int launch_flip_k2(const KParams &p, int ring_max, void *stream) {
    const int blocks = (p.n_chains + kWavesPerBlock - 1) / kWavesPerBlock;
    const size_t lds = (size_t)p.chain_lds_bytes * kWavesPerBlock;
    hipStream_t s = (hipStream_t)stream;
    if (ring_max == 8)
        hipLaunchKernelGGL(flip_k2_kernel<8>, dim3(blocks), dim3(kWave * kWavesPerBlock), lds, s, p);
    else if (ring_max == 16)
        hipLaunchKernelGGL(flip_k2_kernel<16>, dim3(blocks), dim3(kWave * kWavesPerBlock), lds, s, p);
    else
        return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

}  // namespace fc
