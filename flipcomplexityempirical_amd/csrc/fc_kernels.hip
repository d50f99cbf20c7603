// Flip-walk kernels for gfx950 (MI355X).
//
// One chain per wavefront.  The chain's state lives in LDS: int8 district per node, uint8
// count of foreign neighbours per node (so |B| and boundary membership are O(1)), its
// acceptance-threshold table, BFS bitmaps and a 64-slot staging area.  The graph (one
// 32/48-byte record per node: meta, population, degree, packed int16 link ring) is shared by
// all chains and read through L1/L2.
//
// A wave advances its chain in batches:
//   1a. up to NSUB rounds of 64 Philox draws map to nodes (exact Lemire); draws whose node is
//       a boundary node (fcnt[v] > 0) are proposals and are packed, in draw order, into up
//       to 64 slots; other draws are not proposals (rejection sampling of random.choice
//       over b_nodes, grid_chain_sec11.py:143);
//   1b. every slot lane evaluates its proposal against the current state: link-ring reads,
//       contiguity by the planar run rule, population bound, delta-cut, Metropolis threshold;
//   2.  a wave-uniform commit loop walks the slots in draw order as the reference's
//       MarkovChain.__next__ would ([gc-0.2], used grid_chain_sec11.py:340-342,366): invalid
//       proposals are skipped, rejected valid ones re-yield the state, an accepted one is
//       applied; later slots whose ring holds the flipped node (and non-hit draws whose node
//       just entered the boundary) are redrawn in the next batch, so the trajectory is the
//       one-draw-at-a-time chain bit for bit;
//   3.  the per-yield driver diagnostics (grid_chain_sec11.py:366-402) are accumulated
//       lane-parallel from the per-lane status bits.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include <cstdio>

#include "fc_internal.h"
#include "fc_philox.h"
#include "fc_device.h"

namespace fc {

using namespace dev;

// district_rule (the district-graph contiguity rule, k > 2): fc_ring.h, shared with the host
// check tests/native/district_rule_lib.cpp.

// KM = 2: two districts (BI_SIGN, and PAIR with k = 2, which coincide); the outer-face
// exact rule applies.  KM = 0: k <= 32 districts, PAIR proposals, populations in LDS.  KM = 1:
// as KM = 0 with the workgroup-cooperative search (p.coop); a separate instance, because the
// helper waves' code costs the common one its registers (C3: 14 -> 58 spilled VGPRs).  KM = 3:
// as KM = 0 when the district-graph rule decides every proposal (p.dgraph): no search code.
// RMAX = 8: at most 128 VGPRs, four waves per SIMD (C3's 8192 chains per GPU run in two
// rounds of waves instead of three: 1.46e9 against 1.35e9 proposals/s; a handful of VGPRs
// spill; C4's LDS-limited launch with three waves' budget and no spills: 25.4 against 25.1 ms)
// MF (KM = 3): the multi-flip commit below, in an instance of its own so that runs without it
// keep the smaller code
#ifndef FC_K_WAVES8
#define FC_K_WAVES8 4  // RMAX = 8 waves per SIMD the register budget is sized for
#endif
template <int RMAX, int NSUB, int KM, bool FULL, int MF>
__global__ __launch_bounds__(256, (RMAX == 8 ? FC_K_WAVES8 : 1)) void flip_kernel(KParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = (int)(threadIdx.x & 63u);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // p.coop: one chain per workgroup; wave 0 runs it, waves 1.. join its contiguity searches
    const bool coop = KM == 1 && p.coop != 0;  // only the KM = 1 instance carries the helper code
    const int c = coop ? (int)blockIdx.x : (int)blockIdx.x * (int)(blockDim.x >> 6) + wv;
    if (c >= p.n_chains) return;

    const int n = p.n;
    const int npad = (n + 15) & ~15;
    unsigned char *base = smem + (coop ? (size_t)0 : (size_t)wv * p.chain_lds_bytes);
    // KM = 3 packs a node into one byte: district (bits 0-4) | foreign districts nf, saturated
    // at 7 (bits 5-7); the exact nf is recounted from the ring where it matters (the slot
    // filter of a saturated node, the nf histogram).  Half the chain's LDS: C4 / C5 hold about
    // twice the chains per CU.  The HBM state keeps the exact int8 / uint8 arrays.
    constexpr bool PK = KM == 3;
    int8_t *a = (int8_t *)base;
    uint8_t *const pkb = base;                      // PK: the packed bytes (a aliases them)
    uint8_t *fcnt = base + npad;                    // !PK
    uint64_t *T = (uint64_t *)(base + (PK ? 1 : 2) * npad);
    auto dist = [&](int u) -> int { return PK ? (int)(pkb[u] & 31u) : (int)a[u]; };
    BfsScratch bs;                                  // BFS labels, masks, chunk, bitmaps
    bs.lab = (uint32_t *)(T + (2 * RMAX + 2));
    bs.lab_words = p.lab_words;
    bs.mm = bs.lab + p.lab_words;
    bs.cm = bs.mm + 16;
    bs.lcnt = (int32_t *)(bs.cm + 16);
    bs.list = (uint16_t *)(bs.lcnt + 4);
    bs.vis = (uint64_t *)(bs.list + 2 * kBfsList);
    bs.front = bs.vis + p.words;
    bs.nxt = bs.front + p.words;
    bs.W = p.words;
    bs.prof = nullptr;
    // [5][64]: node, word1, word2, draw offset, word3; with the district-graph rule the search
    // never runs and its scratch is not allocated (fc_run_create)
    uint32_t *slot = KM != 2 && p.dgraph ? (uint32_t *)(T + (2 * RMAX + 2)) : (uint32_t *)(bs.nxt + p.words);
    int32_t *popk = (int32_t *)(slot + 5 * 64);    // [32] district populations (KM = 0)
    // PAIR slot bound: fcnt[u] holds nf(u), u's number of foreign districts (its pairs in
    // b_nodes, :151-153), and nfh[j] the nodes with nf = j; the canonical stream draws slots
    // r < wcap = max_u nf(u) (p.wdyn), else r < p.wmax
    int32_t *nfh = popk + kMaxKGeneral;
    // accepted states whose geometric wait is still to be drawn (kWaitQK: creating draw, |B|
    // after the flip, yields so far); as in fc_flip2.hip, drained by wait_flush
    uint64_t *q_d = (uint64_t *)(nfh + kNfh);
    uint32_t *q_nb = (uint32_t *)(q_d + kWaitQK), *q_run = q_nb + kWaitQK;
    // district-graph rule (p.dgraph): pair counts [k * k], adjacency masks [32] (entry 31: the
    // outer face), outer-face nodes per district [32]
    int32_t *mcnt = (int32_t *)(q_run + kWaitQK);
    uint32_t *adj = (uint32_t *)(mcnt + p.k * p.k);
    int32_t *ngk = (int32_t *)(adj + 32);
    const bool dgraph = KM == 3 || (KM != 2 && p.dgraph != 0);  // KM = 3: always, by construction
    // KM = 3 multi-flip commit: marks of the members' neighbours, hashed to 2048 bits (1024 for
    // RMAX = 16, which keeps C5's chain at 11 LDS granules; a collision only ends a group early)
    uint32_t *hb = (uint32_t *)(ngk + 32);
    constexpr int kHbMask = fc::hb_bytes(RMAX) * 8 - 1;
    // MF = 2 (graphs small enough, fc_run_create): exact marks instead, one byte per node (bit g:
    // the g-th candidate of a pass has the node as a neighbour)
    uint8_t *const mk8 = (uint8_t *)(ngk + 32);
    uint32_t *const mk32 = (uint32_t *)mk8;
    // cooperative search control words (coop implies no district tables: they start here)
    int32_t *ctl = (int32_t *)(q_run + kWaitQK);
    const NodeRec<RMAX> *__restrict__ G = (const NodeRec<RMAX> *)p.graph;
    if (coop && wv > 0) {
        coop_helper_loop<RMAX>(G, a, bs, ctl, (int)threadIdx.x, (int)blockDim.x);
        return;
    }

    // ---- load the chain into LDS -------------------------------------------------------
    {
        const uint4 *ga = (const uint4 *)(p.assign + (size_t)c * npad);
        const uint4 *gf = (const uint4 *)(p.fcnt + (size_t)c * npad);
        for (int i = lane; i < npad / 16; i += kWave) {
            if constexpr (PK) {
                const uint4 x = ga[i], y = gf[i];
                const uint32_t xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
                uint32_t o[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t w = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const uint32_t f = (ya[q] >> (8 * b)) & 0xffu;
                        w |= (((xa[q] >> (8 * b)) & 31u) | ((f < 7u ? f : 7u) << 5)) << (8 * b);
                    }
                    o[q] = w;
                }
                ((uint4 *)pkb)[i] = uint4{o[0], o[1], o[2], o[3]};
            } else {
                ((uint4 *)a)[i] = ga[i];
                ((uint4 *)fcnt)[i] = gf[i];
            }
        }
        if (lane < 2 * RMAX + 1) T[lane] = p.thresh[(size_t)c * (2 * RMAX + 1) + lane];
        if (KM != 2 && lane < 32) {
            popk[lane] = p.popk[(size_t)c * 32 + lane];
            nfh[lane] = p.nfh[(size_t)c * kNfh + lane];
        }
        if (dgraph) {
            const int kk = p.k * p.k;
            for (int i = lane; i < kk; i += kWave) mcnt[i] = p.mcnt[(size_t)c * kk + i];
            if (lane < 32) ngk[lane] = p.ngk[(size_t)c * 32 + lane];
            if (KM == 3 && MF == 1 && lane < fc::hb_bytes(RMAX) / 4) hb[lane] = 0u;
            if (KM == 3 && MF == 2)
                for (int i = lane; i < npad / 4; i += kWave) mk32[i] = 0u;
            wave_sync();
            // adj[X] bit Y: some face holds cells of X and Y; bit 31: X touches the outer face
            uint32_t m = 0;
            if (lane < p.k) {
                for (int Y = 0; Y < p.k; ++Y)
                    if (Y != lane && mcnt[min(lane, Y) * p.k + max(lane, Y)] > 0) m |= 1u << Y;
                if (ngk[lane] > 0) m |= 1u << 31;
            }
            const uint32_t om = (uint32_t)__ballot(lane < p.k && ngk[lane] > 0);
            if (lane < 32) adj[lane] = lane == 31 ? om : m;
        }
    }
    // slot bound of the PAIR draws and its Lemire threshold 2^32 mod wcap (wave-uniform)
    int wcap = p.wmax;
    if (KM != 2 && p.wdyn) {
        wave_sync();
        const uint64_t hm = __ballot(lane >= 1 && lane < kNfh && nfh[lane] > 0);
        wcap = hm ? 63 - __builtin_clzll(hm) : 1;
    }
    uint32_t wthr = (0u - (uint32_t)wcap) % (uint32_t)wcap;
    ChainScalars *scp = p.sc + c;
    uint64_t draw = scp->draw;
    int64_t steps = scp->steps;  // index of the current yield
    int64_t bfs_calls = scp->bfs_calls, bfs_levels = scp->bfs_levels;
    int64_t trace_len = scp->trace_len;
    int64_t ev_len = scp->ev_len, hit_time = scp->hit_time;
    int cut = scp->cut, nb = scp->nb;
    int pops0 = scp->pops[0], pops1 = scp->pops[1];
    const int pop_lo = scp->pop_lo, pop_hi = scp->pop_hi;  // this chain's bounds (chain_pop_bounds)
    int ng0 = scp->ngamma[0], ng1 = scp->ngamma[1];
    int64_t wait_cur = scp->wait_cur;
    int last_flip = scp->last_flip;
    int stuck = 0;
    int rem = (int)p.n_steps;  // steps still to take in this launch (host: n_steps < 2^31)
    uint64_t draw_cap = draw + (uint64_t)p.max_draws;
    if (FULL && p.tape && draw_cap > (uint64_t)p.tape_draws) draw_cap = (uint64_t)p.tape_draws;
    const uint32_t chain_gid = p.chain_id_offset + (uint32_t)c;
    const bool force_bfs = (p.flags & FC_FLAG_FORCE_BFS) != 0;
    const bool want_wait = (p.diag & FC_DIAG_WAIT) != 0;
    const bool trace_on = FULL && p.trace && c < p.trace_chains;
    const bool defer = want_wait && !trace_on && !(FULL && p.tape);  // waits drawn later (wait_flush)
    int qn = 0;

    // per-lane accumulators, reduced once per launch
    int64_t acc_cut = 0, acc_nb = 0, acc_wait = 0, acc_cut2 = 0, acc_nb2 = 0;
    uint32_t n_prop = 0, n_acc = 0, n_ic = 0, n_ip = 0;
#ifdef FC_PHASE_PROF
    int64_t *prof_acc = (int64_t *)(base + p.chain_lds_bytes - kProfSlots * 8);
    if (lane < kProfSlots) prof_acc[lane] = 0;
    bs.prof = prof_acc;
#endif
    // the k = 2 kernel's deferred waits (fc_flip2.hip): one full-width pass per queue load
    auto wait_flush = [&]() {
        compiler_fence();
        int64_t w = 0;
        if (lane < qn) {
            const uint64_t dq = q_d[lane];
            const Words4 g = philox4x32_10((uint32_t)dq, (uint32_t)(dq >> 32), chain_gid, 1u, p.seed_lo, p.seed_hi);
            w = geom_from(u53(g.x0, g.x1), p.log1mp[q_nb[lane]]);
            acc_wait += w * (int64_t)q_run[lane];
        }
        wait_cur = (int64_t)__shfl((long long)w, qn - 1);
        qn = 0;
        compiler_fence();
    };
    wave_sync();
    FC_STAMP(t_loop0);

    while (rem > 0) {
        FC_STAMP(t_a);
        FC_PROF(5, 1);
        if (draw >= draw_cap) {
            stuck = 1;
            break;
        }
        const uint64_t room = draw_cap - draw;
        // ---- 1a. draws -> nodes; boundary hits packed, in draw order, into <= 64 slots ----
        int nh = 0;       // boundary hits seen
        int gen = 0;      // draws generated (offsets 0..gen-1 of this batch)
        int rv[NSUB];     // node of this lane's draw in round r (offset 64 r + lane)
        uint64_t nonhit[NSUB];
#pragma unroll
        for (int r = 0; r < NSUB; ++r) {
            rv[r] = -1;
            nonhit[r] = 0;
            if ((r > 0 && nh >= p.hit_stop) || nh >= 64 || (uint64_t)gen >= room) continue;
            const int off = gen + lane;
            const bool inrange = (uint64_t)off < room;
            const uint64_t dr = draw + (uint64_t)off;
            Words4 w;
            if (FULL && p.tape) {
                const uint32_t *t = p.tape + ((size_t)c * (size_t)p.tape_draws + (inrange ? dr : draw)) * 6;
                w = Words4{t[0], t[1], t[2], t[3]};
            } else {
                w = philox4x32_10((uint32_t)dr, (uint32_t)(dr >> 32), chain_gid, 0u, p.seed_lo, p.seed_hi);
            }
            const uint64_t m = (uint64_t)w.x0 * (uint64_t)(uint32_t)n;
            const int v = (int)(m >> 32);
            bool ok = inrange && (uint32_t)m >= p.lemire_thresh;
            bool hit;
            if constexpr (KM != 2) {
                // the draw's district slot r (word 3, exact Lemire over wmax) can only name a
                // foreign district if r < fcnt[v] (foreign neighbours >= foreign districts):
                // slots beyond are non-proposals whatever 1b would find, so they take no slot
                // (a slot rejected by the Lemire map never proposes: not a non-hit either)
                const uint64_t mw = (uint64_t)w.x3 * (uint64_t)(uint32_t)wcap;
                ok = ok && (uint32_t)mw >= wthr;
                if constexpr (PK) {  // a saturated count passes every slot; 1b decides exactly
                    const int nfs = (int)(pkb[v] >> 5);
                    hit = ok && ((int)(mw >> 32) < nfs || nfs == 7);
                } else {
                    hit = ok & ((int)(mw >> 32) < (int)fcnt[v]);  // (v < n: no guard, no branch)
                }
            } else {
                hit = ok & (fcnt[v] != 0);
            }
            const uint64_t hm = __ballot(hit);
            const int pos = nh + __popcll(hm & bits_below(lane));
            if (hit && pos < 64) {
                slot[pos] = (uint32_t)v;
                slot[64 + pos] = w.x1;
                slot[128 + pos] = w.x2;
                slot[192 + pos] = (uint32_t)off;
                slot[256 + pos] = w.x3;
            }
            rv[r] = v;
            uint64_t nm = __ballot(ok && !hit);
            const int cnt = __popcll(hm);
            if (nh + cnt > 64) {  // the 64th hit closes the batch inside this round
                const int last = kth_set_bit(hm, 64 - nh);
                gen += last + 1;
                nm &= bits_below(last + 1);
            } else {
                gen = (uint64_t)(gen + 64) < room ? gen + 64 : (int)room;
            }
            nonhit[r] = nm;
            nh += cnt;
        }
        const int ns = nh < 64 ? nh : 64;
        FC_PROF(17, ns);
        FC_PROF(18, gen);
        compiler_fence();
        FC_STAMP(t_b);
        FC_PROF(1, t_b - t_a);

        // ---- 1b. evaluate every slot against the current state ---------------------------
        const bool has = lane < ns;
        const int off_l = has ? (int)slot[192 + lane] : gen;
        const uint64_t d = draw + (uint64_t)off_l;
        const int v = has ? (int)slot[lane] : 0;
        const uint32_t w1 = slot[64 + lane], w2 = slot[128 + lane];
        const NodeRec<RMAX> rec = G[v];
        const int av = dist(v);
        const int pv = rec.pop;
        const uint32_t Ln = (uint32_t)(rec.meta & kMetaLenMask);
        const uint32_t full = (1u << Ln) - 1u;
        const uint32_t nbr = (uint32_t)(rec.meta >> kMetaNbrShift) & 0xffffu;
        const uint32_t link = (uint32_t)(rec.meta >> kMetaLinkShift) & 0xffffu;
        uint32_t inA = 0;    // ring cells in the old district
        uint32_t tmask;      // neighbours in the target district
        int tgt;             // target district
        bool slot_ok = true;
        int adv[RMAX];       // districts of the ring cells (KM = 0)
        int nf_after = 0;    // KM != 2: foreign districts of v after its flip
        int nf_before = 0;   // ... and before it
        if constexpr (KM == 2) {
#pragma unroll
            for (int i = 0; i < RMAX; ++i) inA |= (uint32_t)(a[ring_entry<RMAX>(rec.ring, i)] == av) << i;
            inA &= full;
            tgt = 1 - av;                       // -1 * assignment, grid_chain_sec11.py:145
            tmask = nbr & ~inA;
        } else {
            uint32_t dall = 0;                  // districts among the neighbours
            // the raw bytes first, every read issued before the first use (the compiler otherwise
            // waited on each), then the districts
#pragma unroll
            for (int i = 0; i < RMAX; ++i) {
                const int u = ring_entry<RMAX>(rec.ring, i);
                adv[i] = PK ? (int)pkb[u] : (int)a[u];
            }
#pragma unroll
            for (int i = 0; i < RMAX; ++i) asm volatile("" : "+v"(adv[i]));
#pragma unroll
            for (int i = 0; i < RMAX; ++i) {
                if constexpr (PK) adv[i] &= 31;
                inA |= (uint32_t)(adv[i] == av) << i;
                dall |= (((nbr >> i) & 1u) << adv[i]);
            }
            const uint32_t dm = dall & ~(1u << av);  // foreign districts among the neighbours
            inA &= full;
            // slow_reversible_propose (:117-130): uniform over (node, district) pairs -- slot
            // r < wmax by an exact Lemire map of word 3; the r-th foreign district is the target
            const uint64_t mw = (uint64_t)slot[256 + lane] * (uint64_t)(uint32_t)wcap;
            const int r = (int)(mw >> 32);
            slot_ok = (uint32_t)mw >= wthr && r < __popc(dm);
            uint32_t dd = dm;
            for (int q = 0; q < r && dd; ++q) dd &= dd - 1u;
            tgt = dd ? __builtin_ctz(dd) : 0;
            nf_after = __popc(dall & ~(1u << tgt));
            nf_before = __popc(dm);
            tmask = 0;
#pragma unroll
            for (int i = 0; i < RMAX; ++i) tmask |= (uint32_t)(adv[i] == tgt) << i;
            tmask &= nbr;
        }
        const uint32_t nbrA = inA & nbr;
        const int nA = __popc(nbrA);
        const int nT = __popc(tmask);
        const bool isprop = has && (rec.deg - nA) > 0 && slot_ok;
        bool s_lin, s_cyc;
        {
            const uint32_t rot = Ln ? (((inA >> 1) | (inA << (Ln - 1))) & full) : 0u;
            const uint32_t lk = inA & rot & link;
            s_lin = one_run(nbrA, full & ~lk, full);
            const uint32_t vlink = (Ln >= 2 && (inA & 1u) && ((inA >> (Ln - 1)) & 1u)) ? (1u << (Ln - 1)) : 0u;
            s_cyc = one_run(nbrA, full & ~(lk | vlink), full);
        }
        const bool exact = KM == 2 && (rec.meta & kMetaExact) && !force_bfs;
        const bool gam = (rec.meta & kMetaGamma) != 0;
        // k > 2 (KM = 0): on an exact interior node (closed, fully linked ring) the flip is
        // decided invalid when some district X != A shows up in two of the gaps between the
        // ring's A-runs that hold old neighbours: v + an X-path closes a Jordan curve with
        // old neighbours on both sides.  Anything else multi-run goes to the device BFS.
        bool s_cut = false;
        if constexpr (KM != 2) {
            if (dgraph) {
                // every multi-run case decided locally (district_rule above)
                s_cut = has && !s_lin && nA > 0 && !district_rule<RMAX>(adv, inA, nbr, Ln, gam, av, adj);
            } else if (has && !s_lin && nA > 0 && !force_bfs && !gam && (rec.meta & kMetaExact) && (link & full) == full) {
                uint32_t relA = 0;
                {
                    const uint32_t rotA = ((inA << 1) | (inA >> (Ln - 1))) & full;
                    uint32_t st0 = inA & ~rotA;
                    const uint32_t a2 = inA | (inA << Ln);
                    while (st0) {
                        const int s0 = __builtin_ctz(st0);
                        st0 &= st0 - 1u;
                        const int len = __builtin_ctz(~(a2 >> s0));
                        uint32_t run = ((1u << len) - 1u) << s0;
                        run = (run | (run >> Ln)) & full;
                        if (run & nbr) relA |= run;
                    }
                }
                const uint32_t gap = full & ~relA;
                const uint32_t rotG = ((gap << 1) | (gap >> (Ln - 1))) & full;
                uint32_t gst = gap & ~rotG;
                const uint32_t g2 = gap | (gap << Ln);
                uint32_t seen = 0;
                while (gst && !s_cut) {
                    const int s0 = __builtin_ctz(gst);
                    gst &= gst - 1u;
                    const int len = __builtin_ctz(~(g2 >> s0));
                    uint32_t run = ((1u << len) - 1u) << s0;
                    run = (run | (run >> Ln)) & full & ~inA;
                    uint32_t dR = 0;
                    while (run) {
                        const int i = __builtin_ctz(run);
                        run &= run - 1u;
                        dR |= 1u << dist(ring_entry<RMAX>(rec.ring, i));
                    }
                    s_cut = (dR & seen) != 0;
                    seen |= dR;
                }
            }
        }
        const int delta = nA - nT;  // cut(S') - cut(S)
        const bool acc = mant53(w1, w2) < T[delta + RMAX];
        // packed for the wave-uniform apply
        const uint32_t pk = (uint32_t)v | ((uint32_t)av << 15) | ((uint32_t)tgt << 21) | ((uint32_t)gam << 27);
        const uint32_t pk2 = inA | (nbr << 16);
        // |delta| <= deg <= 16 (6 bits); nf_after, nf_before <= 16 (5 bits each)
        const uint32_t pk3 = tmask | ((uint32_t)(delta + 32) << 16) | ((uint32_t)nf_after << 22) |
                             ((uint32_t)nf_before << 27);
        FC_STAMP(t_c);
        FC_PROF(2, t_c - t_b);

        // ---- 2. commit loop (wave-uniform) -----------------------------------------------
        uint32_t st = 0;
        int end = ns, pos = 0;
        int trunc_off = gen;  // first draw offset not consumed by this batch
        bool target_hit = false;
        const int cut0 = cut, nb0 = nb, rem0 = rem;
        const int64_t steps0 = steps;
        const int last_flip0 = last_flip;
        const int a_last0 = last_flip0 >= 0 ? dist(last_flip0) : 0;
        int cut_after = 0, nb_after = 0;
        // contiguity undecided by the ring rule at slot f: wave BFS on the current state
        auto run_bfs = [&](int f) -> bool {
            const uint32_t pkf = rlu(pk, f), nbrAf = rlu(pk2, f) & rlu(pk2, f) >> 16;
            int my_target = -1;
#pragma unroll
            for (int k2 = 0; k2 < RMAX / 2; ++k2) {
                const uint32_t wrd = rlu(rec.ring[k2], f);
                if ((lane >> 1) == k2) my_target = (int)((wrd >> (16 * (lane & 1))) & 0xffffu);
            }
            if (!(lane < RMAX && ((nbrAf >> lane) & 1u))) my_target = -1;
            ++bfs_calls;
            FC_STAMP(t_b0);
            bool res;
            if (coop) {
                // hand the search to the whole workgroup (coop_bfs): sources by label order
                const bool srcl = my_target >= 0;
                const uint64_t SM = __ballot(srcl);
                const int nsrc = __popcll(SM);
                if (nsrc <= 1) {
                    res = true;
                } else {
                    if (srcl) ctl[kCtlSrc + count_below(SM)] = my_target;
                    if (lane == 0) {
                        ctl[kCtlCmd] = 1;
                        ctl[kCtlVf] = (int)(pkf & 0x7fffu);
                        ctl[kCtlA] = (int)((pkf >> 15) & 63u);
                        ctl[kCtlNs] = nsrc;
                    }
                    block_sync();
                    res = coop_bfs<RMAX>(G, a, bs, ctl, (int)threadIdx.x, (int)blockDim.x, bfs_levels);
                }
            } else {
                res = wave_bfs<RMAX>(G, a, bs, lane, (int)(pkf & 0x7fffu), (int)((pkf >> 15) & 63u), my_target,
                                     bfs_levels);
            }
            FC_STAMP(t_b1);
            FC_PROF(13, t_b1 - t_b0);
            FC_PROF(14, 1);
            return res;
        };
        while (pos < end) {
            FC_PROF(6, 1);
            const bool prop = isprop && lane >= pos && lane < end;
            // contiguity verdict when the other district does / does not touch the outer face
            bool known = true, okT, okN;
            if (st & ST_BD) {
                okT = okN = (st & ST_BR) != 0;
            } else if (nA == 0) {
                okT = okN = false;
            } else if (exact) {
                okT = s_lin;
                okN = gam ? s_cyc : s_lin;
            } else if (KM != 2 && s_cut) {
                okT = okN = false;
            } else if (KM != 2 && dgraph) {
                okT = okN = true;  // one run, or the district rule found the pieces joined
            } else {
                known = s_lin;
                okT = okN = s_lin;
            }
            int pa, pb;
            if constexpr (KM == 2) {
                pa = av ? pops1 : pops0;
                pb = av ? pops0 : pops1;
            } else {
                pa = popk[av];
                pb = popk[tgt];
            }
            const bool ok = ((av ? ng0 : ng1) > 0) ? okT : okN;
            const bool popok = (pa - pv >= pop_lo) && (pb + pv <= pop_hi);
            const bool valid = prop && known && ok && popok;
            // ---- one event at a time: the first acceptance or undecided slot -----------------
            const uint64_t VAL = __ballot(valid);
            const uint64_t EV = __ballot((valid && acc) || (prop && !known));
            const int f = EV ? __builtin_ctzll(EV) : end;
            const uint64_t segv = VAL & bits_below(f);
            const int nvalid = __popcll(segv);
            const uint32_t bits = valid ? ST_VS : (ok ? ST_IP : ST_IC);
            if (nvalid >= rem) {  // the launch's last step lies in this segment
                const int e = kth_set_bit(segv, rem);
                if (prop && lane <= e) st |= bits;
                rem = 0;
                end = e + 1;
                target_hit = true;
                break;
            }
            if (prop && lane < f) st |= bits;
            rem -= nvalid;
            pos = f;
            if (f >= end) break;
            if (KM != 3 && !((VAL >> f) & 1ull)) {
                // undecided contiguity at slot f: device BFS on the current state
                const bool res = run_bfs(f);
                if (lane == f) st |= ST_BD | (res ? ST_BR : 0u);
                continue;
            }

            // ---- KM = 3: several independent flips in one pass -----------------------------
            // The accepted slots after f are taken in slot order while they stay independent of
            // the ones taken before them: no taken node in a later slot's ring or as its node
            // (that slot's view would change: the batch ends there), no shared neighbour (the
            // neighbours' foreign-district recounts would need an order), no later proposal whose
            // population verdict changes under the taken flips.  Their neighbours' recounts run in
            // parallel (lane group g = the g-th flip), then the district tables and the nf histogram
            // take the flips one by one in slot order, and the first flip that changes an adjacency
            // bit or the slot bound is the last one applied -- exactly the one-flip-at-a-time chain.
            if constexpr (KM == 3 && MF != 0) {
                constexpr int kGrp = 64 / RMAX;  // flips per pass, RMAX lanes each (one per ring cell)
                // RMAX = 16 (MF = 1): the flips taken are packed by ring length instead (flip g owns
                // the lanes [o_g, o_g + L_g)), up to kMaxF of them in 64 lanes -- on the Delaunay
                // dual (rings of ~6) the four-flip cap ended 0.68 selections per pass of the slowest
                // chains; on RMAX = 8 lattices the longer selection cost more than it saved
                constexpr bool kPack = MF == 1 && RMAX == 16;
                // RMAX = 8 (MF = 1): a taken flip that changes a later proposal's population verdict
                // does not end the selection; every later slot's verdict is re-read under the
                // populations after the flips taken before it (vcur), and the next candidate follows
                // from it (C4: 0.39 selections per pass ended there; +6 % per launch.  On C5 the
                // extra registers cost more than the 0.04-0.13 ends per pass it saves)
                constexpr bool kReeval = MF == 1 && !kPack;
                constexpr int kMaxF = kPack ? 16 : kGrp;
                const uint64_t CANDM = __ballot(valid && acc) & lane_range(f, end);
                if (__popcll(CANDM) >= 2) {
                    FC_PROF(21, 1);
                    FC_STAMP(t_m0);
                    uint64_t FM = 0;
                    int nF = 0;
                    int cutA = end;     // first slot whose view a taken flip changed (the batch ends there)
                    int cutP = kWave;   // first proposal whose population verdict changed
                    int dA = 0, dT = 0; // this slot's district populations moved by the taken flips
                    int gi = lane / RMAX, ge = lane % RMAX;
                    uint64_t S = 0;    // kPack: group starts (lane o_g of each flip taken)
                    int cumL = 0;      // kPack: lanes the groups span
                    bool cap_end = false;
                    // lane group g <- the g-th flip (slot order) of mask M: its data, and this lane's
                    // ring cell of it
                    int mg, vm, Am, Tm, um;
                    uint32_t pkm, pk2m, pk3m, nbrm;
#define FC_MAP_GROUPS(M, CNT)                                                                 \
    do {                                                                                      \
        mg = gi < (CNT) ? select_bit64((M), gi) : f;                                          \
        pkm = (uint32_t)__shfl((int)pk, mg);                                                  \
        pk2m = (uint32_t)__shfl((int)pk2, mg);                                                \
        pk3m = (uint32_t)__shfl((int)pk3, mg);                                                \
        vm = (int)(pkm & 0x7fffu);                                                            \
        Am = (int)((pkm >> 15) & 63u);                                                        \
        Tm = (int)((pkm >> 21) & 63u);                                                        \
        nbrm = pk2m >> 16;                                                                    \
        uint32_t selm_ = 0;                                                                   \
        _Pragma("unroll") for (int k2 = 0; k2 < RMAX / 2; ++k2) {                             \
            const uint32_t w_ = (uint32_t)__shfl((int)rec.ring[k2], mg);                      \
            if ((ge >> 1) == k2) selm_ = w_;                                                  \
        }                                                                                     \
        um = (int)((selm_ >> (16 * (ge & 1))) & 0xffffu);                                     \
    } while (0)
                    int nT = kMaxF;  // MF = 2: the first candidate sharing a neighbour with an earlier one
                    bool nb_k = false;  // MF = 2: this lane's cell is a neighbour of its group's candidate
                    NodeRec<RMAX> ru;   // MF = 2: that neighbour's node record, loaded during the selection
                    if constexpr (MF == 2) {
                        // the first kGrp candidates mapped before the selection: their neighbours'
                        // exact marks, all at once (byte u holds the candidates, bit g, having u as a
                        // neighbour: one LDS round trip instead of one per member), and the
                        // neighbours' records for the recount below, whose loads fly meanwhile
                        const int nK = min(__popcll(CANDM), kGrp);
                        FC_MAP_GROUPS(CANDM, nK);
                        nb_k = gi < nK && ((nbrm >> ge) & 1u);
                        ru = G[nb_k ? um : vm];
                        if (nb_k) atomicOr(&mk32[um >> 2], (1u << gi) << (8 * (um & 3)));
                        compiler_fence();
                        const uint32_t mkv = nb_k ? (uint32_t)mk8[um] : 0u;
                        const uint64_t CL = __ballot((mkv & ((1u << gi) - 1u)) != 0u);
                        nT = CL ? (int)(__builtin_ctzll(CL) / RMAX) : nK;
                    }
                    uint64_t CC = CANDM;
                    bool vcur = valid;  // kReeval: this slot's verdict after the flips taken before it
                    while (CC && nF < nT) {
                        const int i = __builtin_ctzll(CC);
                        CC &= CC - 1ull;
                        if (i >= cutA || i >= cutP) {
                            FC_PROF(i >= cutA ? 29 : 30, 1);
                            break;
                        }
                        if constexpr (MF == 1) {  // (statement order kept: hipcc spills 13 more VGPRs otherwise)
                            const int Li = kPack ? max((int)rlu(Ln, i), 1) : RMAX;
                            if (kPack && cumL + Li > kWave) {
                                cap_end = true;
                                break;
                            }
                            const int vi = rl32(v, i);
                            const uint32_t pki = rlu(pk, i), nbri = rlu(pk2, i) >> 16;
                            const int Ai = (int)((pki >> 15) & 63u), Ti = (int)((pki >> 21) & 63u);
                            const int pvi = rl32(pv, i);
                            uint32_t rwi[RMAX / 2];
#pragma unroll
                            for (int k2 = 0; k2 < RMAX / 2; ++k2) rwi[k2] = rlu(rec.ring[k2], i);
                            // its neighbours against the marks of the flips taken before it
                            uint32_t sel = rwi[0];
#pragma unroll
                            for (int k2 = 1; k2 < RMAX / 2; ++k2) sel = ((lane >> 1) == k2) ? rwi[k2] : sel;
                            const int ui = (int)((sel >> (16 * (lane & 1))) & 0xffffu);
                            const bool isn = lane < RMAX && ((nbri >> lane) & 1u);
                            if (nF > 0) {
                                const bool clash = isn && ((hb[(ui & kHbMask) >> 5] >> (ui & 31)) & 1u);
                                if (__any(clash)) {
                                    FC_PROF(31, 1);
                                    break;
                                }
                            }
                            if (isn) atomicOr(&hb[(ui & kHbMask) >> 5], 1u << (ui & 31));
                            FM |= 1ull << i;
                            ++nF;
                            if constexpr (kPack) {
                                S |= 1ull << cumL;
                                cumL += Li;
                            }
                            // later slots whose node is vi or has vi in its own ring (rings are symmetric)
                            bool stl = v == vi;
#pragma unroll
                            for (int k2 = 0; k2 < RMAX / 2; ++k2)
                                stl |= (rec.ring[k2] & 0xffffu) == (uint32_t)vi || (rec.ring[k2] >> 16) == (uint32_t)vi;
                            const uint64_t SM = __ballot(stl && has && lane > i && lane < end);
                            if (SM && __builtin_ctzll(SM) < cutA) cutA = __builtin_ctzll(SM);
                            // the populations of later slots' districts after this flip
                            dA += (av == Ti ? pvi : 0) - (av == Ai ? pvi : 0);
                            dT += (tgt == Ti ? pvi : 0) - (tgt == Ai ? pvi : 0);
                            const bool pok2 = (pa + dA - pv >= pop_lo) && (pb + dT + pv <= pop_hi);
                            if constexpr (kReeval) {
                                if (lane > i) vcur = prop && known && ok && pok2;
                                CC = __ballot(vcur && acc) & lane_range(i + 1, end);
                            } else {
                                const uint64_t PM = __ballot(prop && lane > i && pok2 != popok);
                                if (PM && __builtin_ctzll(PM) < cutP) cutP = __builtin_ctzll(PM);
                            }
                        } else {
                            const int vi = rl32(v, i);
                            const uint32_t pki = rlu(pk, i);
                            const int Ai = (int)((pki >> 15) & 63u), Ti = (int)((pki >> 21) & 63u);
                            const int pvi = rl32(pv, i);
                            FM |= 1ull << i;
                            ++nF;
                            // later slots whose node is vi or has vi in its own ring (rings are symmetric)
                            bool stl = v == vi;
#pragma unroll
                            for (int k2 = 0; k2 < RMAX / 2; ++k2)
                                stl |= (rec.ring[k2] & 0xffffu) == (uint32_t)vi || (rec.ring[k2] >> 16) == (uint32_t)vi;
                            const uint64_t SM = __ballot(stl && has && lane > i && lane < end);
                            if (SM && __builtin_ctzll(SM) < cutA) cutA = __builtin_ctzll(SM);
                            // the populations of later slots' districts after this flip
                            dA += (av == Ti ? pvi : 0) - (av == Ai ? pvi : 0);
                            dT += (tgt == Ti ? pvi : 0) - (tgt == Ai ? pvi : 0);
                            const bool pok2 = (pa + dA - pv >= pop_lo) && (pb + dT + pv <= pop_hi);
                            const uint64_t PM = __ballot(prop && lane > i && pok2 != popok);
                            if (PM && __builtin_ctzll(PM) < cutP) cutP = __builtin_ctzll(PM);
                        }
                    }
                    if (MF == 2 && CC && nF == nT && nT < kGrp) FC_PROF(31, 1);
                    if (CC && (nF == kMaxF || cap_end)) FC_PROF(28, 1);
                    FC_STAMP(t_m1);
                    FC_PROF(23, t_m1 - t_m0);
                    const int f_last = 63 - __builtin_clzll(FM);
                    const uint64_t VALc = kReeval ? __ballot(vcur) : VAL;
                    const int nv = __popcll(VALc & lane_range(f, f_last + 1));
                    if constexpr (MF == 1) {  // the flips taken (mapped here: keeps the selection's registers)
                        if constexpr (kPack) {
                            const uint64_t upS = S & bits_below(lane + 1);
                            gi = lane < cumL ? __popcll(upS) - 1 : kMaxF;
                            ge = lane < cumL ? lane - (63 - __builtin_clzll(upS)) : 0;
                        }
                        mg = gi < nF ? select_bit64(FM, gi) : f;
                        pkm = (uint32_t)__shfl((int)pk, mg);
                        pk2m = (uint32_t)__shfl((int)pk2, mg);
                        pk3m = (uint32_t)__shfl((int)pk3, mg);
                        vm = (int)(pkm & 0x7fffu);
                        Am = (int)((pkm >> 15) & 63u);
                        Tm = (int)((pkm >> 21) & 63u);
                        nbrm = pk2m >> 16;
                        uint32_t selm = 0;
#pragma unroll
                        for (int k2 = 0; k2 < RMAX / 2; ++k2) {
                            const uint32_t w = (uint32_t)__shfl((int)rec.ring[k2], mg);
                            if ((ge >> 1) == k2) selm = w;
                        }
                        um = (int)((selm >> (16 * (ge & 1))) & 0xffffu);
                    }
#undef FC_MAP_GROUPS
                    const bool in_g = gi < nF;
                    const bool nb_m = in_g && ((nbrm >> ge) & 1u);
                    // exact recount of the neighbour's foreign districts before / after its flip,
                    // reading the flipped node's district as Am / Tm (nothing is written yet)
                    int old_m = 0, nfn_m = 0, au_m = 0;
                    if (nb_m) {
                        if constexpr (MF == 1) ru = G[um];
                        au_m = dist(um);
                        const uint32_t nbu = (uint32_t)(ru.meta >> kMetaNbrShift) & 0xffffu;
                        uint32_t du = 0, du0 = 0;
                        // every ring cell read (valid nodes), all issued before the first use;
                        // the neighbour bit masks the district bit in
                        int xr[RMAX];
#pragma unroll
                        for (int k = 0; k < RMAX; ++k) {
                            const int w = ring_entry<RMAX>(ru.ring, k);
                            xr[k] = PK ? (int)pkb[w] : (int)a[w];
                        }
#pragma unroll
                        for (int k = 0; k < RMAX; ++k) asm volatile("" : "+v"(xr[k]));
#pragma unroll
                        for (int k = 0; k < RMAX; ++k) {
                            const int w = ring_entry<RMAX>(ru.ring, k);
                            const uint32_t nk = (nbu >> k) & 1u;
                            const int xd = PK ? (xr[k] & 31) : xr[k];
                            du |= nk << (w == vm ? Tm : xd);
                            du0 |= nk << (w == vm ? Am : xd);
                        }
                        nfn_m = __popc(du & ~(1u << au_m));
                        old_m = __popc(du0 & ~(1u << au_m));
                    }
                    const bool grew_m = nb_m && nfn_m > old_m;
                    // entering non-hit draws: the flip's grown node drawn later as a non-hit
                    int t_na = trunc_off;
                    {
                        const int off_m = __shfl(off_l, mg);
                        uint64_t ge_m = __ballot(grew_m);
                        while (ge_m) {
                            const int ln = __builtin_ctzll(ge_m);
                            ge_m &= ge_m - 1ull;
                            const int u = rl32(um, ln), ofm = rl32(off_m, ln);
#pragma unroll
                            for (int r = 0; r < NSUB; ++r) {
                                const uint64_t m2 = __ballot(((nonhit[r] >> lane) & 1ull) && rv[r] == u && 64 * r + lane > ofm);
                                if (m2 && 64 * r + __builtin_ctzll(m2) < t_na) t_na = 64 * r + __builtin_ctzll(m2);
                            }
                        }
                    }
                    const int e2 = t_na < trunc_off ? __popcll(__ballot(has && off_l < t_na)) : kWave;
                    FC_STAMP(t_m2);
                    FC_PROF(24, t_m2 - t_m1);
                    if (nF < 2 || nv >= rem || e2 <= f_last) {
                        FC_PROF(27, 1);
                        // not worth it, or the launch's last step / an entering draw lies inside:
                        // clear the marks and take f alone
                        if constexpr (MF == 1) {
                            if (nb_m) hb[(um & kHbMask) >> 5] = 0u;
                        } else {
                            if (nb_k) mk8[um] = 0u;
                        }
                        compiler_fence();
                    } else {
                        // district tables and nf histogram: all flips at once, decrements before
                        // increments.  A count that reaches 0 there (or an increment from 0, or a slot
                        // bound move) is the only way some prefix of the flips, taken in slot order, can
                        // change an adjacency bit or the bound; otherwise all apply unchanged.  When
                        // one might, the counts are restored and the flips go one by one.
                        int nA_ = nF;  // flips applied
                        bool adj_chg = false, wcap_chg = false;
                        const int Lm = __shfl((int)Ln, mg);
                        const bool gamm = (pkm >> 27) & 1u;
                        const int nf_af = (int)((pk3m >> 22) & 31u), nf_bf = (int)(pk3m >> 27);
                        const int Xm = (in_g && ge < Lm) ? dist(um) : Am;
                        const bool decA = in_g && ge < Lm && Xm != Am, incT = in_g && ge < Lm && Xm != Tm;
                        const bool gml = in_g && ge == 0 && gamm;
                        const bool hN = nb_m && nfn_m != old_m, hS = in_g && ge == 0 && nf_af != nf_bf;
                        const int pA = min(Am, Xm) * p.k + max(Am, Xm), pT = min(Tm, Xm) * p.k + max(Tm, Xm);
                        int r0 = 2, r1 = 2, r2 = 2, r3 = 2, i0 = 1, i1 = 1;
                        if (decA) r0 = atomicSub(&mcnt[pA], 1);
                        if (gml) r1 = atomicSub(&ngk[Am], 1);
                        if (hN) r2 = atomicSub(&nfh[old_m], 1);
                        if (hS) r3 = atomicSub(&nfh[nf_bf], 1);
                        if (incT) i0 = atomicAdd(&mcnt[pT], 1);
                        if (gml) i1 = atomicAdd(&ngk[Tm], 1);
                        if (hN) atomicAdd(&nfh[nfn_m], 1);
                        if (hS) atomicAdd(&nfh[nf_af], 1);
                        bool risk = r0 == 1 || r1 == 1 || i0 == 0 || i1 == 0;
                        if (p.wdyn)
                            risk = risk || (hN && (nfn_m > wcap || (old_m == wcap && r2 == 1))) ||
                                   (hS && (nf_af > wcap || (nf_bf == wcap && r3 == 1)));
                        if (__any(risk)) {
                            FC_PROF(20, 1);
                            if (decA) atomicAdd(&mcnt[pA], 1);
                            if (gml) atomicAdd(&ngk[Am], 1);
                            if (hN) atomicAdd(&nfh[old_m], 1);
                            if (hS) atomicAdd(&nfh[nf_bf], 1);
                            if (incT) atomicSub(&mcnt[pT], 1);
                            if (gml) atomicSub(&ngk[Tm], 1);
                            if (hN) atomicSub(&nfh[nfn_m], 1);
                            if (hS) atomicSub(&nfh[nf_af], 1);
                            compiler_fence();
                            nA_ = 0;
                            for (int g = 0; g < nF; ++g) {
                                bool chg = false;
                                if (gi == g && ge < Lm) {
                                    if (decA && atomicSub(&mcnt[pA], 1) == 1) {
                                        atomicAnd(&adj[Am], ~(1u << Xm));
                                        atomicAnd(&adj[Xm], ~(1u << Am));
                                        chg = true;
                                    }
                                    if (incT && atomicAdd(&mcnt[pT], 1) == 0) {
                                        atomicOr(&adj[Tm], 1u << Xm);
                                        atomicOr(&adj[Xm], 1u << Tm);
                                        chg = true;
                                    }
                                }
                                if (gi == g && gml) {
                                    if (atomicSub(&ngk[Am], 1) == 1) {
                                        atomicAnd(&adj[Am], ~(1u << 31));
                                        atomicAnd(&adj[31], ~(1u << Am));
                                        chg = true;
                                    }
                                    if (atomicAdd(&ngk[Tm], 1) == 0) {
                                        atomicOr(&adj[Tm], 1u << 31);
                                        atomicOr(&adj[31], 1u << Tm);
                                        chg = true;
                                    }
                                }
                                if (gi == g && hN) {
                                    atomicSub(&nfh[old_m], 1);
                                    atomicAdd(&nfh[nfn_m], 1);
                                }
                                if (gi == g && hS) {
                                    atomicSub(&nfh[nf_bf], 1);
                                    atomicAdd(&nfh[nf_af], 1);
                                }
                                ++nA_;
                                adj_chg = __any(chg);
                                if (p.wdyn) {
                                    compiler_fence();
                                    const uint64_t hm = __ballot(lane >= 1 && lane < kNfh && nfh[lane] > 0);
                                    const int wn = hm ? 63 - __builtin_clzll(hm) : 1;
                                    if (wn != wcap) {
                                        wcap = wn;
                                        wthr = (0u - (uint32_t)wcap) % (uint32_t)wcap;
                                        wcap_chg = true;
                                    }
                                }
                                if (adj_chg || wcap_chg) break;
                            }
                        }
                        FC_STAMP(t_m3);
                        FC_PROF(25, t_m3 - t_m2);
                        // the flips applied: districts and counts, populations, marks cleared
                        const bool app = gi < nA_;
                        const int pvm = __shfl(pv, mg);
                        if constexpr (MF == 1) {
                            if (nb_m) hb[(um & kHbMask) >> 5] = 0u;
                        } else {
                            if (nb_k) mk8[um] = 0u;
                        }
                        if (app && ge == 0) {
                            pkb[vm] = (uint8_t)(Tm | ((nf_af < 7 ? nf_af : 7) << 5));
                            atomicSub(&popk[Am], pvm);
                            atomicAdd(&popk[Tm], pvm);
                        }
                        if (app && nb_m && nfn_m != old_m) pkb[um] = (uint8_t)(au_m | ((nfn_m < 7 ? nfn_m : 7) << 5));
                        const bool ent_m = app && nb_m && old_m == 0 && nfn_m > 0;
                        const bool lev_m = app && nb_m && old_m > 0 && nfn_m == 0;
                        // the slots up to the last flip applied: verdict bits, |cut| / |B| after each flip
                        const int fl = nA_ == nF ? f_last : select_bit64(FM, nA_ - 1);
                        if (prop && lane >= f && lane <= fl) st |= kReeval ? (vcur ? ST_VS : (ok ? ST_IP : ST_IC)) : bits;
                        // flip of rank rk (slot order): |cut| after it = cut + the first rk+1 deltas
                        // (lane group g holds flip g's delta), |B| = nb + the entering / leaving
                        // neighbours of lane groups 0..rk
                        const int rk = count_below(FM);
                        const int dm = (int)((pk3m >> 16) & 0x3fu) - 32;
                        int csum = 0, my_cs = 0, my_up = 0;
                        if constexpr (!kPack) {
#pragma unroll
                            for (int g = 0; g < kGrp; ++g)
                                if (g < nA_) {
                                    csum += rl32(dm, g * RMAX);
                                    my_cs = rk == g ? csum : my_cs;
                                }
                            my_up = (rk + 1) * RMAX;
                        } else {
                            uint64_t SS = S;
                            for (int g = 0; g < nA_; ++g) {
                                const int o = __builtin_ctzll(SS);
                                SS &= SS - 1ull;
                                csum += rl32(dm, o);
                                const int nx = SS ? __builtin_ctzll(SS) : cumL;  // lanes of groups 0..g
                                my_cs = rk == g ? csum : my_cs;
                                my_up = rk == g ? nx : my_up;
                            }
                        }
                        const uint64_t ENT = __ballot(ent_m), LEV = __ballot(lev_m);
                        if (((FM >> lane) & 1ull) && rk < nA_) {
                            const uint64_t upto = bits_below(my_up);
                            st |= ST_VS | ST_AC;
                            cut_after = cut + my_cs;
                            nb_after = nb + __popcll(ENT & upto) - __popcll(LEV & upto);
                        }
                        cut += csum;
                        nb += __popcll(ENT) - __popcll(LEV);
                        rem -= __popcll(VALc & lane_range(f, fl + 1));
                        last_flip = rl32(v, fl);
                        compiler_fence();
                        FC_PROF(7, nA_);
                        FC_PROF(22, nA_);
                        // what ends the batch after them: a changed view, adjacency or slot bound, an
                        // entering draw
                        if (cutA < end) end = cutA;
                        if ((adj_chg || wcap_chg) && fl + 1 < end) end = fl + 1;
                        if (wcap_chg) {
                            const int t_w = rl32(off_l, fl) + 1;
                            if (t_w < trunc_off) trunc_off = t_w;
                        }
                        if (t_na < trunc_off) {
                            trunc_off = t_na;
                            if (e2 < end) end = e2;
                        }
                        pos = fl + 1;
                        FC_STAMP(t_m4);
                        FC_PROF(26, t_m4 - t_m3);
                        continue;
                    }
                }
            }
            // ---- accept slot f: apply the flip -----------------------------------------
            FC_PROF(7, 1);
            const uint32_t pkf = rlu(pk, f), pk2f = rlu(pk2, f), pk3f = rlu(pk3, f);
            const int vf = (int)(pkf & 0x7fffu), Af = (int)((pkf >> 15) & 63u), tf = (int)((pkf >> 21) & 63u);
            const bool gamf = (pkf >> 27) & 1u;
            const int df = (int)((pk3f >> 16) & 0x3fu) - 32;
            const int pvf = rl32(pv, f);
            const uint32_t inAf = pk2f & 0xffffu, nbrf = pk2f >> 16, tmf = pk3f & 0xffffu;
            uint32_t rw[RMAX / 2];
#pragma unroll
            for (int k2 = 0; k2 < RMAX / 2; ++k2) rw[k2] = rlu(rec.ring[k2], f);
            uint32_t sel = rw[0];
#pragma unroll
            for (int k2 = 1; k2 < RMAX / 2; ++k2) sel = ((lane >> 1) == k2) ? rw[k2] : sel;
            const int my_e = (int)((sel >> (16 * (lane & 1))) & 0xffffu);
            const bool is_nbr = lane < RMAX && ((nbrf >> lane) & 1u);
            FC_STAMP(t_g1);
            bool enter = false, leave = false, grew = false;
            bool wcap_chg = false;
            int dpair = 0;  // FC_FLAG_NB_PAIRS: this lane's change of the (node, district) pair count
            if constexpr (KM == 2) {
                // foreign-neighbour counts: u sees v leave A (+1 if u in A) and join t (-1 if u in t)
                const int dlt = (int)((inAf >> lane) & 1u) - (int)((tmf >> lane) & 1u);
                if (is_nbr && dlt != 0) {
                    const int old = fcnt[my_e];
                    fcnt[my_e] = (uint8_t)(old + dlt);
                    enter = dlt > 0 && old == 0;
                    leave = dlt < 0 && old == 1;
                }
                grew = enter;
            } else {
                // foreign districts nf(u) of vf's neighbours, recounted on the new state (v
                // leaving A can drop A from u's foreign set, joining T add T), and vf's own
                // from the evaluation; nfh follows every change, and with it the slot bound
                const int nf_af = (int)((pk3f >> 22) & 31u), nf_bf = (int)(pk3f >> 27);
                if (lane == 0) {
                    if constexpr (PK) pkb[vf] = (uint8_t)(tf | ((nf_af < 7 ? nf_af : 7) << 5));
                    else a[vf] = (int8_t)tf;
                }
                compiler_fence();
                if (is_nbr) {
                    const NodeRec<RMAX> ru = G[my_e];
                    const int au = dist(my_e);
                    const uint32_t nbu = (uint32_t)(ru.meta >> kMetaNbrShift) & 0xffffu;
                    uint32_t du = 0, du0 = 0;  // districts among u's neighbours after / before the flip
                    // (every ring cell read, the reads issued together; the neighbour bit masks)
                    int xr[RMAX];
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) {
                        const int w = ring_entry<RMAX>(ru.ring, i);
                        xr[i] = PK ? (int)pkb[w] : (int)a[w];
                    }
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) asm volatile("" : "+v"(xr[i]));
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) {
                        const int w = ring_entry<RMAX>(ru.ring, i);
                        const uint32_t ni = (nbu >> i) & 1u;
                        const int xw = PK ? (xr[i] & 31) : xr[i];
                        du |= ni << xw;
                        du0 |= ni << (w == vf ? Af : xw);
                    }
                    const int nfn = __popc(du & ~(1u << au));
                    // the old count: exact from the ring when packed (a stored 7 may stand for more)
                    const int old = PK ? __popc(du0 & ~(1u << au)) : (int)fcnt[my_e];
                    if (nfn != old) {
                        if constexpr (PK) pkb[my_e] = (uint8_t)(au | ((nfn < 7 ? nfn : 7) << 5));
                        else fcnt[my_e] = (uint8_t)nfn;
                        atomicSub(&nfh[old], 1);
                        atomicAdd(&nfh[nfn], 1);
                    }
                    enter = old == 0 && nfn > 0;
                    leave = old > 0 && nfn == 0;
                    grew = nfn > old;
                    dpair = nfn - old;
                }
                if (lane == 0) {
                    // vf's own count: before / after from its evaluation (its view was current)
                    const int old = PK ? nf_bf : (int)fcnt[vf];
                    dpair += nf_af - old;
                    if (nf_af != old) {
                        if constexpr (!PK) fcnt[vf] = (uint8_t)nf_af;
                        atomicSub(&nfh[old], 1);
                        atomicAdd(&nfh[nf_af], 1);
                    }
                }
                if (p.wdyn) {
                    compiler_fence();
                    const uint64_t hm = __ballot(lane >= 1 && lane < kNfh && nfh[lane] > 0);
                    const int wn = hm ? 63 - __builtin_clzll(hm) : 1;
                    if (wn != wcap) {  // later draws of the batch map to other slots: end it after f
                        wcap = wn;
                        wthr = (0u - (uint32_t)wcap) % (uint32_t)wcap;
                        wcap_chg = true;
                    }
                }
            }
            FC_STAMP(t_g2);
            FC_PROF(9, t_g2 - t_g1);
            // non-hit draws to re-check below: nodes that entered the boundary; with PAIR
            // slots any node whose foreign-district count grew (its slot may now fall below it)
            uint64_t ent = __ballot(grew);
            int dnb = __popcll(__ballot(enter)) - __popcll(__ballot(leave));
            if constexpr (KM != 2)
                if (p.nb_pairs) dnb = rl32(wave_scan_incl(dpair), 63);
            // district-graph tables: the pairs {vf, w} of vf's face-adjacent cells w move from
            // (Af, a[w]) to (tf, a[w]); a count crossing 0 flips an adjacency bit (as does an
            // outer-face node crossing between districts), which may change the verdict of a
            // later slot: the batch then ends after this flip
            bool adj_chg = false;
            FC_STAMP(t_g0);
            if (dgraph) {
                const int Lf = rl32((int)Ln, f);
                bool chg = false;
                if (lane < Lf) {
                    const int X = dist(my_e);
                    if (X != Af && atomicSub(&mcnt[min(Af, X) * p.k + max(Af, X)], 1) == 1) {
                        atomicAnd(&adj[Af], ~(1u << X));
                        atomicAnd(&adj[X], ~(1u << Af));
                        chg = true;
                    }
                    if (X != tf && atomicAdd(&mcnt[min(tf, X) * p.k + max(tf, X)], 1) == 0) {
                        atomicOr(&adj[tf], 1u << X);
                        atomicOr(&adj[X], 1u << tf);
                        chg = true;
                    }
                }
                if (lane == 0 && gamf) {
                    if (atomicSub(&ngk[Af], 1) == 1) {
                        atomicAnd(&adj[Af], ~(1u << 31));
                        atomicAnd(&adj[31], ~(1u << Af));
                        chg = true;
                    }
                    if (atomicAdd(&ngk[tf], 1) == 0) {
                        atomicOr(&adj[tf], 1u << 31);
                        atomicOr(&adj[31], 1u << tf);
                        chg = true;
                    }
                }
                adj_chg = __any(chg);
            }
            FC_STAMP(t_g4);
            FC_PROF(8, t_g4 - t_g0);
            if (lane == 0) {
                if constexpr (KM == 2) {
                    a[vf] = (int8_t)tf;
                    fcnt[vf] = (uint8_t)(__popc(nbrf) - __popc(tmf));
                } else {
                    popk[Af] -= pvf;
                    popk[tf] += pvf;
                }
            }
            if constexpr (KM == 2) {
                if (Af == 0) { pops0 -= pvf; pops1 += pvf; } else { pops1 -= pvf; pops0 += pvf; }
                if (gamf) { if (Af == 0) { --ng0; ++ng1; } else { --ng1; ++ng0; } }
            }
            cut += df;
            nb += dnb;
            --rem;
            last_flip = vf;
            if (lane == f) {
                st |= ST_VS | ST_AC;
                cut_after = cut;
                nb_after = nb;
            }
            // slots after f whose node lies in R(vf) + {vf} (rings are symmetric) saw a stale
            // neighbourhood
            bool hit = v == vf;
#pragma unroll
            for (int i = 0; i < RMAX; ++i) hit |= v == (int)((rw[i >> 1] >> (16 * (i & 1))) & 0xffffu);
            const uint64_t aff = __ballot(hit && lane > f && lane < end);
            if (aff) end = __builtin_ctzll(aff);
            FC_PROF(11, aff ? 1 : 0);
            FC_PROF(15, adj_chg && f + 1 < end ? 1 : 0);
            FC_PROF(16, wcap_chg && f + 1 < end ? 1 : 0);
            if (adj_chg && f + 1 < end) end = f + 1;
            if (wcap_chg) {  // every later draw of the batch is re-read under the new bound
                if (f + 1 < end) end = f + 1;
                const int t_w = rl32(off_l, f) + 1;
                if (t_w < trunc_off) trunc_off = t_w;
            }
            // non-hit draws after f whose node just entered the boundary would now propose
            if (ent) {
                const int off_f = rl32(off_l, f);
                int t_na = trunc_off;
                while (ent) {
                    const int u = rl32(my_e, __builtin_ctzll(ent));
                    ent &= ent - 1;
#pragma unroll
                    for (int r = 0; r < NSUB; ++r) {
                        const uint64_t m2 = __ballot(((nonhit[r] >> lane) & 1ull) && rv[r] == u && 64 * r + lane > off_f);
                        if (m2) {
                            const int t = 64 * r + __builtin_ctzll(m2);
                            if (t < t_na) t_na = t;
                        }
                    }
                }
                if (t_na < trunc_off) {
                    trunc_off = t_na;
                    const int e2 = __popcll(__ballot(has && off_l < t_na));
                    FC_PROF(12, e2 < end ? 1 : 0);
                    if (e2 < end) end = e2;
                }
            }
            FC_STAMP(t_g3);
            FC_PROF(10, t_g3 - t_g2);
            compiler_fence();
            pos = f + 1;
            if (rem == 0) {
                end = pos;
                target_hit = true;
                break;
            }
        }
        // draws consumed by the committed slots [0, end)
        int consumed;
        if (target_hit) {
            consumed = rl32(off_l, end - 1) + 1;
        } else {
            consumed = end < ns ? rl32(off_l, end) : gen;
            if (trunc_off < consumed) consumed = trunc_off;
        }
        steps = steps0 + (rem0 - rem);
        FC_STAMP(t_d);
        FC_PROF(3, t_d - t_c);

        // ---- 3. lane-parallel bookkeeping of the committed batch ----------------------------
        const bool done = lane < end;
        const bool is_acc = (st & ST_AC) != 0;
        n_prop += (isprop && done) ? 1u : 0u;
        n_acc += is_acc ? 1u : 0u;
        n_ic += (st & ST_IC) ? 1u : 0u;
        n_ip += (st & ST_IP) ? 1u : 0u;
        const uint64_t ACCM = __ballot(is_acc);
        const uint64_t VSM = __ballot((st & ST_VS) != 0);
        const uint64_t later_acc = ACCM & ~bits_below(lane + 1);
        const int next_acc = later_acc ? __builtin_ctzll(later_acc) : end;
        const int run_len = is_acc ? 1 + __popcll(VSM & lane_range(lane + 1, next_acc)) : 0;
        const int first_acc = ACCM ? __builtin_ctzll(ACCM) : end;
        const int r0 = __popcll(VSM & bits_below(first_acc));
        int64_t my_wait = 0;
        const int na = __popcll(ACCM);
        // the start state's r0 further yields: its queue entry if it is queued, else wait_cur
        // (charged below, before anything can change wait_cur)
        const bool r0_queued = qn > 0;
        if (lane == 0 && r0 && r0_queued) q_run[qn - 1] += (uint32_t)r0;
        if (lane == 0 && r0 && !r0_queued) acc_wait += wait_cur * r0;
        // drain a non-empty queue that cannot take this batch (an empty one has nothing to
        // draw, and its flush would leave wait_cur undefined)
        if (defer && na && qn > 0 && qn + na > p.wait_q) wait_flush();
        // a batch with more acceptances than the queue holds draws its waits now (queue empty)
        const bool queue_now = defer && na <= p.wait_q;
        if (want_wait && !queue_now && is_acc) {
            Words4 g;
            if (FULL && p.tape) {
                const uint32_t *t = p.tape + ((size_t)c * (size_t)p.tape_draws + d) * 6;
                g = Words4{t[4], t[5], 0u, 0u};
            } else {
                g = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), chain_gid, 1u, p.seed_lo, p.seed_hi);
            }
            const double U = u53(g.x0, g.x1);
            my_wait = geom_from(U, p.log1mp[nb_after]);
        }
        if (is_acc) {
            acc_cut += (int64_t)cut_after * run_len;
            acc_cut2 += (int64_t)cut_after * cut_after * run_len;
            acc_nb += (int64_t)nb_after * run_len;
            acc_nb2 += (int64_t)nb_after * nb_after * run_len;
            if (!queue_now) acc_wait += my_wait * run_len;
        }
        if (lane == 0 && r0) {
            acc_cut += (int64_t)cut0 * r0;
            acc_cut2 += (int64_t)cut0 * cut0 * r0;
            acc_nb += (int64_t)nb0 * r0;
            acc_nb2 += (int64_t)nb0 * nb0 * r0;
        }
        if (queue_now && na) {
            const int qi = qn + count_below(ACCM);
            if (is_acc) {
                q_d[qi] = d;
                q_nb[qi] = (uint32_t)nb_after;
                q_run[qi] = (uint32_t)run_len;
            }
            qn += na;
            compiler_fence();
        }
        const int64_t t_acc = steps0 + __popcll(VSM & bits_below(lane + 1));  // yield index of this slot
        if (FULL && (p.diag & FC_DIAG_SERIES) && ACCM) {
            const int64_t idx = ev_len + __popcll(ACCM & bits_below(lane));
            if (is_acc && idx < p.ev_cap) {
                fc_event ev;
                ev.t = t_acc;
                ev.v = (uint16_t)v;
                ev.cut = (uint16_t)cut_after;
                ev.nb = (uint16_t)nb_after;
                ev.target = (uint8_t)tgt;
                ev.reserved = 0;
                p.events[(size_t)c * p.ev_cap + idx] = ev;
            }
            ev_len += __popcll(ACCM);
        }
        if (FULL && hit_time < 0 && ACCM) {
            const uint64_t hm = __ballot(is_acc && cut_after >= p.hit_lo && cut_after <= p.hit_hi);
            if (hm) hit_time = (int64_t)__shfl((long long)t_acc, __builtin_ctzll(hm));
        }
        if (FULL && (p.diag & (FC_DIAG_HIST | FC_DIAG_FLIPS | FC_DIAG_FLIPS_EXACT | FC_DIAG_EDGES))) {
            if (p.diag & FC_DIAG_HIST) {
                if (is_acc) {
                    atomicAdd((unsigned long long *)&p.cut_hist[(size_t)c * (p.n_edges + 1) + cut_after], (unsigned long long)run_len);
                    atomicAdd((unsigned long long *)&p.nb_hist[(size_t)c * p.nb_w + nb_after], (unsigned long long)run_len);
                }
                if (lane == 0 && r0) {
                    atomicAdd((unsigned long long *)&p.cut_hist[(size_t)c * (p.n_edges + 1) + cut0], (unsigned long long)r0);
                    atomicAdd((unsigned long long *)&p.nb_hist[(size_t)c * p.nb_w + nb0], (unsigned long long)r0);
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
                    const int64_t t_last = t_acc + run_len - 1;
                    const int64_t old = (int64_t)atomicExch(lf + v, (unsigned long long)t_last);
                    atomicAdd((unsigned long long *)(ps + v), (unsigned long long)(-(int64_t)p.labels[tgt] * (t_last - old)));
                    atomicAdd((unsigned long long *)(nf + v), (unsigned long long)run_len);
                }
            }
            if ((p.diag & FC_DIAG_FLIPS_EXACT) && is_acc) {
                // corrected companions (App. A.6), as in fc_flip2.hip
                const size_t o = (size_t)c * n + v;
                const int64_t dl = (int64_t)p.labels[tgt] - (int64_t)p.labels[av];
                atomicAdd((unsigned long long *)(p.flip_count + o), 1ull);
                atomicAdd((unsigned long long *)(p.occ_acc + o), (unsigned long long)(-dl * t_acc));
                atomicMax((unsigned long long *)(p.last_accept + o), (unsigned long long)t_acc);
            }
            if ((p.diag & FC_DIAG_EDGES) && is_acc) {
                // cut_times[e] = sum of the yields at which e turns uncut - sum of those at which
                // it turns cut (+ the yield count while it is cut: fc_run_read_edges)
                int64_t *ea = p.edge_acc + (size_t)c * p.n_edges;
                for (int i = 0; i < RMAX; ++i) {
                    if (!((nbr >> i) & 1u)) continue;
                    const int e = p.ring_eid[(size_t)v * RMAX + i];
                    if ((inA >> i) & 1u) {
                        atomicAdd((unsigned long long *)(ea + e), (unsigned long long)(-t_acc));  // becomes cut
                    } else if ((tmask >> i) & 1u) {
                        atomicAdd((unsigned long long *)(ea + e), (unsigned long long)t_acc);     // becomes uncut
                    }
                }
            }
        }
        if (trace_on) {
            const uint64_t P = __ballot(isprop && done);
            const uint64_t mine = ACCM & bits_below(lane + 1);
            const int src = mine ? 63 - __builtin_clzll(mine) : 0;
            const int c_j = __shfl(cut_after, src), n_j = __shfl(nb_after, src);
            const long long w_j = __shfl((long long)my_wait, src);
            const int64_t idx = trace_len + __popcll(P & bits_below(lane));
            if (isprop && done && idx < p.trace_cap) {
                fc_record &rr = p.trace[(size_t)c * p.trace_cap + idx];
                const bool valid = (st & ST_VS) != 0;
                rr.draw = (int64_t)d;
                rr.v = v;
                rr.flags = (valid ? (1 | (is_acc ? 2 : 0)) : ((st & ST_IC) ? 4 : 8)) | (tgt << 8);
                rr.cut = mine ? c_j : cut0;
                rr.nb = mine ? n_j : nb0;
                rr.wait = valid ? (mine ? (int64_t)w_j : wait_cur) : 0;
            }
            trace_len += __popcll(P);
        }
        if (ACCM && !queue_now) wait_cur = (int64_t)__shfl((long long)my_wait, 63 - __builtin_clzll(ACCM));
        draw += (uint64_t)consumed;
        compiler_fence();
        FC_STAMP(t_e);
        FC_PROF(4, t_e - t_d);
    }
    if (defer && qn > 0) wait_flush();
    if (coop) {  // release the helper waves (every path of the chain's loop ends here)
        if (lane == 0) ctl[kCtlCmd] = 0;
        block_sync();
    }
    FC_STAMP(t_loop1);
    FC_PROF(0, t_loop1 - t_loop0);
#ifdef FC_PHASE_PROF
    wave_sync();
    if (p.prof && lane == 0)
        for (int i = 0; i < kProfSlots; ++i) p.prof[(size_t)c * kProfSlots + i] = prof_acc[i];  // after wave_sync
#endif

    // ---- write back ---------------------------------------------------------------------
    {
        uint4 *ga = (uint4 *)(p.assign + (size_t)c * npad);
        uint4 *gf = (uint4 *)(p.fcnt + (size_t)c * npad);
        for (int i = lane; i < npad / 16; i += kWave) {
            if constexpr (PK) {
                const uint4 x = ((const uint4 *)pkb)[i];
                const uint32_t xa[4] = {x.x, x.y, x.z, x.w};
                uint32_t oa[4], of[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    oa[q] = xa[q] & 0x1f1f1f1fu;
                    of[q] = (xa[q] >> 5) & 0x07070707u;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        if (((of[q] >> (8 * b)) & 0xffu) != 7u) continue;
                        // saturated: the exact count from the ring (rare)
                        const int u = 16 * i + 4 * q + b;
                        const NodeRec<RMAX> ru = G[u];
                        const int au = (int)(pkb[u] & 31u);
                        const uint32_t nbu = (uint32_t)(ru.meta >> kMetaNbrShift) & 0xffffu;
                        uint32_t du = 0;
                        for (int j = 0; j < RMAX; ++j)
                            if ((nbu >> j) & 1u) du |= 1u << dist(ring_entry<RMAX>(ru.ring, j));
                        of[q] = (of[q] & ~(0xffu << (8 * b))) | ((uint32_t)__popc(du & ~(1u << au)) << (8 * b));
                    }
                ga[i] = uint4{oa[0], oa[1], oa[2], oa[3]};
                gf[i] = uint4{of[0], of[1], of[2], of[3]};
            } else {
                ga[i] = ((const uint4 *)a)[i];
                gf[i] = ((const uint4 *)fcnt)[i];
            }
        }
        if (KM != 2 && lane < 32) {
            p.popk[(size_t)c * 32 + lane] = popk[lane];
            p.nfh[(size_t)c * kNfh + lane] = nfh[lane];
        }
        if (dgraph) {
            const int kk = p.k * p.k;
            for (int i = lane; i < kk; i += kWave) p.mcnt[(size_t)c * kk + i] = mcnt[i];
            if (lane < 32) p.ngk[(size_t)c * 32 + lane] = ngk[lane];
        }
    }
    int64_t cnt_prop = n_prop, cnt_acc = n_acc, cnt_ic = n_ic, cnt_ip = n_ip;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        acc_cut += __shfl_xor((long long)acc_cut, off);
        acc_nb += __shfl_xor((long long)acc_nb, off);
        acc_wait += __shfl_xor((long long)acc_wait, off);
        acc_cut2 += __shfl_xor((long long)acc_cut2, off);
        acc_nb2 += __shfl_xor((long long)acc_nb2, off);
        cnt_prop += __shfl_xor((long long)cnt_prop, off);
        cnt_acc += __shfl_xor((long long)cnt_acc, off);
        cnt_ic += __shfl_xor((long long)cnt_ic, off);
        cnt_ip += __shfl_xor((long long)cnt_ip, off);
    }
    if (lane == 0) {
        scp->draw = draw;
        scp->steps = steps;
        scp->proposals += cnt_prop;
        scp->accepted += cnt_acc;
        scp->inv_contig += cnt_ic;
        scp->inv_pop += cnt_ip;
        scp->bfs_calls = bfs_calls;
        scp->bfs_levels = bfs_levels;
        scp->trace_len = trace_len;
        scp->ev_len = ev_len;
        scp->hit_time = hit_time;
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

int launch_flip_k2(const KParams &p, int ring_max, void *stream, char *name, size_t name_cap) {
    // one chain (wave) per workgroup, as in fc_flip2.hip (C3 on one MI355X: 1.35e9 proposals/s
    // against 1.29e9 with four chains per workgroup); tune_chains_per_block = 2 / 4 restores larger ones
    const int wpb = p.wpb;  // fc_params.tune_chains_per_block (resolved by fc_run_create)
    const int blocks = p.coop ? p.n_chains : (p.n_chains + wpb - 1) / wpb;
    const size_t lds = (size_t)p.chain_lds_bytes * (p.coop ? 1 : wpb);
    hipStream_t s = (hipStream_t)stream;
    // cooperative search: one chain per 256-thread workgroup (wave 0 + three search helpers)
    const dim3 grid(blocks), block(p.coop ? kWave * kWavesPerBlock : kWave * wpb);
    // FULL: replay tapes, traces, event logs, histograms, per-node/per-edge tallies or a
    // hitting-time window; the lean instance (proposals, steps, sums, waits) keeps its
    // register budget for the hot loop.
    const bool full = p.tape || p.trace || (p.diag & ~(uint32_t)FC_DIAG_WAIT) || p.hit_lo <= p.hit_hi;
#define FC_LAUNCHM(R, S, K, F, M)                                                                       \
    do {                                                                                                \
        if (lds > 65536)                                                                                \
            (void)hipFuncSetAttribute((const void *)flip_kernel<R, S, K, F, M>,                         \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);            \
        if (name)                                                                                       \
            snprintf(name, name_cap, "fc::flip_kernel<%d, %d, %d, %s, %d>", R, S, K, F ? "true" : "false", \
                     (int)(M));                                                                         \
        hipLaunchKernelGGL((flip_kernel<R, S, K, F, M>), grid, block, lds, s, p);                       \
    } while (0)
    // the multi-flip instance: district-graph rule, when the run asks for it
    // (1: hashed marks; 2: exact marks, when fc_run_create found room for a byte per node)
#define FC_LAUNCH(R, S, K, F)                                                     \
    do {                                                                          \
        if (K == 3 && p.multi_flip == 2) FC_LAUNCHM(R, S, K, F, (K == 3 ? 2 : 0)); \
        else if (K == 3 && p.multi_flip) FC_LAUNCHM(R, S, K, F, (K == 3 ? 1 : 0)); \
        else FC_LAUNCHM(R, S, K, F, 0);                                            \
    } while (0)
#define FC_FULL_SWITCH(R, S, K)                          \
    do {                                                 \
        if (full) FC_LAUNCH(R, S, K, true);              \
        else FC_LAUNCH(R, S, K, false);                  \
    } while (0)
#define FC_NSUB_SWITCH(R, K)                          \
    switch (p.nsub) {                                 \
        case 1: FC_FULL_SWITCH(R, 1, K); break;       \
        case 2: FC_FULL_SWITCH(R, 2, K); break;       \
        case 4: FC_FULL_SWITCH(R, 4, K); break;       \
        default: return (int)hipErrorInvalidValue;    \
    }
    // (p.dgraph is off under FC_FLAG_FORCE_BFS, and coop needs it off)
    if (ring_max == 8) {
        if (p.coop) {
            FC_NSUB_SWITCH(8, 1)
        } else if (p.dgraph) {
            FC_NSUB_SWITCH(8, 3)
        } else {
            FC_NSUB_SWITCH(8, 0)
        }
    } else if (ring_max == 16) {
        if (p.coop) {
            FC_NSUB_SWITCH(16, 1)
        } else if (p.dgraph) {
            FC_NSUB_SWITCH(16, 3)
        } else {
            FC_NSUB_SWITCH(16, 0)
        }
    } else {
        return (int)hipErrorInvalidValue;
    }
#undef FC_NSUB_SWITCH
#undef FC_FULL_SWITCH
#undef FC_LAUNCH
#undef FC_LAUNCHM
    return (int)hipGetLastError();
}

}  // namespace fc
