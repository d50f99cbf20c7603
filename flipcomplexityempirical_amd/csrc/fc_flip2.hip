// Two-district flip-walk kernel for gfx950 (MI355X): the headline path.
//
// Reference step: MarkovChain.__next__ [gc-0.2] driving slow_reversible_propose_bi,
// single_flip_contiguous + within_percent_of_ideal_population and cut_accept
// (grid_chain_sec11.py:132-179, 299-342), plus the driver's per-yield diagnostics
// (:366-402).  k = 2 is the reference's only configuration; PAIR proposals with k = 2
// coincide with it (one foreign district).
//
// One chain per wavefront, state in LDS (int8 district, uint8 foreign-neighbour count per
// node; |B| and boundary membership are O(1)).  A wave advances its chain in batches:
//   1. a window of up to 64 NSUB draws maps to nodes (exact Lemire; the node words of four
//      draws come from one Philox call per lane); draws on boundary nodes are
//      proposals (rejection sampling of random.choice over b_nodes, grid_chain_sec11.py:143)
//      and are packed, in draw order, into up to 64 slots; the nodes of the other ("non-hit")
//      draws stay in registers;
//   2. every slot is evaluated against the current state: ring districts, contiguity by the
//      planar run rule, population bound, delta-cut, Metropolis threshold;
//   3. commit in draw order.  One event at a time when few slots of the batch accept: the
//      first acceptance is applied and every later slot whose view it changed (the flipped
//      node in its ring or as its node) is evaluated again against the new state; the first
//      later non-hit draw whose node it pulled into the boundary ends the batch.  When many
//      accept, a segment-parallel commit (commit marks in LDS + prefix scans, below) applies
//      them in one pass.  Either way the committed sequence is the one-draw-at-a-time chain,
//      bit for bit;
//   4. the per-yield diagnostics are accumulated lane-parallel from per-slot status bits.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>

#include "fc_device.h"
#include "fc_internal.h"
#include "fc_philox.h"

namespace fc {

using namespace dev;

// SEARCH = false: every node is exact and FC_FLAG_FORCE_BFS is off (p.all_exact), so the run
// rule decides every proposal and the instance carries no search code (its registers are the
// hot loop's).  XTRA (FULL only): replay tapes, per-proposal traces, accept / constraint
// variants and frozen nodes; the diagnostics instance without them keeps its registers too.
//
// BAND (FC_STREAM_BAND): a draw picks the i-th member of the chain's band S (b_nodes and their
// neighbours, an LDS bitmap) instead of one of all n nodes.  S only changes when an accepted flip
// puts a node outside S into b_nodes; the batch then ends after that flip and S is rebuilt, so
// within a batch the draw -> node map is fixed, as the speculative evaluation needs.
// the issue priority is re-chosen every 2^FC_PRIO_EVERY_LOG2 batches (scheduling only)
#ifndef FC_PRIO_EVERY_LOG2
#define FC_PRIO_EVERY_LOG2 4  // profiles/r04p_prio_period_ab.txt: 55.0 ms against 55.4 every 4 batches, 56.3 every batch
#endif
// The per-yield tallies of the reference's loop body (grid_chain_sec11.py:367-400) for one
// accepted state and its run (kind 0: a flushed queue entry -- yield t of the flip, `run` yields,
// node u | old-district ring bits << 16, |cut| | target << 31, |B|) or for the yields a batch's
// start state adds right after a flush (kind 1: yields steps0 + 1 .. steps0 + r0 of the state
// the last flip created; node last_flip | its district << 16, 0xffff: none).  Every update
// commutes (sums and maxima), so where and in which order they are applied leaves the results
// bit-identical: inside the flip kernel (a full log) or by tally_reduce after the launch.
template <int RMAX>
__device__ __forceinline__ void tally_apply(const KParams &p, int c, int64_t t, int run, uint32_t qv, uint32_t qc,
                                            uint32_t nbk, int64_t lab0, int64_t lab1) {
    const int n = p.n;
    const int cq = (int)(qc & 0x7fffffffu), nbq = (int)(nbk & 0x7fffffffu);
    if (p.diag & FC_DIAG_HIST) {
        atomicAdd((unsigned long long *)&p.cut_hist[(size_t)c * (p.n_edges + 1) + cq], (unsigned long long)run);
        atomicAdd((unsigned long long *)&p.nb_hist[(size_t)c * (n + 1) + nbq], (unsigned long long)run);
    }
    const int u = (int)(qv & 0xffffu);
    if (nbk >> 31) {  // kind 1: the start state's further yields (the per-batch form in flip2_kernel)
        if ((p.diag & FC_DIAG_FLIPS) && u != 0xffff) {
            const size_t o = (size_t)c * n + u;
            atomicMax((unsigned long long *)(p.last_flipped + o), (unsigned long long)(t + run));
            atomicAdd((unsigned long long *)(p.part_sum + o), (unsigned long long)(((qv >> 16) & 1u ? lab0 - lab1 : lab1 - lab0) * run));
            atomicAdd((unsigned long long *)(p.num_flips + o), (unsigned long long)run);
        }
        return;
    }
    const int tg = (int)(qc >> 31);
    const int64_t lab_t = tg ? lab1 : lab0, lab_o = tg ? lab0 : lab1;
    const uint32_t up = qv >> 16;  // neighbours in the old district: their edges turn cut
    if (p.diag & FC_DIAG_FLIPS) {  // the run's share (fc_run_read_flips closes the last run)
        const size_t o = (size_t)c * n + u;
        const int64_t t_last = t + run - 1;
        atomicMax((unsigned long long *)(p.last_flipped + o), (unsigned long long)t_last);
        atomicAdd((unsigned long long *)(p.part_sum + o), (unsigned long long)((lab_o - lab_t) * t_last));
        atomicAdd((unsigned long long *)(p.num_flips + o), (unsigned long long)run);
    }
    if (p.diag & FC_DIAG_FLIPS_EXACT) {
        const size_t o = (size_t)c * n + u;
        atomicAdd((unsigned long long *)(p.flip_count + o), 1ull);
        atomicAdd((unsigned long long *)(p.occ_acc + o), (unsigned long long)(-(lab_t - lab_o) * t));
        atomicMax((unsigned long long *)(p.last_accept + o), (unsigned long long)t);
    }
    if (p.diag & FC_DIAG_EDGES) {
        const int4 *er = (const int4 *)(p.ring_eid + (size_t)u * RMAX);
        int eid[RMAX];
#pragma unroll
        for (int j = 0; j < RMAX / 4; ++j) {
            const int4 e4 = er[j];
            eid[4 * j] = e4.x;
            eid[4 * j + 1] = e4.y;
            eid[4 * j + 2] = e4.z;
            eid[4 * j + 3] = e4.w;
        }
        int64_t *ea = p.edge_acc + (size_t)c * p.n_edges;
#pragma unroll
        for (int i = 0; i < RMAX; ++i)
            if (eid[i] >= 0) atomicAdd((unsigned long long *)(ea + eid[i]), (unsigned long long)(((up >> i) & 1u) ? -t : t));
    }
}

// One tally-log entry in 16 B (one coalesced store per lane): dt = t - t0 (< 2^24: launches
// with the log are at most 2^23 steps), run (< 2^24), |B| (< 2^16), node | ring bits << 16,
// |cut| (< 2^24), target, kind (0: a queue entry, 1: a start state's further yields).
__device__ __forceinline__ uint4 tally_pack(int64_t dt, int run, uint32_t qv, uint32_t qc, uint32_t nbk) {
    const uint32_t r = (uint32_t)run, kind = nbk >> 31;
    return make_uint4(((uint32_t)dt & 0xffffffu) | (r << 24), (r >> 8) | ((nbk & 0xffffu) << 16), qv,
                      (qc & 0xffffffu) | ((qc >> 31) << 24) | (kind << 25));
}

// Apply every chain's tally log and reset it: one workgroup per chain, after the flip kernel on
// the same stream, so the chain's serial stream never waits on these updates.  Each pass keeps
// the arrays of its mask (TR_* bits) privatised in LDS -- zeroed, every entry of the log applied
// with LDS atomics, then added (maxed) into the chain's global rows -- and applies the arrays of
// `gmask` with global atomics (those too large for any pass).  Global atomics from a separate
// kernel, for all arrays, took 62 ms per C2 launch: the chains' rows do not stay in L2.
enum : uint32_t { TR_CUT = 1, TR_NB = 2, TR_EDGE = 4, TR_NF = 8, TR_PS = 16, TR_LF = 32, TR_FC = 64, TR_OCC = 128, TR_LA = 256 };
constexpr int kTrArrays = 9;

__device__ __forceinline__ int64_t tr_len(const KParams &p, int a) {  // entries of array a per chain
    return a == 0 ? (int64_t)p.n_edges + 1 : a == 1 ? (int64_t)p.n + 1 : a == 2 ? (int64_t)p.n_edges : (int64_t)p.n;
}
__device__ __forceinline__ int64_t *tr_row(const KParams &p, int a, int c) {  // chain c's global row
    int64_t *b = a == 0 ? p.cut_hist : a == 1 ? p.nb_hist : a == 2 ? p.edge_acc : a == 3 ? p.num_flips
               : a == 4 ? p.part_sum : a == 5 ? p.last_flipped : a == 6 ? p.flip_count : a == 7 ? p.occ_acc : p.last_accept;
    return b + (size_t)c * (size_t)tr_len(p, a);
}

template <int RMAX>
__global__ __launch_bounds__(1024) void tally_reduce_kernel(KParams p, uint32_t lmask, uint32_t gmask, int last) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long *acc = (unsigned long long *)smem;
    const int c = (int)blockIdx.x;
    const int tid = (int)threadIdx.x, nt = (int)blockDim.x;
    const int64_t len = p.tl_len[c];
    const int64_t lab0 = p.labels[0], lab1 = p.labels[1];
    // LDS offsets (in entries) of the arrays of this pass, in TR order
    int64_t off[kTrArrays];
    int64_t tot = 0;
#pragma unroll
    for (int a = 0; a < kTrArrays; ++a) {
        off[a] = tot;
        if ((lmask >> a) & 1u) tot += tr_len(p, a);
    }
    for (int64_t i = tid; i < tot; i += nt) acc[i] = 0ull;
    __syncthreads();
    const uint4 *lg = (const uint4 *)p.tl + (size_t)c * (size_t)p.tl_cap;
    const int64_t t0 = p.tl_t0[c];
    // one update: LDS when the array is in this pass, global when it is in gmask
    auto add = [&](int a, int64_t i, int64_t v) {
        if ((lmask >> a) & 1u) atomicAdd(acc + off[a] + i, (unsigned long long)v);
        else if ((gmask >> a) & 1u) atomicAdd((unsigned long long *)(tr_row(p, a, c) + i), (unsigned long long)v);
    };
    auto mx = [&](int a, int64_t i, int64_t v) {
        if ((lmask >> a) & 1u) atomicMax(acc + off[a] + i, (unsigned long long)v);
        else if ((gmask >> a) & 1u) atomicMax((unsigned long long *)(tr_row(p, a, c) + i), (unsigned long long)v);
    };
    const uint32_t want = lmask | gmask;
    // kU entries per thread in flight: their log loads, then their ring-edge loads, are issued
    // together (2.24 -> 2.11 ms per C2 launch; contiguous stretches per thread instead, so one
    // instruction's lanes carry entries from 64 stretches of the launch: 2.54 ms)
    constexpr int kU = 8;
    const bool edges = (want & TR_EDGE) != 0;
    for (int64_t b0 = tid; b0 < len; b0 += (int64_t)nt * kU) {
        uint4 e[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const int64_t i = b0 + (int64_t)k * nt;
            e[k] = i < len ? lg[i] : make_uint4(0u, 0u, 0u, 0u);
        }
        int4 er[kU][RMAX / 4];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const int64_t i = b0 + (int64_t)k * nt;
            const bool need = edges && i < len && !((e[k].w >> 25) & 1u);
            const int4 *rp = (const int4 *)(p.ring_eid + (size_t)(e[k].z & 0xffffu) * RMAX);
#pragma unroll
            for (int j = 0; j < RMAX / 4; ++j) er[k][j] = need ? rp[j] : make_int4(-1, -1, -1, -1);
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            if (b0 + (int64_t)k * nt >= len) break;
            const uint4 ek = e[k];  // (tally_pack)
            const int64_t t = t0 + (int64_t)(ek.x & 0xffffffu);
            const int run = (int)((ek.x >> 24) | ((ek.y & 0xffffu) << 8));
            const uint32_t qv = ek.z, qc = (ek.w & 0xffffffu) | (((ek.w >> 24) & 1u) << 31);
            const int u = (int)(qv & 0xffffu);
            if (want & TR_CUT) add(0, (int64_t)(qc & 0x7fffffffu), run);
            if (want & TR_NB) add(1, (int64_t)(ek.y >> 16), run);
            if ((ek.w >> 25) & 1u) {  // kind 1 (tally_apply)
                if (u != 0xffff) {
                    if (want & TR_LF) mx(5, u, t + run);
                    if (want & TR_PS) add(4, u, ((qv >> 16) & 1u ? lab0 - lab1 : lab1 - lab0) * run);
                    if (want & TR_NF) add(3, u, run);
                }
                continue;
            }
            const int tg = (int)(qc >> 31);
            const int64_t lab_t = tg ? lab1 : lab0, lab_o = tg ? lab0 : lab1;
            const int64_t t_last = t + run - 1;
            if (want & TR_LF) mx(5, u, t_last);
            if (want & TR_PS) add(4, u, (lab_o - lab_t) * t_last);
            if (want & TR_NF) add(3, u, run);
            if (want & TR_FC) add(6, u, 1);
            if (want & TR_OCC) add(7, u, -(lab_t - lab_o) * t);
            if (want & TR_LA) mx(8, u, t);
            if (edges) {
                const uint32_t up = qv >> 16;
#pragma unroll
                for (int j = 0; j < RMAX / 4; ++j) {
                    const int ev[4] = {er[k][j].x, er[k][j].y, er[k][j].z, er[k][j].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (ev[q] >= 0) add(2, ev[q], ((up >> (4 * j + q)) & 1u) ? -t : t);
                }
            }
        }
    }
    __syncthreads();
    // the pass's sums (maxima) into the chain's rows: one workgroup per chain, so no atomics
#pragma unroll
    for (int a = 0; a < kTrArrays; ++a) {
        if (!((lmask >> a) & 1u)) continue;
        int64_t *row = tr_row(p, a, c);
        const int64_t L = tr_len(p, a);
        const bool is_max = a == 5 || a == 8;
        // four rows' entries per thread in flight (their loads issued together)
        for (int64_t b0 = tid; b0 < L; b0 += (int64_t)nt * 4) {
            int64_t cur[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int64_t i = b0 + (int64_t)k * nt;
                cur[k] = i < L ? row[i] : 0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int64_t i = b0 + (int64_t)k * nt;
                if (i >= L) break;
                const int64_t v = (int64_t)acc[off[a] + i];
                if (is_max) {
                    if (v > cur[k]) row[i] = v;
                } else if (v) {
                    row[i] = cur[k] + v;
                }
            }
        }
    }
    if (last) {
        __syncthreads();
        if (tid == 0) p.tl_len[c] = 0;
    }
}

int launch_tally_reduce(const KParams &p, int ring_max, void *stream) {
    if (!p.tl_len || p.n_chains <= 0) return (int)hipSuccess;
    // the arrays this run keeps, their per-chain bytes, packed greedily into passes of at most
    // 160 KiB of LDS (sec11 with every tally: one pass of 139 KiB, one 1024-thread workgroup per
    // CU: the log is read once); an array above 160 KiB goes to global atomics
    uint32_t have = 0;
    if (p.diag & FC_DIAG_HIST) have |= TR_CUT | TR_NB;
    if (p.diag & FC_DIAG_EDGES) have |= TR_EDGE;
    if (p.diag & FC_DIAG_FLIPS) have |= TR_NF | TR_PS | TR_LF;
    if (p.diag & FC_DIAG_FLIPS_EXACT) have |= TR_FC | TR_OCC | TR_LA;
    auto bytes = [&](int a) -> size_t {
        return 8 * (size_t)(a == 0 ? p.n_edges + 1 : a == 1 ? p.n + 1 : a == 2 ? p.n_edges : p.n);
    };
    // the device's LDS per workgroup (gfx950: 160 KiB), queried, not assumed
    int dev = 0, optin = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || optin <= 0)
        optin = 65536;
    const size_t kPass = (size_t)optin, kMaxLds = (size_t)optin;
    std::vector<std::pair<uint32_t, size_t>> passes;
    uint32_t gmask = 0;
    for (int a = 0; a < kTrArrays; ++a) {
        if (!((have >> a) & 1u)) continue;
        const size_t b = bytes(a);
        if (b > kMaxLds) {
            gmask |= 1u << a;
            continue;
        }
        bool put = false;
        for (auto &ps : passes)
            if (ps.second + b <= std::max(kPass, b)) {
                ps.first |= 1u << a;
                ps.second += b;
                put = true;
                break;
            }
        if (!put) passes.emplace_back(1u << a, b);
    }
    if (passes.empty()) passes.emplace_back(0u, 0);
    for (size_t i = 0; i < passes.size(); ++i) {
        size_t lds = passes[i].second;
        uint32_t lmask = passes[i].first, g = i == 0 ? gmask : 0u;
        const int last = i + 1 == passes.size() ? 1 : 0;
        const void *fn = ring_max <= 8 ? (const void *)tally_reduce_kernel<8> : (const void *)tally_reduce_kernel<16>;
        if (lds > 65536 &&
            hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
            // the device refuses this much dynamic LDS: the pass's arrays take the global atomics
            (void)hipGetLastError();
            g |= lmask;
            lmask = 0;
            lds = 0;
        }
        if (ring_max <= 8)
            hipLaunchKernelGGL(tally_reduce_kernel<8>, dim3(p.n_chains), dim3(1024), lds, (hipStream_t)stream, p,
                               lmask, g, last);
        else
            hipLaunchKernelGGL(tally_reduce_kernel<16>, dim3(p.n_chains), dim3(1024), lds, (hipStream_t)stream, p,
                               lmask, g, last);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return (int)hipSuccess;
}

template <int RMAX, int NSUB, bool FULL, bool SEARCH, bool XTRA, bool BAND>
__global__ __launch_bounds__(256, (RMAX == 8 ? 4 : 1)) void flip2_kernel(KParams p) {
    static_assert(FULL || !XTRA, "XTRA is a FULL instance");
    // non-hit draws held per lane: the node stream's four words per Philox call, BAND's rounds
    constexpr int kRV = BAND ? NSUB : 4;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = (int)(threadIdx.x & 63u);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int wave = (int)blockIdx.x * (int)(blockDim.x >> 6) + wv;
    if (wave >= p.n_chains) return;
    const int c = p.order ? deal_chain(p, lane) : wave;  // chain dealing (fc_deal.hip)

    const int n = p.n;
    const int npad = (n + 15) & ~15;
    unsigned char *base = smem + (size_t)wv * p.chain_lds_bytes;
    int8_t *a = (int8_t *)base;                    // [npad] district of each node
    uint8_t *fcnt = base + npad;                   // [npad] foreign neighbours of each node
    uint64_t *T = (uint64_t *)(base + 2 * npad);   // [2 RMAX + 2] acceptance thresholds by delta-cut
    BfsScratch bs{};                                // wave_bfs_single: the three bitmaps only
    bs.vis = (uint64_t *)(T + (2 * RMAX + 2));
    bs.front = bs.vis + p.words;
    bs.nxt = bs.front + p.words;
    bs.W = p.words;
    bs.prof = nullptr;
    uint32_t *slot = (uint32_t *)(bs.nxt + p.words);  // [5][64]: node, word1, word2, draw offset, ring link | len
    uint8_t *smark = (uint8_t *)(slot + 5 * 64);   // [npad] lowest slot of a segment flip at the node
    uint8_t *nmark = smark + npad;                 // [npad] ... having the node as a neighbour
    uint8_t *const dum = nmark + npad + (lane & 15);  // [16] sink for masked-off stores
    // a store only some lanes make: the others write the sink (no branch; storing under exec
    // masks instead measured no faster, profiles/r03c_ab_masked_stores)
#define FC_ST(cond, ref, val) (*((cond) ? (uint8_t *)&(ref) : dum) = (uint8_t)(val))
    // accepted states whose geometric wait is still to be drawn (kWaitQ of them:
    // creating draw, |B| after the flip, yields so far); see wait_flush below
    uint64_t *q_d = (uint64_t *)(nmark + npad + 16);
    uint32_t *q_nb = (uint32_t *)(q_d + kWaitQ), *q_run = q_nb + kWaitQ;
    // FULL: the per-flip tallies of a queued state, applied by the same pass (tally_flush):
    // node | old-district neighbours (ring bits) << 16, |cut| | target district << 31
    uint32_t *q_v = q_run + kWaitQ, *q_c = q_v + kWaitQ;
    // [5]: launch start time, previous launch's pace (read back, not held), yield of the first
    // queued state, FULL: tally-log entries written this launch, the launch's first yield
    uint64_t *misc = (uint64_t *)(q_c + kWaitQ);
    uint64_t *const sb = misc + 5;  // BAND: [words] the band S (bit u: node u in S)
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
        for (int i = lane; i < npad / 4 + 2; i += kWave) ((uint64_t *)smark)[i] = ~0ull;  // marks + sink
        if (BAND && lane < p.words) sb[lane] = p.sbits[(size_t)c * p.words + lane];
    }
    ChainScalars *scp = p.sc + c;
    uint64_t draw = scp->draw;
    int64_t steps = scp->steps;  // index of the current yield
    int64_t trace_len = FULL ? scp->trace_len : 0;
    int64_t ev_len = FULL ? scp->ev_len : 0, hit_time = FULL ? scp->hit_time : 0;
    int cut = scp->cut, nb = scp->nb;
    int pops0 = scp->pops[0], pops1 = scp->pops[1];
    const int pop_lo = scp->pop_lo, pop_hi = scp->pop_hi;  // this chain's bounds (chain_pop_bounds)
    int ng0 = scp->ngamma[0], ng1 = scp->ngamma[1];
    int64_t wait_cur = scp->wait_cur;
    int qn = 0;  // queued accepted states (lean instance); the last one is the current state
    int last_flip = scp->last_flip;
    int stuck = 0;
    int rem = (int)p.n_steps;  // steps still to take in this launch (host: n_steps < 2^31)
    uint64_t draw_cap = draw + (uint64_t)p.max_draws;
    if (XTRA && p.tape && draw_cap > (uint64_t)p.tape_draws) draw_cap = (uint64_t)p.tape_draws;
    const uint32_t chain_gid = p.chain_id_offset + (uint32_t)c;
    const bool force_bfs = (p.flags & FC_FLAG_FORCE_BFS) != 0;
    const bool want_wait = (p.diag & FC_DIAG_WAIT) != 0;
    const bool trace_on = XTRA && p.trace && c < p.trace_chains;
    // accepted states queued (wait_flush: their waits drawn, FULL: their tallies applied later)
    // unless a trace or a replay tape needs the waits per batch
    const bool defer = (want_wait || FULL) && !trace_on && !(XTRA && p.tape);

    // per-lane accumulators, reduced once per launch
    int64_t acc_cut = 0, acc_nb = 0, acc_wait = 0, acc_cut2 = 0, acc_nb2 = 0;
    int64_t n_prop = 0, n_acc = 0, n_ic = 0, n_ip = 0;  // wave-uniform (scalar) counters
#ifdef FC_PHASE_PROF
    int64_t *prof_acc = (int64_t *)(base + p.chain_lds_bytes - kProfSlots * 8);
    if (lane < kProfSlots) prof_acc[lane] = 0;
#endif
    wave_sync();
    // BAND: |S| and the Lemire threshold 2^32 mod |S| (scalars, changed only by band_rebuild)
    uint32_t nS = 1u, thrS = 0u;
    auto band_count = [&]() {
        const int cw = lane < p.words ? (int)__popcll(sb[lane]) : 0;
        nS = (uint32_t)rl32(wave_scan_incl(cw), kWave - 1);
        thrS = (0u - nS) % nS;
    };
    // S := b_nodes of the current state and their neighbours (the oracle's band_build)
    auto band_rebuild = [&]() {
        compiler_fence();
        if (lane < p.words) sb[lane] = 0ull;
        compiler_fence();
        for (int j = 0; j < p.words; ++j) {
            const int u = 64 * j + lane;
            const bool isB = u < n && fcnt[u] != 0;
            const uint64_t mb = __ballot(isB);
            if (!mb) continue;
            if (lane == 0) atomicOr((unsigned long long *)&sb[j], (unsigned long long)mb);
            if (isB) {
                const NodeRec<RMAX> ru = G[u];
                const uint32_t nbm = (uint32_t)(ru.meta >> kMetaNbrShift) & 0xffffu;
#pragma unroll
                for (int i = 0; i < RMAX; ++i)
                    if ((nbm >> i) & 1u) {
                        const int w = ring_entry<RMAX>(ru.ring, i);
                        atomicOr((uint32_t *)sb + (w >> 5), 1u << (w & 31));
                    }
            }
        }
        compiler_fence();
        band_count();
    };
    if constexpr (BAND) band_count();
#ifdef FC_PHASE_PROF
    {  // slot 20: the wave's SIMD (XCC_ID . HW_ID[15:4], as deal_chain keys it)
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        FC_PROF(20, (int64_t)(((xcc & 7u) << 12) | ((hw >> 4) & 0xfffu)));
    }
#endif
    FC_STAMP(t_loop0);

    // issue priority among the waves sharing a SIMD (scheduling only: trajectories are
    // unchanged).  The launch lasts as long as its slowest chain, so the chains projected to
    // finish last get the issue slots: a chain's projected finish (elapsed / steps taken so
    // far x steps to take) against the previous launch's slowest chain, or, before it has
    // taken 1/16 of its steps, its |B| (a short boundary needs many draws per proposal).
    // The wait of an accepted state (geom_wait, grid_chain_sec11.py:147-148) only enters the
    // run-length-weighted sum of waits, so it is drawn later (no trace, no tape): a batch accepts
    // 1-3 states, and a per-batch pass would run the purpose-1 Philox and the f64 log on a
    // nearly idle wave in every chain's serial path.  The queue is drained by one full-width
    // pass when it would overflow and at the end of the launch; the current state's wait is then
    // known (wait_cur) and the yields it still lasts are charged to it directly.  The sums are
    // the per-batch ones, term by term.
    // FULL: the per-yield tallies of the queued states (grid_chain_sec11.py:367-400), in the
    // same pass.  Issued per batch they were global atomics in every chain's serial path, and
    // the next batch's first vector-memory wait (vmcnt counts them) waited for all of them; here
    // the loads go first and the atomics follow back to back, once per queue.  Each entry holds
    // its whole run: the batches that continue the queued current state add to its run length
    // instead of issuing their own updates.  Every update commutes (sums and maxima), so the
    // order differs from the per-batch one and the results do not.
    auto tally_flush = [&]() {
        if constexpr (FULL) {
            const bool in = lane < qn;
            const int run = in ? (int)q_run[lane] : 0;  // a launch's runs sum below 2^31
            const int64_t t = (int64_t)misc[2] + (int64_t)(wave_scan_incl(run) - run);  // yield of the flip
            const uint32_t qv = in ? q_v[lane] : 0u, qc = in ? q_c[lane] : 0u;
            const int nbq = in ? (int)q_nb[lane] : 0;
            if (in && (p.diag & FC_DIAG_SERIES)) {
                const int64_t idx = ev_len + lane;
                if (idx < p.ev_cap) {
                    fc_event ev;
                    ev.t = t;
                    ev.v = (uint16_t)(qv & 0xffffu);
                    ev.cut = (uint16_t)(qc & 0x7fffffffu);
                    ev.nb = (uint16_t)nbq;
                    ev.target = (uint8_t)(qc >> 31);
                    ev.reserved = 0;
                    p.events[(size_t)c * p.ev_cap + idx] = ev;
                }
            }
            if (p.diag & (FC_DIAG_HIST | FC_DIAG_FLIPS | FC_DIAG_FLIPS_EXACT | FC_DIAG_EDGES)) {
                // the entries go to the chain's tally log (two coalesced stores; tally_reduce applies
                // them after the launch): issued here, the atomics held up the next batch's first
                // vector-memory wait (vmcnt counts them and completes in order), C2 full diagnostics
                // 62.6 -> 54.8 ms per launch (profiles/r05e_tally_log_ab.txt).  A full log: atomics.
                const int64_t lbase = (int64_t)misc[3];
                if (p.tl && lbase + qn <= p.tl_cap) {
                    if (in)
                        ((uint4 *)p.tl)[(size_t)c * (size_t)p.tl_cap + (size_t)(lbase + lane)] =
                            tally_pack(t - (int64_t)misc[4], run, qv, qc, (uint32_t)nbq);
                    if (lane == 0) misc[3] = (uint64_t)(lbase + qn);
                } else if (in) {
                    tally_apply<RMAX>(p, c, t, run, qv, qc, (uint32_t)nbq, p.labels[0], p.labels[1]);
                }
            }
            if (p.diag & FC_DIAG_SERIES) ev_len += qn;
        }
    };
    auto wait_flush = [&]() {
        compiler_fence();
        int64_t w = 0;  // (waits off: 0, as the per-batch form leaves them)
        if (want_wait && lane < qn) {  // the loads before the tallies' atomics (vmcnt completes in order)
            const uint64_t dq = q_d[lane];
            const Words4 g = philox4x32_10((uint32_t)dq, (uint32_t)(dq >> 32), chain_gid, 1u, p.seed_lo, p.seed_hi);
            w = geom_wait_of(g.x0, g.x1, p.log1mp[q_nb[lane]]);
            acc_wait += w * (int64_t)q_run[lane];
        }
        tally_flush();
        wait_cur = (int64_t)(((uint64_t)(uint32_t)rl32((int)(uint32_t)w, qn - 1)) |
                             ((uint64_t)(uint32_t)rl32((int)(w >> 32), qn - 1) << 32));
        qn = 0;
        compiler_fence();
    };
    int prio = 0;  // bits 0-1: the issue priority set; bits 2 and up: batches since it was last chosen
    if (lane == 0) {
        misc[3] = 0;  // the tally log starts empty (tally_reduce emptied it)
        misc[4] = (uint64_t)steps;
        if (FULL && p.tl_t0) p.tl_t0[c] = steps;
        misc[0] = __builtin_amdgcn_s_memrealtime();
        // the previous launch's slowest-chain pace, scaled to this launch (0: none yet)
        const float eta0 = p.eta ? (float)p.eta[p.eta_parity ^ 1] * (float)p.n_steps * (1.0f / 1024.0f) : 0.0f;
        misc[1] = (uint64_t)__float_as_uint(eta0);
    }
    compiler_fence();
    while (rem > 0) {
        // re-chosen every 2^FC_PRIO_EVERY_LOG2 batches (it moves slowly; scheduling only)
        if (p.prio_nb[0] > 0 && ((prio += 4) & (((1 << FC_PRIO_EVERY_LOG2) - 1) << 2)) == 0) {
            const int done = (int)p.n_steps - rem;
            const float eta = __uint_as_float((uint32_t)misc[1]);
            int lv;
            if (eta > 0.0f && done * 16 >= (int)p.n_steps) {
                const float pr = (float)(__builtin_amdgcn_s_memrealtime() - misc[0]) * (float)p.n_steps / ((float)done * eta);
                lv = (pr > p.prio_th[0]) + (pr > p.prio_th[1]) + (pr > p.prio_th[2]);
            } else {
                lv = (nb < p.prio_nb[0]) + (nb < p.prio_nb[1]) + (nb < p.prio_nb[2]);
            }
            if (lv != (prio & 3)) {
                prio = (prio & ~3) | lv;
                switch (lv) {
                    case 0: __builtin_amdgcn_s_setprio(0); break;
                    case 1: __builtin_amdgcn_s_setprio(1); break;
                    case 2: __builtin_amdgcn_s_setprio(2); break;
                    default: __builtin_amdgcn_s_setprio(3); break;
                }
            }
        }
        FC_STAMP(t_a);
        FC_PROF(5, 1);
        if (draw >= draw_cap) {
            stuck = 1;
            break;
        }
        const uint64_t room = draw_cap - draw;
        // ---- 1. draws -> nodes; boundary hits packed, in draw order, into <= 64 slots ----
        int nh = 0;   // boundary hits seen
        int gen = 0;  // draws generated (offsets 0..gen-1 of this batch)
        // the nodes of this lane's non-hit draws: node | (slots drawn before it << 16), -1: none.
        // "slot s precedes the draw" is then s < rv >> 16.  Node stream: word j of this lane's
        // Philox call (draw offset 4 lane + j - (draw mod 4)); BAND: round j (offset 64 j + lane).
        int rv[kRV];
        // draw offset of entry j of lane l
        auto rv_off = [&](int j, int l) { return BAND ? 64 * j + l : 4 * l + j - (int)(draw & 3u); };
        if constexpr (!BAND) {
            // node stream: the node words of draws 4q .. 4q+3 are the four words of
            // one Philox call (ctr = q, chain, purpose 3): lane l holds q = draw / 4 + l, so one
            // call per lane covers the batch's window of up to 64 NSUB draws, in draw order
            // lane-major.  The acceptance words of the hits come from their own call (phase 2).
            const int s0 = (int)(draw & 3u);
            // (the window never passes the last lane's words: 4 * 64 - s0 draws at most)
            const int wcap = 64 * NSUB < 4 * kWave - s0 ? 64 * NSUB : 4 * kWave - s0;
            const int win = (uint64_t)wcap < room ? wcap : (int)room;
            const uint64_t q = (draw >> 2) + (uint64_t)lane;
            uint32_t nw[4];
            if (XTRA && p.tape) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int off = 4 * lane + j - s0;
                    const bool inr = off >= 0 && off < win;
                    nw[j] = p.tape[((size_t)c * (size_t)p.tape_draws + (inr ? draw + (uint64_t)off : draw)) * 6];
                }
            } else {
                const Words4 w = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), chain_gid, 3u, p.seed_lo, p.seed_hi);
                nw[0] = w.x0;
                nw[1] = w.x1;
                nw[2] = w.x2;
                nw[3] = w.x3;
            }
            int vdj[4];
            uint32_t okm = 0u, hb = 0u;  // this lane's draws: Lemire-accepted, boundary hits
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int off = 4 * lane + j - s0;
                const uint64_t m = (uint64_t)nw[j] * (uint64_t)(uint32_t)n;
                vdj[j] = (int)(m >> 32);
                const bool ok = (off >= 0) & (off < win) & ((uint32_t)m >= p.lemire_thresh);
                // (vdj < n on every lane: the read needs no guard)
                okm |= (uint32_t)ok << j;
                hb |= (uint32_t)(ok & (fcnt[vdj[j]] != 0)) << j;
            }
            const int hc = __popc(hb);
            const int incl = wave_scan_incl(hc);
            const int excl = incl - hc;
            const int tot = rl32(incl, kWave - 1);
            gen = win;
            int lim = 4 * kWave;  // draws of the window consumed, as an offset bound
            if (tot > 64) {  // the 64th hit closes the batch
                const int L = __builtin_ctzll(__ballot(incl >= 64));
                const uint32_t hbL = rlu(hb, L);
                const int k = 64 - rl32(excl, L);  // its rank among lane L's hits (1-based)
                uint32_t mk = hbL;  // its word: the k-th set bit of lane L's hits (wave-uniform)
                for (int i = 1; i < k; ++i) mk &= mk - 1u;
                const int jj = __builtin_ctz(mk);
                lim = 4 * L + jj - s0 + 1;
                gen = lim;
            }
            // the slot lanes' sink for masked-off stores: row 4 of the slots (phase 2 writes it)
            uint32_t *const ssink = slot + 256 + lane;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int off = 4 * lane + j - s0;
                const int sp = excl + __popc(hb & ((1u << j) - 1u));
                const bool hit = (hb >> j) & 1u;
                const bool put = hit & (sp < 64);
                *(put ? slot + sp : ssink) = (uint32_t)vdj[j];
                *(put ? slot + 192 + sp : ssink) = (uint32_t)off;
                rv[j] = (((okm >> j) & 1u) & !hit & (off < lim)) ? (vdj[j] | (sp << 16)) : -1;
            }
            nh = tot;
        } else {
            // BAND: lane l < words holds the members of S in the words below l (the rank search's keys)
            int bpre = 0x7fffffff;
            {
                const int cw = lane < p.words ? (int)__popcll(sb[lane]) : 0;
                const int inc = wave_scan_incl(cw);
                if (lane < p.words) bpre = inc - cw;
            }
#pragma unroll
            for (int r = 0; r < NSUB; ++r) {
                rv[r] = -1;
                if ((r > 0 && nh >= p.hit_stop) || nh >= 64 || (uint64_t)gen >= room) continue;
                const int off = gen + lane;
                const bool inrange = (uint64_t)off < room;
                const uint64_t dr = draw + (uint64_t)off;
                const Words4 w = philox4x32_10((uint32_t)dr, (uint32_t)(dr >> 32), chain_gid, 0u, p.seed_lo, p.seed_hi);
                // exact Lemire over |S|, then the idx-th member of S: the word by a binary search
                // over the lanes' prefix counts, the bit by popcount halvings
                const uint64_t m = (uint64_t)w.x0 * (uint64_t)nS;
                const int idx = (int)(m >> 32);
                const bool okd = inrange && (uint32_t)m >= thrS;
                int bw = 0, bb = 0;
                for (int st2 = p.band_step0; st2 >= 1; st2 >>= 1) {
                    const int cand = bw + st2;
                    const int pc = __builtin_amdgcn_ds_bpermute(cand << 2, bpre);
                    if (pc <= idx) {
                        bw = cand;
                        bb = pc;
                    }
                }
                const int vd = 64 * bw + select_bit64(sb[bw], idx - bb);
                const bool hitd = okd & (fcnt[vd] != 0);
                const uint64_t hm = __ballot(hitd);
                const int sp = nh + count_below(hm);
                if (hitd && sp < 64) {
                    slot[sp] = (uint32_t)vd;
                    slot[64 + sp] = w.x1;
                    slot[128 + sp] = w.x2;
                    slot[192 + sp] = (uint32_t)off;
                }
                const int cnt = __popcll(hm);
                int used = kWave;  // lanes of this round consumed by the batch
                if (nh + cnt > 64) {  // the 64th hit closes the batch inside this round
                    used = kth_set_bit(hm, 64 - nh) + 1;
                    gen += used;
                } else {
                    gen = (uint64_t)(gen + 64) < room ? gen + 64 : (int)room;
                }
                rv[r] = (okd & !hitd & (lane < used)) ? (vd | (sp << 16)) : rv[r];
                nh += cnt;
            }
        }
        const int ns = nh < 64 ? nh : 64;
        compiler_fence();
        FC_STAMP(t_b);
        FC_PROF(1, t_b - t_a);

        // ---- 2. every slot against the current state --------------------------------------
        const bool has = lane < ns;
        // (the slot array is always readable: unconditional reads and a select, no exec-mask branch)
        const int off_r = (int)slot[192 + lane], v_r = (int)slot[lane];
        int off_l = has ? off_r : gen;
        const uint64_t d = draw + (uint64_t)off_l;
        int v = has ? v_r : 0;
        uint32_t w1, w2;  // the draw's acceptance words (random(), grid_chain_sec11.py:179)
        if constexpr (BAND) {
            w1 = slot[64 + lane];
            w2 = slot[128 + lane];
        } else {
            // node stream: words 1-2 of the draw's own Philox call (ctr = draw, chain, purpose 0),
            // made for the hits only; kept in the slots for the re-evaluations
            if (XTRA && p.tape) {
                const uint32_t *t = p.tape + ((size_t)c * (size_t)p.tape_draws + (has ? d : draw)) * 6;
                w1 = t[1];
                w2 = t[2];
            } else {
                const Words4 g = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), chain_gid, 0u, p.seed_lo, p.seed_hi);
                w1 = g.x1;
                w2 = g.x2;
            }
            slot[64 + lane] = w1;
            slot[128 + lane] = w2;
        }
        const NodeRec<RMAX> rec = G[v];
        int av = a[v];
        int pv = rec.pop;
        const uint32_t Ln = (uint32_t)(rec.meta & kMetaLenMask);
        const uint32_t full = (1u << Ln) - 1u;
        uint32_t nbr = (uint32_t)(rec.meta >> kMetaNbrShift) & 0xffffu;
        const uint32_t link = (uint32_t)(rec.meta >> kMetaLinkShift) & 0xffffu;
        int cell[RMAX];  // ring cells (padded with the node itself)
        // districts are 0 / 1: pack the ring's district-1 bits, then A's bits are those or
        // their complement (shift-ors, no compare / select per cell)
        uint32_t in1 = 0;
        int ad[RMAX];
#pragma unroll
        for (int i = 0; i < RMAX; ++i) {
            cell[i] = ring_entry<RMAX>(rec.ring, i);
            ad[i] = a[cell[i]];
        }
        // every read issued before the first use (the compiler otherwise waited on each read
        // before issuing the next: eight LDS round trips in a row)
#pragma unroll
        for (int i = 0; i < RMAX; ++i) asm volatile("" : "+v"(ad[i]));
#pragma unroll
        for (int i = 0; i < RMAX; ++i) in1 |= (uint32_t)ad[i] << i;
        uint32_t inA = (av ? in1 : ~in1) & full;
        slot[256 + lane] = link | (Ln << 16);  // for re-evaluations inside the commit
        // target district: 1 - av (-1 * assignment, grid_chain_sec11.py:145)
        const uint32_t nbrA = inA & nbr;        // old-district neighbours
        uint32_t tmask = nbr & ~inA;            // target-district neighbours
        int nA = __popc(nbrA);
        int delta = nA - __popc(tmask);         // cut(S') - cut(S)
        const bool hit = has && tmask != 0u;    // v in b_nodes: a proposal
        bool s_lin, s_cyc;
        {
            const uint32_t rot = Ln ? (((inA >> 1) | (inA << (Ln - 1))) & full) : 0u;
            const uint32_t lk = inA & rot & link;
            s_lin = one_run_flat(nbrA, full & ~lk, full);
            // the ring's closing step (cell Ln-1 to cell 0), when both ends are in A
            const uint32_t vlink = (Ln >= 2) ? ((inA & (inA >> (Ln - 1)) & 1u) << (Ln - 1)) : 0u;
            s_cyc = one_run_flat(nbrA, full & ~(lk | vlink), full);
        }
        const bool exact = SEARCH ? (rec.meta & kMetaExact) && !force_bfs : true;
        const bool gam = (rec.meta & kMetaGamma) != 0;
        const bool acc = mant53(w1, w2) < T[delta + RMAX];
        // per-slot predicates live as bits of one VGPR (st) through the commit; the compiler
        // would otherwise hold each as a 64-bit lane mask in SGPRs for the whole loop
        uint32_t st = (hit ? LF_HIT : 0u) | (acc ? LF_ACC : 0u) | (s_lin ? LF_SLIN : 0u) | (s_cyc ? LF_SCYC : 0u) |
                      (exact ? LF_EXACT : 0u) | (gam ? LF_GAM : 0u) | (has ? LF_HAS : 0u);
        if (XTRA && (rec.meta & kMetaFrozen)) st |= LF_FRZ;
#ifdef FC_PHASE_PROF
        bool first_it = true;
#endif
        FC_STAMP(t_c);
        FC_PROF(2, t_c - t_b);

        // ---- 3. commit in draw order ----------------------------------------------------
        int end = ns, pos = 0;
        int trunc_off = gen;  // first draw offset not consumed by this batch
        bool target_hit = false;
        bool rebuild = false;  // BAND: a committed flip put a node outside S into b_nodes
        const int cut0 = cut, nb0 = nb, rem0 = rem;
        const int64_t steps0 = steps;
        const int last_flip0 = last_flip;
        const int a_last0 = FULL && last_flip0 >= 0 ? (int)a[last_flip0] : 0;
        int cut_after = 0, nb_after = 0;
        // pops0 change of this lane's flip, ngamma0 change (derived from av / st: a
        // re-evaluation changes them)
        auto dp_of = [&]() { return av == 0 ? -pv : pv; };
        auto dg_of = [&]() { return (st & LF_GAM) ? (av == 0 ? -1 : 1) : 0; };

        // A committed flip that changes the view of later slots (its node, or a node of their
        // ring) no longer ends the batch: the slots from `from` on are evaluated again against
        // the current state (phase 2 once more, from registers and LDS) and the commit goes
        // on.  A slot whose node left the boundary is then a non-proposal draw, as it is in
        // the one-draw-at-a-time chain.  The commit marks of the segment passes so far are
        // cleared first: every slot's view is current again.
        // vfx >= 0 (one event at a time): node vfx is the only one flipped since the slots' last
        // evaluation, and eqx marks it in this lane's ring, so the view is updated in registers
        // (no ring reads; the threshold read issues beside the slot reads)
        auto reeval = [&](int from, int vfx, uint32_t eqx) {
            FC_STAMP(t_re0);
            // (no marks to clear: every segment pass clears its own before anything else runs)
            compiler_fence();
            if (has && lane >= from) {
                const uint32_t lkl = slot[256 + lane];
                const uint32_t w1r = slot[64 + lane], w2r = slot[128 + lane];
                if (vfx < 0) {
                    av = a[v];
                    uint32_t i1 = 0;
                    int ad[RMAX];
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) ad[i] = a[cell[i]];
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) asm volatile("" : "+v"(ad[i]));  // (reads issued together)
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) i1 |= (uint32_t)ad[i] << i;
                    inA = av ? i1 : ~i1;
                } else {
                    const bool self = v == vfx;  // its own node flipped: every ring relation inverts
                    av = self ? 1 - av : av;
                    inA = (self ? ~inA : inA) ^ eqx;
                }
                // nbr has no bits at or above the ring length: these need no length mask
                const uint32_t nbA = inA & nbr;
                tmask = nbr & ~inA;
                nA = __popc(nbA);
                delta = nA - __popc(tmask);
                const uint64_t th = T[delta + RMAX];
                const uint32_t lnk = lkl & 0xffffu, L2 = lkl >> 16;
                const uint32_t fl = (1u << L2) - 1u;
                inA &= fl;
                const uint32_t rot = L2 ? (((inA >> 1) | (inA << (L2 - 1))) & fl) : 0u;
                const uint32_t lk = inA & rot & lnk;
                const bool sl = one_run_flat(nbA, fl & ~lk, fl);
                const uint32_t vlink = (L2 >= 2) ? ((inA & (inA >> (L2 - 1)) & 1u) << (L2 - 1)) : 0u;
                const bool sc = one_run_flat(nbA, fl & ~(lk | vlink), fl);
                const bool ac = mant53(w1r, w2r) < th;
                st = (st & (LF_EXACT | LF_GAM | LF_HAS | LF_FRZ)) | (tmask != 0u ? LF_HIT : 0u) | (ac ? LF_ACC : 0u) |
                     (sl ? LF_SLIN : 0u) | (sc ? LF_SCYC : 0u);
            }
            compiler_fence();
            FC_STAMP(t_re1);
            FC_PROF(16, t_re1 - t_re0);
            FC_PROF(17, 1);
        };

        // contiguity undecided by the ring rule at lane f: wave BFS on the current state
        auto run_bfs = [&](int f) -> bool {
            const uint32_t nbrAf = rlu(inA & nbr, f);
            int my_target = -1, start = -1;
#pragma unroll
            for (int k2 = 0; k2 < RMAX / 2; ++k2) {
                const uint32_t wrd = rlu(rec.ring[k2], f);
                if ((lane >> 1) == k2) my_target = (int)((wrd >> (16 * (lane & 1))) & 0xffffu);
                if (start < 0 && ((nbrAf >> (2 * k2)) & 1u)) start = (int)(wrd & 0xffffu);
                if (start < 0 && ((nbrAf >> (2 * k2 + 1)) & 1u)) start = (int)(wrd >> 16);
            }
            if (!(lane < RMAX && ((nbrAf >> lane) & 1u))) my_target = -1;
            // the (rare) search counts go straight to the chain's record: as loop-carried values
            // they cost the hot loop two 64-bit registers
            int64_t lv = 0;
            const bool res = wave_bfs_single<RMAX>(G, a, bs, lane, rl32(v, f), rl32(av, f), my_target, start, lv);
            if (lane == 0) {
                atomicAdd((unsigned long long *)&scp->bfs_calls, 1ull);
                atomicAdd((unsigned long long *)&scp->bfs_levels, (unsigned long long)lv);
            }
            return res;
        };

        while (pos < end) {
            FC_PROF(6, 1);
            FC_STAMP(t_it0);
#ifdef FC_PHASE_PROF
            if (first_it) FC_PROF(27, t_it0 - t_c);  // the commit's set-up
            first_it = false;
#endif
            // re-derive the predicates each iteration: loop-invariant lane values would otherwise
            // be hoisted as lane masks into SGPRs and spilled
            asm volatile("" : "+v"(st), "+v"(inA), "+v"(tmask), "+v"(nbr), "+v"(delta), "+v"(nA), "+v"(av), "+v"(pv),
                         "+v"(v), "+v"(off_l));
            // (SEARCH = false: every node exact and no search verdicts -- compile-time constants,
            // so the lean instance carries no undecided-slot logic)
            const bool hit = (st & LF_HIT) != 0, acc = (st & LF_ACC) != 0, s_lin = (st & LF_SLIN) != 0,
                       s_cyc = (st & LF_SCYC) != 0, exact = SEARCH ? (st & LF_EXACT) != 0 : true,
                       gam = (st & LF_GAM) != 0, has = (st & LF_HAS) != 0;
            const bool prop = hit & (lane >= pos) & (lane < end);
            // contiguity verdict when the other district does (okT) / does not (okN) touch
            // the outer face -- the outer-face counts are chain-global
            // (selects, not an if-chain: the chain compiled to nested exec-mask branches)
            // BFS verdict if any; no old-district neighbour: invalid; else the run rule, exact
            // or (not exact) deciding only "one run"
            const bool bd = SEARCH && (st & ST_BD) != 0, br = SEARCH && (st & ST_BR) != 0, nz = nA != 0;
            const bool okT = bd ? br : (nz & s_lin);
            const bool okN = bd ? br : (nz & ((exact & gam) ? s_cyc : s_lin));
            const bool known = bd | !nz | exact | s_lin;
            const bool ok = ((av ? ng0 : ng1) > 0) ? okT : okN;
            const int pa = av ? pops1 : pops0, pb = av ? pops0 : pops1;
            const bool popok = (pa - pv >= pop_lo) & (pb + pv <= pop_hi);
            bool valid = prop & known & ok & popok;
            bool acc_now = acc;
            bool inv_contig = !ok;  // reason of an invalid proposal: contiguity, else "pop"
            if constexpr (XTRA) {
                if (p.variant) {
                    // Validator members re-draw, accept-callable constraints reject the step
                    // (grid_chain_sec11.py:39-52,81-110,159-165); contiguity / populations as
                    // above, boundary_condition from the outer-face counts, fixed_endpoints
                    // from the frozen bit
                    const int gm = gam ? 1 : 0;
                    const bool b_ok = ((av ? ng1 : ng0) - gm > 0) && ((av ? ng0 : ng1) + gm > 0);
                    const bool f_ok = !(st & LF_FRZ);
                    auto pass = [&](uint32_t M) {
                        return (!(M & FC_CON_CONTIG) || ok) && (!(M & FC_CON_POP) || popok) &&
                               (!(M & FC_CON_BOUNDARY) || b_ok) && (!(M & FC_CON_FIXED) || f_ok);
                    };
                    valid = prop && known && pass(p.con_valid);
                    inv_contig = (p.con_valid & FC_CON_CONTIG) && !ok;
                    bool au = acc;
                    if (p.accept == FC_ACCEPT_UNIFORM) {
                        au = true;  // random() < 1
                    } else if (p.accept == FC_ACCEPT_ANNEAL) {
                        // bound = base ** (beta (cut - cut')) * (|B'| / |B|), :99; |B'| from the
                        // foreign counts of v's neighbours (v stays a boundary node iff nA > 0)
                        int dnb_l = nA == 0 ? -1 : 0;
#pragma unroll
                        for (int i = 0; i < RMAX; ++i) {
                            const int oc = fcnt[cell[i]];
                            const bool nb_i = (nbr >> i) & 1u;
                            dnb_l += nb_i ? (int)(((inA >> i) & 1u) && oc == 0) - (int)(((tmask >> i) & 1u) && oc == 1) : 0;
                        }
                        const double bw = __longlong_as_double((long long)T[delta + RMAX]);
                        const double bound = bw * ((double)(nb + dnb_l) / (double)nb);
                        au = (double)mant53(w1, w2) * 0x1p-53 < bound;
                    }
                    acc_now = pass(p.con_accept) && au;
                }
            }
            const uint64_t C0 = __ballot(valid && acc_now);
            FC_STAMP(t_it1);
            FC_PROF(8, t_it1 - t_it0);
            if (__popcll(C0) >= p.par_min) {
                FC_PROF(12, 1);
                // ---- segment-parallel commit ---------------------------------------------
                // A lane's verdict reads only a[] on its node and ring, so it stays exact until
                // a flip lands there (alpha: the batch ends at that lane; a non-hit lane ends
                // it when a flip lands on a neighbour, its node entering the boundary); two
                // flips sharing a neighbour would need ordered foreign-count updates (beta: the
                // batch ends at the later one).  Inside a segment the flips then commute except
                // through the chain-global populations and outer-face counts: a prefix scan over
                // the speculative acceptances gives every lane its sequential view, and the
                // first lane whose verdict changes under that view closes the segment (it is
                // itself exact).  Flips committed one at a time (below) leave no marks: they cut
                // the batch at every lane they affect themselves.
                const bool cand0 = valid && acc;
                const int dp_l = dp_of(), dg_l = dg_of();
                const int x0 = cand0 ? dp_l : 0;
                const int P = wave_scan_incl(x0) - x0;
                const int Gp = count_below(__ballot(cand0 && dg_l > 0)) - count_below(__ballot(cand0 && dg_l < 0));
                const bool ok1 = ((av ? ng0 + Gp : ng1 - Gp) > 0) ? okT : okN;
                const int q0 = pops0 + P, q1 = pops1 - P;
                const bool valid1 = prop & known & ok1 & ((av ? q1 : q0) - pv >= pop_lo) &
                                    ((av ? q0 : q1) + pv <= pop_hi);
                const bool cand1 = valid1 && acc;
                const uint64_t MM = __ballot(prop && cand1 != cand0);
                const uint64_t UU = __ballot(prop && !known);
                int sg = end;
                if (MM) sg = min(sg, __builtin_ctzll(MM) + 1);
                const int u = UU ? __builtin_ctzll(UU) : kWave;
                if (u < sg) sg = u;
                uint64_t VAL = __ballot(valid1) & lane_range(pos, sg);
                bool last_step = false;
                if (__popcll(VAL) >= rem) {  // the launch's last step lies in this segment
                    sg = kth_set_bit(VAL, rem) + 1;
                    VAL &= bits_below(sg);
                    last_step = true;
                }
                const uint64_t K = __ballot(cand1) & lane_range(pos, sg);
                int x = kWave;  // first lane that must not be committed
                bool stale_seg = false;
                if (K) {
                    const bool inK = (K >> lane) & 1ull;
                    st |= inK ? LF_WROTE : 0u;
                    // marks: smark[node] / nmark[neighbour] = lowest candidate lane (0xff: none).
                    // Every segment pass clears its marks (below), so the first round writes without
                    // reading.  Stores to one byte from later instructions win (a node is a
                    // neighbour of two candidates at different ring positions), so a lane that finds
                    // a higher lane in one of its marks writes again.  Each round also reads what the
                    // checks below need (the last round's values are the final ones): alpha (later
                    // slots), beta (later candidates), entering non-hits.  Every lane reads (cells
                    // are valid nodes on idle lanes too), so the reads issue back to back.
                    bool need = inK;
                    // the neighbour marks only as two ring masks: cells whose mark is above / below
                    // this lane (8 values live across the rounds made the compiler read them one
                    // LDS round trip at a time)
                    int ms = 0xff, mk[kRV];
                    uint32_t gtm = 0xffffu, ltm = 0u;
                    for (;;) {
                        FC_PROF(21, 1);
                        FC_ST(need && ms > lane, smark[v], lane);
                        const uint32_t wm = need ? (nbr & gtm) : 0u;
#pragma unroll
                        for (int i = 0; i < RMAX; ++i) FC_ST((wm >> i) & 1u, nmark[cell[i]], lane);
                        compiler_fence();
                        ms = smark[v];
                        int mn[RMAX];
#pragma unroll
                        for (int i = 0; i < RMAX; ++i) mn[i] = nmark[cell[i]];
#pragma unroll
                        for (int r = 0; r < kRV; ++r) mk[r] = nmark[rv[r] < 0 ? 0 : (rv[r] & 0xffff)];
                        gtm = 0u;
                        ltm = 0u;
#pragma unroll
                        for (int i = 0; i < RMAX; ++i) {
                            gtm |= (uint32_t)(mn[i] > lane) << i;
                            ltm |= (uint32_t)(mn[i] < lane) << i;
                        }
                        const bool again = (ms > lane) | ((nbr & gtm) != 0u);
                        need = need & again;
                        if (!__any(need)) break;
                    }
                    FC_STAMP(t_mk);
                    FC_PROF(18, t_mk - t_it1);
                    // alpha: this slot's node or a ring cell is an earlier candidate's node; beta: a
                    // neighbour shared with an earlier candidate
                    bool conf = (ms < lane) | (inK & ((nbr & ltm) != 0u));
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) conf |= (int)smark[cell[i]] < lane;
                    conf &= has;
                    const uint64_t XX = __ballot(conf && lane > pos && lane < end);
                    if (XX) {
                        x = __builtin_ctzll(XX);
                        stale_seg = true;
                        FC_PROF(13, 1);
                    }
                    // non-hit draws whose node a committed flip (a candidate before the draw)
                    // pulls into the boundary would now be proposals: the batch ends before the
                    // first of them
                    int t = trunc_off;
#pragma unroll
                    for (int r = 0; r < kRV; ++r) {
                        const bool tr = (rv[r] >= 0) & (mk[r] < x) & (mk[r] < (rv[r] >> 16));
                        const uint64_t TR = __ballot(tr);
                        if (TR) t = min(t, rv_off(r, __builtin_ctzll(TR)));
                    }
                    if (t < trunc_off) {
                        trunc_off = t;
                        const int e2 = __popcll(__ballot(has && off_l < t));
                        if (e2 < x) x = e2;
                        if (e2 < end) end = e2;  // the batch ends before the first entering draw
                        FC_PROF(14, 1);
                    }
                }
                FC_STAMP(t_cf);
                FC_PROF(19, t_cf - t_it1);
                int ce = min(sg, x);  // commit lanes [pos, ce)
                bool seg_out = false;
                if constexpr (BAND) {
                    // the first candidate whose flip puts a neighbour outside S into b_nodes is the
                    // segment's last commit (later draws map through the rebuilt S).  Inside a
                    // segment no two flips share a neighbour (beta), so the counts read here are
                    // each flip's own sequential view
                    const uint64_t K0 = K & bits_below(ce);
                    if (K0) {
                        bool out = false;
                        if ((K0 >> lane) & 1ull) {
#pragma unroll
                            for (int i = 0; i < RMAX; ++i) {
                                const int u = cell[i];
                                const uint32_t oc = fcnt[u];
                                const uint64_t swd = sb[u >> 6];
                                out |= ((nbr & inA) >> i & 1u) && oc == 0u && !((swd >> (u & 63)) & 1ull);
                            }
                        }
                        const uint64_t IV = __ballot(out);
                        if (IV) {
                            ce = __builtin_ctzll(IV) + 1;
                            seg_out = true;
                            if (ce < sg) last_step = false;
                        }
                    }
                }
                if (x < sg) last_step = false;
                if (prop && lane < ce) st |= valid1 ? (cand1 ? (ST_VS | ST_AC) : ST_VS) : (ok1 ? ST_IP : ST_IC);
                rem -= __popcll(VAL & bits_below(ce));
                const uint64_t AP = K & bits_below(ce);
                if (AP) {
                    FC_PROF(7, __popcll(AP));
                    const bool me = (AP >> lane) & 1ull;
                    // foreign-neighbour counts: u sees v leave A (+1 if u in A) and join t (-1 if u
                    // in t); beta leaves every u to one flip of the segment
                    int oldc[RMAX];
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) oldc[i] = fcnt[cell[i]];
                    compiler_fence();
                    int dnb = 0;
                    // (bit masks, not short-circuit tests: those compiled to a branch per cell)
                    // two districts: a neighbour in A gains v as a foreign neighbour (+1), one in T
                    // loses it (-1); |B| changes by the neighbours whose count leaves or reaches 0
                    const uint32_t nbm = me ? nbr : 0u;
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) {
                        const int nw = oldc[i] + 2 * (int)((inA >> i) & 1u) - 1;
                        const uint32_t nb_i = (nbm >> i) & 1u;
                        FC_ST(nb_i, fcnt[cell[i]], nw);
                        dnb += (min(nw, 1) - min(oldc[i], 1)) & -(int)nb_i;
                    }
                    FC_ST(me, *(uint8_t *)&a[v], 1 - av);
                    FC_ST(me, fcnt[v], nA);
                    const int pkd = me ? ((delta + 32) | ((dnb + 32) << 16)) : 0;
                    const int S = wave_scan_incl(pkd);
                    const int cntA = count_below(AP) + 1;
                    cut_after = me ? cut + (S & 0xffff) - 32 * cntA : cut_after;
                    nb_after = me ? nb + (S >> 16) - 32 * cntA : nb_after;
                    const int L = 63 - __builtin_clzll(AP);
                    cut = rl32(cut_after, L);
                    nb = rl32(nb_after, L);
                    const int dP = rl32(P + dp_l, L), dG = rl32(Gp + dg_l, L);
                    pops0 += dP;
                    pops1 -= dP;
                    ng0 += dG;
                    ng1 -= dG;
                    last_flip = rl32(v, L);
                    compiler_fence();
                }
                // clear this pass's marks: the next pass (and the next batch) starts clean.  Every
                // mark is 0xff between passes, so the lanes that wrote clear their whole ring
                // (cells that are not neighbours hold 0xff already; padding cells are the node)
                if (st & LF_WROTE) {
                    smark[v] = 0xff;
#pragma unroll
                    for (int i = 0; i < RMAX; ++i) nmark[cell[i]] = 0xff;
                    st &= ~LF_WROTE;
                }
                FC_STAMP(t_sg1);
                FC_PROF(11, t_sg1 - t_it1);
                pos = ce;
                if (BAND && seg_out) rebuild = true;
                if (last_step) {
                    end = pos;
                    target_hit = true;
                    break;
                }
                if (BAND && seg_out) {
                    end = pos;
                    trunc_off = rl32(off_l, pos - 1) + 1;
                    break;
                }
                if (pos >= end) break;
                if (stale_seg && AP) {  // a committed flip changed the view of a later slot
                    reeval(pos, -1, 0u);
                    FC_STAMP(t_sg2);
                    FC_PROF(29, t_sg2 - t_sg1);
                    continue;
                }
                if (SEARCH && u == pos) {
                    const bool res = run_bfs(u);
                    if (lane == u) st |= ST_BD | (res ? ST_BR : 0u);
                }
                FC_STAMP(t_sg3);
                FC_PROF(29, t_sg3 - t_sg1);
                continue;
            }
            // ---- one event at a time: the first acceptance or undecided lane -----------------
            const uint64_t VAL = __ballot(valid);
            const uint64_t EV = C0 | __ballot(prop && !known);
            const int f = EV ? __builtin_ctzll(EV) : end;
            const uint64_t segv = VAL & bits_below(f);
            const int nvalid = __popcll(segv);
            const uint32_t bits = valid ? ST_VS : (inv_contig ? ST_IC : ST_IP);
            if (nvalid >= rem) {  // the launch's last step lies before f
                const int e = kth_set_bit(segv, rem);
                st |= (prop & (lane <= e)) ? bits : 0u;
                rem = 0;
                end = e + 1;
                target_hit = true;
                break;
            }
            st |= (prop & (lane < f)) ? bits : 0u;
            rem -= nvalid;
            pos = f;
            if (f >= end) {
                FC_STAMP(t_fx);
                FC_PROF(25, t_fx - t_it1);  // the last iteration: no event left
                break;
            }
            if (SEARCH && !((VAL >> f) & 1ull)) {
                const bool res = run_bfs(f);
                if (lane == f) st |= ST_BD | (res ? ST_BR : 0u);
                continue;
            }
            // ---- accept lane f: apply the flip -------------------------------------------------
            FC_PROF(7, 1);
            FC_STAMP(t_ap0);
            FC_PROF(9, t_ap0 - t_it1);
            const int vf = rl32(v, f), Af = rl32(av, f), pvf = rl32(pv, f), df = rl32(delta, f);
            const uint32_t inAf = rlu(inA, f), nbrf = rlu(nbr, f), tmf = rlu(tmask, f);
            const bool gamf = rl32((int)gam, f) != 0;
            uint32_t rw[RMAX / 2];
#pragma unroll
            for (int k2 = 0; k2 < RMAX / 2; ++k2) rw[k2] = rlu(rec.ring[k2], f);
            uint32_t sel = rw[0];
#pragma unroll
            for (int k2 = 1; k2 < RMAX / 2; ++k2) sel = ((lane >> 1) == k2) ? rw[k2] : sel;
            const int my_e = (int)((sel >> (16 * (lane & 1))) & 0xffffu);
            const bool is_nbr = lane < RMAX && ((nbrf >> lane) & 1u);
            // foreign-neighbour counts: u sees v leave A (+1 if u in A) and join t (-1 if u in t)
            const int dlt = (int)((inAf >> lane) & 1u) - (int)((tmf >> lane) & 1u);
            // (my_e is a valid node on every lane: the read needs no guard, the store goes to the
            // sink off the neighbour lanes)
            const int old = fcnt[my_e];
            FC_ST(is_nbr, fcnt[my_e], old + dlt);
            const bool enter = is_nbr & (dlt > 0) & (old == 0);
            const bool leave = is_nbr & (dlt < 0) & (old == 1);
            bool outS = false;
            if constexpr (BAND) {
                const uint64_t swd = sb[my_e >> 6];
                outS = enter && !((swd >> (my_e & 63)) & 1ull);
            }
            if (lane == 0) {
                a[vf] = (int8_t)(1 - Af);
                fcnt[vf] = (uint8_t)__popc(nbrf & inAf);
            }
            // later lanes whose view the flip changed: proposals with vf in their ring or as
            // their node (rings are symmetric), non-hits with vf as a neighbour
            uint32_t eqm = 0;
#pragma unroll
            for (int i = 0; i < RMAX; ++i) eqm |= (uint32_t)(cell[i] == vf) << i;
            const bool stale = has & ((v == vf) | (eqm != 0u));
            const uint64_t aff = __ballot(stale && lane > f && lane < end);
            if (aff) FC_PROF(13, 1);
            uint64_t ent = __ballot(enter);
            const int dnb = __popcll(ent) - __popcll(__ballot(leave));
            // non-hit draws after f whose node just entered the boundary would now propose
            // (the counts written above are read back: a non-hit node had no foreign neighbour
            // when it was drawn, and a flip before f that gave it one has cut the batch already)
            if (ent) {
                int t_na = trunc_off;
                int fr[kRV];
#pragma unroll
                for (int r = 0; r < kRV; ++r) fr[r] = fcnt[rv[r] < 0 ? 0 : (rv[r] & 0xffff)];
#pragma unroll
                for (int r = 0; r < kRV; ++r) {
                    const bool tr = (rv[r] >= 0) & ((rv[r] >> 16) > f) & (fr[r] != 0);
                    const uint64_t m2 = __ballot(tr);
                    if (m2) t_na = min(t_na, rv_off(r, __builtin_ctzll(m2)));
                }
                if (t_na < trunc_off) {
                    trunc_off = t_na;
                    const int e2 = __popcll(__ballot(has && off_l < t_na));
                    if (e2 < end) end = e2;
                    FC_PROF(14, 1);
                }
            }
            if (Af == 0) {
                pops0 -= pvf;
                pops1 += pvf;
            } else {
                pops1 -= pvf;
                pops0 += pvf;
            }
            if (gamf) {
                const int dg = Af == 0 ? -1 : 1;
                ng0 += dg;
                ng1 -= dg;
            }
            cut += df;
            nb += dnb;
            --rem;
            last_flip = vf;
            const bool me_f = lane == f;
            st |= me_f ? (ST_VS | ST_AC) : 0u;
            cut_after = me_f ? cut : cut_after;
            nb_after = me_f ? nb : nb_after;
            compiler_fence();
            FC_STAMP(t_ap1);
            FC_PROF(10, t_ap1 - t_ap0);
            pos = f + 1;
            const bool f_out = BAND && __ballot(outS) != 0ull;  // S is rebuilt after this flip
            if (f_out) rebuild = true;
            if (rem == 0) {
                end = pos;
                target_hit = true;
                break;
            }
            if (f_out) {
                end = pos;
                trunc_off = rl32(off_l, f) + 1;
                break;
            }
            if (aff && pos < end) reeval(pos, vf, eqm);
            FC_STAMP(t_ap2);
            FC_PROF(30, t_ap2 - t_ap1);
        }
        compiler_fence();  // (the marks: cleared by each segment pass)
        steps = steps0 + (rem0 - rem);
        FC_STAMP(t_d);
        FC_PROF(3, t_d - t_c);

        FC_PROF(15, (end == ns && !target_hit && trunc_off == gen) ? 1 : 0);  // every slot committed
        // ---- 4. lane-parallel bookkeeping of the committed draws [0, end) ------------------
        const bool done = lane < end;
        const bool is_acc = (st & ST_AC) != 0;
        const bool proposed = (st & LF_HIT) && done;
        n_prop += __popcll(__ballot(proposed));
        n_acc += __popcll(__ballot(is_acc));
        n_ic += __popcll(__ballot((st & ST_IC) != 0));
        n_ip += __popcll(__ballot((st & ST_IP) != 0));
        const uint64_t ACCM = __ballot(is_acc);
        const uint64_t VSM = __ballot((st & ST_VS) != 0);
        int ln = lane;  // opaque copy: lane masks derived from it are recomputed, not hoisted and spilled
        asm volatile("" : "+v"(ln));
        const uint64_t later_acc = ACCM & ~bits_below(ln + 1);
        const int next_acc = later_acc ? __builtin_ctzll(later_acc) : end;
        const int run_len = is_acc ? 1 + __popcll(VSM & lane_range(ln + 1, next_acc)) : 0;
        const int first_acc = ACCM ? __builtin_ctzll(ACCM) : end;
        const int r0 = __popcll(VSM & bits_below(first_acc));
        int64_t my_wait = 0;
        if (XTRA && want_wait && !defer && is_acc) {
            Words4 g;
            if (XTRA && p.tape) {
                const uint32_t *t = p.tape + ((size_t)c * (size_t)p.tape_draws + d) * 6;
                g = Words4{t[4], t[5], 0u, 0u};
            } else {
                g = philox4x32_10((uint32_t)d, (uint32_t)(d >> 32), chain_gid, 1u, p.seed_lo, p.seed_hi);
            }
            my_wait = geom_from(u53(g.x0, g.x1), p.log1mp[nb_after]);
        }
        // (run_len is 0 off the accepting lanes: no guard, no exec-mask branch)
        {
            const int cr = cut_after * run_len, br = nb_after * run_len;  // < 2^31: |cut| < 2^24, runs <= 64
            acc_cut += cr;
            acc_cut2 += (int64_t)cr * cut_after;
            acc_nb += br;
            acc_nb2 += (int64_t)br * nb_after;
        }
        if (!defer) acc_wait += my_wait * run_len;
        if (lane == 0 && r0) {
            acc_cut += (int64_t)cut0 * r0;
            acc_cut2 += (int64_t)cut0 * cut0 * r0;
            acc_nb += (int64_t)nb0 * r0;
            acc_nb2 += (int64_t)nb0 * nb0 * r0;
            if (!defer || qn == 0) acc_wait += wait_cur * r0;  // else: the queued current state's run
        }
        const int64_t t_acc = FULL ? steps0 + __popcll(VSM & bits_below(ln + 1)) : 0;  // yield index of this lane
        if constexpr (FULL) {
            // the run of the batch's start state goes on: a queued state takes it into its run
            // (below), else it is tallied here
            if (lane == 0 && r0 && (!defer || qn == 0) && (p.diag & (FC_DIAG_HIST | FC_DIAG_FLIPS))) {
                // (kind 1 of tally_apply: to the tally log like the queue entries, else applied here)
                const uint32_t qv0 = (last_flip0 >= 0 ? (uint32_t)last_flip0 : 0xffffu) | ((uint32_t)(a_last0 & 1) << 16);
                const int64_t lbase = (int64_t)misc[3];
                if (p.tl && lbase < p.tl_cap) {
                    ((uint4 *)p.tl)[(size_t)c * (size_t)p.tl_cap + (size_t)lbase] =
                        tally_pack(steps0 - (int64_t)misc[4], r0, qv0, (uint32_t)cut0, (uint32_t)nb0 | 0x80000000u);
                    misc[3] = (uint64_t)(lbase + 1);
                } else {
                    tally_apply<RMAX>(p, c, steps0, r0, qv0, (uint32_t)cut0, (uint32_t)nb0 | 0x80000000u, p.labels[0],
                                      p.labels[1]);
                }
            }
        }
        if (defer) {
            if (lane == 0 && r0 && qn > 0) q_run[qn - 1] += (uint32_t)r0;
            const int na = __popcll(ACCM);
            if (na) {
                if (qn > 0 && qn + na > p.wait_q) wait_flush();  // na <= 64 = kWaitQ always fits an empty queue
                const int qi = qn + count_below(ACCM);
                if (is_acc) {
                    q_d[qi] = d;
                    q_nb[qi] = (uint32_t)nb_after;
                    q_run[qi] = (uint32_t)run_len;
                    if constexpr (FULL) {
                        q_v[qi] = (uint32_t)v | ((inA & nbr) << 16);
                        q_c[qi] = (uint32_t)cut_after | ((uint32_t)(1 - av) << 31);
                        if (qi == 0) misc[2] = (uint64_t)t_acc;
                    }
                }
                qn += na;
                compiler_fence();
            }
        }
        if constexpr (FULL) {
            // per batch only with a trace or a tape (XTRA); else in tally_flush
            if (XTRA && !defer && (p.diag & FC_DIAG_SERIES) && ACCM) {
                const int64_t idx = ev_len + __popcll(ACCM & bits_below(ln));
                if (is_acc && idx < p.ev_cap) {
                    fc_event ev;
                    ev.t = t_acc;
                    ev.v = (uint16_t)v;
                    ev.cut = (uint16_t)cut_after;
                    ev.nb = (uint16_t)nb_after;
                    ev.target = (uint8_t)(1 - av);
                    ev.reserved = 0;
                    p.events[(size_t)c * p.ev_cap + idx] = ev;
                }
                ev_len += __popcll(ACCM);
            }
            if (hit_time < 0 && ACCM) {
                const uint64_t hm = __ballot(is_acc && cut_after >= p.hit_lo && cut_after <= p.hit_hi);
                if (hm) {
                    const int hl = __builtin_ctzll(hm);
                    hit_time = steps0 + __popcll(VSM & bits_below(hl + 1));
                }
            }
            // per batch only when the queue is off (trace, tape): else tally_flush
            if (XTRA && !defer && (p.diag & FC_DIAG_HIST) && is_acc) {
                atomicAdd((unsigned long long *)&p.cut_hist[(size_t)c * (p.n_edges + 1) + cut_after], (unsigned long long)run_len);
                atomicAdd((unsigned long long *)&p.nb_hist[(size_t)c * (n + 1) + nb_after], (unsigned long long)run_len);
            }
            if (XTRA && !defer && (p.diag & FC_DIAG_FLIPS) && is_acc) {
                // part.flips is stale on rejected steps: every yield of a run repeats the update
                // part_sum[f] -= a[f] * (t - last_flipped[f]) for the node f whose flip created
                // the state (grid_chain_sec11.py:396-400).  With two districts a node's label
                // alternates between its runs, so summed over the runs r of f (last yield t_r,
                // label a_r) part_sum = init - a_R t_R + sum_{r<R} (L0 + L1 - 2 a_r) t_r: every
                // run adds (L0 + L1 - 2 a_r) per yield it lasts, and the read-out replaces the
                // last run's share (fc_run_read_flips).  Only commuting adds and a max remain,
                // so flips of one batch may share nodes.
                // (the start state's run: above)
                int64_t *nf = p.num_flips + (size_t)c * n, *ps = p.part_sum + (size_t)c * n;
                unsigned long long *lf = (unsigned long long *)(p.last_flipped + (size_t)c * n);
                const int64_t lsum = (int64_t)p.labels[0] + (int64_t)p.labels[1];
                const int64_t t_last = t_acc + run_len - 1;
                atomicMax(lf + v, (unsigned long long)t_last);
                atomicAdd((unsigned long long *)(ps + v), (unsigned long long)((lsum - 2 * (int64_t)p.labels[1 - av]) * t_last));
                atomicAdd((unsigned long long *)(nf + v), (unsigned long long)run_len);
            }
            if (XTRA && !defer && (p.diag & FC_DIAG_FLIPS_EXACT) && is_acc) {
                // the corrected companions: one count per accepted
                // flip, the label's time integral as -(L_new - L_old) t per flip (+ L_now T at
                // read-out, fc_run_read_flips_exact), the flip's yield; commuting updates only
                const size_t o = (size_t)c * n + v;
                const int64_t dl = (int64_t)p.labels[1 - av] - (int64_t)p.labels[av];
                atomicAdd((unsigned long long *)(p.flip_count + o), 1ull);
                atomicAdd((unsigned long long *)(p.occ_acc + o), (unsigned long long)(-dl * t_acc));
                atomicMax((unsigned long long *)(p.last_accept + o), (unsigned long long)t_acc);
            }
            if (XTRA && !defer && (p.diag & FC_DIAG_EDGES) && is_acc) {
                // cut_times[e] (yields with e cut, :383-384) = sum of the yields at which e turns
                // uncut - sum of those at which it turns cut (+ the yield count while it is cut:
                // fc_run_read_edges); commuting adds only
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
            if (trace_on) {
                const uint64_t PM = __ballot(proposed);
                const uint64_t mine = ACCM & bits_below(ln + 1);
                const int src = mine ? 63 - __builtin_clzll(mine) : 0;
                const int c_j = __shfl(cut_after, src), n_j = __shfl(nb_after, src);
                const long long w_j = __shfl((long long)my_wait, src);
                const int64_t idx = trace_len + __popcll(PM & bits_below(ln));
                if (proposed && idx < p.trace_cap) {
                    fc_record &rr = p.trace[(size_t)c * p.trace_cap + idx];
                    const bool valid = (st & ST_VS) != 0;
                    rr.draw = (int64_t)d;
                    rr.v = v;
                    rr.flags = (valid ? (1 | (is_acc ? 2 : 0)) : ((st & ST_IC) ? 4 : 8)) | ((1 - av) << 8);
                    rr.cut = mine ? c_j : cut0;
                    rr.nb = mine ? n_j : nb0;
                    rr.wait = valid ? (mine ? (int64_t)w_j : wait_cur) : 0;
                }
                trace_len += __popcll(PM);
            }
        }
        if (!defer && ACCM) {
            const int la = 63 - __builtin_clzll(ACCM);
            wait_cur = (int64_t)(((uint64_t)(uint32_t)rl32((int)(uint32_t)my_wait, la)) |
                                 ((uint64_t)(uint32_t)rl32((int)(my_wait >> 32), la) << 32));
        }
        // draws consumed by the committed slots [0, end)
        int consumed;
        if (target_hit) {
            consumed = rl32(off_l, end - 1) + 1;
        } else {
            consumed = end < ns ? rl32(off_l, end) : gen;
            if (trunc_off < consumed) consumed = trunc_off;
        }
        draw += (uint64_t)consumed;
        if constexpr (BAND) {
            if (rebuild) {
                FC_STAMP(t_rb0);
                band_rebuild();
                FC_STAMP(t_rb1);
                FC_PROF(22, 1);
                FC_PROF(23, t_rb1 - t_rb0);
            }
        }
        FC_PROF(24, ns);
        compiler_fence();
        FC_STAMP(t_e);
        FC_PROF(4, t_e - t_d);
    }
    if (defer && qn > 0) wait_flush();
    FC_STAMP(t_loop1);
    FC_PROF(0, t_loop1 - t_loop0);
    // the chain's own work this launch (draws: a short boundary costs many per step), not its
    // duration, which its SIMD-mates stretch
    if (p.ctime && lane == 0) p.ctime[c] = (uint32_t)min(draw - scp->draw, (uint64_t)0xffffffffu);
    if (p.eta && rem == 0 && lane == 0) {  // this launch's pace, for the next one's priorities
        const uint64_t el = __builtin_amdgcn_s_memrealtime() - misc[0];
        atomicMax(&p.eta[p.eta_parity], (uint32_t)min(el * 1024ull / (uint64_t)max((int)p.n_steps, 1), 0xffffffffull));
    }
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
            ga[i] = ((const uint4 *)a)[i];
            gf[i] = ((const uint4 *)fcnt)[i];
        }
        if (BAND && lane < p.words) p.sbits[(size_t)c * p.words + lane] = sb[lane];
    }
    const int64_t cnt_prop = n_prop, cnt_acc = n_acc, cnt_ic = n_ic, cnt_ip = n_ip;  // already wave totals
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        acc_cut += __shfl_xor((long long)acc_cut, off);
        acc_nb += __shfl_xor((long long)acc_nb, off);
        acc_wait += __shfl_xor((long long)acc_wait, off);
        acc_cut2 += __shfl_xor((long long)acc_cut2, off);
        acc_nb2 += __shfl_xor((long long)acc_nb2, off);
    }
    if (FULL && p.tl_len && lane == 0) p.tl_len[c] = (int64_t)misc[3];
    if (lane == 0) {
        scp->draw = draw;
        scp->steps = steps;
        scp->proposals += cnt_prop;
        scp->accepted += cnt_acc;
        scp->inv_contig += cnt_ic;
        scp->inv_pop += cnt_ip;
        if (FULL) {
            scp->trace_len = trace_len;
            scp->ev_len = ev_len;
            scp->hit_time = hit_time;
        }
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

int launch_flip2(const KParams &p, int ring_max, void *stream, char *name, size_t name_cap) {
    // one chain (wave) per workgroup: the dispatcher then deals consecutive chains, whose
    // bases differ, round-robin over the XCDs, CUs and SIMDs, and the short-boundary chains
    // that set the launch time spread more evenly over the SIMDs than four to a workgroup
    // (C2 on one MI355X: 8.46 ms per 10,000-step launch against 9.0 with four, 9.5 with two).
    // tune_chains_per_block = 2 / 4 restores the larger workgroups (diagnostic).
    const int wpb = p.wpb;  // fc_params.tune_chains_per_block (resolved by fc_run_create)
    const int blocks = (p.n_chains + wpb - 1) / wpb;
    const size_t lds = (size_t)p.chain_lds_bytes * wpb;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(blocks), block(kWave * wpb);
    // FULL: replay tapes, traces, event logs, histograms, per-node/per-edge tallies or a
    // hitting-time window; the lean instance keeps its registers for the hot loop.
    const bool full = p.tape || p.trace || (p.diag & ~(uint32_t)FC_DIAG_WAIT) || p.hit_lo <= p.hit_hi || p.variant;
    // replay tapes, traces, accept / constraint variants, frozen nodes
    const bool xtra = p.tape || p.trace || p.variant;
    // no search code when the run rule decides every proposal (all nodes exact, no forced search)
    const bool search = !p.all_exact || (p.flags & FC_FLAG_FORCE_BFS);
#define FC_LAUNCH2B(R, S, F, X, Y, B)                                                                      \
    do {                                                                                                    \
        if (lds > 65536)                                                                                    \
            (void)hipFuncSetAttribute((const void *)flip2_kernel<R, S, F, X, Y, B>,                         \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                \
        if (name)                                                                                           \
            snprintf(name, name_cap, "fc::flip2_kernel<%d, %d, %s, %s, %s, %s>", R, S, F ? "true" : "false", \
                     X ? "true" : "false", Y ? "true" : "false", B ? "true" : "false");                    \
        hipLaunchKernelGGL((flip2_kernel<R, S, F, X, Y, B>), grid, block, lds, s, p);                       \
    } while (0)
#define FC_LAUNCH2(R, S, F, X, Y)                        \
    do {                                                 \
        if (p.band) FC_LAUNCH2B(R, S, F, X, Y, true);    \
        else FC_LAUNCH2B(R, S, F, X, Y, false);          \
    } while (0)
#define FC_SEARCH2(R, S, F, Y)                    \
    do {                                          \
        if (search) FC_LAUNCH2(R, S, F, true, Y);  \
        else FC_LAUNCH2(R, S, F, false, Y);        \
    } while (0)
#define FC_FULL2(R, S)                                \
    do {                                              \
        if (xtra) FC_SEARCH2(R, S, true, true);        \
        else if (full) FC_SEARCH2(R, S, true, false);  \
        else FC_SEARCH2(R, S, false, false);           \
    } while (0)
#define FC_NSUB2(R)                                \
    switch (p.nsub) {                              \
        case 1: FC_FULL2(R, 1); break;             \
        case 2: FC_FULL2(R, 2); break;             \
        case 4: FC_FULL2(R, 4); break;             \
        default: return (int)hipErrorInvalidValue; \
    }
    if (ring_max == 8) {
        FC_NSUB2(8)
    } else if (ring_max == 16) {
        FC_NSUB2(16)
    } else {
        return (int)hipErrorInvalidValue;
    }
#undef FC_NSUB2
#undef FC_FULL2
#undef FC_SEARCH2
#undef FC_LAUNCH2
#undef FC_LAUNCH2B
    return (int)hipGetLastError();
}

}  // namespace fc
