// Internal structures shared by the host graph builder, the C-ABI layer and the kernels.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/flipchain.h"

namespace fc {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;   // one chain per wave, 4 chains per 256-thread workgroup
constexpr int kBigChainLds = 16 * 1024;  // above this, one chain per 64-thread workgroup (occupancy)
// LDS bytes of one chain's BFS scratch (dev::BfsScratch): labels, masks, counters, 2 lists, 3 bitmaps
inline int bfs_lab_words(int n) { return ((n + 3) / 4 + 1) & ~1; }
inline int bfs_bytes(int n) { return 4 * bfs_lab_words(n) + 128 + 16 + 2 * 2 * 512 + 24 * ((n + 63) / 64); }
inline int waves_per_block(int chain_lds_bytes) { return chain_lds_bytes > kBigChainLds ? 1 : kWavesPerBlock; }
constexpr int kMaxK = 2;            // districts held in ChainScalars (k = 2 fast path)
constexpr int kMaxKGeneral = 32;    // districts of the general (PAIR) kernel
constexpr int kMaxKDistrictRule = 31;  // district-graph rule: bit 31 of a district mask is the outer face
// LDS bytes of the district-graph rule's per-chain tables: pair counts, adjacency masks, outer counts
inline int dgraph_lds_bytes(int k) { return 4 * k * k + 4 * 32 + 4 * 32; }
// the multi-flip commit's hashed neighbour marks (fc_kernels.hip), after the district tables
constexpr int hb_bytes(int ring_max) { return ring_max == 8 ? 256 : 128; }

// meta word layout (also exported by fc_graph_rings)
constexpr uint64_t kMetaLenMask = 0xffull;
constexpr uint64_t kMetaExact = 1ull << 8;
constexpr uint64_t kMetaGamma = 1ull << 9;
constexpr uint64_t kMetaFrozen = 1ull << 10;  // FC_CON_FIXED: endpoint of a pinned cut edge (per run)
constexpr int kMetaNbrShift = 16;
constexpr int kMetaLinkShift = 32;

// Device node record: everything one proposal needs about its node, in one cache sector.
// ring[] holds int16 node ids packed two per u32, padded with the node itself.
template <int RMAX>
struct alignas(16) NodeRec {
    uint64_t meta;
    int32_t pop;
    int32_t deg;
    uint32_t ring[RMAX / 2];
};
static_assert(sizeof(NodeRec<8>) == 32, "NodeRec<8> must be 32 B");
static_assert(sizeof(NodeRec<16>) == 48, "NodeRec<16> must be 48 B");

struct HostGraph {
    int32_t n = 0, n_edges = 0, ring_max = 8, max_degree = 0;
    std::vector<int32_t> row_ptr, col_idx, pop;
    std::vector<double> pos;          // [2n] or empty
    std::vector<int32_t> eu, ev;      // canonical edges
    std::vector<int32_t> ring;        // [n * ring_max]
    std::vector<uint64_t> meta;       // [n]
    std::vector<int32_t> ring_eid;    // [n * ring_max] edge id of neighbour entries, else -1
    int32_t n_exact = 0, n_gamma = 0;
    bool planar = false, outer_simple = false, connected = false;
};

// Builds rings / exactness (fc_graph.cpp).  Returns an error message or "".
std::string build_host_graph(int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                             const int32_t *pop, const double *pos_xy, uint32_t flags, HostGraph &g);

// Per-chain persistent scalars (device, one struct per chain).
struct ChainScalars {
    uint64_t draw;          // next draw index
    int64_t steps, proposals, accepted, inv_contig, inv_pop;
    int64_t sum_cut, sum_nb, sum_wait, sum_cut2, sum_nb2;
    int64_t wait_cur;
    int64_t bfs_calls, bfs_levels;
    int64_t trace_len;
    int64_t ev_len;         // FC_DIAG_SERIES events in the current window
    int64_t hit_time;       // first yield with hit_lo <= cut <= hit_hi, -1: not yet
    int64_t ser_t0;         // yield index starting the series window
    int32_t cut, nb;
    int32_t pops[kMaxK];
    int32_t ngamma[kMaxK];
    int32_t last_flip;
    int32_t stuck;
    int32_t ser_cut0, ser_nb0;  // |cut|, |B| at ser_t0
    int32_t pop_lo, pop_hi;     // this chain's inclusive population bounds (fc_params.chain_pop_bounds)
};

// Kernel parameters (passed by value).
struct KParams {
    const void *graph;          // NodeRec<RMAX>[n]
    const int32_t *ring_eid;    // [n * RMAX] (FC_DIAG_EDGES)
    int32_t n, n_edges, n_chains, k;
    int32_t chain_lds_bytes;    // LDS bytes per chain
    int32_t words;              // ceil(n / 64) bitmap words
    int32_t lab_words;          // BFS label bytes, in u32 words (even)
    uint32_t lemire_thresh;     // 2^32 mod n
    uint32_t chain_id_offset;
    uint32_t seed_lo, seed_hi;
    int32_t pop_lo, pop_hi;     // (unused by the kernels: each chain's bounds are in ChainScalars)
    int64_t n_steps;            // steps to advance per chain in this launch
    int64_t max_draws;          // per chain per launch
    int8_t *assign;             // [n_chains * n]
    uint8_t *fcnt;              // [n_chains * n] foreign-neighbour counts
    ChainScalars *sc;           // [n_chains]
    const uint64_t *thresh;     // [n_chains * (2*RMAX+1)] acceptance thresholds (U53 mantissa)
    const double *log1mp;       // [nb_w]
    const int32_t *labels;      // [k]
    uint32_t diag;              // FC_DIAG_*
    uint32_t flags;             // FC_FLAG_*
    // optional diagnostics
    int64_t *cut_hist;          // [n_chains * (E+1)]
    int64_t *nb_hist;           // [n_chains * nb_w]
    int32_t nb_w;               // |B| histogram row: n + 1, or the largest pair count + 1 (nb_pairs)
    int32_t nb_pairs;           // k > 2, FC_FLAG_NB_PAIRS: |B| counts (node, district) pairs
    int64_t *edge_acc;          // [n_chains * E]
    int64_t *num_flips;         // [n_chains * n]
    int64_t *part_sum;          // [n_chains * n]
    int64_t *last_flipped;      // [n_chains * n]
    int64_t *flip_count;        // [n_chains * n] FC_DIAG_FLIPS_EXACT: accepted flips
    int64_t *occ_acc;           // [n_chains * n] ... -sum over flips of (L_new - L_old) * t
    int64_t *last_accept;       // [n_chains * n] ... yield of the last accepted flip
    fc_record *trace;           // [trace_chains * trace_cap]
    int32_t trace_chains;
    int64_t trace_cap;
    const uint32_t *tape;       // replay tape or null
    int64_t tape_draws;
    int32_t *popk;              // [n_chains * 32] district populations (k > 2)
    int32_t wmax;               // PAIR: fixed slot bound per node draw (wdyn == 0)
    int32_t wdyn;               // PAIR: slot bound = the state's largest foreign-district count
    int32_t *nfh;               // [n_chains * kNfh] PAIR: nodes per foreign-district count
    fc_event *events;           // [n_chains * ev_cap] (FC_DIAG_SERIES)
    int64_t ev_cap;
    int32_t hit_lo, hit_hi;     // hitting-time window on |cut| (lo > hi: off)
    int32_t nsub;               // max draw rounds of 64 per batch (1, 2, 4)
    int32_t hit_stop;           // start another round only while fewer boundary hits than this
    int64_t *prof;              // [n_chains * kProfSlots] phase cycles (FC_PHASE_PROF builds only)
    int32_t par_min;            // k = 2: segment-parallel commit from this many acceptances on
    int32_t variant;            // accept / constraint variants in use (FULL k = 2 instance)
    int32_t accept;             // FC_ACCEPT_*
    uint32_t con_valid;         // FC_CON_* of the Validator
    uint32_t con_accept;        // FC_CON_* of the accept callable
    int32_t prio_nb[3];         // k = 2: issue priority 1/2/3 below these |B| (0: off)
    uint32_t *eta;              // k = 2: [2] slowest chain's s_memrealtime ticks per 1024 steps, by launch parity
    int32_t eta_parity;         // this launch writes eta[parity] and reads eta[parity ^ 1]
    float prio_th[3];           // ... projected-finish / previous launch thresholds for priority 1/2/3
    int32_t wait_q;             // deferred-wait queue capacity in use (<= kWaitQ / kWaitQK)
    int32_t wpb;                // chains (waves) per workgroup: 1, 2 or 4
    // k > 2 district-graph contiguity rule (every node exact, planar, simple outer face,
    // k <= kMaxKDistrictRule): per chain, face-adjacent cell pairs per district pair and
    // outer-face nodes per district (fc_kernels.hip district_rule)
    int32_t all_exact;          // every node's contiguity is decided by the local rules (k = 2 run rule)
    int32_t dgraph;
    int32_t *mcnt;              // [n_chains * k * k] pair counts, cell [min(X, Y) * k + max(X, Y)]
    int32_t *ngk;               // [n_chains * 32] outer-face nodes per district
    int32_t coop;               // k > 2 large graphs without the district rule: one chain per
                                // 256-thread workgroup, contiguity searches by the whole workgroup
    // chain dealing (k = 2): a wave takes its chain by its arrival slot on its SIMD, from the
    // slot's quarter of `order` (chains by the previous launch's duration, slowest first), so
    // that every SIMD runs one chain of each quarter instead of whatever the dispatcher's
    // order piles onto it (fc_deal.hip)
    uint32_t *deal;             // [kDealKeys + 4]: arrivals per SIMD key, claims per quarter (zeroed per launch)
    const uint32_t *order;      // [n_chains] chain ids, slowest first (null: no dealing)
    uint32_t *ctime;            // [n_chains] draws each chain took in its last launch (the dealing key)
    // k = 2 band stream (FC_STREAM_BAND): per chain the band S = b_nodes + neighbours as a
    // bitmap of `words` u64; a draw selects the i-th member (fc_flip2.hip)
    int32_t multi_flip;         // k > 2 district-rule instance: several independent flips per commit pass
    // k = 2 full diagnostics: the per-flip tallies of the flushed wait / tally queue, logged per
    // chain (two coalesced stores per entry) and applied by tally_reduce after the launch, so
    // the chain's serial stream carries no global atomics (fc_flip2.hip tally_flush).  A full
    // log falls back to the atomics; tl_len is 0 at every launch start (tally_reduce resets it)
    uint32_t *tl;               // [n_chains * tl_cap][4], 16 B per entry (fc_flip2.hip tally_pack)
    int64_t *tl_t0;             // [n_chains] yield index at the launch's start (entries hold t - t0)
    int64_t *tl_len;            // [n_chains] entries logged this launch
    int64_t tl_cap;             // entries per chain
    int32_t band;
    int32_t band_step0;         // largest power of two below `words` (rank search over the words)
    uint64_t *sbits;            // [n_chains * words]
};

// chain dealing: SIMD keys are XCC_ID[2:0] . HW_ID[15:4] (SIMD, pipe, CU, SH, SE)
constexpr int kDealKeys = 1 << 15;

// Diagnostic build (-DFC_PHASE_PROF): s_memtime cycles per kernel phase, per chain.
// slots: 0 loop total, 1 draws, 2 evaluate, 3 commit, 4 bookkeeping, 5 batches,
//        6 commit-loop iterations, 7 applied flips; k = 2 commit detail: 8 verdicts,
//        9 one-event classify, 10 one-event apply, 11 segment-parallel, 12 segments
constexpr int kProfSlots = 32;
// k = 2 lean kernel: accepted states queued for their geometric wait (fc_flip2.hip wait_flush)
constexpr int kWaitQ = 64;
// k > 2 kernel: 32 entries, so that sec11 chains keep four waves per SIMD in 160 KB of LDS
constexpr int kWaitQK = 32;
// k > 2 kernel: histogram bins of the per-node foreign-district counts (0..31)
constexpr int kNfh = 32;

// ReCom kernel parameters (fc_recom.hip).
struct RecomParams {
    const void *graph;             // NodeRec<RMAX>[n]
    const uint32_t *nbe;           // [n * nb_d] neighbours, ring order: id | edge id << 16 (pad ~0u)
    const uint32_t *eslot;         // [n_edges] k_u | k_v << 8: each end's index in the other's nbe row
    const int32_t *eu, *ev;        // [n_edges] canonical edge list
    int32_t nb_d;                  // nbe row length: max degree rounded up to a multiple of 4
    int32_t n, n_edges, n_chains, chain_lds_bytes;
    uint32_t chain_id_offset, seed_lo, seed_hi;
    int32_t pop_lo, pop_hi;
    double pop_target, epsilon;
    int32_t node_repeats, max_attempts;
    int64_t n_steps, max_draws;
    int8_t *assign;
    ChainScalars *sc;              // attempts in bfs_calls, spanning trees in bfs_levels
    const uint64_t *accept_thresh; // [2 n_edges + 1]: U53 thresholds of base ** (cut - cut')
    fc_recom_record *trace;
    int32_t trace_chains;
    int64_t trace_cap;
    int64_t *prof;                 // [n_chains * kProfSlots] phase cycles (FC_PHASE_PROF builds only)
};
// fc_recom.hip's layout: 8 B (keys / tree CSR + parents / subtree populations) + component +
// order (2 + 2 B) + tree-edge bits (1 B for RMAX = 8, else 2) + assignment (1 B) per node
inline int recom_lds_bytes(int n, int ring_max) { return (ring_max == 8 ? 14 : 15) * ((n + 15) & ~15); }
int launch_recom(const RecomParams &p, int ring_max, void *stream, char *name, size_t name_cap);

// Launch wrappers (fc_kernels.hip).  Return a hipError_t as int.
// `name` (may be null) receives the launched instance, spelled as rocprofv3 reports it.
int launch_flip_k2(const KParams &p, int ring_max, void *stream, char *name, size_t name_cap);  // k > 2
int launch_flip2(const KParams &p, int ring_max, void *stream, char *name, size_t name_cap);    // k = 2
// k = 2 full diagnostics: apply every chain's tally log (KParams tl_*) to the per-chain
// histograms / per-node / per-edge arrays and reset the logs (fc_flip2.hip)
int launch_tally_reduce(const KParams &p, int ring_max, void *stream);
// chain dealing (fc_deal.hip): order[] = chains by descending key (ctime, the last launch's
// draws, if `timed`, else the boundary length's complement n - |B|: a short boundary needs
// many draws per proposal), and the deal counters zeroed, for the next flip launch
int launch_deal_order(const uint32_t *ctime, const ChainScalars *sc, int n, int n_chains, int timed,
                      uint32_t *order, uint32_t *deal, void *stream);

// Series diagnostics (fc_series.hip): expand the event logs of chains [c0, c0 + nc) into
// dense |cut| series x[(c - c0) * stride + t], t < len[c], then accumulate per lag
// P = sum x_t x_{t+L}, H = sum_{t < len-L} x_t, G = sum_{t >= L} x_t into sums[c][lag][3].
int launch_series_expand(const fc_event *events, int64_t ev_cap, const int64_t *ev_len, const int64_t *t0,
                         const int32_t *cut0, const int64_t *len, int32_t c0, int32_t nc, int64_t stride,
                         int64_t max_len, uint16_t *x, void *stream);
int launch_series_lagsums(const uint16_t *x, const int64_t *len, int32_t c0, int32_t nc, int64_t stride,
                          int64_t max_len, const int32_t *lags, int32_t nlags, unsigned long long *sums,
                          void *stream);
// Frame-edge slope / angle series of chains [c0, c0 + nc), k = 2 (fc_series.hip): entry 0 is
// the window start (assignment a0), entry i + 1 the state after event i.  tog_idx[node] is the
// node's row in tog_mask[.][4] (frame edges incident to it) or -1.  n_frame <= 256.
int launch_frame_series(const int8_t *a0, int32_t npad, const fc_event *events, int64_t ev_cap,
                        const int64_t *ev_len, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *fu,
                        const int32_t *fv, const double *mid, double cx, double cy, const int32_t *tog_idx,
                        const uint64_t *tog_mask, int32_t n_rows, int32_t n_nodes, int64_t cap, double *slope,
                        double *angle, int32_t *cnt, void *stream);
// Change points of the same series (fc_run_frame_series_changes): cp_off == nullptr counts them
// per chain into cp_cnt[cl]; otherwise writes (t, slope, angle) at cp_off[cl].  n_rows: rows of
// tog_mask, n_nodes: entries of tog_idx (the tables are staged in LDS when they fit).
int launch_frame_changes(const int8_t *a0, int32_t npad, const fc_event *events, int64_t ev_cap,
                         const int64_t *ev_len, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *fu,
                         const int32_t *fv, const double *mid, double cx, double cy, const int32_t *tog_idx,
                         const uint64_t *tog_mask, int32_t n_rows, int32_t n_nodes, const int64_t *t0,
                         int64_t *cp_cnt, const int64_t *cp_off, int64_t *t_out, double *slope, double *angle,
                         int64_t *wcnt, void *stream);
constexpr int kFrameWaves = 4;  // waves per chain of the frame-series kernels (wcnt: [nc][kFrameWaves])
// One-pass form of the above (count and write together): each chain's waves stage their change
// points at st_* + cl * stage_cap + w * (stage_cap / kFrameWaves), counts in wcnt / cp_cnt; then
// launch_frame_compact packs them at cp_off.  stage_cap / kFrameWaves must exceed the events of any
// wave's range: 64 * ceil(ceil(ev_cap / 64) / kFrameWaves) + 1.
int launch_frame_stage(const int8_t *a0, int32_t npad, const fc_event *events, int64_t ev_cap,
                       const int64_t *ev_len, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *fu,
                       const int32_t *fv, const double *mid, double cx, double cy, const int32_t *tog_idx,
                       const uint64_t *tog_mask, int32_t n_rows, int32_t n_nodes, const int64_t *t0,
                       int64_t *cp_cnt, int64_t stage_cap, int64_t *st_t, double *st_s, double *st_a,
                       int64_t *wcnt, void *stream);
int launch_frame_compact(int32_t nc, int64_t stage_cap, const int64_t *st_t, const double *st_s,
                         const double *st_a, const int64_t *wcnt, const int64_t *cp_off, int64_t *t_out,
                         double *slope, double *angle, void *stream);

}  // namespace fc
