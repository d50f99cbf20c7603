// C-ABI of libflipchain.so (include/flipchain.h): graph and run lifetime, initial-state
// validation and set-up on the host, kernel launches and readouts.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "fc_internal.h"
#include "fc_philox.h"

struct fc_graph {
    fc::HostGraph h;
};

struct fc_run {
    fc::HostGraph g;  // host copy (sizes, edges, rings for readouts)
    fc_params p{};
    std::vector<int32_t> labels;
    std::vector<double> log1mp;
    int32_t nb_w = 0;   // entries of the |B| histogram / log(1 - p) table: n + 1, or with
                        // FC_FLAG_NB_PAIRS (k > 2) the largest pair count + 1
    int32_t n_chains = 0;
    int32_t npad = 0;
    int32_t words = 0;
    int32_t chain_lds_bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> launch_events;  // pool
    size_t n_launch_events = 0;                                      // recorded since last read
    // device buffers
    void *d_graph = nullptr;
    int32_t *d_ring_eid = nullptr;
    int8_t *d_assign = nullptr;
    uint8_t *d_fcnt = nullptr;
    fc::ChainScalars *d_sc = nullptr;
    uint64_t *d_thresh = nullptr;
    double *d_log1mp = nullptr;
    int32_t *d_labels = nullptr;
    int64_t *d_cut_hist = nullptr, *d_nb_hist = nullptr;
    int64_t *d_edge_acc = nullptr;
    // k = 2 full diagnostics: the per-chain tally log (KParams tl_*), grown by fc_run_steps
    uint32_t *d_tl = nullptr;
    int64_t *d_tl_len = nullptr, *d_tl_t0 = nullptr;
    int64_t tl_cap = 0;
    int64_t tl_want = 0;           // entries per chain the last launch asked for (tl_cap: granted)
    int32_t series_staged = -1;    // last fc_run_frame_series_changes: 1 one staged pass, 0 two passes
    int64_t *d_num_flips = nullptr, *d_part_sum = nullptr, *d_last_flipped = nullptr;
    int64_t *d_flip_count = nullptr, *d_occ_acc = nullptr, *d_last_accept = nullptr;  // FC_DIAG_FLIPS_EXACT
    int32_t *d_popk = nullptr;
    int32_t *d_nfh = nullptr;   // k > 2: per chain, nodes per foreign-district count (PAIR slot bound)
    uint64_t *d_sbits = nullptr;  // k = 2 band stream: per chain, the band S as a bitmap (words u64)
    int32_t *d_mcnt = nullptr, *d_ngk = nullptr;  // k > 2 district-graph rule tables
    bool dgraph = false;
    int32_t mf_marks = 0;        // k > 2 multi-flip commit: 0 off, 1 hashed neighbour marks, 2 exact marks
    int32_t wmax = 1;
    fc_event *d_events = nullptr;
    int64_t ev_cap = 0;
    fc_record *d_trace = nullptr;
    uint32_t *d_tape = nullptr;
    int64_t tape_draws = 0;
    int64_t *d_prof = nullptr;  // FC_PHASE_PROF builds
    uint32_t *d_eta = nullptr;  // k = 2: per-launch pace of the slowest chain (issue priorities)
    uint32_t *d_deal = nullptr, *d_order = nullptr, *d_ctime = nullptr;  // k = 2 chain dealing (fc_deal.hip)
    bool deal_timed = false;    // d_ctime holds a launch's per-chain durations
    int64_t n_flip_launches = 0;
    int32_t *d_eu = nullptr, *d_ev = nullptr;  // recom: canonical edge list
    uint32_t *d_nbe = nullptr, *d_eslot = nullptr;  // recom: neighbour rows, edge ends' row indices
    int32_t nb_d = 4;                          // recom: nbe row length
    uint64_t *d_recom_thresh = nullptr;        // recom: [2E+1] acceptance thresholds
    int8_t *d_ser_a0 = nullptr;  // FC_DIAG_SERIES: assignment at the series window start
    double *d_fs_out = nullptr;  // fc_run_frame_series output (slope, angle), grown on demand
    int32_t *d_fs_cnt = nullptr; // ... frame-cut counts
    size_t fs_cap = 0;           // entries per output array held
    // fc_run_frame_series_changes, kept across calls (one call per launch in the driver loop):
    // the frame tables (re-uploaded only when the frame changes), per-chain lengths / window
    // starts / counts / offsets, and the (t, slope, angle) outputs, grown on demand
    uint64_t fc_frame_hash = 0;
    int32_t fc_rows = 0;  // rows of d_fc_tog
    int64_t *d_fc_wcnt = nullptr;  // change points per chain and frame-series wave
    int64_t *d_st_t = nullptr;     // one-pass change points: per-wave staging ranges (t; slope, angle)
    double *d_st_sa = nullptr;
    size_t fc_stage_cap = 0;
    int32_t *d_fc_fuv = nullptr, *d_fc_tidx = nullptr;
    uint64_t *d_fc_tog = nullptr;
    double *d_fc_mid = nullptr;
    int64_t *d_fc_len = nullptr, *d_fc_t0 = nullptr, *d_fc_cnt = nullptr, *d_fc_off = nullptr;
    int64_t *d_fc_t = nullptr;
    double *d_fc_sa = nullptr;
    size_t fc_cap = 0;           // change points the outputs hold
    char kname[96] = {0};        // last launched flip-kernel instance
    uint64_t param_hash = 0;     // FNV-1a of every trajectory-determining parameter (checkpoint check)
    bool variant = false;        // accept / constraint variants (FULL k = 2 instance)
    struct {                     // fc_params.tune_* with the defaults filled in
        int32_t nsub, hit_stop, par_min, wait_q, wpb, coop, deal, multi;
        int32_t prio_div[3];     // prio_div[0] <= 0: priorities off
        float prio_th[3];
    } tune{};
    size_t ev_head = 0;          // launch_events: oldest recorded pair (ring of kMaxLaunchEvents)
};

namespace {

constexpr int kWaveSlots = 64;
constexpr size_t kMaxLaunchEvents = 4096;  // per-launch HIP event pairs kept (fc_run_timings)
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(FC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <typename T>
int dalloc(T **p, size_t count) {
    *p = nullptr;
    if (count == 0) return FC_OK;
    hipError_t e = hipMalloc((void **)p, count * sizeof(T));
    if (e != hipSuccess) return fail(FC_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    return FC_OK;
}

void free_run(fc_run *r) {
    if (!r) return;
    void *bufs[] = {r->d_graph, r->d_ring_eid, r->d_assign, r->d_fcnt, r->d_sc, r->d_thresh, r->d_log1mp,
                    r->d_labels, r->d_cut_hist, r->d_nb_hist, r->d_edge_acc,
                    r->d_num_flips, r->d_part_sum, r->d_last_flipped, r->d_flip_count, r->d_occ_acc, r->d_last_accept, r->d_trace, r->d_tape, r->d_popk, r->d_nfh, r->d_sbits, r->d_mcnt, r->d_ngk, r->d_events, r->d_prof, r->d_eta, r->d_deal, r->d_order, r->d_ctime, r->d_ser_a0, r->d_eu, r->d_ev, r->d_nbe, r->d_eslot, r->d_recom_thresh, r->d_tl, r->d_tl_len, r->d_tl_t0,
                    r->d_fs_out, r->d_fs_cnt, r->d_fc_fuv, r->d_fc_tidx, r->d_fc_tog, r->d_fc_mid, r->d_fc_len,
                    r->d_fc_t0, r->d_fc_cnt, r->d_fc_off, r->d_fc_t, r->d_fc_sa, r->d_fc_wcnt, r->d_st_t, r->d_st_sa};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (auto &pr : r->launch_events) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
}

// FNV-1a over a byte range (checkpoint parameter hash)
uint64_t fnv1a(uint64_t h, const void *data, size_t bytes) {
    const unsigned char *b = (const unsigned char *)data;
    for (size_t i = 0; i < bytes; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

bool district_contiguous(const fc::HostGraph &g, const int8_t *a, int k, std::vector<int32_t> &q,
                         std::vector<uint8_t> &seen) {
    std::fill(seen.begin(), seen.end(), 0);
    for (int d = 0; d < k; ++d) {
        int32_t start = -1, size = 0;
        for (int32_t u = 0; u < g.n; ++u)
            if (a[u] == d) { if (start < 0) start = u; ++size; }
        if (start < 0) continue;
        q.clear();
        q.push_back(start);
        seen[start] = 1;
        for (size_t h = 0; h < q.size(); ++h) {
            const int32_t u = q[h];
            for (int32_t j = g.row_ptr[u]; j < g.row_ptr[u + 1]; ++j) {
                const int32_t w = g.col_idx[j];
                if (a[w] == d && !seen[w]) { seen[w] = 1; q.push_back(w); }
            }
        }
        if ((int32_t)q.size() != size) return false;
    }
    return true;
}

template <int RMAX>
std::vector<fc::NodeRec<RMAX>> pack_records(const fc::HostGraph &g) {
    std::vector<fc::NodeRec<RMAX>> recs(g.n);
    for (int32_t v = 0; v < g.n; ++v) {
        auto &r = recs[v];
        std::memset(&r, 0, sizeof r);
        r.meta = g.meta[v];
        r.pop = g.pop[v];
        r.deg = g.row_ptr[v + 1] - g.row_ptr[v];
        for (int j = 0; j < RMAX; ++j) {
            const uint32_t x = (uint32_t)g.ring[(size_t)v * g.ring_max + j] & 0xffffu;
            r.ring[j >> 1] |= x << (16 * (j & 1));
        }
    }
    return recs;
}

}  // namespace

extern "C" {

const char *fc_last_error(void) { return g_err.c_str(); }

#ifndef FC_BUILD_ID
#define FC_BUILD_ID "unknown"
#endif
// the marker lets build.py read the id from the .so bytes without loading the library
static const char kBuildIdMarker[] = "FC_BUILD_ID=" FC_BUILD_ID;

const char *fc_build_id(void) { return kBuildIdMarker + 12; }

uint32_t fc_build_flags(void) {
    uint32_t f = 0;
#ifdef FC_PHASE_PROF
    f |= FC_BUILD_PHASE_PROF;
#endif
#ifdef FC_PHASE_SYNC
    f |= FC_BUILD_PHASE_SYNC;
#endif
#ifdef FC_VARIANT_BUILD
    f |= FC_BUILD_VARIANT;
#endif
    return f;
}

int fc_device_count(int32_t *n) {
    if (!n) return fail(FC_ERR_ARG, "fc_device_count: null output");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        return fail(FC_ERR_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *n = c;
    return FC_OK;
}

int fc_device_pci_id(int32_t device, char *buf, int32_t cap) {
    if (!buf || cap < 13) return fail(FC_ERR_ARG, "fc_device_pci_id: null buffer or cap < 13");
    HIP_TRY(hipDeviceGetPCIBusId(buf, cap, device));
    return FC_OK;
}

int fc_graph_create(int32_t n, const int32_t *row_ptr, const int32_t *col_idx, const int32_t *pop,
                    const double *pos_xy, uint32_t flags, fc_graph **out) {
    if (!out) return fail(FC_ERR_ARG, "fc_graph_create: null output");
    *out = nullptr;
    auto *g = new (std::nothrow) fc_graph();
    if (!g) return fail(FC_ERR_NOMEM, "fc_graph_create: out of memory");
    std::string err;
    try {
        err = fc::build_host_graph(n, row_ptr, col_idx, pop, pos_xy, flags, g->h);
    } catch (const std::exception &ex) {
        err = std::string("fc_graph_create: ") + ex.what();
    }
    if (!err.empty()) {
        delete g;
        return fail(err.rfind("graph: round-1", 0) == 0 ? FC_ERR_UNSUPPORTED : FC_ERR_ARG, err);
    }
    *out = g;
    return FC_OK;
}

int fc_graph_get_info(const fc_graph *g, fc_graph_info *out) {
    if (!g || !out) return fail(FC_ERR_ARG, "fc_graph_get_info: null argument");
    out->n_nodes = g->h.n;
    out->n_edges = g->h.n_edges;
    out->ring_max = g->h.ring_max;
    out->max_degree = g->h.max_degree;
    out->n_exact = g->h.n_exact;
    out->n_gamma = g->h.n_gamma;
    out->planar = g->h.planar ? 1 : 0;
    out->outer_simple = g->h.outer_simple ? 1 : 0;
    return FC_OK;
}

int fc_graph_edges(const fc_graph *g, int32_t *eu, int32_t *ev) {
    if (!g || !eu || !ev) return fail(FC_ERR_ARG, "fc_graph_edges: null argument");
    std::copy(g->h.eu.begin(), g->h.eu.end(), eu);
    std::copy(g->h.ev.begin(), g->h.ev.end(), ev);
    return FC_OK;
}

int fc_graph_rings(const fc_graph *g, int32_t *ring, uint64_t *meta) {
    if (!g || !ring || !meta) return fail(FC_ERR_ARG, "fc_graph_rings: null argument");
    std::copy(g->h.ring.begin(), g->h.ring.end(), ring);
    std::copy(g->h.meta.begin(), g->h.meta.end(), meta);
    return FC_OK;
}

void fc_graph_destroy(fc_graph *g) { delete g; }

int fc_params_init(fc_params *p, uint32_t struct_size) {
    if (!p) return fail(FC_ERR_ARG, "fc_params_init: null argument");
    if (struct_size != sizeof(fc_params))
        return fail(FC_ERR_ARG, "fc_params_init: struct_size " + std::to_string(struct_size) + " != sizeof(fc_params) " +
                                    std::to_string(sizeof(fc_params)) + " (the caller's flipchain.h is another version)");
    std::memset(p, 0, sizeof *p);
    p->struct_size = (uint32_t)sizeof(fc_params);
    p->abi_version = FC_ABI_VERSION;
    p->k = 2;
    p->base = 1.0;
    p->pop_lo = 0;
    p->pop_hi = INT32_MAX;
    p->hit_lo = 1;  // hitting-time window off (hit_lo > hit_hi)
    p->hit_hi = 0;
    return FC_OK;
}

int32_t fc_run_n_chains(const fc_run *r) { return r ? r->n_chains : 0; }

int32_t fc_run_chain_lds_bytes(const fc_run *r) { return r ? r->chain_lds_bytes : 0; }

int32_t fc_run_nb_width(const fc_run *r) { return r ? r->nb_w : 0; }

int fc_run_diag_paths(const fc_run *r, int64_t *tally_log_cap, int64_t *tally_log_wanted, int32_t *series_staged) {
    if (!r || !tally_log_cap || !tally_log_wanted || !series_staged) return fail(FC_ERR_ARG, "fc_run_diag_paths: null argument");
    *tally_log_cap = r->tl_cap;
    *tally_log_wanted = r->tl_want;
    *series_staged = r->series_staged;
    return FC_OK;
}

int fc_run_create(const fc_graph *gr, const fc_params *p, int32_t n_chains, const int8_t *init_assign,
                  const double *bases, fc_run **out) {
    if (!out) return fail(FC_ERR_ARG, "fc_run_create: null output");
    *out = nullptr;
    if (!gr || !p || !init_assign || n_chains <= 0) return fail(FC_ERR_ARG, "fc_run_create: null argument or n_chains <= 0");
    // the caller's fc_params layout must be this library's: nothing past struct_size is read
    if (p->struct_size != sizeof(fc_params) || p->abi_version != FC_ABI_VERSION)
        return fail(FC_ERR_ARG, "fc_run_create: fc_params.struct_size " + std::to_string(p->struct_size) +
                                    " / abi_version " + std::to_string(p->abi_version) + " do not match this library (" +
                                    std::to_string(sizeof(fc_params)) + " / " + std::to_string(FC_ABI_VERSION) +
                                    "): set them with fc_params_init or sizeof / FC_ABI_VERSION of the same flipchain.h");
    if (p->k < 2 || p->k > fc::kMaxKGeneral)
        return fail(FC_ERR_UNSUPPORTED, "fc_run_create: k must be in [2, 32]");
    if (p->proposal == FC_PROPOSE_BI_SIGN && p->k != 2)
        return fail(FC_ERR_ARG, "fc_run_create: slow_reversible_propose_bi flips between two districts (k == 2)");
    if (p->proposal != FC_PROPOSE_BI_SIGN && p->proposal != FC_PROPOSE_PAIR && p->proposal != FC_PROPOSE_RECOM)
        return fail(FC_ERR_UNSUPPORTED, "fc_run_create: unsupported proposal");
    const bool recom = p->proposal == FC_PROPOSE_RECOM;
    if (p->stream != FC_STREAM_NODE && p->stream != FC_STREAM_BAND)
        return fail(FC_ERR_ARG, "fc_run_create: stream must be FC_STREAM_NODE or FC_STREAM_BAND");
    if (p->stream == FC_STREAM_BAND && (p->k != 2 || recom || gr->h.n > 4096))
        return fail(FC_ERR_UNSUPPORTED, "fc_run_create: the band stream is for k = 2 flip runs on n <= 4096 nodes");
    if (recom) {
        if (p->accept != FC_ACCEPT_CUT || p->con_valid != 0 || p->con_accept != 0 || p->n_frozen > 0)
            return fail(FC_ERR_UNSUPPORTED, "fc_run_create: recom runs with the population Validator and cut_accept");
        if (!(p->recom_epsilon >= 0.0) || !(p->recom_pop_target > 0.0))
            return fail(FC_ERR_ARG, "fc_run_create: recom needs pop_target > 0 and epsilon >= 0");
        if (gr->h.n > 8000)
            return fail(FC_ERR_UNSUPPORTED, "fc_run_create: recom keeps a chain's spanning tree in LDS (n <= 8000)");
        if (bases)
            for (int32_t c = 1; c < n_chains; ++c)
                if (bases[c] != bases[0]) return fail(FC_ERR_UNSUPPORTED, "fc_run_create: recom takes one base");
    }
    const fc::HostGraph &g = gr->h;
    const int32_t n = g.n, E = g.n_edges, R = g.ring_max, k = p->k;
    // accept / constraint variants (uniform_accept, annealing_cut_accept_backwards,
    // boundary_condition, fixed_endpoints: grid_chain_sec11.py:39-52,81-110,159-165)
    const bool variant = p->accept != FC_ACCEPT_CUT || p->con_valid != 0 || p->con_accept != 0 || p->n_frozen > 0;
    const uint32_t con_valid = p->con_valid ? p->con_valid : (FC_CON_CONTIG | FC_CON_POP);
    const uint32_t con_all = FC_CON_CONTIG | FC_CON_POP | FC_CON_BOUNDARY | FC_CON_FIXED | FC_CON_EMPTY;
    if (variant) {
        if (k != 2) return fail(FC_ERR_UNSUPPORTED, "fc_run_create: accept / constraint variants need k == 2");
        if (p->accept < FC_ACCEPT_CUT || p->accept > FC_ACCEPT_ANNEAL)
            return fail(FC_ERR_ARG, "fc_run_create: unknown accept kind");
        if ((con_valid | p->con_accept) & ~con_all) return fail(FC_ERR_ARG, "fc_run_create: unknown constraint bits");
        if (!((con_valid | p->con_accept) & FC_CON_CONTIG))
            return fail(FC_ERR_UNSUPPORTED, "fc_run_create: single_flip_contiguous must be a Validator or accept "
                                            "constraint (the device keeps districts connected)");
        if (((con_valid | p->con_accept) & FC_CON_BOUNDARY) && g.n_gamma == 0)
            return fail(FC_ERR_UNSUPPORTED, "fc_run_create: boundary_condition needs a planar graph with a simple "
                                            "outer face (its nodes are the boundary set)");
        if (p->n_frozen < 0 || (p->n_frozen > 0 && !p->frozen)) return fail(FC_ERR_ARG, "fc_run_create: frozen nodes");
        for (int32_t i = 0; i < p->n_frozen; ++i)
            if (p->frozen[i] < 0 || p->frozen[i] >= n) return fail(FC_ERR_ARG, "fc_run_create: frozen node out of range");
    }
    // population bounds per chain (fc_params.chain_pop_bounds, else pop_lo / pop_hi for all)
    std::vector<int64_t> pop_bounds(2 * (size_t)n_chains);
    for (int32_t c = 0; c < n_chains; ++c) {
        pop_bounds[2 * (size_t)c] = p->chain_pop_bounds ? p->chain_pop_bounds[2 * (size_t)c] : p->pop_lo;
        pop_bounds[2 * (size_t)c + 1] = p->chain_pop_bounds ? p->chain_pop_bounds[2 * (size_t)c + 1] : p->pop_hi;
        for (int j = 0; j < 2; ++j)
            if (pop_bounds[2 * (size_t)c + j] > INT32_MAX || pop_bounds[2 * (size_t)c + j] < INT32_MIN)
                return fail(FC_ERR_UNSUPPORTED, "fc_run_create: population bounds must fit int32");
    }
    for (int64_t i = 0; i < (int64_t)n_chains * n; ++i)
        if (init_assign[i] < 0 || init_assign[i] >= k) return fail(FC_ERR_ARG, "fc_run_create: district id out of range");

    std::unique_ptr<fc_run, void (*)(fc_run *)> r(new (std::nothrow) fc_run(), free_run);
    if (!r) return fail(FC_ERR_NOMEM, "fc_run_create: out of memory");
    r->g = g;
    r->p = *p;
    r->labels.resize(k);
    for (int i = 0; i < k; ++i) r->labels[i] = p->labels ? p->labels[i] : i;
    r->p.labels = nullptr;
    // |b_nodes| as the driver's len(partition["b_nodes"]) counts it: nodes (b_nodes_bi, :155-156),
    // or with FC_FLAG_NB_PAIRS the (node, district) pairs of the pair updater b_nodes (:151-153)
    // a k > 2 driver registers for slow_reversible_propose (:117-130) -- at most
    // sum_u min(deg u, k - 1).  With k = 2 both counts are the same.
    const bool nb_pairs = (p->flags & FC_FLAG_NB_PAIRS) && k > 2;
    if ((p->flags & FC_FLAG_NB_PAIRS) && recom)
        return fail(FC_ERR_UNSUPPORTED, "fc_run_create: FC_FLAG_NB_PAIRS is for flip proposals");
    r->nb_w = n + 1;
    if (nb_pairs) {
        int64_t mx = 0;
        for (int32_t u = 0; u < n; ++u) mx += std::min<int64_t>(g.row_ptr[u + 1] - g.row_ptr[u], k - 1);
        if (mx > 65535)  // fc_event.nb is 16 bits
            return fail(FC_ERR_UNSUPPORTED, "fc_run_create: FC_FLAG_NB_PAIRS: more than 65535 possible pairs");
        r->nb_w = (int32_t)mx + 1;
    }
    const int32_t nbw = r->nb_w;
    r->log1mp.resize(nbw);
    if (p->log1mp) {
        std::copy(p->log1mp, p->log1mp + nbw, r->log1mp.begin());
    } else {
        const double denom = std::pow((double)n, (double)k) - 1.0;
        for (int32_t b = 0; b < nbw; ++b) r->log1mp[b] = std::log(1.0 - (double)b / denom);
    }
    r->p.log1mp = nullptr;
    r->p.frozen = nullptr;
    r->p.chain_pop_bounds = nullptr;
    r->p.con_valid = con_valid;
    r->variant = variant;
    r->n_chains = n_chains;
    r->npad = (n + 15) & ~15;
    r->words = (n + 63) / 64;
    if (g.max_degree > 16)  // dev::wave_bfs labels each old neighbour with a 4-bit id
        return fail(FC_ERR_UNSUPPORTED, "fc_run_create: node degree above 16");
    if (recom)   // fc_recom.hip: keys / tree CSR + parents / subtree populations, component /
                 // levels, order, tree-edge bits, a
        r->chain_lds_bytes = fc::recom_lds_bytes(n, g.ring_max);
    else if (k == 2)  // fc_flip2.hip: a, fcnt, thresholds, 3 BFS bitmaps, slots, commit marks (2 npad + 16),
                      // wait / tally queue (24 B per entry), launch start time, pace, first queued yield,
                      // tally-log length, launch's first yield (40) (sec11: 10,032 B, so 16 chains still
                      // fill a CU's 160 KB at the 1280-B allocation granule)
        r->chain_lds_bytes = 4 * r->npad + (2 * R + 2) * 8 + 24 * r->words + 5 * 64 * 4 + 16 + fc::kWaitQ * 24 + 40 +
                             (p->stream == FC_STREAM_BAND ? 8 * r->words : 0);  // the band bitmap (sec11: 200 B)
    // k > 2: with every node's ring exact (all bounded faces triangles / quadrilaterals, so the
    // rings list every face-adjacent cell) contiguity is decided by the district-graph rule
    // (fc_kernels.hip district_rule) instead of the device search, whose scratch is then not
    // allocated; FC_FLAG_FORCE_BFS keeps the search (cross-check)
    r->dgraph = !recom && k > 2 && k <= fc::kMaxKDistrictRule && g.n_exact == n && g.planar && g.outer_simple &&
                !(p->flags & FC_FLAG_FORCE_BFS);
    if (!recom && k > 2)  // fc_kernels.hip: a, fcnt (one packed byte per node with the district-graph
                          // rule), thresholds, [BFS scratch | district tables], slots, district
                          // populations, wait queue; the multi-flip commit's hashed marks (last)
                          // only when it is on, so an "off" run keeps its residency
    {
        const int base_b = (r->dgraph ? 1 : 2) * r->npad + (2 * R + 2) * 8 +
                           (r->dgraph ? fc::dgraph_lds_bytes(k) : fc::bfs_bytes(n)) + 5 * 64 * 4 +
                           fc::kMaxKGeneral * 4 + fc::kNfh * 4 + fc::kWaitQK * 16;
        // chains per CU the LDS holds (granule 1280 B per one-wave workgroup, measured: DESIGN.md
        // §4), capped by the 16 waves the k > 2 instances' registers allow
        auto per_cu = [](int b) { return std::min(16, 160 * 1024 / (((b + 15) / 16 * 16 + 1279) / 1280 * 1280)); };
        const int mf = p->tune_multi_flip;
        r->mf_marks = 0;
        // FC_FLAG_NB_PAIRS runs take the one-flip-at-a-time commit: the multi-flip pass counts
        // |B| as nodes only (its pair count would cost the C5 instance the register that keeps
        // three waves per SIMD)
        if (!recom && k > 2 && r->dgraph && mf != -1 && !nb_pairs) {
            // exact marks (a byte per node) when they cost no residency, else the hashed set
            const bool fits = per_cu(base_b + r->npad) >= per_cu(base_b + fc::hb_bytes(R));
            r->mf_marks = mf == 2 ? 1 : mf == 3 ? 2 : (fits ? 2 : 1);
        }
        if (!recom && k > 2)  // (k = 2 above)
            r->chain_lds_bytes = base_b + (r->mf_marks == 2 ? r->npad : r->mf_marks == 1 ? fc::hb_bytes(R) : 0);
    }
    // PAIR slot bound: fc_params.wmax > 0 fixes it; otherwise the canonical stream's bound is
    // the state's largest foreign-district count (kept on the device, r->wmax = 0)
    r->wmax = 1;
    if (k > 2) r->wmax = p->wmax > 0 ? p->wmax : 0;
    if (k > 2 && p->wmax > 0 && p->wmax < std::min(g.max_degree, k - 1))  // would skew the proposal
        return fail(FC_ERR_ARG, "fc_run_create: a fixed PAIR slot bound (wmax) must be >= min(max degree, k - 1) = " +
                                    std::to_string(std::min(g.max_degree, k - 1)) + " (<= 0: the canonical dynamic bound)");
#ifdef FC_PHASE_PROF
    r->chain_lds_bytes += fc::kProfSlots * 8;  // phase-cycle accumulators (diagnostic build)
#endif
    r->chain_lds_bytes = (r->chain_lds_bytes + 15) & ~15;
    if ((size_t)r->chain_lds_bytes * fc::waves_per_block(r->chain_lds_bytes) > 160 * 1024)
        return fail(FC_ERR_UNSUPPORTED, "fc_run_create: graph too large for the wave-per-chain LDS layout");

    // ---- launch tuning (scheduling only; 0 = default) --------------------------------------
    // k = 2 node stream: a window of up to 64 * nsub = 256 draws per batch (the four node words
    // of one Philox call per lane), closed by the 64th boundary hit -- no round cut-off (the band
    // stream keeps rounds of 64 with the hit_stop cut-off).  Before round 4, C2 sweeps on one MI355X, ms per launch: before stale slots were re-evaluated
    // in place, 2 rounds / 32 hits 10.7, 4 / 12 10.3 (4 / 8 10.55, 4 / 24 10.8); with the
    // re-evaluation, 4 / 12 9.33, 4 / 20..64 8.9-9.0, 2 / 32 10.3, 8 / 32..64 9.45-9.55
    {
        auto &t = r->tune;
        // k > 2 (one MI355X, 2000-step launches): C3 (wmax 3) 1.80 / 2.14 / 2.09e9 proposals/s with
        // 1 / 2 / 4 rounds, C4 (wmax 6) 6.6 / 7.9 / 7.6e8, C5 (wmax 16, ~39 draws per
        // proposal) 3.0 / 4.1 / 4.8e8
        const int wmax_k = k > 2 ? (p->wmax > 0 ? p->wmax : std::max(1, std::min(g.max_degree, k - 1))) : 1;
        t.nsub = p->tune_nsub ? p->tune_nsub : (k == 2 ? 4 : wmax_k > 8 ? 4 : 2);
        if (!recom && !(t.nsub == 1 || t.nsub == 2 || t.nsub == 4))
            return fail(FC_ERR_ARG, std::string("fc_run_create: tune_nsub must be 1, 2 or 4 for the ") +
                                        (k == 2 ? "k = 2" : "k > 2") + " kernel (got " + std::to_string(t.nsub) + ")");
        // the round cut-off applies to the k > 2 rounds and the k = 2 band stream; the k = 2 node
        // stream takes a window of 64 * nsub draws (four node words per lane's Philox call)
        // closed by the 64th hit, so a cut-off there would silently change nothing
        if (k == 2 && !recom && p->stream == FC_STREAM_NODE && p->tune_hit_stop != 0)
            return fail(FC_ERR_ARG, "fc_run_create: tune_hit_stop has no effect on the k = 2 node stream (its batch window "
                                    "is 64 * tune_nsub draws, closed by the 64th boundary hit); leave it 0");
        t.hit_stop = p->tune_hit_stop ? p->tune_hit_stop : 32;
        if (t.hit_stop < 1) return fail(FC_ERR_ARG, "fc_run_create: tune_hit_stop must be >= 1");
        t.par_min = p->tune_par_min ? p->tune_par_min : 3;
        if (t.par_min < 1) return fail(FC_ERR_ARG, "fc_run_create: tune_par_min must be >= 1");
        // k > 2 with the district-graph rule: commit several independent flips per pass (64 /
        // RMAX of them).  Auto (0) = on (C4 +32 %, C3 +3.5 %)
        if (p->tune_multi_flip < -1 || p->tune_multi_flip > 3)
            return fail(FC_ERR_ARG, "fc_run_create: tune_multi_flip must be 0 (auto), 1 (on), -1 (off), 2 (on, hashed "
                                    "marks) or 3 (on, exact marks)");
        t.multi = p->tune_multi_flip != -1;
        const int qmax = k == 2 ? fc::kWaitQ : fc::kWaitQK;
        t.wait_q = p->tune_wait_queue ? p->tune_wait_queue : qmax;
        if (t.wait_q < 1 || t.wait_q > qmax)
            return fail(FC_ERR_ARG, "fc_run_create: tune_wait_queue must be in [1, " + std::to_string(qmax) + "]");
        t.wpb = p->tune_chains_per_block ? p->tune_chains_per_block : 1;
        if (t.wpb != 1 && t.wpb != 2 && t.wpb != 4)
            return fail(FC_ERR_ARG, "fc_run_create: tune_chains_per_block must be 1, 2 or 4");
        t.wpb = std::min(t.wpb, fc::waves_per_block(r->chain_lds_bytes));
        // large k > 2 chains that need the search: 4 = one chain per 256-thread workgroup,
        // searched by all of it.  Default 1: the workgroup's helper waves carry the kernel's
        // VGPR count, so a chain then holds four waves' registers and fewer chains are
        // resident, and these searches are short (≈ 2 levels from the C4 / C5 start plans):
        // C4 forced search 5.7 ms (1 wave) against 7.3 ms (workgroup), C5 7.9 against 16.8,
        // C5 without positions 11.7 against 28.1 (1024 chains x 1000 steps, one MI355X)
        const int sw = p->tune_search_waves ? p->tune_search_waves : 1;
        if (sw != 1 && sw != 4) return fail(FC_ERR_ARG, "fc_run_create: tune_search_waves must be 1 or 4");
        t.coop = !recom && k > 2 && !r->dgraph && r->chain_lds_bytes > fc::kBigChainLds && sw == 4;
        if (t.coop) r->chain_lds_bytes += 32 * 4;  // control words of the cooperative search
        // k = 2: chains with a short boundary need many draws per proposal and set the launch
        // time; they get the SIMD's issue priority over the chains sharing it (s_setprio 1/2/3
        // below |B| = n/2, n/5, n/10); once a chain has taken 1/16 of its steps, its projected
        // finish against the previous launch's slowest chain sets the priority instead
        const bool div_default = !p->tune_prio_div[0] && !p->tune_prio_div[1] && !p->tune_prio_div[2];
        for (int i = 0; i < 3; ++i) t.prio_div[i] = div_default ? (i == 0 ? 2 : i == 1 ? 5 : 10) : p->tune_prio_div[i];
        if (t.prio_div[0] > 0 && (t.prio_div[1] <= 0 || t.prio_div[2] <= 0))
            return fail(FC_ERR_ARG, "fc_run_create: tune_prio_div needs three positive divisors (or [0] < 0: off)");
        // k = 2: deal chains to SIMDs by the previous launch's draws (fc_deal.hip).  Off by
        // default: C2's dispatch order already gives every SIMD one or two of its slow chains
        // (chain dealing)
        t.deal = p->tune_deal ? p->tune_deal : -1;
        if (t.deal != 1 && t.deal != -1) return fail(FC_ERR_ARG, "fc_run_create: tune_deal must be 1 or -1");
        t.deal = t.deal > 0 && k == 2 && !recom;
        const bool th_default = p->tune_prio_th[0] == 0.0f && p->tune_prio_th[1] == 0.0f && p->tune_prio_th[2] == 0.0f;
        const float th0[3] = {0.95f, 1.0f, 1.05f};  // tools/archive/gpu_knobs_r04.sh: 55.3 against 55.8 ms at {0.9, 1.0, 1.1}
        for (int i = 0; i < 3; ++i) t.prio_th[i] = th_default ? th0[i] : p->tune_prio_th[i];
    }

    // ---- host-side initial state (validated like MarkovChain.__init__ [gc-0.2]) ---------
    std::vector<int8_t> assign((size_t)n_chains * r->npad, 0);
    std::vector<uint8_t> fcnt((size_t)n_chains * r->npad, 0);
    std::vector<fc::ChainScalars> sc(n_chains);
    std::vector<int32_t> popk((size_t)n_chains * fc::kMaxKGeneral, 0);
    std::vector<int32_t> nfh(k > 2 && !recom ? (size_t)n_chains * fc::kNfh : 0, 0);
    const bool band = p->stream == FC_STREAM_BAND;
    std::vector<uint64_t> sbits(band ? (size_t)n_chains * r->words : 0, 0);
    std::vector<int32_t> mcnt(r->dgraph ? (size_t)n_chains * k * k : 0, 0), ngk(r->dgraph ? (size_t)n_chains * 32 : 0, 0);
    std::vector<uint64_t> thresh((size_t)n_chains * (2 * R + 1));
    std::vector<int32_t> q;
    std::vector<uint8_t> seen(n);
    const bool want_hist = p->diag_mask & FC_DIAG_HIST, want_edges = p->diag_mask & FC_DIAG_EDGES,
               want_flips = p->diag_mask & FC_DIAG_FLIPS;
    std::vector<int64_t> cut_hist, nb_hist, part_sum;
    if (want_hist) { cut_hist.assign((size_t)n_chains * (E + 1), 0); nb_hist.assign((size_t)n_chains * nbw, 0); }
    if (want_flips) part_sum.assign((size_t)n_chains * n, 0);
    for (int32_t c = 0; c < n_chains; ++c) {
        const int8_t *a = init_assign + (size_t)c * n;
        std::memcpy(&assign[(size_t)c * r->npad], a, n);
        int64_t pops[fc::kMaxKGeneral] = {0};
        int32_t ng[fc::kMaxKGeneral] = {0};
        for (int32_t u = 0; u < n; ++u) {
            if (a[u] < 0 || a[u] >= k)
                return fail(FC_ERR_ARG, "chain " + std::to_string(c) + ": district id out of range [0, k)");
            pops[a[u]] += g.pop[u];
            if (g.meta[u] & fc::kMetaGamma) ng[a[u]] += 1;
        }
        if (con_valid & FC_CON_POP)
            for (int d = 0; d < k; ++d)
                if (pops[d] < pop_bounds[2 * (size_t)c] || pops[d] > pop_bounds[2 * (size_t)c + 1])
                    return fail(FC_ERR_INVALID_STATE, "chain " + std::to_string(c) +
                                                          ": The given initial_state is not valid according is_valid (population).");
        if ((con_valid & FC_CON_BOUNDARY) && (ng[0] == 0 || ng[1] == 0))
            return fail(FC_ERR_INVALID_STATE, "chain " + std::to_string(c) +
                                                  ": The given initial_state is not valid according is_valid (boundary_condition).");
        if (!district_contiguous(g, a, k, q, seen))
            return fail(FC_ERR_INVALID_STATE, "chain " + std::to_string(c) +
                                                  ": The given initial_state is not valid according is_valid (contiguity).");
        int32_t cut = 0, nb = 0;
        for (int32_t e = 0; e < E; ++e) cut += a[g.eu[e]] != a[g.ev[e]];
        for (int32_t u = 0; u < n; ++u) {
            // k = 2: foreign neighbours; k > 2: foreign districts nf(u) (the PAIR slot count)
            int32_t f = 0;
            uint32_t dm = 0;
            for (int32_t j = g.row_ptr[u]; j < g.row_ptr[u + 1]; ++j) {
                f += a[g.col_idx[j]] != a[u];
                if (a[g.col_idx[j]] != a[u]) dm |= 1u << a[g.col_idx[j]];
            }
            if (k > 2 && !recom) {
                f = __builtin_popcount(dm);
                nfh[(size_t)c * fc::kNfh + f] += 1;
            }
            fcnt[(size_t)c * r->npad + u] = (uint8_t)f;
            nb += nb_pairs ? f : f > 0;
        }
        if (band) {  // the band S of the initial state: b_nodes and their neighbours
            uint64_t *sb = &sbits[(size_t)c * r->words];
            for (int32_t u = 0; u < n; ++u) {
                if (!fcnt[(size_t)c * r->npad + u]) continue;
                sb[u >> 6] |= 1ull << (u & 63);
                for (int32_t j = g.row_ptr[u]; j < g.row_ptr[u + 1]; ++j) sb[g.col_idx[j] >> 6] |= 1ull << (g.col_idx[j] & 63);
            }
        }
        fc::ChainScalars &s = sc[c];
        std::memset(&s, 0, sizeof s);
        s.cut = cut;
        s.nb = nb;
        s.pops[0] = (int32_t)pops[0];
        s.pops[1] = (int32_t)pops[1];
        for (int d = 0; d < fc::kMaxKGeneral; ++d) popk[(size_t)c * fc::kMaxKGeneral + d] = (int32_t)pops[d];
        if (r->dgraph) {
            // face-adjacent cell pairs {u, w} (w in ring(u), counted once: u < w) per district pair
            int32_t *mc = &mcnt[(size_t)c * k * k];
            for (int32_t u = 0; u < n; ++u) {
                const int32_t L = (int32_t)(g.meta[u] & fc::kMetaLenMask);
                for (int32_t j = 0; j < L; ++j) {
                    const int32_t w = g.ring[(size_t)u * R + j];
                    if (w <= u || a[w] == a[u]) continue;
                    const int32_t X = std::min(a[u], a[w]), Y = std::max(a[u], a[w]);
                    ++mc[X * k + Y];
                }
            }
            for (int d = 0; d < k; ++d) ngk[(size_t)c * 32 + d] = ng[d];
        }
        s.ngamma[0] = ng[0];
        s.ngamma[1] = ng[1];
        s.last_flip = -1;
        s.pop_lo = (int32_t)pop_bounds[2 * (size_t)c];
        s.pop_hi = (int32_t)pop_bounds[2 * (size_t)c + 1];
        int64_t wait0 = 0;
        if (p->diag_mask & FC_DIAG_WAIT) {
            const uint32_t gid = p->chain_id_offset + (uint32_t)c;
            fc::Words4 w = fc::philox4x32_10(0u, 0u, gid, 2u, (uint32_t)p->seed, (uint32_t)(p->seed >> 32));
            wait0 = fc::geom_from(fc::u53(w.x0, w.x1), r->log1mp[nb]);
        }
        s.wait_cur = wait0;
        s.hit_time = (cut >= p->hit_lo && cut <= p->hit_hi) ? 0 : -1;
        s.ser_t0 = 0;
        s.ser_cut0 = cut;
        s.ser_nb0 = nb;
        // yield #0 (the initial state) enters every per-yield sum
        s.sum_cut = cut;
        s.sum_nb = nb;
        s.sum_cut2 = (int64_t)cut * cut;
        s.sum_nb2 = (int64_t)nb * nb;
        s.sum_wait = wait0;
        if (want_hist) {
            cut_hist[(size_t)c * (E + 1) + cut] = 1;
            nb_hist[(size_t)c * nbw + nb] = 1;
        }
        if (want_flips)
            for (int32_t u = 0; u < n; ++u) part_sum[(size_t)c * n + u] = r->labels[a[u]];  // :219
        const double base = bases ? bases[c] : p->base;
        for (int dd = -R; dd <= R; ++dd) {
            if (p->accept == FC_ACCEPT_ANNEAL) {
                // annealing_cut_accept_backwards, :99: base ** (beta * (-(cut' - cut))); the
                // |B'| / |B| factor is applied on the device (the table holds the double)
                const double bw = std::pow(base, p->beta * (double)(-dd));
                uint64_t t;
                std::memcpy(&t, &bw, 8);
                thresh[(size_t)c * (2 * R + 1) + (dd + R)] = t;
                continue;
            }
            // cut_accept: random() < base ** (-(cut' - cut)), grid_chain_sec11.py:175,179
            const double bound = std::pow(base, (double)(-dd));
            uint64_t t;
            if (!(bound < 1.0)) t = 1ull << 53;                     // always accepted
            else if (!(bound > 0.0)) t = 0;
            else t = (uint64_t)std::ceil(bound * 9007199254740992.0);
            thresh[(size_t)c * (2 * R + 1) + (dd + R)] = t;
        }
    }

    // every parameter a trajectory depends on besides seed / chain ids, for fc_run_restore
    {
        uint64_t h = 0xcbf29ce484222325ull;
        h = fnv1a(h, thresh.data(), thresh.size() * 8);
        h = fnv1a(h, pop_bounds.data(), pop_bounds.size() * 8);
        h = fnv1a(h, r->labels.data(), r->labels.size() * 4);
        h = fnv1a(h, r->log1mp.data(), r->log1mp.size() * 8);
        const int64_t scal[] = {k, p->proposal, p->accept, (int64_t)con_valid, (int64_t)p->con_accept, p->flags,
                                r->wmax, p->hit_lo, p->hit_hi, p->recom_node_repeats, p->recom_max_attempts,
                                p->stream};
        h = fnv1a(h, scal, sizeof scal);
        const double dscal[] = {p->beta, p->recom_pop_target, p->recom_epsilon, bases ? bases[0] : p->base};
        h = fnv1a(h, dscal, sizeof dscal);
        if (p->n_frozen > 0) h = fnv1a(h, p->frozen, (size_t)p->n_frozen * 4);
        r->param_hash = h;
    }

    // ---- device ---------------------------------------------------------------------------
    HIP_TRY(hipSetDevice(p->device));
    HIP_TRY(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
    int rc;
    if (R == 8) {
        auto recs = pack_records<8>(g);
        for (int32_t i = 0; i < p->n_frozen; ++i) recs[p->frozen[i]].meta |= fc::kMetaFrozen;
        if ((rc = dalloc((fc::NodeRec<8> **)&r->d_graph, recs.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_graph, recs.data(), recs.size() * sizeof(recs[0]), hipMemcpyHostToDevice));
    } else {
        auto recs = pack_records<16>(g);
        for (int32_t i = 0; i < p->n_frozen; ++i) recs[p->frozen[i]].meta |= fc::kMetaFrozen;
        if ((rc = dalloc((fc::NodeRec<16> **)&r->d_graph, recs.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_graph, recs.data(), recs.size() * sizeof(recs[0]), hipMemcpyHostToDevice));
    }
    if ((rc = dalloc(&r->d_ring_eid, g.ring_eid.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_ring_eid, g.ring_eid.data(), g.ring_eid.size() * 4, hipMemcpyHostToDevice));
    if ((rc = dalloc(&r->d_assign, assign.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_assign, assign.data(), assign.size(), hipMemcpyHostToDevice));
    if ((rc = dalloc(&r->d_fcnt, fcnt.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_fcnt, fcnt.data(), fcnt.size(), hipMemcpyHostToDevice));
    if ((rc = dalloc(&r->d_popk, popk.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_popk, popk.data(), popk.size() * 4, hipMemcpyHostToDevice));
    if (band) {
        if ((rc = dalloc(&r->d_sbits, sbits.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_sbits, sbits.data(), sbits.size() * 8, hipMemcpyHostToDevice));
    }
    if (!nfh.empty()) {
        if ((rc = dalloc(&r->d_nfh, nfh.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_nfh, nfh.data(), nfh.size() * 4, hipMemcpyHostToDevice));
    }
    if (r->dgraph) {
        if ((rc = dalloc(&r->d_mcnt, mcnt.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_mcnt, mcnt.data(), mcnt.size() * 4, hipMemcpyHostToDevice));
        if ((rc = dalloc(&r->d_ngk, ngk.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_ngk, ngk.data(), ngk.size() * 4, hipMemcpyHostToDevice));
    }
    if ((rc = dalloc(&r->d_sc, sc.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_sc, sc.data(), sc.size() * sizeof(sc[0]), hipMemcpyHostToDevice));
    if ((rc = dalloc(&r->d_thresh, thresh.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_thresh, thresh.data(), thresh.size() * 8, hipMemcpyHostToDevice));
    if ((rc = dalloc(&r->d_log1mp, r->log1mp.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_log1mp, r->log1mp.data(), r->log1mp.size() * 8, hipMemcpyHostToDevice));
    if ((rc = dalloc(&r->d_labels, r->labels.size()))) return rc;
    HIP_TRY(hipMemcpy(r->d_labels, r->labels.data(), r->labels.size() * 4, hipMemcpyHostToDevice));
    if (want_hist) {
        if ((rc = dalloc(&r->d_cut_hist, cut_hist.size()))) return rc;
        if ((rc = dalloc(&r->d_nb_hist, nb_hist.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_cut_hist, cut_hist.data(), cut_hist.size() * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(r->d_nb_hist, nb_hist.data(), nb_hist.size() * 8, hipMemcpyHostToDevice));
    }
    if (want_edges) {
        if ((rc = dalloc(&r->d_edge_acc, (size_t)n_chains * E))) return rc;
        HIP_TRY(hipMemset(r->d_edge_acc, 0, (size_t)n_chains * E * 8));
    }
    if (want_flips) {
        if ((rc = dalloc(&r->d_num_flips, (size_t)n_chains * n))) return rc;
        if ((rc = dalloc(&r->d_part_sum, (size_t)n_chains * n))) return rc;
        if ((rc = dalloc(&r->d_last_flipped, (size_t)n_chains * n))) return rc;
        HIP_TRY(hipMemset(r->d_num_flips, 0, (size_t)n_chains * n * 8));
        HIP_TRY(hipMemset(r->d_last_flipped, 0, (size_t)n_chains * n * 8));
        HIP_TRY(hipMemcpy(r->d_part_sum, part_sum.data(), part_sum.size() * 8, hipMemcpyHostToDevice));
    }
    if (p->diag_mask & FC_DIAG_FLIPS_EXACT) {
        if (recom) return fail(FC_ERR_UNSUPPORTED, "fc_run_create: FC_DIAG_FLIPS_EXACT is kept by the flip kernels, not ReCom");
        for (int64_t **b : {&r->d_flip_count, &r->d_occ_acc, &r->d_last_accept}) {
            if ((rc = dalloc(b, (size_t)n_chains * n))) return rc;
            HIP_TRY(hipMemset(*b, 0, (size_t)n_chains * n * 8));
        }
    }
    if ((p->diag_mask & FC_DIAG_SERIES) && p->event_cap > 0) {
        if (E > 65535) return fail(FC_ERR_UNSUPPORTED, "fc_run_create: FC_DIAG_SERIES stores |cut| in 16 bits (E <= 65535)");
        r->ev_cap = p->event_cap;
        if ((rc = dalloc(&r->d_events, (size_t)n_chains * (size_t)p->event_cap))) return rc;
        if ((rc = dalloc(&r->d_ser_a0, assign.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_ser_a0, r->d_assign, assign.size(), hipMemcpyDeviceToDevice));
    } else {
        r->p.diag_mask &= ~FC_DIAG_SERIES;
    }
    if (recom) {
        if ((rc = dalloc(&r->d_eu, (size_t)std::max(E, 1)))) return rc;
        if ((rc = dalloc(&r->d_ev, (size_t)std::max(E, 1)))) return rc;
        if (E) {
            HIP_TRY(hipMemcpy(r->d_eu, g.eu.data(), (size_t)E * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(r->d_ev, g.ev.data(), (size_t)E * 4, hipMemcpyHostToDevice));
        }
        // the neighbours of each node in ring order with their edge ids (node ids and edge ids
        // < 65535: n <= 8000, degree <= 16), and each edge end's index in the other end's row:
        // the spanning-tree scan reads one row per node instead of its ring and ring edge ids
        {
            const int R = g.ring_max;
            r->nb_d = std::max(4, (g.max_degree + 3) / 4 * 4);
            std::vector<uint32_t> nbe((size_t)n * r->nb_d, ~0u), es((size_t)std::max(E, 1), 0u);
            for (int32_t x = 0; x < n; ++x) {
                int k = 0;
                for (int j = 0; j < R; ++j) {
                    const int32_t e = g.ring_eid[(size_t)x * R + j];
                    if (e < 0) continue;
                    nbe[(size_t)x * r->nb_d + k] = (uint32_t)g.ring[(size_t)x * R + j] | ((uint32_t)e << 16);
                    es[e] |= (uint32_t)k << (g.eu[e] == x ? 0 : 8);
                    ++k;
                }
            }
            if ((rc = dalloc(&r->d_nbe, nbe.size()))) return rc;
            if ((rc = dalloc(&r->d_eslot, es.size()))) return rc;
            HIP_TRY(hipMemcpy(r->d_nbe, nbe.data(), nbe.size() * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(r->d_eslot, es.data(), es.size() * 4, hipMemcpyHostToDevice));
        }
        // cut_accept: random() < base ** (cut - cut'), cut - cut' in [-E, E]
        const double rb = bases ? bases[0] : p->base;
        std::vector<uint64_t> th(2 * (size_t)E + 1);
        for (int32_t dd = -E; dd <= E; ++dd) {
            const double bound = std::pow(rb, (double)dd);
            th[dd + E] = !(bound < 1.0) ? (1ull << 53) : !(bound > 0.0) ? 0 : (uint64_t)std::ceil(bound * 9007199254740992.0);
        }
        if ((rc = dalloc(&r->d_recom_thresh, th.size()))) return rc;
        HIP_TRY(hipMemcpy(r->d_recom_thresh, th.data(), th.size() * 8, hipMemcpyHostToDevice));
    }
    if (p->trace_chains > 0 && p->trace_cap > 0) {
        const int32_t tc = std::min(p->trace_chains, n_chains);
        r->p.trace_chains = tc;
        if ((rc = dalloc(&r->d_trace, (size_t)tc * p->trace_cap))) return rc;
    } else {
        r->p.trace_chains = 0;
    }
    HIP_TRY(hipDeviceSynchronize());
    *out = r.release();
    return FC_OK;
}

int fc_run_set_tape(fc_run *r, const uint32_t *tape, int64_t n_draws) {
    if (!r) return fail(FC_ERR_ARG, "fc_run_set_tape: null run");
    if (r->d_sbits && tape && n_draws > 0)  // a tape's word 0 is a node of all n (the node-tape map)
        return fail(FC_ERR_ARG, "fc_run_set_tape: replay tapes need the node stream (FC_STREAM_NODE)");
    HIP_TRY(hipSetDevice(r->p.device));
    if (r->d_tape) { HIP_TRY(hipFree(r->d_tape)); r->d_tape = nullptr; }
    r->tape_draws = 0;
    if (!tape || n_draws <= 0) return FC_OK;
    const size_t words = (size_t)r->n_chains * (size_t)n_draws * 6;
    int rc;
    if ((rc = dalloc(&r->d_tape, words))) return rc;
    HIP_TRY(hipMemcpy(r->d_tape, tape, words * 4, hipMemcpyHostToDevice));
    r->tape_draws = n_draws;
    return FC_OK;
}

int fc_run_set_initial_wait(fc_run *r, const uint32_t *words) {
    if (!r || !words) return fail(FC_ERR_ARG, "fc_run_set_initial_wait: null argument");
    if (!(r->p.diag_mask & FC_DIAG_WAIT)) return fail(FC_ERR_ARG, "fc_run_set_initial_wait: FC_DIAG_WAIT is off");
    if (r->p.proposal == FC_PROPOSE_RECOM) return fail(FC_ERR_UNSUPPORTED, "fc_run_set_initial_wait: flip runs only");
    if (int rc = fc_run_sync(r)) return rc;
    std::vector<fc::ChainScalars> sc(r->n_chains);
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    for (const auto &s : sc)
        if (s.steps != 0 || s.draw != 0) return fail(FC_ERR_ARG, "fc_run_set_initial_wait: a chain has stepped");
    for (int32_t c = 0; c < r->n_chains; ++c) {
        fc::ChainScalars &s = sc[c];
        const int64_t w = fc::geom_from(fc::u53(words[2 * c], words[2 * c + 1]), r->log1mp[s.nb]);
        s.sum_wait += w - s.wait_cur;  // yield #0's term
        s.wait_cur = w;
    }
    HIP_TRY(hipMemcpy(r->d_sc, sc.data(), sc.size() * sizeof(sc[0]), hipMemcpyHostToDevice));
    return FC_OK;
}

#ifdef FC_PHASE_PROF
// diagnostic build: the launch's per-chain phase cycles appended to $FC_PROF_OUT
static int dump_prof(fc_run *r, hipStream_t s) {
    if (const char *path = std::getenv("FC_PROF_OUT")) {
        std::vector<int64_t> h((size_t)r->n_chains * fc::kProfSlots);
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(hipMemcpy(h.data(), r->d_prof, h.size() * 8, hipMemcpyDeviceToHost));
        if (FILE *f = std::fopen(path, "ab")) {
            std::fwrite(h.data(), 8, h.size(), f);
            std::fclose(f);
        }
    }
    return FC_OK;
}
#endif

int fc_run_steps(fc_run *r, int64_t n_steps, int64_t max_draws, void *hip_stream) {
    if (!r) return fail(FC_ERR_ARG, "fc_run_steps: null run");
    if (n_steps < 0) return fail(FC_ERR_ARG, "fc_run_steps: n_steps must be >= 0");
    if (n_steps == 0) return FC_OK;
    HIP_TRY(hipSetDevice(r->p.device));
    fc::KParams k{};
    k.graph = r->d_graph;
    k.ring_eid = r->d_ring_eid;
    k.n = r->g.n;
    k.n_edges = r->g.n_edges;
    k.n_chains = r->n_chains;
    k.k = r->p.k;
    k.popk = r->d_popk;
    k.all_exact = r->g.n_exact == r->g.n ? 1 : 0;
    k.dgraph = r->dgraph ? 1 : 0;
    k.mcnt = r->d_mcnt;
    k.ngk = r->d_ngk;
    k.wmax = r->wmax > 0 ? r->wmax : 1;
    k.wdyn = r->p.k > 2 && r->wmax <= 0 ? 1 : 0;
    k.nfh = r->d_nfh;
    k.band = r->d_sbits ? 1 : 0;
    k.sbits = r->d_sbits;
    k.band_step0 = 1;
    while (k.band_step0 * 2 < r->words) k.band_step0 *= 2;
    k.chain_lds_bytes = r->chain_lds_bytes;
    k.words = r->words;
    k.lab_words = fc::bfs_lab_words(r->g.n);
    k.lemire_thresh = (uint32_t)((1ull << 32) % (uint64_t)r->g.n);
    k.chain_id_offset = r->p.chain_id_offset;
    k.seed_lo = (uint32_t)r->p.seed;
    k.seed_hi = (uint32_t)(r->p.seed >> 32);
    k.pop_lo = (int32_t)r->p.pop_lo;
    k.pop_hi = (int32_t)r->p.pop_hi;
    k.n_steps = n_steps;
    k.max_draws = max_draws > 0 ? max_draws : 65536 * std::max<int64_t>(n_steps, 1);
    k.assign = r->d_assign;
    k.fcnt = r->d_fcnt;
    k.sc = r->d_sc;
    k.thresh = r->d_thresh;
    k.log1mp = r->d_log1mp;
    k.labels = r->d_labels;
    k.diag = r->p.diag_mask;
    k.flags = r->p.flags;
    k.cut_hist = r->d_cut_hist;
    k.nb_hist = r->d_nb_hist;
    k.nb_w = r->nb_w;
    k.nb_pairs = (r->p.flags & FC_FLAG_NB_PAIRS) && r->p.k > 2;
    k.edge_acc = r->d_edge_acc;
    k.num_flips = r->d_num_flips;
    k.part_sum = r->d_part_sum;
    k.last_flipped = r->d_last_flipped;
    k.flip_count = r->d_flip_count;
    k.occ_acc = r->d_occ_acc;
    k.last_accept = r->d_last_accept;
    k.trace = r->d_trace;
    k.trace_chains = r->p.trace_chains;
    k.trace_cap = r->p.trace_cap;
    k.tape = r->d_tape;
    k.tape_draws = r->tape_draws;
    k.events = r->d_events;
    k.ev_cap = r->ev_cap;
    k.hit_lo = r->p.hit_lo;
    k.hit_hi = r->p.hit_hi;
    // launch tuning (fc_params.tune_*, resolved and checked by fc_run_create; scheduling only)
    k.nsub = r->tune.nsub;
    k.hit_stop = r->tune.hit_stop;
    k.par_min = r->tune.par_min;
    k.multi_flip = r->tune.multi ? r->mf_marks : 0;
    k.wait_q = r->tune.wait_q;
    k.wpb = r->tune.wpb;
    k.coop = r->tune.coop ? 1 : 0;
    k.variant = r->variant ? 1 : 0;
    k.accept = r->p.accept;
    k.con_valid = r->p.con_valid;
    k.con_accept = r->p.con_accept;
    if (r->variant) k.par_min = kWaveSlots + 1;  // variants commit one event at a time
    for (int i = 0; i < 3; ++i) {
        k.prio_nb[i] = r->tune.prio_div[0] > 0 && r->p.k == 2 ? k.n / r->tune.prio_div[i] : 0;
        k.prio_th[i] = r->tune.prio_th[i];
    }
    k.eta = nullptr;
    k.eta_parity = 0;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : r->stream;
    k.prof = nullptr;
#ifdef FC_PHASE_PROF
    if (!r->d_prof) {
        if (int rc = dalloc(&r->d_prof, (size_t)r->n_chains * fc::kProfSlots)) return rc;
    }
    HIP_TRY(hipMemsetAsync(r->d_prof, 0, (size_t)r->n_chains * fc::kProfSlots * 8, s));
    k.prof = r->d_prof;
#endif
    // per-launch event pairs: a pool that grows to kMaxLaunchEvents, then a ring that keeps
    // the most recent ones (an iterator stepping one launch at a time never reads timings)
    size_t slot_i;
    if (r->n_launch_events < r->launch_events.size()) {
        slot_i = (r->ev_head + r->n_launch_events) % r->launch_events.size();
        ++r->n_launch_events;
    } else if (r->launch_events.size() < kMaxLaunchEvents) {  // pool full and not wrapped (ev_head == 0)
        hipEvent_t a, b;
        HIP_TRY(hipEventCreate(&a));
        HIP_TRY(hipEventCreate(&b));
        r->launch_events.emplace_back(a, b);
        slot_i = r->launch_events.size() - 1;
        ++r->n_launch_events;
    } else {  // ring full: overwrite the oldest
        slot_i = r->ev_head;
        r->ev_head = (r->ev_head + 1) % r->launch_events.size();
    }
    auto &evp = r->launch_events[slot_i];
    HIP_TRY(hipEventRecord(evp.first, s));
    if (r->p.proposal == FC_PROPOSE_RECOM) {
        fc::RecomParams q{};
        q.graph = r->d_graph;
        q.nbe = r->d_nbe;
        q.eslot = r->d_eslot;
        q.nb_d = r->nb_d;
        q.eu = r->d_eu;
        q.ev = r->d_ev;
        q.n = r->g.n;
        q.n_edges = r->g.n_edges;
        q.n_chains = r->n_chains;
        q.chain_lds_bytes = r->chain_lds_bytes;
        q.chain_id_offset = r->p.chain_id_offset;
        q.seed_lo = (uint32_t)r->p.seed;
        q.seed_hi = (uint32_t)(r->p.seed >> 32);
        q.pop_lo = (int32_t)r->p.pop_lo;
        q.pop_hi = (int32_t)r->p.pop_hi;
        q.pop_target = r->p.recom_pop_target;
        q.epsilon = r->p.recom_epsilon;
        q.node_repeats = r->p.recom_node_repeats > 0 ? r->p.recom_node_repeats : 1;
        q.max_attempts = r->p.recom_max_attempts > 0 ? r->p.recom_max_attempts : 10000;
        q.n_steps = n_steps;
        q.max_draws = max_draws > 0 ? max_draws : 1024 * std::max<int64_t>(n_steps, 1);
        q.assign = r->d_assign;
        q.sc = r->d_sc;
        q.accept_thresh = r->d_recom_thresh;
        q.trace = (fc_recom_record *)r->d_trace;
        q.trace_chains = r->p.trace_chains;
        q.trace_cap = r->p.trace_cap;
        q.prof = k.prof;
        const int e = fc::launch_recom(q, r->g.ring_max, s, r->kname, sizeof r->kname);
        if (e != 0) return fail(FC_ERR_HIP, std::string("recom kernel launch: ") + hipGetErrorString((hipError_t)e));
        HIP_TRY(hipEventRecord(evp.second, s));
#ifdef FC_PHASE_PROF
        if (int rc = dump_prof(r, s)) return rc;
#endif
        r->ev0 = evp.first;
        r->ev1 = evp.second;
        r->timed = true;
        return FC_OK;
    }
    // the kernel keeps per-launch step and per-lane counters in 32 bits: launch in chunks
    constexpr int64_t kChunk = int64_t(1) << 24;
    if (r->p.k == 2 && k.prio_nb[0] > 0 && k.prio_th[0] >= 0.0f) {  // tune_prio_th[0] < 0: |B| rule only
        if (!r->d_eta) {
            if (int rc = dalloc(&r->d_eta, 2)) return rc;
            HIP_TRY(hipMemsetAsync(r->d_eta, 0, 2 * sizeof(uint32_t), s));
        }
        k.eta = r->d_eta;
    }
    k.deal = nullptr;
    k.order = nullptr;
    k.ctime = nullptr;
    if (r->tune.deal) {
        if (!r->d_deal) {
            if (int rc = dalloc(&r->d_deal, (size_t)fc::kDealKeys + 4)) return rc;
            if (int rc = dalloc(&r->d_order, (size_t)r->n_chains)) return rc;
            if (int rc = dalloc(&r->d_ctime, (size_t)r->n_chains)) return rc;
        }
        k.deal = r->d_deal;
        k.order = r->d_order;
        k.ctime = r->d_ctime;
    }
    // k = 2 full diagnostics: the tally log (16 B per entry), sized for this call's launches (a
    // state's entries: one per accepted flip, plus a start-state entry per batch right after a
    // queue flush -- n_steps + n_steps / 8 + 256 per chain covers what the reference's sweeps
    // produce; a chain whose log fills applies the rest of its launch's tallies itself) within a
    // tenth of the device's free memory; launches of at most 2^23 steps (an entry holds t - t0
    // in 24 bits)
    k.tl = nullptr;
    k.tl_t0 = k.tl_len = nullptr;
    k.tl_cap = 0;
    int64_t chunk = kChunk;
    if (r->p.k == 2 && (r->p.diag_mask & (FC_DIAG_HIST | FC_DIAG_FLIPS | FC_DIAG_FLIPS_EXACT | FC_DIAG_EDGES)) &&
        r->g.n < 65535 && r->g.n_edges < (1 << 24)) {
        chunk = int64_t(1) << 23;
        const int64_t steps1 = std::min(chunk, n_steps);
        int64_t want = steps1 + steps1 / 8 + 256;
        if (r->p.flags & FC_FLAG_TALLY_LOG_SMALL) want = std::min<int64_t>(want, 64);
        r->tl_want = want;
        if (want > r->tl_cap) {
            size_t free_b = 0, total_b = 0;
            HIP_TRY(hipMemGetInfo(&free_b, &total_b));
            const int64_t per_chain = (int64_t)((free_b / 10) / ((size_t)r->n_chains * 16));
            want = std::min(want, std::max<int64_t>(per_chain, 0));
            if (want > r->tl_cap) {
                HIP_TRY(hipStreamSynchronize(s));
                if (r->d_tl) { HIP_TRY(hipFree(r->d_tl)); r->d_tl = nullptr; }
                r->tl_cap = 0;
                if (int rc = dalloc(&r->d_tl, (size_t)r->n_chains * (size_t)want * 4)) return rc;
                r->tl_cap = want;
            }
        }
        if (!r->d_tl_len) {
            if (int rc = dalloc(&r->d_tl_len, (size_t)r->n_chains)) return rc;
            if (int rc = dalloc(&r->d_tl_t0, (size_t)r->n_chains)) return rc;
            HIP_TRY(hipMemsetAsync(r->d_tl_len, 0, (size_t)r->n_chains * 8, s));
        }
        if (r->tl_cap > 0) {
            k.tl = r->d_tl;
            k.tl_t0 = r->d_tl_t0;
            k.tl_len = r->d_tl_len;
            k.tl_cap = r->tl_cap;
        }
    }
    for (int64_t done = 0; done < n_steps; done += chunk) {
        k.n_steps = std::min(chunk, n_steps - done);
        if (max_draws <= 0) k.max_draws = 65536 * k.n_steps;
        if (k.order) {  // this launch's deal: chains by the last one's durations (first: by |B|)
            const int e = fc::launch_deal_order(r->d_ctime, r->d_sc, k.n, r->n_chains, r->deal_timed ? 1 : 0,
                                                r->d_order, r->d_deal, s);
            if (e != 0) return fail(FC_ERR_HIP, std::string("deal kernel launch: ") + hipGetErrorString((hipError_t)e));
            r->deal_timed = true;
        }
        if (k.eta) {
            k.eta_parity = (int32_t)(r->n_flip_launches++ & 1);
            HIP_TRY(hipMemsetAsync(r->d_eta + k.eta_parity, 0, sizeof(uint32_t), s));
        }
        const int e = r->p.k == 2 ? fc::launch_flip2(k, r->g.ring_max, s, r->kname, sizeof r->kname)
                                    : fc::launch_flip_k2(k, r->g.ring_max, s, r->kname, sizeof r->kname);
        if (e != 0) return fail(FC_ERR_HIP, std::string("flip kernel launch: ") + hipGetErrorString((hipError_t)e));
        if (k.tl_len) {  // the launch's logged tallies, applied and the logs emptied
            const int er = fc::launch_tally_reduce(k, r->g.ring_max, s);
            if (er != 0) return fail(FC_ERR_HIP, std::string("tally reduce launch: ") + hipGetErrorString((hipError_t)er));
        }
    }
    HIP_TRY(hipEventRecord(evp.second, s));
#ifdef FC_PHASE_PROF
    if (int rc = dump_prof(r, s)) return rc;
#endif
    r->ev0 = evp.first;
    r->ev1 = evp.second;
    r->timed = true;
    return FC_OK;
}

int fc_run_sync(fc_run *r) {
    if (!r) return fail(FC_ERR_ARG, "fc_run_sync: null run");
    HIP_TRY(hipSetDevice(r->p.device));
    HIP_TRY(hipDeviceSynchronize());
    return FC_OK;
}

int fc_run_last_ms(fc_run *r, float *ms) {
    if (!r || !ms) return fail(FC_ERR_ARG, "fc_run_last_ms: null argument");
    if (!r->timed) return fail(FC_ERR_ARG, "fc_run_last_ms: no launch recorded");
    HIP_TRY(hipEventSynchronize(r->ev1));
    HIP_TRY(hipEventElapsedTime(ms, r->ev0, r->ev1));
    return FC_OK;
}

int fc_run_timings(fc_run *r, float *ms, int32_t cap, int32_t *n) {
    if (!r || !n || (cap > 0 && !ms)) return fail(FC_ERR_ARG, "fc_run_timings: null argument");
    HIP_TRY(hipSetDevice(r->p.device));
    const size_t cnt = r->n_launch_events, sz = r->launch_events.size();
    if (cnt) HIP_TRY(hipEventSynchronize(r->launch_events[(r->ev_head + cnt - 1) % sz].second));
    int32_t m = 0;
    for (size_t i = 0; i < cnt && m < cap; ++i, ++m) {
        const auto &pr = r->launch_events[(r->ev_head + i) % sz];
        HIP_TRY(hipEventElapsedTime(&ms[m], pr.first, pr.second));
    }
    *n = (int32_t)cnt;
    // the next launch records into slot 0 again; fc_run_last_ms keeps reading ev0 / ev1 (the
    // most recent pair) until then
    r->n_launch_events = 0;
    r->ev_head = 0;
    return FC_OK;
}

namespace {

// Version of the canonical random stream a checkpoint's chains continue on:
// 3 = round 4's k = 2 node words, four draws per purpose-3 Philox call.  A blob written under
// another stream (magic "FCCKPT02": one call per draw) is refused, not continued on a stream
// its trajectory never used.
constexpr uint32_t kStreamVersion = 3;

struct CkptHeader {
    char magic[8];          // "FCCKPT03"
    uint32_t stream_version, reserved;
    int32_t n_chains, n, n_edges, k, ring_max, proposal, npad, dgraph;
    uint32_t diag_mask;
    uint32_t chain_id_offset;
    int64_t ev_cap, payload;
    uint64_t seed, param_hash;  // the random stream and every trajectory-determining parameter
};

// (device pointer, bytes) of every buffer a checkpoint carries, in blob order
static std::vector<std::pair<void *, size_t>> ckpt_sections(fc_run *r) {
    const size_t C = (size_t)r->n_chains, n = (size_t)r->g.n, E = (size_t)r->g.n_edges, k = (size_t)r->p.k;
    const size_t R = (size_t)r->g.ring_max;
    std::vector<std::pair<void *, size_t>> v;
    v.emplace_back(r->d_assign, C * r->npad);
    v.emplace_back(r->d_sc, C * sizeof(fc::ChainScalars));
    if (r->p.proposal != FC_PROPOSE_RECOM) {
        v.emplace_back(r->d_fcnt, C * r->npad);
        v.emplace_back(r->d_popk, C * fc::kMaxKGeneral * 4);
        if (r->d_nfh) v.emplace_back(r->d_nfh, C * fc::kNfh * 4);
        if (r->d_sbits) v.emplace_back(r->d_sbits, C * (size_t)r->words * 8);
        v.emplace_back(r->d_thresh, C * (2 * R + 1) * 8);
        if (r->dgraph) {
            v.emplace_back(r->d_mcnt, C * k * k * 4);
            v.emplace_back(r->d_ngk, C * 32 * 4);
        }
    }
    if (r->d_cut_hist) v.emplace_back(r->d_cut_hist, C * (E + 1) * 8);
    if (r->d_nb_hist) v.emplace_back(r->d_nb_hist, C * (size_t)r->nb_w * 8);
    if (r->d_edge_acc) v.emplace_back(r->d_edge_acc, C * E * 8);
    if (r->d_num_flips) {
        v.emplace_back(r->d_num_flips, C * n * 8);
        v.emplace_back(r->d_part_sum, C * n * 8);
        v.emplace_back(r->d_last_flipped, C * n * 8);
    }
    if (r->d_flip_count) {
        v.emplace_back(r->d_flip_count, C * n * 8);
        v.emplace_back(r->d_occ_acc, C * n * 8);
        v.emplace_back(r->d_last_accept, C * n * 8);
    }
    if (r->d_events) {
        v.emplace_back(r->d_events, C * (size_t)r->ev_cap * sizeof(fc_event));
        v.emplace_back(r->d_ser_a0, C * r->npad);
    }
    return v;
}

CkptHeader ckpt_header(const fc_run *r, int64_t payload) {
    CkptHeader h{};
    std::memcpy(h.magic, "FCCKPT03", 8);
    h.stream_version = kStreamVersion;
    h.n_chains = r->n_chains;
    h.n = r->g.n;
    h.n_edges = r->g.n_edges;
    h.k = r->p.k;
    h.ring_max = r->g.ring_max;
    h.proposal = r->p.proposal;
    h.npad = r->npad;
    h.dgraph = r->dgraph ? 1 : 0;
    h.diag_mask = r->p.diag_mask;
    h.ev_cap = r->ev_cap;
    h.payload = payload;
    h.chain_id_offset = r->p.chain_id_offset;
    h.seed = r->p.seed;
    h.param_hash = r->param_hash;
    return h;
}

}  // namespace

int fc_run_checkpoint(fc_run *r, void *buf, int64_t cap, int64_t *len) {
    if (!r || !len) return fail(FC_ERR_ARG, "fc_run_checkpoint: null argument");
    const auto secs = ckpt_sections(r);
    int64_t payload = 0;
    for (const auto &sc : secs) payload += (int64_t)sc.second;
    const int64_t total = (int64_t)sizeof(CkptHeader) + payload;
    *len = total;
    if (!buf) return FC_OK;
    if (cap < total) return fail(FC_ERR_ARG, "fc_run_checkpoint: buffer too small (" + std::to_string(total) + " bytes needed)");
    if (int rc = fc_run_sync(r)) return rc;
    const CkptHeader h = ckpt_header(r, payload);
    unsigned char *out = (unsigned char *)buf;
    std::memcpy(out, &h, sizeof h);
    size_t off = sizeof h;
    for (const auto &sc : secs) {
        if (sc.second) HIP_TRY(hipMemcpy(out + off, sc.first, sc.second, hipMemcpyDeviceToHost));
        off += sc.second;
    }
    return FC_OK;
}

int fc_run_restore(fc_run *r, const void *buf, int64_t len) {
    if (!r || !buf) return fail(FC_ERR_ARG, "fc_run_restore: null argument");
    if (len < (int64_t)sizeof(CkptHeader)) return fail(FC_ERR_ARG, "fc_run_restore: blob too short");
    CkptHeader h;
    std::memcpy(&h, buf, sizeof h);
    const auto secs = ckpt_sections(r);
    int64_t payload = 0;
    for (const auto &sc : secs) payload += (int64_t)sc.second;
    const CkptHeader want = ckpt_header(r, payload);
    if (std::memcmp(h.magic, "FCCKPT02", 8) == 0)
        return fail(FC_ERR_ARG, "fc_run_restore: the checkpoint was written under an earlier random stream (FCCKPT02: one "
                                "Philox call per k = 2 node draw); its chains cannot continue on this build's stream");
    if (std::memcmp(h.magic, want.magic, 8) != 0) return fail(FC_ERR_ARG, "fc_run_restore: not a flipchain checkpoint");
    if (h.stream_version != kStreamVersion)
        return fail(FC_ERR_ARG, "fc_run_restore: the checkpoint's random-stream version (" + std::to_string(h.stream_version) +
                                    ") differs from this build's (" + std::to_string(kStreamVersion) + ")");
    if (h.n_chains != want.n_chains || h.n != want.n || h.n_edges != want.n_edges || h.k != want.k ||
        h.ring_max != want.ring_max || h.proposal != want.proposal || h.npad != want.npad || h.dgraph != want.dgraph ||
        h.diag_mask != want.diag_mask || h.ev_cap != want.ev_cap || h.payload != payload)
        return fail(FC_ERR_ARG, "fc_run_restore: the checkpoint was taken from a run with another graph or fc_params");
    if (h.seed != want.seed || h.chain_id_offset != want.chain_id_offset)
        return fail(FC_ERR_ARG, "fc_run_restore: the checkpoint's seed / chain_id_offset differ from this run's "
                                "(its chains would continue on another random stream)");
    if (h.param_hash != want.param_hash)
        return fail(FC_ERR_ARG, "fc_run_restore: the checkpoint's bases / thresholds, population bounds, labels, "
                                "log(1 - p) table or accept / constraint / ReCom settings differ from this run's");
    if (len != (int64_t)sizeof(CkptHeader) + payload) return fail(FC_ERR_ARG, "fc_run_restore: blob size mismatch");
    if (int rc = fc_run_sync(r)) return rc;
    const unsigned char *in = (const unsigned char *)buf;
    size_t off = sizeof h;
    for (size_t i = 0; i < secs.size(); ++i) {
        const auto &sc = secs[i];
        if (i == 1) {  // ChainScalars: traces are outputs and restart empty
            std::vector<fc::ChainScalars> s((size_t)r->n_chains);
            std::memcpy(s.data(), in + off, sc.second);
            for (auto &x : s) x.trace_len = 0;
            HIP_TRY(hipMemcpy(sc.first, s.data(), sc.second, hipMemcpyHostToDevice));
        } else if (sc.second) {
            HIP_TRY(hipMemcpy(sc.first, in + off, sc.second, hipMemcpyHostToDevice));
        }
        off += sc.second;
    }
    r->deal_timed = false;  // the restored chains' pace is not the last launch's
    return FC_OK;
}

int fc_run_read_stats(fc_run *r, fc_chain_stats *out) {
    if (!r || !out) return fail(FC_ERR_ARG, "fc_run_read_stats: null argument");
    if (int rc = fc_run_sync(r)) return rc;
    std::vector<fc::ChainScalars> sc(r->n_chains);
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    for (int32_t c = 0; c < r->n_chains; ++c) {
        const fc::ChainScalars &s = sc[c];
        fc_chain_stats &o = out[c];
        o.steps = s.steps;
        o.proposals = s.proposals;
        o.draws = (int64_t)s.draw;
        o.accepted = s.accepted;
        o.inv_contig = s.inv_contig;
        o.inv_pop = s.inv_pop;
        o.sum_cut = s.sum_cut;
        o.sum_nb = s.sum_nb;
        o.sum_wait = s.sum_wait;
        o.sum_cut2 = s.sum_cut2;
        o.sum_nb2 = s.sum_nb2;
        o.wait_cur = s.wait_cur;
        o.bfs_calls = s.bfs_calls;
        o.bfs_levels = s.bfs_levels;
        o.cut = s.cut;
        o.nb = s.nb;
        o.last_flip = s.last_flip;
        o.stuck = s.stuck;
        o.hit_time = s.hit_time;
        o.events = s.ev_len;
        o.series_t0 = s.ser_t0;
        o.series_cut0 = s.ser_cut0;
        o.series_nb0 = s.ser_nb0;
    }
    return FC_OK;
}

int fc_run_read_state(fc_run *r, int8_t *assign_out) {
    if (!r || !assign_out) return fail(FC_ERR_ARG, "fc_run_read_state: null argument");
    if (int rc = fc_run_sync(r)) return rc;
    std::vector<int8_t> a((size_t)r->n_chains * r->npad);
    HIP_TRY(hipMemcpy(a.data(), r->d_assign, a.size(), hipMemcpyDeviceToHost));
    for (int32_t c = 0; c < r->n_chains; ++c)
        std::memcpy(assign_out + (size_t)c * r->g.n, &a[(size_t)c * r->npad], r->g.n);
    return FC_OK;
}

int fc_run_read_pops(fc_run *r, int64_t *pops_out) {
    if (!r || !pops_out) return fail(FC_ERR_ARG, "fc_run_read_pops: null argument");
    if (int rc = fc_run_sync(r)) return rc;
    const int k = r->p.k;
    if (k == 2) {
        std::vector<fc::ChainScalars> sc(r->n_chains);
        HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
        for (int32_t c = 0; c < r->n_chains; ++c) {
            pops_out[2 * c] = sc[c].pops[0];
            pops_out[2 * c + 1] = sc[c].pops[1];
        }
    } else {
        std::vector<int32_t> pk((size_t)r->n_chains * fc::kMaxKGeneral);
        HIP_TRY(hipMemcpy(pk.data(), r->d_popk, pk.size() * 4, hipMemcpyDeviceToHost));
        for (int32_t c = 0; c < r->n_chains; ++c)
            for (int d = 0; d < k; ++d) pops_out[(size_t)c * k + d] = pk[(size_t)c * fc::kMaxKGeneral + d];
    }
    return FC_OK;
}

int fc_run_read_trace(fc_run *r, int32_t chain, fc_record *out, int64_t cap, int64_t *len) {
    if (!r || !out || !len) return fail(FC_ERR_ARG, "fc_run_read_trace: null argument");
    if (chain < 0 || chain >= r->p.trace_chains) return fail(FC_ERR_ARG, "fc_run_read_trace: chain is not traced");
    if (int rc = fc_run_sync(r)) return rc;
    fc::ChainScalars s;
    HIP_TRY(hipMemcpy(&s, r->d_sc + chain, sizeof s, hipMemcpyDeviceToHost));
    const int64_t n = std::min<int64_t>({s.trace_len, r->p.trace_cap, cap});
    HIP_TRY(hipMemcpy(out, r->d_trace + (size_t)chain * r->p.trace_cap, (size_t)n * sizeof(fc_record),
                      hipMemcpyDeviceToHost));
    *len = s.trace_len;
    return FC_OK;
}

int fc_run_read_recom_trace(fc_run *r, int32_t chain, fc_recom_record *out, int64_t cap, int64_t *len) {
    if (!r || !out || !len) return fail(FC_ERR_ARG, "fc_run_read_recom_trace: null argument");
    if (r->p.proposal != FC_PROPOSE_RECOM) return fail(FC_ERR_ARG, "fc_run_read_recom_trace: not a recom run");
    if (chain < 0 || chain >= r->p.trace_chains) return fail(FC_ERR_ARG, "fc_run_read_recom_trace: chain is not traced");
    if (int rc = fc_run_sync(r)) return rc;
    fc::ChainScalars s;
    HIP_TRY(hipMemcpy(&s, r->d_sc + chain, sizeof s, hipMemcpyDeviceToHost));
    const int64_t n = std::min<int64_t>({s.trace_len, r->p.trace_cap, cap});
    static_assert(sizeof(fc_recom_record) == sizeof(fc_record), "trace slots are shared");
    HIP_TRY(hipMemcpy(out, (const fc_recom_record *)r->d_trace + (size_t)chain * r->p.trace_cap,
                      (size_t)n * sizeof(fc_recom_record), hipMemcpyDeviceToHost));
    *len = s.trace_len;
    return FC_OK;
}

int fc_run_trace_reset(fc_run *r) {
    if (!r) return fail(FC_ERR_ARG, "fc_run_trace_reset: null run");
    if (int rc = fc_run_sync(r)) return rc;
    std::vector<fc::ChainScalars> sc(r->n_chains);
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    for (auto &s : sc) s.trace_len = 0;
    HIP_TRY(hipMemcpy(r->d_sc, sc.data(), sc.size() * sizeof(sc[0]), hipMemcpyHostToDevice));
    return FC_OK;
}

int fc_run_read_events(fc_run *r, int32_t chain, fc_event *out, int64_t cap, int64_t *len) {
    if (!r || !len || (cap > 0 && !out)) return fail(FC_ERR_ARG, "fc_run_read_events: null argument");
    if (!r->d_events) return fail(FC_ERR_ARG, "fc_run_read_events: FC_DIAG_SERIES not enabled");
    if (chain < 0 || chain >= r->n_chains) return fail(FC_ERR_ARG, "fc_run_read_events: chain out of range");
    if (int rc = fc_run_sync(r)) return rc;
    fc::ChainScalars s;
    HIP_TRY(hipMemcpy(&s, r->d_sc + chain, sizeof s, hipMemcpyDeviceToHost));
    const int64_t n = std::min<int64_t>({s.ev_len, r->ev_cap, cap});
    if (n > 0)
        HIP_TRY(hipMemcpy(out, r->d_events + (size_t)chain * r->ev_cap, (size_t)n * sizeof(fc_event),
                          hipMemcpyDeviceToHost));
    *len = s.ev_len;
    return FC_OK;
}

int fc_run_series_reset(fc_run *r) {
    if (!r) return fail(FC_ERR_ARG, "fc_run_series_reset: null run");
    if (int rc = fc_run_sync(r)) return rc;
    std::vector<fc::ChainScalars> sc(r->n_chains);
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    for (auto &s : sc) {
        s.ev_len = 0;
        s.ser_t0 = s.steps;
        s.ser_cut0 = s.cut;
        s.ser_nb0 = s.nb;
    }
    HIP_TRY(hipMemcpy(r->d_sc, sc.data(), sc.size() * sizeof(sc[0]), hipMemcpyHostToDevice));
    if (r->d_ser_a0)
        HIP_TRY(hipMemcpy(r->d_ser_a0, r->d_assign, (size_t)r->n_chains * r->npad, hipMemcpyDeviceToDevice));
    return FC_OK;
}

int fc_run_autocorr(fc_run *r, const int32_t *lags, int32_t nlags, int64_t *lag_sums, double *acf) {
    if (!r || !lags || nlags <= 0 || !lag_sums) return fail(FC_ERR_ARG, "fc_run_autocorr: null argument");
    if (!r->d_events) return fail(FC_ERR_ARG, "fc_run_autocorr: FC_DIAG_SERIES not enabled");
    for (int32_t j = 0; j < nlags; ++j)
        if (lags[j] < 0) return fail(FC_ERR_ARG, "fc_run_autocorr: negative lag");
    if (int rc = fc_run_sync(r)) return rc;
    const int32_t C = r->n_chains;
    std::vector<fc::ChainScalars> sc(C);
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    std::vector<int64_t> ev_len(C), t0(C), len(C);
    std::vector<int32_t> cut0(C);
    int64_t max_len = 0;
    for (int32_t c = 0; c < C; ++c) {
        if (sc[c].ev_len > r->ev_cap)
            return fail(FC_ERR_ARG, "fc_run_autocorr: chain " + std::to_string(c) +
                                        " overflowed event_cap; reset the series window more often");
        ev_len[c] = sc[c].ev_len;
        t0[c] = sc[c].ser_t0;
        cut0[c] = sc[c].ser_cut0;
        len[c] = sc[c].steps - sc[c].ser_t0 + 1;  // yields t0 .. steps
        max_len = std::max(max_len, len[c]);
    }
    // lag 0 is always evaluated first: it yields the window totals Sx = H_0 and Sxx = P_0
    std::vector<int32_t> lg(nlags + 1);
    lg[0] = 0;
    std::copy(lags, lags + nlags, lg.begin() + 1);
    const int32_t nl = nlags + 1;
    // device scratch: metadata + dense series for a batch of chains (<= 1 GiB)
    const int64_t stride = (max_len + 7) & ~int64_t(7);
    const int32_t batch = (int32_t)std::max<int64_t>(1, std::min<int64_t>({C, 65535, (int64_t(1) << 29) / stride}));
    int64_t *d_meta = nullptr;
    int32_t *d_cut0 = nullptr, *d_lags = nullptr;
    uint16_t *d_x = nullptr;
    unsigned long long *d_sums = nullptr;
    auto cleanup = [&]() {
        for (void *b : {(void *)d_meta, (void *)d_cut0, (void *)d_lags, (void *)d_x, (void *)d_sums})
            if (b) (void)hipFree(b);
    };
    auto run = [&]() -> int {
        int q;
        if ((q = dalloc(&d_meta, (size_t)3 * C))) return q;
        if ((q = dalloc(&d_cut0, (size_t)C))) return q;
        if ((q = dalloc(&d_lags, (size_t)nl))) return q;
        if ((q = dalloc(&d_x, (size_t)batch * stride))) return q;
        if ((q = dalloc(&d_sums, (size_t)C * nl * 3))) return q;
        HIP_TRY(hipMemcpy(d_meta, ev_len.data(), (size_t)C * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_meta + C, t0.data(), (size_t)C * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_meta + 2 * C, len.data(), (size_t)C * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_cut0, cut0.data(), (size_t)C * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_lags, lg.data(), (size_t)nl * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemsetAsync(d_sums, 0, (size_t)C * nl * 3 * 8, r->stream));
        for (int32_t c0 = 0; c0 < C; c0 += batch) {
            const int32_t nc = std::min(batch, C - c0);
            int e = fc::launch_series_expand(r->d_events, r->ev_cap, d_meta, d_meta + C, d_cut0, d_meta + 2 * C, c0,
                                             nc, stride, max_len, d_x, r->stream);
            if (e) return fail(FC_ERR_HIP, std::string("series expand: ") + hipGetErrorString((hipError_t)e));
            e = fc::launch_series_lagsums(d_x, d_meta + 2 * C, c0, nc, stride, max_len, d_lags, nl, d_sums,
                                          r->stream);
            if (e) return fail(FC_ERR_HIP, std::string("series lag sums: ") + hipGetErrorString((hipError_t)e));
        }
        std::vector<int64_t> sums((size_t)C * nl * 3);
        HIP_TRY(hipMemcpyAsync(sums.data(), d_sums, sums.size() * 8, hipMemcpyDeviceToHost, r->stream));
        HIP_TRY(hipStreamSynchronize(r->stream));
        for (int32_t c = 0; c < C; ++c) {
            const int64_t *s0 = &sums[(size_t)c * nl * 3];
            const __int128 Sxx = s0[0], Sx = s0[1], T = len[c];
            for (int32_t j = 0; j < nlags; ++j) {
                const int64_t *s = s0 + 3 * (j + 1);
                lag_sums[(size_t)c * nlags + j] = s[0];
                if (!acf) continue;
                const __int128 L = lags[j];
                double v = 0.0;
                if (L < T) {
                    // T^2 * sum_{t < T-L} (x_t - m)(x_{t+L} - m), m = Sx / T, in exact integers
                    const __int128 num = T * T * (__int128)s[0] - T * Sx * ((__int128)s[1] + s[2]) + (T - L) * Sx * Sx;
                    const __int128 den = T * (T * Sxx - Sx * Sx);
                    if (den != 0) v = (double)num / (double)den;
                }
                acf[(size_t)c * nlags + j] = v;
            }
        }
        return FC_OK;
    };
    const int rc = run();
    cleanup();
    return rc;
}

int fc_run_frame_series(fc_run *r, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *frame_u,
                        const int32_t *frame_v, const double *mid_xy, double cx, double cy, int64_t cap,
                        double *slope, double *angle, int32_t *n_cut, int64_t *len) {
    if (!r || !frame_u || !frame_v || !mid_xy || !slope || !angle || !n_cut || !len)
        return fail(FC_ERR_ARG, "fc_run_frame_series: null argument");
    if (!r->d_events) return fail(FC_ERR_ARG, "fc_run_frame_series: FC_DIAG_SERIES not enabled");
    if (r->p.k != 2)
        return fail(FC_ERR_UNSUPPORTED, "fc_run_frame_series: the frame series follows k = 2 flips (the reference "
                                        "computes boundary_slope only in its two-district drivers)");
    if (c0 < 0 || nc < 0 || c0 + nc > r->n_chains) return fail(FC_ERR_ARG, "fc_run_frame_series: chain range");
    if (n_frame < 0 || n_frame > 256) return fail(FC_ERR_UNSUPPORTED, "fc_run_frame_series: at most 256 frame edges");
    const int32_t n = r->g.n;
    std::vector<int32_t> tog_idx(n, -1);
    std::vector<uint64_t> tog;
    for (int32_t j = 0; j < n_frame; ++j) {
        const int32_t ends[2] = {frame_u[j], frame_v[j]};
        if (ends[0] < 0 || ends[0] >= n || ends[1] < 0 || ends[1] >= n || ends[0] == ends[1])
            return fail(FC_ERR_ARG, "fc_run_frame_series: frame edge " + std::to_string(j) + " out of range");
        for (int32_t x : ends) {
            if (tog_idx[x] < 0) {
                tog_idx[x] = (int32_t)(tog.size() / 4);
                tog.insert(tog.end(), 4, 0);
            }
            tog[(size_t)tog_idx[x] * 4 + (j >> 6)] |= uint64_t(1) << (j & 63);
        }
    }
    if (nc == 0) return FC_OK;
    if (int rc = fc_run_sync(r)) return rc;
    std::vector<fc::ChainScalars> sc(nc);
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc + c0, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    std::vector<int64_t> ev_len(r->n_chains, 0);
    for (int32_t i = 0; i < nc; ++i) {
        if (sc[i].ev_len > r->ev_cap)
            return fail(FC_ERR_ARG, "fc_run_frame_series: chain " + std::to_string(c0 + i) +
                                        " overflowed event_cap; reset the series window more often");
        if (sc[i].ev_len + 1 > cap)
            return fail(FC_ERR_ARG, "fc_run_frame_series: cap < events + 1 for chain " + std::to_string(c0 + i));
        ev_len[c0 + i] = sc[i].ev_len;
        len[i] = sc[i].ev_len + 1;
    }
    int32_t *d_fuv = nullptr, *d_tidx = nullptr;
    int64_t *d_len = nullptr;
    uint64_t *d_tog = nullptr;
    double *d_mid = nullptr;
    auto cleanup = [&]() {
        for (void *b : {(void *)d_fuv, (void *)d_tidx, (void *)d_len, (void *)d_tog, (void *)d_mid})
            if (b) (void)hipFree(b);
    };
    auto run = [&]() -> int {
        int q;
        const size_t outn = (size_t)nc * cap;
        if ((q = dalloc(&d_fuv, (size_t)2 * std::max(n_frame, 1)))) return q;
        if ((q = dalloc(&d_tidx, (size_t)n))) return q;
        if ((q = dalloc(&d_tog, std::max<size_t>(tog.size(), 4)))) return q;
        if ((q = dalloc(&d_mid, (size_t)2 * std::max(n_frame, 1)))) return q;
        if ((q = dalloc(&d_len, (size_t)r->n_chains))) return q;
        // the large outputs are kept by the run (chunked callers ask for similar sizes)
        if (outn > r->fs_cap) {
            if (r->d_fs_out) (void)hipFree(r->d_fs_out);
            if (r->d_fs_cnt) (void)hipFree(r->d_fs_cnt);
            r->d_fs_out = nullptr;
            r->d_fs_cnt = nullptr;
            r->fs_cap = 0;
            if ((q = dalloc(&r->d_fs_out, 2 * outn))) return q;
            if ((q = dalloc(&r->d_fs_cnt, outn))) return q;
            r->fs_cap = outn;
        }
        double *const d_out = r->d_fs_out;
        int32_t *const d_cnt = r->d_fs_cnt;
        if (n_frame) {
            HIP_TRY(hipMemcpy(d_fuv, frame_u, (size_t)n_frame * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(d_fuv + n_frame, frame_v, (size_t)n_frame * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(d_mid, mid_xy, (size_t)n_frame * 16, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(d_tog, tog.data(), tog.size() * 8, hipMemcpyHostToDevice));
        }
        HIP_TRY(hipMemcpy(d_tidx, tog_idx.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_len, ev_len.data(), ev_len.size() * 8, hipMemcpyHostToDevice));
        int e = fc::launch_frame_series(r->d_ser_a0, r->npad, r->d_events, r->ev_cap, d_len, c0, nc, n_frame, d_fuv,
                                        d_fuv + n_frame, d_mid, cx, cy, d_tidx, d_tog, (int32_t)(tog.size() / 4), n,
                                        cap, d_out, d_out + outn,
                                        d_cnt, r->stream);
        if (e) return fail(FC_ERR_HIP, std::string("frame series: ") + hipGetErrorString((hipError_t)e));
        HIP_TRY(hipStreamSynchronize(r->stream));
        HIP_TRY(hipMemcpy(slope, d_out, outn * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(angle, d_out + outn, outn * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(n_cut, d_cnt, outn * 4, hipMemcpyDeviceToHost));
        return FC_OK;
    };
    const int rc = run();
    cleanup();
    return rc;
}

int fc_run_frame_series_changes(fc_run *r, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *frame_u,
                                const int32_t *frame_v, const double *mid_xy, double cx, double cy, int64_t cap,
                                int64_t *offsets, int64_t *t, double *slope, double *angle) {
    if (!r || !frame_u || !frame_v || !mid_xy || !offsets)
        return fail(FC_ERR_ARG, "fc_run_frame_series_changes: null argument");
    const bool query = !t && !slope && !angle;
    if (!query && (!t || !slope || !angle)) return fail(FC_ERR_ARG, "fc_run_frame_series_changes: null output");
    if (!r->d_events) return fail(FC_ERR_ARG, "fc_run_frame_series_changes: FC_DIAG_SERIES not enabled");
    if (r->p.k != 2) return fail(FC_ERR_UNSUPPORTED, "fc_run_frame_series_changes: k = 2 runs only");
    if (c0 < 0 || nc < 0 || c0 + nc > r->n_chains) return fail(FC_ERR_ARG, "fc_run_frame_series_changes: chain range");
    if (n_frame < 0 || n_frame > 256)
        return fail(FC_ERR_UNSUPPORTED, "fc_run_frame_series_changes: at most 256 frame edges");
    const int32_t n = r->g.n;
    for (int32_t j = 0; j < n_frame; ++j)
        if (frame_u[j] < 0 || frame_u[j] >= n || frame_v[j] < 0 || frame_v[j] >= n || frame_u[j] == frame_v[j])
            return fail(FC_ERR_ARG, "fc_run_frame_series_changes: frame edge " + std::to_string(j) + " out of range");
    offsets[0] = 0;
    if (nc == 0) return FC_OK;
    if (int rc = fc_run_sync(r)) return rc;
    int q;
    // the frame tables: uploaded when the frame differs from the last call's
    uint64_t h = fnv1a(0xcbf29ce484222325ull, &n_frame, sizeof n_frame);
    h = fnv1a(h, frame_u, (size_t)n_frame * 4);
    h = fnv1a(h, frame_v, (size_t)n_frame * 4);
    h = fnv1a(h, mid_xy, (size_t)n_frame * 16);
    if (!r->d_fc_fuv || h != r->fc_frame_hash) {
        std::vector<int32_t> tog_idx(n, -1);
        std::vector<uint64_t> tog;
        for (int32_t j = 0; j < n_frame; ++j) {
            const int32_t ends[2] = {frame_u[j], frame_v[j]};
            for (int32_t x : ends) {
                if (tog_idx[x] < 0) {
                    tog_idx[x] = (int32_t)(tog.size() / 4);
                    tog.insert(tog.end(), 4, 0);
                }
                tog[(size_t)tog_idx[x] * 4 + (j >> 6)] |= uint64_t(1) << (j & 63);
            }
        }
        for (void *b : {(void *)r->d_fc_fuv, (void *)r->d_fc_tidx, (void *)r->d_fc_tog, (void *)r->d_fc_mid})
            if (b) (void)hipFree(b);
        r->d_fc_fuv = r->d_fc_tidx = nullptr;
        r->d_fc_tog = nullptr;
        r->d_fc_mid = nullptr;
        if ((q = dalloc(&r->d_fc_fuv, (size_t)2 * 256))) return q;
        if ((q = dalloc(&r->d_fc_tidx, (size_t)n))) return q;
        if ((q = dalloc(&r->d_fc_tog, (size_t)4 * 512))) return q;
        if ((q = dalloc(&r->d_fc_mid, (size_t)2 * 256))) return q;
        if (n_frame) {
            HIP_TRY(hipMemcpy(r->d_fc_fuv, frame_u, (size_t)n_frame * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(r->d_fc_fuv + n_frame, frame_v, (size_t)n_frame * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(r->d_fc_mid, mid_xy, (size_t)n_frame * 16, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(r->d_fc_tog, tog.data(), tog.size() * 8, hipMemcpyHostToDevice));
        }
        HIP_TRY(hipMemcpy(r->d_fc_tidx, tog_idx.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        r->fc_frame_hash = h;
        r->fc_rows = (int32_t)(tog.size() / 4);
    }
    if (!r->d_fc_len) {
        const size_t C = (size_t)r->n_chains;
        if ((q = dalloc(&r->d_fc_len, C))) return q;
        if ((q = dalloc(&r->d_fc_t0, C))) return q;
        if ((q = dalloc(&r->d_fc_cnt, C))) return q;
        if ((q = dalloc(&r->d_fc_off, C))) return q;
        if ((q = dalloc(&r->d_fc_wcnt, C * fc::kFrameWaves))) return q;
    }
    std::vector<fc::ChainScalars> sc(nc);
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc + c0, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    std::vector<int64_t> ev_len(nc), t0(nc);
    for (int32_t i = 0; i < nc; ++i) {
        if (sc[i].ev_len > r->ev_cap)
            return fail(FC_ERR_ARG, "fc_run_frame_series_changes: chain " + std::to_string(c0 + i) +
                                        " overflowed event_cap; reset the series window more often");
        ev_len[i] = sc[i].ev_len;
        t0[i] = sc[i].ser_t0;
    }
    // the kernels index the per-chain arrays by global chain id
    HIP_TRY(hipMemcpyAsync(r->d_fc_len + c0, ev_len.data(), (size_t)nc * 8, hipMemcpyHostToDevice, r->stream));
    HIP_TRY(hipMemcpyAsync(r->d_fc_t0 + c0, t0.data(), (size_t)nc * 8, hipMemcpyHostToDevice, r->stream));
    int32_t *const d_fuv = r->d_fc_fuv;
    // one pass (count and write together) into per-wave staging ranges when they fit a tenth of
    // the free device memory: sized by event_cap, kept by the run
    const int64_t nk = (r->ev_cap + 63) / 64;
    const int64_t sub = 64 * ((nk + fc::kFrameWaves - 1) / fc::kFrameWaves) + 1;
    const int64_t stage_cap = sub * fc::kFrameWaves;
    bool staged = false;
    if (!query && !(r->p.flags & FC_FLAG_SERIES_TWO_PASS)) {
        const size_t want = (size_t)r->n_chains * (size_t)stage_cap;
        if (want > r->fc_stage_cap) {
            size_t free_b = 0, total_b = 0;
            HIP_TRY(hipMemGetInfo(&free_b, &total_b));
            if (want * 24 <= free_b / 10) {
                for (void *b : {(void *)r->d_st_t, (void *)r->d_st_sa})
                    if (b) (void)hipFree(b);
                r->d_st_t = nullptr;
                r->d_st_sa = nullptr;
                r->fc_stage_cap = 0;
                if ((q = dalloc(&r->d_st_t, want))) return q;
                if ((q = dalloc(&r->d_st_sa, 2 * want))) return q;
                r->fc_stage_cap = want;
            }
        }
        staged = want <= r->fc_stage_cap;
    }
    if (!query) r->series_staged = staged ? 1 : 0;
    const size_t stn = r->fc_stage_cap;  // staging: slope at d_st_sa, angle at d_st_sa + stn
    int e;
    if (staged)
        e = fc::launch_frame_stage(r->d_ser_a0, r->npad, r->d_events, r->ev_cap, r->d_fc_len, c0, nc, n_frame, d_fuv,
                                   d_fuv + n_frame, r->d_fc_mid, cx, cy, r->d_fc_tidx, r->d_fc_tog, r->fc_rows, n,
                                   r->d_fc_t0, r->d_fc_cnt, stage_cap, r->d_st_t, r->d_st_sa, r->d_st_sa + stn,
                                   r->d_fc_wcnt, r->stream);
    else  // pass 1: change points per chain -> offsets
        e = fc::launch_frame_changes(r->d_ser_a0, r->npad, r->d_events, r->ev_cap, r->d_fc_len, c0, nc, n_frame, d_fuv,
                                     d_fuv + n_frame, r->d_fc_mid, cx, cy, r->d_fc_tidx, r->d_fc_tog, r->fc_rows, n,
                                     r->d_fc_t0, r->d_fc_cnt, nullptr, nullptr, nullptr, nullptr, r->d_fc_wcnt, r->stream);
    if (e) return fail(FC_ERR_HIP, std::string(staged ? "frame changes (stage): " : "frame changes (count): ") +
                                       hipGetErrorString((hipError_t)e));
    std::vector<int64_t> cnt(nc);
    HIP_TRY(hipMemcpyAsync(cnt.data(), r->d_fc_cnt, (size_t)nc * 8, hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    for (int32_t i = 0; i < nc; ++i) offsets[i + 1] = offsets[i] + cnt[i];
    const int64_t total = offsets[nc];
    if (query) return FC_OK;
    if (cap < total)  // offsets are filled: the caller can size its buffers and call again
        return fail(FC_ERR_ARG, "fc_run_frame_series_changes: cap " + std::to_string(cap) + " < " +
                                    std::to_string(total) + " change points (offsets[nc])");
    if ((size_t)total > r->fc_cap) {
        if (r->d_fc_t) (void)hipFree(r->d_fc_t);
        if (r->d_fc_sa) (void)hipFree(r->d_fc_sa);
        r->d_fc_t = nullptr;
        r->d_fc_sa = nullptr;
        r->fc_cap = 0;
        const size_t want = (size_t)total + (size_t)total / 4 + 1024;  // headroom: one allocation per run
        if ((q = dalloc(&r->d_fc_t, want))) return q;
        if ((q = dalloc(&r->d_fc_sa, 2 * want))) return q;
        r->fc_cap = want;
    }
    // pass 2: (t, slope, angle) at the offsets, then one copy per array
    HIP_TRY(hipMemcpyAsync(r->d_fc_off, offsets, (size_t)nc * 8, hipMemcpyHostToDevice, r->stream));
    double *const d_sl = r->d_fc_sa, *const d_an = r->d_fc_sa + r->fc_cap;
    if (staged)  // the staged ranges packed at the offsets
        e = fc::launch_frame_compact(nc, stage_cap, r->d_st_t, r->d_st_sa, r->d_st_sa + stn, r->d_fc_wcnt, r->d_fc_off,
                                     r->d_fc_t, d_sl, d_an, r->stream);
    else
        e = fc::launch_frame_changes(r->d_ser_a0, r->npad, r->d_events, r->ev_cap, r->d_fc_len, c0, nc, n_frame, d_fuv,
                                     d_fuv + n_frame, r->d_fc_mid, cx, cy, r->d_fc_tidx, r->d_fc_tog, r->fc_rows, n,
                                     r->d_fc_t0, r->d_fc_cnt, r->d_fc_off, r->d_fc_t, d_sl, d_an, r->d_fc_wcnt, r->stream);
    if (e) return fail(FC_ERR_HIP, std::string("frame changes (write): ") + hipGetErrorString((hipError_t)e));
    HIP_TRY(hipMemcpyAsync(t, r->d_fc_t, (size_t)total * 8, hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipMemcpyAsync(slope, d_sl, (size_t)total * 8, hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipMemcpyAsync(angle, d_an, (size_t)total * 8, hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    return FC_OK;
}

int fc_host_register(void *ptr, int64_t bytes) {
    if (!ptr || bytes <= 0) return fail(FC_ERR_ARG, "fc_host_register: null or empty buffer");
    HIP_TRY(hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault));
    return FC_OK;
}

int fc_host_unregister(void *ptr) {
    if (!ptr) return fail(FC_ERR_ARG, "fc_host_unregister: null buffer");
    HIP_TRY(hipHostUnregister(ptr));
    return FC_OK;
}

int fc_run_kernel_name(const fc_run *r, char *buf, int32_t cap) {
    if (!r || !buf || cap <= 0) return fail(FC_ERR_ARG, "fc_run_kernel_name: null argument");
    std::snprintf(buf, (size_t)cap, "%s", r->kname);
    return FC_OK;
}

int fc_run_read_hist(fc_run *r, int64_t *cut_hist, int64_t *nb_hist) {
    if (!r || !cut_hist || !nb_hist) return fail(FC_ERR_ARG, "fc_run_read_hist: null argument");
    if (!r->d_cut_hist) return fail(FC_ERR_ARG, "fc_run_read_hist: FC_DIAG_HIST not enabled");
    if (int rc = fc_run_sync(r)) return rc;
    HIP_TRY(hipMemcpy(cut_hist, r->d_cut_hist, (size_t)r->n_chains * (r->g.n_edges + 1) * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(nb_hist, r->d_nb_hist, (size_t)r->n_chains * r->nb_w * 8, hipMemcpyDeviceToHost));
    return FC_OK;
}

int fc_run_read_edges(fc_run *r, int64_t *cut_times) {
    if (!r || !cut_times) return fail(FC_ERR_ARG, "fc_run_read_edges: null argument");
    if (!r->d_edge_acc) return fail(FC_ERR_ARG, "fc_run_read_edges: FC_DIAG_EDGES not enabled");
    if (int rc = fc_run_sync(r)) return rc;
    const size_t E = r->g.n_edges, C = r->n_chains;
    std::vector<int64_t> acc(C * E);
    std::vector<int8_t> a(C * r->npad);
    std::vector<fc::ChainScalars> sc(C);
    HIP_TRY(hipMemcpy(acc.data(), r->d_edge_acc, acc.size() * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(a.data(), r->d_assign, a.size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    for (size_t c = 0; c < C; ++c) {
        const int8_t *ac = &a[c * r->npad];
        const int64_t T = sc[c].steps + 1;  // yields so far
        for (size_t e = 0; e < E; ++e) {
            const bool is_cut = ac[r->g.eu[e]] != ac[r->g.ev[e]];
            // the kernels add the yield at which e turns uncut and subtract the one at which it
            // turns cut; an edge cut now is cut through the last yield
            cut_times[c * E + e] = acc[c * E + e] + (is_cut ? T : 0);
        }
    }
    return FC_OK;
}

int fc_run_read_flips(fc_run *r, int64_t *num_flips, int64_t *part_sum, int64_t *last_flipped) {
    if (!r || !num_flips || !part_sum || !last_flipped) return fail(FC_ERR_ARG, "fc_run_read_flips: null argument");
    if (!r->d_num_flips) return fail(FC_ERR_ARG, "fc_run_read_flips: FC_DIAG_FLIPS not enabled");
    if (int rc = fc_run_sync(r)) return rc;
    const size_t n = r->g.n, C = r->n_chains;
    std::vector<int8_t> a(C * r->npad);
    std::vector<fc::ChainScalars> sc(C);
    HIP_TRY(hipMemcpy(num_flips, r->d_num_flips, C * n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(part_sum, r->d_part_sum, C * n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(last_flipped, r->d_last_flipped, C * n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(a.data(), r->d_assign, a.size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    const int64_t lsum = (int64_t)r->labels[0] + (int64_t)r->labels[1];
    for (size_t c = 0; c < C; ++c) {
        const int64_t T = sc[c].steps + 1;
        for (size_t u = 0; u < n; ++u) {
            const int64_t lab = r->labels[a[c * r->npad + u]];
            const int64_t t_r = last_flipped[c * n + u];
            // k = 2 (fc_flip2.hip): every run of u added (L0 + L1 - 2 a_r) per yield; the last
            // run's share is -a_R t_R instead
            if (r->p.k == 2 && t_r != 0) part_sum[c * n + u] += (lab - lsum) * t_r;
            if (t_r == 0) part_sum[c * n + u] = T * lab;  // grid_chain_sec11.py:416-418
        }
    }
    return FC_OK;
}

int fc_run_read_flips_exact(fc_run *r, int64_t *flip_count, int64_t *occupancy, int64_t *last_accept) {
    if (!r || !flip_count || !occupancy || !last_accept) return fail(FC_ERR_ARG, "fc_run_read_flips_exact: null argument");
    if (!r->d_flip_count) return fail(FC_ERR_ARG, "fc_run_read_flips_exact: FC_DIAG_FLIPS_EXACT not enabled");
    if (int rc = fc_run_sync(r)) return rc;
    const size_t n = r->g.n, C = r->n_chains;
    std::vector<int8_t> a(C * r->npad);
    std::vector<fc::ChainScalars> sc(C);
    HIP_TRY(hipMemcpy(flip_count, r->d_flip_count, C * n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(occupancy, r->d_occ_acc, C * n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(last_accept, r->d_last_accept, C * n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(a.data(), r->d_assign, a.size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(sc.data(), r->d_sc, sc.size() * sizeof(sc[0]), hipMemcpyDeviceToHost));
    for (size_t c = 0; c < C; ++c) {
        // sum_t L(a_t) = L(a_0) s_1 + L(a_1)(s_2 - s_1) + ... = L(a_now) T - sum_flips (L_new - L_old) s
        const int64_t T = sc[c].steps + 1;
        for (size_t u = 0; u < n; ++u) occupancy[c * n + u] += (int64_t)r->labels[a[c * r->npad + u]] * T;
    }
    return FC_OK;
}

int fc_run_read_wait_expected(fc_run *r, double *out) {
    if (!r || !out) return fail(FC_ERR_ARG, "fc_run_read_wait_expected: null argument");
    if (!r->d_nb_hist) return fail(FC_ERR_ARG, "fc_run_read_wait_expected: FC_DIAG_HIST not enabled");
    if (int rc = fc_run_sync(r)) return rc;
    const size_t n = r->g.n, C = r->n_chains, W = (size_t)r->nb_w;
    std::vector<int64_t> h(C * W);
    HIP_TRY(hipMemcpy(h.data(), r->d_nb_hist, h.size() * 8, hipMemcpyDeviceToHost));
    // geom_wait (:147-148): np.random.geometric(p) - 1 with p = |B| / (N^k - 1): mean 1/p - 1
    const double M = std::pow((double)n, (double)r->p.k) - 1.0;
    for (size_t c = 0; c < C; ++c) {
        double s = 0.0;
        for (size_t b = 1; b < W; ++b)
            if (h[c * W + b]) s += (double)h[c * W + b] * (M / (double)b - 1.0);
        out[c] = s;
    }
    return FC_OK;
}

void fc_run_destroy(fc_run *r) {
    if (!r) return;
    (void)hipSetDevice(r->p.device);
    (void)hipDeviceSynchronize();
    free_run(r);
}

}  // extern "C"
