/*
 * flipchain.h -- C-ABI of the MI355X-native flip-walk engine (libflipchain.so).
 *
 * This is the drop-in boundary for the reference's hot path: the gerrychain MarkovChain
 * protocol as the reference drives it,
 *
 *   exp_chain = MarkovChain(slow_reversible_propose_bi,
 *                           Validator([single_flip_contiguous, popbound]),
 *                           accept=cut_accept, initial_state=grid_partition,
 *                           total_steps=100000)          grid_chain_sec11.py:340-342
 *   for part in exp_chain: ...                           grid_chain_sec11.py:366-402
 *
 * Each entry point below names the reference interface it replaces.  Plain pointers and
 * sizes only; no C++ exceptions cross this boundary; every call returns an int status
 * (FC_OK = 0, < 0 error) and leaves a thread-local message in fc_last_error().
 *
 * Threading: one fc_run per host thread at a time.  The library has no global mutable
 * state besides the thread-local error string.  fc_run_steps is asynchronous on the given
 * HIP stream (NULL = the run's own stream); every fc_run_read_* call synchronises.
 *
 * Ownership: fc_graph_create / fc_run_create copy all host arrays; the library owns its
 * device buffers and frees them in *_destroy.
 */
#ifndef FLIPCHAIN_H
#define FLIPCHAIN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FC_OK 0
#define FC_ERR_ARG (-1)          /* bad argument (TypeError / IndexError analogues)        */
#define FC_ERR_INVALID_STATE (-2) /* initial state not valid: MarkovChain raises ValueError */
#define FC_ERR_HIP (-3)          /* HIP runtime failure or no GPU                           */
#define FC_ERR_UNSUPPORTED (-4)  /* configuration outside what the kernels implement        */
#define FC_ERR_NOMEM (-5)

/* fc_params.struct_size / abi_version: a caller built against another layout of fc_params is
 * rejected (FC_ERR_ARG) instead of read past.  Bumped whenever fc_params changes.           */
#define FC_ABI_VERSION 5u

/* fc_graph_create flags */
#define FC_GRAPH_NO_EXACT 0x1u   /* never trust the planar local contiguity rule            */

/* fc_params.proposal */
#define FC_PROPOSE_BI_SIGN 0     /* slow_reversible_propose_bi, grid_chain_sec11.py:132-145 */
#define FC_PROPOSE_PAIR 1        /* slow_reversible_propose,    grid_chain_sec11.py:117-130 */
#define FC_PROPOSE_RECOM 2       /* recom tree proposal built at grid_chain_sec11.py:328-335:
                                    spanning-tree bipartition of two merged districts       */

/* fc_params.diag_mask: per-yield driver diagnostics kept on the device
 * (grid_chain_sec11.py:350-419).  The streaming sums are always kept.                    */
#define FC_DIAG_WAIT 0x1u        /* geometric waits, geom_wait :147-148 -> wait.txt          */
#define FC_DIAG_HIST 0x2u        /* per-chain histograms of |cut| and |B| over yields        */
#define FC_DIAG_EDGES 0x4u       /* per-edge cut_times, :383-384                             */
#define FC_DIAG_FLIPS 0x8u       /* per-node num_flips / part_sum / last_flipped, :396-400   */
#define FC_DIAG_SERIES 0x10u     /* per-chain log of accepted flips (fc_event): the rce / rbn
                                    series of :367-369 in run-length form; feeds
                                    fc_run_autocorr and the slope / angle series (:371-392)  */
#define FC_DIAG_FLIPS_EXACT 0x20u /* the corrected companions of FC_DIAG_FLIPS (SURVEY App. A.6
                                    quirks 1-2): accepted flips per node, the time integral of
                                    each node's label over all yields, and the yield of its last
                                    accepted flip -- fc_run_read_flips_exact                   */

/* fc_params.accept: the accept callable (k = 2).  The variants are the reference's
 * alternatives, built but unused by its sweeps.                           */
#define FC_ACCEPT_CUT 0          /* cut_accept: random() < base ** (cut - cut'), :171-179     */
#define FC_ACCEPT_UNIFORM 1      /* uniform_accept: 1 if its constraints hold, :159-165        */
#define FC_ACCEPT_ANNEAL 2       /* annealing_cut_accept_backwards: random() <
                                    base ** (beta (cut - cut')) * |B'| / |B|, :81-110          */

/* Constraint sets (fc_params.con_valid / con_accept).  A constraint in con_valid is a
 * Validator member: a proposal failing it is re-drawn (no step).  One in con_accept is
 * tested inside the accept callable: failing it rejects the step (the state re-yields).  */
#define FC_CON_CONTIG 0x1u       /* single_flip_contiguous                                  */
#define FC_CON_POP 0x2u          /* within_percent_of_ideal_population (pop_lo / pop_hi)   */
#define FC_CON_BOUNDARY 0x4u     /* boundary_condition, :43-52: both districts keep a node of
                                    the outer face (the reference's boundary_node set)      */
#define FC_CON_FIXED 0x8u        /* fixed_endpoints, :39-40: pinned edges stay cut; passed as
                                    the pinned edges' endpoints (`frozen`), which may not flip */
#define FC_CON_EMPTY 0x100u      /* con_valid: an empty Validator (0 selects CONTIG | POP)   */

/* fc_params.flags */
#define FC_FLAG_FORCE_BFS 0x1u   /* resolve every multi-run contiguity case by device BFS   */
#define FC_FLAG_SERIES_TWO_PASS 0x2u /* fc_run_frame_series_changes: the two-pass form (count, then
                                    write at the offsets) instead of one staged pass -- the form a
                                    run whose staging exceeds a tenth of free device memory takes;
                                    same output (a cross-check)                                 */
#define FC_FLAG_TALLY_LOG_SMALL 0x4u /* k = 2 full diagnostics: a 64-entry tally log per chain, so
                                    chains fill it and apply the rest of a launch's tallies with
                                    atomics -- the path a device short of memory takes; same
                                    output (a cross-check)                                      */
#define FC_FLAG_NB_PAIRS 0x8u    /* k > 2 PAIR runs: |b_nodes| (stats nb / sum_nb, the |B| histogram,
                                    geom_wait's p = |b_nodes| / (N^k - 1)) counts the (node,
                                    district) pairs of the pair updater b_nodes (:151-153), which a
                                    k > 2 driver running slow_reversible_propose (:117-130)
                                    registers as "b_nodes", instead of the nodes of b_nodes_bi
                                    (:155-156).  The histogram and log1mp then have
                                    fc_run_nb_width entries; no-op for k = 2.  Such runs commit
                                    one flip at a time (tune_multi_flip has no effect)           */

typedef struct fc_graph fc_graph;
typedef struct fc_run fc_run;

typedef struct fc_graph_info {
    int32_t n_nodes;
    int32_t n_edges;
    int32_t ring_max;     /* entries per node record (8 or 16)                            */
    int32_t max_degree;
    int32_t n_exact;      /* nodes whose local contiguity rule is exact (k = 2)          */
    int32_t n_gamma;      /* nodes on the outer face                                      */
    int32_t planar;       /* positions given and no two edges cross                       */
    int32_t outer_simple; /* outer face boundary is a simple cycle                        */
} fc_graph_info;

typedef struct fc_params {
    uint32_t struct_size;      /* sizeof(fc_params) as the caller compiled it (fc_params_init) */
    uint32_t abi_version;      /* FC_ABI_VERSION as the caller compiled it                  */
    int32_t k;                 /* districts: 2 (BI_SIGN or PAIR) or 3..32 (PAIR)            */
    int32_t proposal;          /* FC_PROPOSE_*                                              */
    double base;               /* cut_accept base when `bases` is NULL (:171-179, :279-280) */
    int64_t pop_lo, pop_hi;    /* inclusive integer bounds equivalent to
                                  within_percent_of_ideal_population (:319); every chain's
                                  unless chain_pop_bounds is given                          */
    uint64_t seed;             /* Philox key (DESIGN.md "Random stream")                    */
    uint32_t chain_id_offset;  /* global id of local chain 0 (multi-GPU sharding)           */
    uint32_t diag_mask;        /* FC_DIAG_*                                                 */
    uint32_t flags;            /* FC_FLAG_*                                                 */
    int32_t device;            /* HIP device ordinal                                        */
    int32_t trace_chains;      /* chains 0..trace_chains-1 record per-proposal traces      */
    int64_t trace_cap;         /* records per traced chain                                  */
    const int32_t *labels;     /* [k] reference district labels (e.g. -1, 1); NULL = 0..k-1 */
    const double *log1mp;      /* [n+1] log(1 - b/(N^k - 1)) ([fc_run_nb_width] with
                                  FC_FLAG_NB_PAIRS); NULL = computed in double               */
    int32_t wmax;              /* PAIR: district slots per node draw (<= 0: min(max deg, k-1)) */
    int32_t hit_lo, hit_hi;    /* hitting time: first yield with hit_lo <= |cut| <= hit_hi
                                  (hit_lo > hit_hi: off)                                     */
    int64_t event_cap;         /* FC_DIAG_SERIES: events kept per chain per series window    */
    /* accept / constraint variants (k = 2; all zero = Validator([single_flip_contiguous,
       popbound]) + cut_accept, the reference's configuration)                               */
    int32_t accept;            /* FC_ACCEPT_*                                                */
    uint32_t con_valid;        /* FC_CON_* in the Validator (0 = CONTIG | POP)               */
    uint32_t con_accept;       /* FC_CON_* tested by the accept callable                      */
    double beta;               /* FC_ACCEPT_ANNEAL exponent factor (the reference: 5)       */
    const int32_t *frozen;     /* FC_CON_FIXED: [n_frozen] endpoints of the pinned edges    */
    int32_t n_frozen;
    /* FC_PROPOSE_RECOM: recom(pop_target, epsilon, node_repeats) [gc-0.2]; the Validator is
       the population bound, acceptance is cut_accept with `base` (1: always_accept)        */
    double recom_pop_target;
    double recom_epsilon;
    int32_t recom_node_repeats;  /* roots tried per spanning tree (<= 0: 1)                */
    int32_t recom_max_attempts;  /* roots tried per proposal before giving up (<= 0: 10000) */
    /* Launch tuning.  Scheduling only: no trajectory, statistic or trace depends on these
     * (tests/test_parity_gpu.py::test_sec11_batch_shapes, test_pair_gpu.py::test_k4_wait_queue_lengths). 0 = the default;
     * the library reads no environment variables.                                          */
    int32_t tune_nsub;          /* draws per batch in units of 64, in {1, 2, 4}: k = 2 default 4
                                   (a window of 64 nsub draws, four node words per Philox call;
                                   band stream: rounds of 64); k > 2 default 2 (4 when the slot
                                   bound wmax exceeds 8); anything else FC_ERR_ARG              */
    int32_t tune_hit_stop;      /* rounds of 64 (k > 2, k = 2 band stream): no further round
                                   once a batch holds this many boundary hits (default 32).
                                   The k = 2 node stream has no rounds (a 64 * nsub window closed
                                   by the 64th hit): nonzero there is FC_ERR_ARG                */
    int32_t tune_par_min;       /* k = 2: segment-parallel commit from this many acceptances on
                                   (default 3; > 64 = one event at a time)                     */
    int32_t tune_wait_queue;    /* accepted states queued for their geometric wait before one
                                   full-width draw pass (default and maximum: 64 for k = 2, 32
                                   for k > 2)                                                  */
    int32_t tune_chains_per_block; /* chains (wavefronts) per workgroup: 1 (default), 2 or 4   */
    int32_t tune_prio_div[3];   /* k = 2 SIMD issue priority 1/2/3 for chains with |B| below
                                   n / div (default {2, 5, 10}); tune_prio_div[0] < 0: off      */
    float tune_prio_th[3];      /* ... and, once a chain has taken 1/16 of the launch's steps,
                                   for projected finish / previous launch's slowest above these
                                   (default {0.95, 1.0, 1.05}); tune_prio_th[0] < 0: |B| rule only */
    int32_t tune_search_waves;  /* k > 2, chains of more than 16 KB LDS whose contiguity needs the
                                   device search (no district-graph rule): 4 = one chain per
                                   256-thread workgroup, searches by the whole workgroup;
                                   1 = one-wave workgroups, wave search (default: faster on
                                   the short searches of C4 / C5)                */
    int32_t tune_deal;          /* k = 2 chain dealing: each SIMD runs one chain of every quarter
                                   of the previous launch's draws (most first) instead of the
                                   dispatcher's order; 1 = on, -1 = off (default).  Changes
                                   which wave runs which chain, never a trajectory              */
    /* Per-chain configuration.  The reference sweeps population tolerance x base x alignment
     * (grid_chain_sec11.py:182-184); with per-chain bases (fc_run_create `bases`) and bounds the
     * whole sweep is one run.                                                                   */
    const int64_t *chain_pop_bounds; /* [2 * n_chains]: chain c's inclusive (pop_lo, pop_hi), or
                                        NULL for pop_lo / pop_hi                                 */
    /* Node stream of k = 2 runs.  Both are rejection sampling of the reference's
     * random.choice(list(b_nodes)) (grid_chain_sec11.py:143), so the chain's law is the same;
     * the trajectories differ.  FC_STREAM_NODE (0): a draw picks one of all n nodes.
     * FC_STREAM_BAND: a draw picks the i-th node (ascending) of the band S = b_nodes plus their
     * neighbours, which the chain keeps lazily: after an accepted flip that puts a node outside
     * S into b_nodes, S is rebuilt from that state.  Short boundaries then waste few draws.
     * k = 2, n <= 4096, no replay tape; oracle: fr_params.stream                               */
    int32_t stream;
    int32_t tune_multi_flip;    /* k > 2 with the district-graph rule: commit several independent
                                   accepted flips per pass (0: auto = on; 1: on; -1: one at a
                                   time; 2: on with the hashed neighbour marks; 3: on with exact
                                   marks, one LDS byte per node -- on (0 / 1) takes the exact marks
                                   when they cost no residency, fc_run_kernel_name shows which).
                                   Scheduling only, like every tune_* field                    */
} fc_params;

#define FC_STREAM_NODE 0
#define FC_STREAM_BAND 1

/* Zero *p, then set struct_size / abi_version and the defaults a zeroed struct does not give:
 * k = 2, base 1, pop bounds [0, INT32_MAX], hitting-time window off.  FC_ERR_ARG when struct_size is
 * not this library's sizeof(fc_params) (the caller's header is another version).            */
int fc_params_init(fc_params *p, uint32_t struct_size);

/* Per-chain statistics.  "Yields" are the states a `for part in exp_chain` loop sees:
 * the initial state plus one per valid step; every sum runs over all yields. */
typedef struct fc_chain_stats {
    int64_t steps;        /* valid steps (MarkovChain steps after the initial yield)      */
    int64_t proposals;    /* proposals: draws that hit a boundary node                    */
    int64_t draws;        /* raw random draws                                             */
    int64_t accepted;
    int64_t inv_contig;   /* rejected by single_flip_contiguous                           */
    int64_t inv_pop;      /* rejected by the population bound                             */
    int64_t sum_cut;      /* sum over yields of |cut_edges|       (rce)                   */
    int64_t sum_nb;       /* sum over yields of |b_nodes|         (rbn)                   */
    int64_t sum_wait;     /* sum over yields of geom              (wait.txt)              */
    int64_t sum_cut2;
    int64_t sum_nb2;
    int64_t wait_cur;     /* geometric wait of the current state                          */
    int64_t bfs_calls;    /* contiguity cases resolved by device BFS                      */
    int64_t bfs_levels;
    int32_t cut;          /* current |cut_edges|                                           */
    int32_t nb;           /* current |b_nodes|                                             */
    int32_t last_flip;    /* node flipped to create the current state (-1: initial)       */
    int32_t stuck;        /* a launch hit max_draws before finishing its steps            */
    int64_t hit_time;     /* first yield index with |cut| in [hit_lo, hit_hi], -1: not yet  */
    int64_t events;       /* accepted flips in the current series window (may exceed cap) */
    int64_t series_t0;    /* yield index at which the series window starts                */
    int32_t series_cut0;  /* |cut| of that yield                                           */
    int32_t series_nb0;   /* |B| of that yield                                             */
} fc_chain_stats;

/* One accepted flip (FC_DIAG_SERIES): yield t is the first state with a[v] = target;
 * |cut| and |B| hold from yield t until the next event's t (16 B). */
typedef struct fc_event {
    int64_t t;
    uint16_t v;
    uint16_t cut;
    uint16_t nb;
    uint8_t target;
    uint8_t reserved;
} fc_event;

/* One record per proposal (trace mode), identical in layout to the oracle's. */
typedef struct fc_record {
    int64_t draw;
    int32_t v;
    int32_t flags;        /* 1 valid, 2 accepted, 4 invalid: contiguity, 8 invalid: pop   */
    int32_t cut;          /* state after this proposal                                     */
    int32_t nb;
    int64_t wait;         /* geometric wait of the yielded state (valid proposals)        */
} fc_record;

/* One ReCom proposal (trace mode, FC_PROPOSE_RECOM), identical in layout to the oracle's. */
typedef struct fc_recom_record {
    int64_t draw;
    int32_t edge;         /* cut edge chosen (canonical edge id): its two districts merge   */
    int32_t root;         /* spanning-tree root of the successful attempt                   */
    int32_t child;        /* the cut's child: subtree(child) -> district of edge's first end */
    int32_t attempts;     /* roots tried                                                     */
    int32_t flags;        /* 1 valid, 2 accepted, 8 invalid: population                      */
    int32_t cut;          /* |cut edges| after the proposal                                  */
} fc_recom_record;

/* ---- graph: replaces gerrychain Graph + the networkx lattice (:186-260) ------------ */
/* CSR adjacency (symmetric, no self loops), node populations (Tally('population'),
 * :299), optional planar positions [2n] from which the per-node link rings and the
 * exactness of the local contiguity rule are derived. */
int fc_graph_create(int32_t n, const int32_t *row_ptr, const int32_t *col_idx, const int32_t *pop,
                    const double *pos_xy, uint32_t flags, fc_graph **out);
int fc_graph_get_info(const fc_graph *g, fc_graph_info *out);
/* Canonical edge list (u < v, CSR order): the order of cut_times / cut_edges. */
int fc_graph_edges(const fc_graph *g, int32_t *eu, int32_t *ev);
/* Debug export of the rings: entries [n * ring_max] (padded with the node itself) and
 * meta [n] (bits 0-7 length, 8 exact, 9 outer-face, 16-31 neighbour mask, 32-47 link mask). */
int fc_graph_rings(const fc_graph *g, int32_t *ring, uint64_t *meta);
void fc_graph_destroy(fc_graph *g);

/* ---- run: replaces Partition(graph, assignment, updaters) + MarkovChain(...) --------- */
/* init_assign: [n_chains * n] district ids 0..k-1 (one initial plan per chain).
 * bases: [n_chains] per-chain cut_accept base, or NULL for params->base.
 * Validates every initial state like MarkovChain.__init__ (FC_ERR_INVALID_STATE) against its
 * chain's population bounds.  FC_ERR_ARG when p->struct_size != sizeof(fc_params) or
 * p->abi_version != FC_ABI_VERSION (a caller compiled against another fc_params layout). */
int fc_run_create(const fc_graph *g, const fc_params *p, int32_t n_chains, const int8_t *init_assign,
                  const double *bases, fc_run **out);
/* Advance every chain by n_steps valid steps (the reference's step semantics: invalid
 * proposals are re-drawn and not counted).  max_draws caps the draws per chain per call
 * (<= 0: 64 * 1024 * n_steps); a capped chain sets stats.stuck.  Asynchronous. */
int fc_run_steps(fc_run *r, int64_t n_steps, int64_t max_draws, void *hip_stream);
/* Replay mode: chain c reads its random words from tape[c * n_draws * 6 ...] (6 u32 per
 * draw: 4 proposal words, 2 geometric words) instead of Philox.  NULL detaches. */
int fc_run_set_tape(fc_run *r, const uint32_t *tape, int64_t n_draws);
/* Replay of the initial state's geometric wait (geom_wait :147-148, drawn by numpy for the
 * yielded initial state in the reference): chain c's wait becomes the inversion of the 53-bit
 * uniform in words[2c], words[2c + 1] (same layout as tape words 4-5) instead of the
 * purpose-2 Philox draw.  Together with a node tape this replays a
 * trajectory of the reference's own random streams bit for bit.  Only before the first
 * fc_run_steps (FC_ERR_ARG after); needs FC_DIAG_WAIT.                                     */
int fc_run_set_initial_wait(fc_run *r, const uint32_t *words);
int fc_run_sync(fc_run *r);
/* Device time of the last fc_run_steps launch, from HIP events on its stream. */
int fc_run_last_ms(fc_run *r, float *ms);
/* Device times (ms) of every fc_run_steps launch since the previous call (up to cap;
 * *n receives the count); synchronises on the last launch and resets the record. */
int fc_run_timings(fc_run *r, float *ms, int32_t cap, int32_t *n);
int fc_run_read_stats(fc_run *r, fc_chain_stats *out);
int fc_run_read_state(fc_run *r, int8_t *assign_out);
/* District populations [c * k] (Tally('population'), :299). */
int fc_run_read_pops(fc_run *r, int64_t *pops_out);
int fc_run_read_trace(fc_run *r, int32_t chain, fc_record *out, int64_t cap, int64_t *len);
/* ReCom runs: the per-proposal records of a traced chain (*len may exceed cap). */
int fc_run_read_recom_trace(fc_run *r, int32_t chain, fc_recom_record *out, int64_t cap, int64_t *len);
/* Restart every traced chain's record buffer at 0 (chunked per-step iteration). */
int fc_run_trace_reset(fc_run *r);
int fc_run_read_hist(fc_run *r, int64_t *cut_hist, int64_t *nb_hist);      /* [c*(E+1)], [c*nb_width] */
int fc_run_read_edges(fc_run *r, int64_t *cut_times);                     /* [c*E], finalised     */
/* num_flips / part_sum / last_flipped [c*n], finalised as grid_chain_sec11.py:416-418. */
int fc_run_read_flips(fc_run *r, int64_t *num_flips, int64_t *part_sum, int64_t *last_flipped);
/* FC_DIAG_FLIPS_EXACT, [c*n] each (the statistics the driver's :396-400 / :416-418 aim at,
 * without its quirks; App. A.6):
 *   flip_count[u]  = accepted flips of u (the driver's num_flips counts every yield of the state
 *                    u's flip created, because part.flips is stale on rejected steps);
 *   occupancy[u]   = sum over all yields t of labels[a_t(u)] (the driver's part_sum drops the
 *                    final segment of every node that flipped at least once);
 *   last_accept[u] = yield index of u's last accepted flip (0: never flipped).
 * FC_ERR_ARG if FC_DIAG_FLIPS_EXACT is off; ReCom runs do not keep them (FC_ERR_UNSUPPORTED at
 * fc_run_create). */
int fc_run_read_flips_exact(fc_run *r, int64_t *flip_count, int64_t *occupancy, int64_t *last_accept);
/* Rao-Blackwellised companion of wait.txt (App. A.6 quirk 3: the cached geometric sample repeats
 * on rejected steps): out[c] = sum over yields of E[geom_wait | |B|] = (N^k - 1) / |B| - 1
 * (geom_wait :147-148), from the |B| histogram.  Needs FC_DIAG_HIST (FC_ERR_ARG otherwise). */
int fc_run_read_wait_expected(fc_run *r, double *out);
/* ---- series diagnostics (FC_DIAG_SERIES): the per-yield lists rce / rbn (:367-369) ----- */
/* Events of one chain's current window (*len = events recorded, may exceed cap). */
int fc_run_read_events(fc_run *r, int32_t chain, fc_event *out, int64_t cap, int64_t *len);
/* Start a new window at the current yield (events dropped; hit_time is kept). */
int fc_run_series_reset(fc_run *r);
/* Autocorrelation of the |cut| series over the window's yields t0..steps, on the device:
 * lag_sums[c * nlags + j] = sum_t x_t x_{t + lags[j]} (exact int64), and, if acf != NULL,
 * acf[c * nlags + j] = sum_t (x_t - m)(x_{t+L} - m) / sum_t (x_t - m)^2 with m the window
 * mean (the biased sample ACF, statsmodels' acf default), formed on the host from exact
 * integer sums.  FC_ERR_ARG if a chain's event log overflowed event_cap. */
int fc_run_autocorr(fc_run *r, const int32_t *lags, int32_t nlags, int64_t *lag_sums, double *acf);
/* Frame-edge slope / angle series of chains [c0, c0 + nc) over the current window
 * (boundary_slope + the driver's loop body, grid_chain_sec11.py:55-78,371-394;
 * Frankenstein_chain.py:55-78,399-422).  k = 2 only (FC_ERR_UNSUPPORTED otherwise).
 *   frame_u/v [n_frame <= 256]: the frame edges boundary_slope can return, in the order
 *                               whose first two cut members are used;
 *   mid_xy [2 n_frame]:          their midpoints (enda / endb) in the reference's node
 *                               coordinates; (cx, cy) the angle centre ((20, 20) there).
 * Output [i * cap + j] for chain c0 + i: j = 0 the window start yield, j >= 1 the state
 * created by event j - 1 (it holds for yields event.t .. next event.t - 1); entries j >= len[i]
 * are padding and left undefined (the outputs are copied whole from a device buffer):
 *   slope (+inf when the two midpoints share x), angle = arccos(clip(cos)), n_cut = frame
 *   cut edges (< 2: slope = angle = NaN, where the reference raises IndexError).
 * len[i] = events + 1.  FC_ERR_ARG when cap is too small or a log overflowed event_cap. */
int fc_run_frame_series(fc_run *r, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *frame_u,
                        const int32_t *frame_v, const double *mid_xy, double cx, double cy, int64_t cap,
                        double *slope, double *angle, int32_t *n_cut, int64_t *len);
/* Change points of the same slope / angle series: what the reference's slope / angle plots
 * (grid_chain_sec11.py:476-484, plt.plot(slopes) / plt.plot(angles)) draw, without one entry
 * per event.  For chain c0 + i, entries offsets[i] .. offsets[i + 1] - 1 hold (t, slope,
 * angle): the values the per-yield lists (:382,394) take from yield t up to the next entry's t
 * (the last up to the current yield); the first entry is the window start, and every later one
 * is an event whose slope or angle differs (bitwise) from the previous entry's.  offsets
 * [nc + 1] is always filled; with t, slope and angle all NULL the call only sizes the output,
 * otherwise cap (entries per output array) must be >= offsets[nc] (FC_ERR_ARG, offsets still
 * filled, so a caller with buffers of a guessed size calls once and only re-calls on a miss).
 * The run keeps the device tables and outputs between calls (one call per launch of a driver
 * loop costs two kernel passes, one small round trip for the offsets and three copies).  k = 2. */
int fc_run_frame_series_changes(fc_run *r, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *frame_u,
                                const int32_t *frame_v, const double *mid_xy, double cx, double cy, int64_t cap,
                                int64_t *offsets, int64_t *t, double *slope, double *angle);
/* Page-lock (pin) a caller's host buffer for faster device-to-host copies of the readers above
 * (hipHostRegister); unregister before freeing it. */
int fc_host_register(void *ptr, int64_t bytes);
int fc_host_unregister(void *ptr);
/* ---- checkpoint / resume ---------------------------------------------------- */
/* Everything later fc_run_steps calls depend on -- every chain's assignment, foreign-neighbour
 * counts, draw counter, counters and sums, populations, acceptance thresholds, district-graph
 * tables, and the enabled per-yield accumulators (histograms, cut_times, flips, the series
 * window and event log) -- as one byte blob.  fc_run_checkpoint with buf == NULL (or cap too
 * small) stores the size in *len (FC_ERR_ARG when cap is too small).  fc_run_restore loads it
 * into a run created with the same graph and fc_params (n_chains, k, proposal, diag_mask,
 * event_cap, seed, chain_id_offset and a hash of every trajectory-determining parameter --
 * per-chain bases / thresholds and population bounds, labels, the log(1 - p) table, accept /
 * constraint settings, frozen nodes, ReCom settings -- are checked; FC_ERR_ARG otherwise); the
 * chains then continue bit for bit as if never interrupted.  Per-proposal traces are outputs: they restart empty after a restore. */
int fc_run_checkpoint(fc_run *r, void *buf, int64_t cap, int64_t *len);
int fc_run_restore(fc_run *r, const void *buf, int64_t len);
/* Name of the last launched flip-kernel instance, as rocprofv3 spells it. */
int fc_run_kernel_name(const fc_run *r, char *buf, int32_t cap);
int32_t fc_run_n_chains(const fc_run *r);
/* LDS bytes one chain's state takes on the device (one chain per wavefront; the chains a CU
 * holds at once is 160 KiB / this, or the VGPR limit) -- for sizing launches to one wave of
 * resident chains. */
int32_t fc_run_chain_lds_bytes(const fc_run *r);
/* Entries of a chain's |B| histogram row and of the log1mp table: n + 1, or with
 * FC_FLAG_NB_PAIRS (k > 2) sum_u min(deg u, k - 1) + 1, the largest pair count + 1. */
int32_t fc_run_nb_width(const fc_run *r);
/* Which paths the memory-dependent diagnostics took (outputs are the same either way):
 * the k = 2 tally log's entries per chain granted (*tally_log_cap; 0 = none, every tally by
 * global atomics) against those the last launch asked for (*tally_log_wanted: a granted size
 * below it means chains may have filled the log and applied the rest by atomics), and whether
 * the last fc_run_frame_series_changes ran one staged pass (*series_staged = 1), the two-pass
 * form (0) or none yet (-1). */
int fc_run_diag_paths(const fc_run *r, int64_t *tally_log_cap, int64_t *tally_log_wanted, int32_t *series_staged);
void fc_run_destroy(fc_run *r);

int fc_device_count(int32_t *n);
/* PCI bus id ("dddd:bb:dd.f") of HIP device `device` (hipDeviceGetPCIBusId): an N-GPU bench line
 * lists every rank's, so it shows that N distinct GPUs did the work. */
int fc_device_pci_id(int32_t device, char *buf, int32_t cap);
const char *fc_last_error(void);

/* What this library was built with (FC_BUILD_* bits; 0 = the product build).  A profiling or
 * experiment build counts phases in the kernels or was compiled with extra flags: its timings
 * are not the product's, so the Python loader refuses it unless asked (_lib.load(allow_variant)). */
#define FC_BUILD_PHASE_PROF 0x1u   /* -DFC_PHASE_PROF: per-phase s_memtime counters per chain   */
#define FC_BUILD_PHASE_SYNC 0x2u   /* -DFC_PHASE_SYNC: each stamp drains outstanding memory     */
#define FC_BUILD_VARIANT 0x4u      /* built with FC_LIB_VARIANT / FC_HIPCC_FLAGS (tools only)   */
uint32_t fc_build_flags(void);
/* Identity of the sources this library was compiled from: the hex SHA-256 of every source and
 * header plus the compiler flags, passed in by the build (flipcomplexityempirical_amd/build.py).
 * The in-tree loader rebuilds when it differs from the current sources' id (never by file
 * times), and profiles record it so counters are matched to the kernel revision they measured. */
const char *fc_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
