/*
 * flipref.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement (plain C) of the reference's
 * flip-walk step, used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * as the checker.  The product (flipcomplexityempirical_amd/) never links or calls this.
 *
 * Semantics restated (reference files under /root/reference):
 *   proposal   slow_reversible_propose_bi   grid_chain_sec11.py:132-145
 *   boundary   b_nodes_bi                   grid_chain_sec11.py:155-156
 *   accept     cut_accept                   grid_chain_sec11.py:171-179
 *   wait       geom_wait                    grid_chain_sec11.py:147-148
 *   chain      MarkovChain(..., Validator([single_flip_contiguous, popbound]), cut_accept)
 *                                           grid_chain_sec11.py:319,340-342   [gc-0.2]
 *   driver     per-yield diagnostics        grid_chain_sec11.py:365-419
 *
 * Random stream (the shared canonical spec, see DESIGN.md "Random stream"): draw d of
 * chain c uses Philox4x32-10(ctr = (lo32 d, hi32 d, c, 0), key = (lo32 seed, hi32 seed)).
 * Node = Lemire multiply-shift of word 0 over N (exact: reject low < 2^32 mod N); a draw
 * whose node is not a boundary node is not a proposal.  k = 2 node stream: word 0 of draw d is
 * instead word d mod 4 of Philox(ctr = (lo32 q, hi32 q, c, 3)), q = d / 4 (four draws' node
 * words per call; words 1-3 stay the draw's own).  Band stream (FR_STREAM_BAND): the
 * same map over |S| picks the i-th node of the band S in ascending order instead.  Acceptance U53 = CPython random()
 * from words (1, 2).  The geometric wait of the state created by draw d uses purpose 1,
 * the initial state's purpose 2 at d = 0; U53 from words (0, 1).
 * A tape (6 u32 per draw: the 4 proposal words then the 2 geometric words) may replace
 * Philox -- the replay mode; the initial state's wait still comes from Philox purpose 2.
 *
 * Parity pins: tests/test_oracle_golden.py (known answers of the reference's start plans,
 * the 174 decoded end-state artifacts, the 174 wait.txt sums) -- see DESIGN.md.
 */
#ifndef FLIPREF_H
#define FLIPREF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fr_record {
    int64_t draw;   /* draw index of this proposal                          */
    int32_t v;      /* proposed node (canonical index)                      */
    int32_t flags;  /* 1 valid, 2 accepted, 4 invalid: contiguity, 8 invalid: population;
                       bits 8-15: target district                                  */
    int32_t cut;    /* |cut edges| of the state after this proposal           */
    int32_t nb;     /* |boundary nodes| after this proposal                   */
    int64_t wait;   /* geometric wait of the yielded state (valid proposals) */
} fr_record;

typedef struct fr_stats {
    int64_t steps;       /* valid proposals = yields after the initial one         */
    int64_t proposals;   /* draws that hit a boundary node                         */
    int64_t draws;       /* raw draws                                              */
    int64_t accepted;
    int64_t inv_contig;
    int64_t inv_pop;
    int64_t sum_cut;     /* sums over all yields t = 0..steps (initial included)   */
    int64_t sum_nb;
    int64_t sum_wait;    /* == sum(waits) written to wait.txt                      */
    double  sum_cut2;
    double  sum_nb2;
    int32_t cut;         /* current state                                          */
    int32_t nb;
    int64_t wait0;       /* geometric wait of the initial state                    */
    int64_t wait_cur;    /* geometric wait of the current state                    */
    int32_t last_flip;   /* node flipped to create the current state, -1 for S0    */
    int32_t stuck;       /* 1 if max_draws was reached before n_steps              */
} fr_stats;

typedef struct fr_params {
    int32_t n;                 /* nodes                                            */
    const int32_t *row_ptr;    /* CSR [n+1]                                        */
    const int32_t *col_idx;    /* CSR [2E]                                         */
    const int32_t *pop;        /* [n] node populations                             */
    int32_t k;                 /* districts (k == 2: BI_SIGN proposal)             */
    const int32_t *labels;     /* [k] reference labels (e.g. -1, +1) for part_sum  */
    double base;               /* cut_accept base                                  */
    int64_t pop_lo, pop_hi;    /* inclusive integer population bounds              */
    uint64_t seed;
    uint32_t chain_id;
    const uint32_t *tape;      /* NULL => Philox; else 6 words per draw            */
    int64_t tape_draws;
    int64_t n_steps;           /* valid steps to advance                           */
    int64_t max_draws;         /* stuck cap (<=0: unlimited)                       */
    const double *log1mp;      /* [n+1] log(1-|B|/(N^k-1)); NULL => waits are 0    */
    int32_t proposal;          /* FR_PROPOSE_BI_SIGN (k == 2) or FR_PROPOSE_PAIR   */
    int32_t wmax;              /* PAIR slot bound: > 0 a fixed count (>= every node's
                                  foreign districts); <= 0 the canonical dynamic bound
                                  = the state's largest foreign-district count      */
    /* accept / constraint variants (grid_chain_sec11.py:39-52,81-110,159-165); zero =
     * Validator([single_flip_contiguous, popbound]) + cut_accept                           */
    int32_t accept;            /* FR_ACCEPT_*                                      */
    uint32_t con_valid;        /* FR_CON_* in the Validator (0: CONTIG | POP)      */
    uint32_t con_accept;       /* FR_CON_* tested inside the accept callable       */
    double beta;               /* annealing exponent factor                        */
    const uint8_t *boundary;   /* [n] boundary_node flags (boundary_condition)     */
    const int32_t *pinned;     /* [2 n_pinned] edges fixed_endpoints keeps cut     */
    int32_t n_pinned;
    /* node-tape replay: the two words of the initial state's geometric
     * wait (numpy's draw in the reference, geom_wait :147-148); NULL = Philox purpose 2   */
    const uint32_t *wait0_words;
    /* node stream (k = 2 BI_SIGN): FR_STREAM_NODE draws the node uniformly over all N nodes;
     * FR_STREAM_BAND uniformly over the band S, a superset of b_nodes kept lazily: S = b_nodes
     * plus their neighbours, recomputed after an accepted flip only when a node enters b_nodes
     * outside S.  Either is rejection sampling of random.choice(b_nodes)   */
    int32_t stream;
    /* |b_nodes| counted as the (node, district) pairs of the pair updater b_nodes
     * (grid_chain_sec11.py:151-153) instead of the nodes of b_nodes_bi (:155-156): what
     * len(partition["b_nodes"]) is in a k > 2 driver that runs slow_reversible_propose (:117-130),
     * in stats.nb, sum_nb, the |B| histogram ([nb_max + 1], nb_max = sum_u min(deg u, k - 1)) and
     * geom_wait's p (:147-148, log1mp then [nb_max + 1]).  With k = 2 both counts coincide. */
    int32_t nb_pairs;
} fr_params;

#define FR_STREAM_NODE 0
#define FR_STREAM_BAND 1

#define FR_ACCEPT_CUT 0        /* cut_accept                          :171-179 */
#define FR_ACCEPT_UNIFORM 1    /* uniform_accept                      :159-165 */
#define FR_ACCEPT_ANNEAL 2     /* annealing_cut_accept_backwards      :81-110  */
#define FR_CON_CONTIG 1u       /* single_flip_contiguous                       */
#define FR_CON_POP 2u          /* within_percent_of_ideal_population           */
#define FR_CON_BOUNDARY 4u     /* boundary_condition                  :43-52   */
#define FR_CON_FIXED 8u        /* fixed_endpoints                     :39-40   */
#define FR_CON_EMPTY 0x100u    /* con_valid: an empty Validator                */

#define FR_PROPOSE_BI_SIGN 0   /* slow_reversible_propose_bi, grid_chain_sec11.py:132-145 */
#define FR_PROPOSE_PAIR 1      /* slow_reversible_propose,    grid_chain_sec11.py:117-130 */

typedef struct fr_outputs {
    fr_record *trace; int64_t trace_cap; int64_t trace_len;   /* nullable trace      */
    int8_t *final_assign;                                     /* [n]                 */
    int64_t *cut_hist;                                        /* [E+1] nullable      */
    int64_t *nb_hist;                                         /* [n+1] nullable ([nb_max+1]
                                                                 with nb_pairs)      */
    int64_t *cut_times;                                       /* [E]   nullable      */
    int64_t *num_flips, *part_sum, *last_flipped;             /* [n]   nullable      */
    /* corrected companions, [n] nullable together:
     * accepted flips, sum over yields of labels[a_t], yield of the last accepted flip  */
    int64_t *flip_count, *occupancy, *last_accept;
} fr_outputs;

/* 0 ok; -1 initial state invalid (ValueError in MarkovChain.__init__); -2 bad args;
 * 1 stuck (max_draws reached).  init_assign holds district ids 0..k-1. */
int fr_run(const fr_params *p, const int8_t *init_assign, fr_stats *st, fr_outputs *out);

/* Reference validity checks on a full assignment (gerrychain contiguous() + Bounds). */
int fr_districts_contiguous(int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                            int32_t k, const int8_t *assign);
/* single_flip_contiguous restated: flipping v out of its district keeps it connected. */
int fr_flip_contiguous(int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                       const int8_t *assign, int32_t v);

void fr_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
