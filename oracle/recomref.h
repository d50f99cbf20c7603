/*
 * recomref.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement (plain C) of the ReCom tree
 * proposal the reference builds beside its flip chain (grid_chain_sec11.py:328-335:
 * partial(recom, pop_col="population", pop_target=ideal_population, epsilon=0.05,
 * node_repeats=1)), driven by gerrychain 0.2's MarkovChain loop [gc-0.2].  Used by tests/
 * as the checker of the HIP ReCom kernel; the product never links or calls it.
 *
 * gerrychain 0.2 (not vendored in the reference) restated:
 *   recom:  edge = choice(cut_edges); parts = (a[edge[0]], a[edge[1]]);
 *           subset = bipartition_tree(subgraph of the two parts, pop_target, epsilon,
 *           node_repeats); subset -> parts[0], the rest -> parts[1]
 *   bipartition_tree: random spanning tree (random edge weights, maximum spanning tree),
 *           root = choice(nodes of tree degree > 1), subtree populations from the root,
 *           cuts = tree edges (child, parent) with |pop(subtree(child)) - pop_target| <
 *           epsilon * pop_target; none -> new root (same tree) until node_repeats roots,
 *           then a new tree; subset = choice(cuts).subtree
 * Canonical random stream (the parity spec shared with the device): proposal
 * draw d of chain c uses Philox4x32-10(ctr = (lo d, hi d, c, 0)): cut edge = cut edges in
 * edge-id order, index mulhi64((x3:x0), |cut|); acceptance U53(x1, x2).  Tree i of the
 * draw: key = (y1:y0) of Philox(d, c, 0x80000000 | i); edge e weighs
 * splitmix64(key + e) >> 32, ties to the lower edge id.  Attempt t (root / cut choice):
 * Philox(d, c, 0x40000000 | t): root index mulhi64((y1:y0), #roots), cut index
 * mulhi64((y3:y2), #cuts), both over ascending node ids.
 */
#ifndef RECOMREF_H
#define RECOMREF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rr_params {
    int32_t n;
    const int32_t *row_ptr, *col_idx, *pop;
    int32_t k;
    double pop_target;        /* recom pop_target (the ideal population)            */
    double epsilon;           /* recom epsilon                                      */
    int32_t node_repeats;     /* roots tried per spanning tree                      */
    int32_t max_attempts;     /* give up (stuck) after this many attempts per draw  */
    int64_t pop_lo, pop_hi;   /* Validator population bound (inclusive integers)    */
    double base;              /* cut_accept base (1: every valid step accepted)     */
    uint64_t seed;
    uint32_t chain_id;
    int64_t n_steps;
    int64_t max_draws;
} rr_params;

typedef struct rr_stats {
    int64_t steps, proposals, accepted, inv_pop, attempts, trees;
    int64_t sum_cut, sum_nb;
    int32_t cut, nb, stuck, pad;
} rr_stats;

typedef struct rr_record {
    int64_t draw;
    int32_t edge;     /* chosen cut edge id                                    */
    int32_t root;
    int32_t child;    /* the cut's child node (its subtree goes to parts[0])   */
    int32_t attempts; /* roots tried for this draw                             */
    int32_t flags;    /* 1 valid, 2 accepted, 8 invalid: population            */
    int32_t cut;      /* |cut edges| after the proposal                        */
} rr_record;

/* 0 ok, 1 stuck, -1 invalid initial state, -2 bad arguments. */
int rr_run(const rr_params *p, const int8_t *init_assign, rr_stats *st, int8_t *final_assign, rr_record *trace,
           int64_t trace_cap, int64_t *trace_len);

#ifdef __cplusplus
}
#endif
#endif
