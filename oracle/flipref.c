/*
 * flipref.c -- TEST INFRASTRUCTURE ONLY (see flipref.h).  A deliberately plain CPU
 * restatement of the reference flip chain: every per-step quantity is recomputed the
 * obvious way (BFS contiguity, neighbour scans, per-yield loops), mirroring the
 * reference's own per-step work, so that it can serve as the checker for the HIP path.
 */
#include "flipref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------- Philox4x32-10 (Salmon et al., SC'11; Random123 constants) -------- */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void fr_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* CPython random.random(): two 32-bit words a, b (Lib/random.py / _randommodule.c). */
static double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

/* ---------------- chain context ---------------------------------------------------- */
typedef struct {
    const fr_params *p;
    int8_t *a;
    int64_t *pops;
    int32_t *stamp;     /* BFS visited stamps */
    int32_t stamp_id;
    int32_t *queue;
    int32_t cut, nb;
    int32_t n_edges;
    int32_t *eu, *ev;   /* canonical edges (u < v, CSR order) */
} ctx_t;

/* number of distinct foreign districts among u's neighbours (the PAIR slots of u) */
static int32_t n_foreign(const ctx_t *c, int32_t u) {
    const fr_params *p = c->p;
    uint64_t dm = 0;
    for (int32_t j = p->row_ptr[u]; j < p->row_ptr[u + 1]; ++j) {
        const int8_t aw = c->a[p->col_idx[j]];
        if (aw != c->a[u]) dm |= 1ull << aw;
    }
    return (int32_t)__builtin_popcountll(dm);
}

static int in_boundary(const ctx_t *c, int32_t u) {
    const fr_params *p = c->p;
    for (int32_t j = p->row_ptr[u]; j < p->row_ptr[u + 1]; ++j)
        if (c->a[p->col_idx[j]] != c->a[u]) return 1;
    return 0;
}

/* u's share of |b_nodes|: 1 if u is a boundary node (b_nodes_bi, :155-156), or with
 * nb_pairs its number of (u, district) pairs in b_nodes (:151-153) */
static int32_t nb_of(const ctx_t *c, int32_t u) {
    return c->p->nb_pairs ? n_foreign(c, u) : in_boundary(c, u);
}

/* single_flip_contiguous [gc-0.2] restated: old_nbrs = neighbours still in v's old
 * district; empty => invalid; else every old neighbour must reach one fixed old neighbour
 * through the old district with v removed (the canonical stream omits the random.choice
 * of the start neighbour: the outcome does not depend on it). */
static int flip_contiguous_ctx(ctx_t *c, int32_t v) {
    const fr_params *p = c->p;
    const int8_t A = c->a[v];
    int32_t n_old = 0, start = -1;
    for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1]; ++j) {
        int32_t w = p->col_idx[j];
        if (c->a[w] == A) { if (start < 0) start = w; ++n_old; }
    }
    if (n_old == 0) return 0;
    if (n_old == 1) return 1;
    if (++c->stamp_id == 0x7fffffff) { memset(c->stamp, 0, sizeof(int32_t) * (size_t)p->n); c->stamp_id = 1; }
    const int32_t sid = c->stamp_id;
    int32_t head = 0, tail = 0, reached = 0;
    c->stamp[v] = sid;       /* v is removed from the district */
    c->stamp[start] = sid;
    c->queue[tail++] = start;
    /* BFS over A - v from one old neighbour; a dequeued node adjacent to v is an old
       neighbour reached.  All reached <=> every old neighbour is connected to `start`
       (the Dijkstra calls of single_flip_contiguous [gc-0.2] ask exactly this), so the
       search may stop there; otherwise it exhausts start's component. */
    while (head < tail) {
        int32_t u = c->queue[head++];
        for (int32_t j = p->row_ptr[u]; j < p->row_ptr[u + 1]; ++j) {
            int32_t w = p->col_idx[j];
            if (w == v) {
                if (++reached == n_old) return 1;
                continue;
            }
            if (c->a[w] != A || c->stamp[w] == sid) continue;
            c->stamp[w] = sid;
            c->queue[tail++] = w;
        }
    }
    return 0;
}

int fr_flip_contiguous(int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                       const int8_t *assign, int32_t v) {
    fr_params p; memset(&p, 0, sizeof p);
    p.n = n; p.row_ptr = row_ptr; p.col_idx = col_idx;
    ctx_t c; memset(&c, 0, sizeof c);
    c.p = &p;
    c.a = (int8_t *)assign;
    c.stamp = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    c.queue = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int r = (c.stamp && c.queue) ? flip_contiguous_ctx(&c, v) : -2;
    free(c.stamp); free(c.queue);
    return r;
}

/* gerrychain contiguous(): every district induces a connected subgraph. */
int fr_districts_contiguous(int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                            int32_t k, const int8_t *assign) {
    int32_t *seen = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    int32_t *q = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    if (!seen || !q) { free(seen); free(q); return -2; }
    int ok = 1;
    for (int32_t d = 0; d < k && ok; ++d) {
        int32_t start = -1, size = 0;
        for (int32_t u = 0; u < n; ++u) if (assign[u] == d) { if (start < 0) start = u; ++size; }
        if (start < 0) continue; /* empty district: gerrychain would not list it */
        int32_t head = 0, tail = 0;
        seen[start] = 1; q[tail++] = start;
        while (head < tail) {
            int32_t u = q[head++];
            for (int32_t j = row_ptr[u]; j < row_ptr[u + 1]; ++j) {
                int32_t w = col_idx[j];
                if (assign[w] == d && !seen[w]) { seen[w] = 1; q[tail++] = w; }
            }
        }
        if (tail != size) ok = 0;
    }
    free(seen); free(q);
    return ok;
}

static void draw_words(const fr_params *p, int64_t d, uint32_t purpose, uint32_t w[4]) {
    if (purpose == 2 && p->wait0_words) {  /* replayed initial-state wait */
        w[0] = p->wait0_words[0]; w[1] = p->wait0_words[1]; w[2] = 0; w[3] = 0;
        return;
    }
    if (p->tape && purpose != 2) {   /* a tape's initial-state wait is Philox unless wait0_words */
        const uint32_t *t = p->tape + 6 * d;
        if (purpose == 0) { w[0] = t[0]; w[1] = t[1]; w[2] = t[2]; w[3] = t[3]; }
        else { w[0] = t[4]; w[1] = t[5]; w[2] = 0; w[3] = 0; }
        return;
    }
    uint32_t ctr[4] = {(uint32_t)(uint64_t)d, (uint32_t)((uint64_t)d >> 32), p->chain_id, purpose};
    uint32_t key[2] = {(uint32_t)p->seed, (uint32_t)(p->seed >> 32)};
    fr_philox4x32_10(ctr, key, w);
    if (purpose == 0 && p->k == 2 && p->stream == FR_STREAM_NODE) {
        /* k = 2 node stream: the node word of draw d is word d mod 4 of the
         * purpose-3 call at counter d / 4 (four draws' node words per call); words 1-3 stay the
         * draw's own (the device makes that call for the boundary hits only). */
        const uint64_t q = (uint64_t)d >> 2;
        uint32_t cq[4] = {(uint32_t)q, (uint32_t)(q >> 32), p->chain_id, 3u}, wq[4];
        fr_philox4x32_10(cq, key, wq);
        w[0] = wq[d & 3];
    }
}

/* geom_wait (grid_chain_sec11.py:147-148): int(np.random.geometric(p, 1)) - 1 with the
 * legacy inversion ceil(log(1 - U) / log(1 - p)), U = legacy random_sample(). */
static int64_t geom_wait(const fr_params *p, int64_t d, uint32_t purpose, int32_t nb) {
    if (!p->log1mp) return 0;
    uint32_t w[4];
    draw_words(p, d, purpose, w);
    double U = u53(w[0], w[1]);
    double q = log(1.0 - U) / p->log1mp[nb];
    if (!(fabs(q) < 4611686018427387904.0)) return (int64_t)4611686018427387904LL; /* saturate: 2^62 */
    return (int64_t)ceil(q) - 1;
}

/* One driver-loop iteration (grid_chain_sec11.py:366-402) for the yielded state. */
static void yield_state(ctx_t *c, fr_stats *st, fr_outputs *o, int64_t t) {
    const fr_params *p = c->p;
    st->sum_cut += c->cut;
    st->sum_cut2 += (double)c->cut * (double)c->cut;
    st->sum_nb += c->nb;
    st->sum_nb2 += (double)c->nb * (double)c->nb;
    st->sum_wait += st->wait_cur;
    if (o) {
        if (o->cut_hist) o->cut_hist[c->cut] += 1;
        if (o->nb_hist) o->nb_hist[c->nb] += 1;
        if (o->cut_times)
            for (int32_t e = 0; e < c->n_edges; ++e)
                if (c->a[c->eu[e]] != c->a[c->ev[e]]) o->cut_times[e] += 1;
        /* part.flips is stale on rejected steps: the update repeats for the last accepted
         * node (grid_chain_sec11.py:396-400, App. A.6 quirk 1). */
        if (st->last_flip >= 0 && o->num_flips) {
            int32_t f = st->last_flip;
            o->part_sum[f] -= (int64_t)p->labels[(int)c->a[f]] * (t - o->last_flipped[f]);
            o->last_flipped[f] = t;
            o->num_flips[f] += 1;
        }
        if (o->occupancy)                                   /* the label's time integral  */
            for (int32_t u = 0; u < p->n; ++u) o->occupancy[u] += p->labels[(int)c->a[u]];
    }
}

/* boundary_condition (grid_chain_sec11.py:43-52) of the state with a[v] = T: some
 * boundary node lies in another district than blist[0]. */
static int boundary_ok_after(const ctx_t *c, int32_t v, int8_t T) {
    const fr_params *p = c->p;
    int32_t first = -1;
    int8_t o_part = 0;
    for (int32_t u = 0; u < p->n; ++u) {
        if (!p->boundary[u]) continue;
        const int8_t au = u == v ? T : c->a[u];
        if (first < 0) { first = u; o_part = au; continue; }
        if (au != o_part) return 1;
    }
    return 0;
}

/* fixed_endpoints (:39-40) of the state with a[v] = T: every pinned edge is cut. */
static int fixed_ok_after(const ctx_t *c, int32_t v, int8_t T) {
    const fr_params *p = c->p;
    for (int32_t i = 0; i < p->n_pinned; ++i) {
        const int32_t x = p->pinned[2 * i], y = p->pinned[2 * i + 1];
        const int8_t ax = x == v ? T : c->a[x], ay = y == v ? T : c->a[y];
        if (ax == ay) return 0;
    }
    return 1;
}

/* |b_nodes| of the state with a[v] = T, by flipping and restoring (the b_nodes of
 * partition and partition.parent in annealing_cut_accept_backwards, :82-83). */
static int32_t nb_after_flip(ctx_t *c, int32_t v, int8_t T) {
    const fr_params *p = c->p;
    int32_t before = nb_of(c, v), after;
    for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1]; ++j) before += nb_of(c, p->col_idx[j]);
    const int8_t A = c->a[v];
    c->a[v] = T;
    after = nb_of(c, v);
    for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1]; ++j) after += nb_of(c, p->col_idx[j]);
    c->a[v] = A;
    return c->nb + after - before;
}

/* Band stream: S = b_nodes and their neighbours, as an ascending node list (the rank a draw
 * selects) and a membership flag per node.  Returns |S|. */
static int32_t band_build(const ctx_t *c, uint8_t *ins, int32_t *slist) {
    const fr_params *p = c->p;
    memset(ins, 0, (size_t)p->n);
    for (int32_t u = 0; u < p->n; ++u) {
        if (!in_boundary(c, u)) continue;
        ins[u] = 1;
        for (int32_t j = p->row_ptr[u]; j < p->row_ptr[u + 1]; ++j) ins[p->col_idx[j]] = 1;
    }
    int32_t ns = 0;
    for (int32_t u = 0; u < p->n; ++u)
        if (ins[u]) slist[ns++] = u;
    return ns;
}

int fr_run(const fr_params *p, const int8_t *init_assign, fr_stats *st, fr_outputs *o) {
    if (!p || !init_assign || !st || p->n <= 0 || p->k < 2 || p->k > 64 || !p->row_ptr || !p->col_idx || !p->pop)
        return -2;
    if (p->proposal == FR_PROPOSE_BI_SIGN && p->k != 2) return -2;
    if (p->proposal != FR_PROPOSE_BI_SIGN && p->proposal != FR_PROPOSE_PAIR) return -2;
    if (p->stream != FR_STREAM_NODE && p->stream != FR_STREAM_BAND) return -2;
    if (p->stream == FR_STREAM_BAND && (p->k != 2 || p->tape)) return -2;
    if (o && o->num_flips && (!o->part_sum || !o->last_flipped || !p->labels)) return -2;
    if (o && o->occupancy && (!o->flip_count || !o->last_accept || !p->labels)) return -2;
    const int32_t n = p->n;
    memset(st, 0, sizeof *st);
    st->last_flip = -1;

    ctx_t c; memset(&c, 0, sizeof c);
    int32_t *nf = NULL, nfh[65];  /* PAIR: foreign districts per node, and their histogram */
    uint8_t *ins = NULL;          /* band stream: membership of S, and S ascending          */
    int32_t *slist = NULL, ns = 0;
    memset(nfh, 0, sizeof nfh);
    c.p = p;
    c.a = (int8_t *)malloc((size_t)n);
    c.pops = (int64_t *)calloc((size_t)p->k, sizeof(int64_t));
    c.stamp = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    c.queue = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    c.n_edges = p->row_ptr[n] / 2;
    c.eu = (int32_t *)malloc(sizeof(int32_t) * (size_t)(c.n_edges + 1));
    c.ev = (int32_t *)malloc(sizeof(int32_t) * (size_t)(c.n_edges + 1));
    int rc = 0;
    if (!c.a || !c.pops || !c.stamp || !c.queue || !c.eu || !c.ev) { rc = -2; goto done; }
    memcpy(c.a, init_assign, (size_t)n);
    {
        int32_t e = 0;
        for (int32_t u = 0; u < n; ++u)
            for (int32_t j = p->row_ptr[u]; j < p->row_ptr[u + 1]; ++j)
                if (p->col_idx[j] > u) { c.eu[e] = u; c.ev[e] = p->col_idx[j]; ++e; }
    }
    for (int32_t u = 0; u < n; ++u) {
        if (c.a[u] < 0 || c.a[u] >= p->k) { rc = -2; goto done; }
        c.pops[(int)c.a[u]] += p->pop[u];
    }
    /* MarkovChain.__init__ validates the initial state with the Validator [gc-0.2]; the
     * districts must be connected in any case (the chain keeps them so). */
    const uint32_t con_valid = p->con_valid ? p->con_valid : (FR_CON_CONTIG | FR_CON_POP);
    if ((con_valid | p->con_accept) & FR_CON_BOUNDARY && !p->boundary) { rc = -2; goto done; }
    if (con_valid & FR_CON_POP)
        for (int32_t d = 0; d < p->k; ++d)
            if (c.pops[d] < p->pop_lo || c.pops[d] > p->pop_hi) { rc = -1; goto done; }
    if (fr_districts_contiguous(n, p->row_ptr, p->col_idx, p->k, c.a) != 1) { rc = -1; goto done; }
    if ((con_valid & FR_CON_BOUNDARY) && !boundary_ok_after(&c, 0, c.a[0])) { rc = -1; goto done; }
    if ((con_valid & FR_CON_FIXED) && !fixed_ok_after(&c, 0, c.a[0])) { rc = -1; goto done; }

    for (int32_t e = 0; e < c.n_edges; ++e) c.cut += c.a[c.eu[e]] != c.a[c.ev[e]];
    int32_t nb_max = n;
    if (p->nb_pairs) {
        nb_max = 0;
        for (int32_t u = 0; u < n; ++u) {
            const int32_t dg = p->row_ptr[u + 1] - p->row_ptr[u];
            nb_max += dg < p->k - 1 ? dg : p->k - 1;
        }
    }
    for (int32_t u = 0; u < n; ++u) c.nb += nb_of(&c, u);
    if (o) {
        if (o->cut_times) memset(o->cut_times, 0, sizeof(int64_t) * (size_t)c.n_edges);
        if (o->cut_hist) memset(o->cut_hist, 0, sizeof(int64_t) * (size_t)(c.n_edges + 1));
        if (o->nb_hist) memset(o->nb_hist, 0, sizeof(int64_t) * (size_t)(nb_max + 1));
        if (o->num_flips)
            for (int32_t u = 0; u < n; ++u) {
                o->num_flips[u] = 0; o->last_flipped[u] = 0;
                o->part_sum[u] = p->labels[(int)c.a[u]];       /* grid_chain_sec11.py:219 */
            }
        if (o->occupancy)
            for (int32_t u = 0; u < n; ++u) { o->flip_count[u] = 0; o->occupancy[u] = 0; o->last_accept[u] = 0; }
        o->trace_len = 0;
    }

    st->wait0 = geom_wait(p, 0, 2, c.nb);
    st->wait_cur = st->wait0;
    yield_state(&c, st, o, 0);                                   /* yield #0 = S0 */

    const uint32_t thresh = (uint32_t)((0x100000000ull) % (uint64_t)n);
    /* PAIR: draw d is a node (word 0) and a slot r < wcap (word 3); it proposes the pair
     * (v, r-th foreign district of v) iff r < nf(v), the number of v's foreign districts.
     * Any wcap >= max_u nf(u) makes the proposal uniform over b_nodes' pairs (:151-153).
     * Canonical stream: wcap = the current state's max_u nf(u) (kept through a histogram of
     * nf), so compact states waste few slot draws; fc_params.wmax > 0 fixes it instead. */
    int32_t wcap = 1;
    const int dyn = p->proposal == FR_PROPOSE_PAIR && p->wmax <= 0;
    if (p->proposal == FR_PROPOSE_PAIR) {
        nf = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
        if (!nf) { rc = -2; goto done; }
        for (int32_t u = 0; u < n; ++u) { nf[u] = n_foreign(&c, u); nfh[nf[u]] += 1; }
        if (dyn) {
            for (int32_t j = 64; j >= 1; --j) if (nfh[j] > 0) { wcap = j; break; }
        } else {
            wcap = p->wmax;
        }
    }
    uint32_t wthresh = (uint32_t)((0x100000000ull) % (uint64_t)wcap);
    uint32_t sthresh = 0;
    if (p->stream == FR_STREAM_BAND) {
        ins = (uint8_t *)malloc((size_t)n);
        slist = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
        if (!ins || !slist) { rc = -2; goto done; }
        ns = band_build(&c, ins, slist);
        sthresh = (uint32_t)((0x100000000ull) % (uint64_t)ns);
    }
    int64_t d = 0;
    while (st->steps < p->n_steps) {
        if ((p->max_draws > 0 && st->draws >= p->max_draws) || (p->tape && d >= p->tape_draws)) {
            st->stuck = 1; rc = 1; break;
        }
        uint32_t w[4];
        draw_words(p, d, 0, w);
        const int64_t draw = d++;
        st->draws += 1;
        int32_t v;
        if (ins) {                                              /* band: i-th node of S     */
            const uint64_t m = (uint64_t)w[0] * (uint64_t)ns;
            if ((uint32_t)m < sthresh) continue;
            v = slist[m >> 32];
        } else {
            const uint64_t m = (uint64_t)w[0] * (uint64_t)n;
            if ((uint32_t)m < thresh) continue;               /* Lemire: exact uniform node */
            v = (int32_t)(m >> 32);
        }
        if (!in_boundary(&c, v)) continue;                      /* not in b_nodes_bi        */
        const int8_t A = c.a[v];
        int8_t T;
        if (p->proposal == FR_PROPOSE_BI_SIGN) {
            T = (int8_t)(1 - A);                                /* -1 * assignment (:145)   */
        } else {
            /* slow_reversible_propose (:117-130): uniform over (node, foreign district)
             * pairs = uniform node, then slot r < wmax accepted iff r < |D(v)|; D(v) in
             * ascending district order. */
            const uint64_t mw = (uint64_t)w[3] * (uint64_t)wcap;
            if ((uint32_t)mw < wthresh) continue;
            const int32_t r = (int32_t)(mw >> 32);
            uint64_t dm = 0;
            for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1]; ++j) {
                int8_t aw = c.a[p->col_idx[j]];
                if (aw != A) dm |= 1ull << aw;
            }
            int32_t cnt = 0;
            T = -1;
            for (int32_t dd = 0; dd < p->k; ++dd)
                if (dm >> dd & 1ull) { if (cnt == r) { T = (int8_t)dd; break; } ++cnt; }
            if (T < 0) continue;                                 /* slot beyond |D(v)|      */
        }
        st->proposals += 1;
        int32_t flags = 0;
        /* constraint verdicts of the proposed state (Validator order: contiguity first) */
        const int contig_ok = flip_contiguous_ctx(&c, v);
        int pop_ok = 1;
        for (int32_t dd = 0; dd < p->k; ++dd) {
            int64_t pp = c.pops[dd] - (dd == A ? p->pop[v] : 0) + (dd == T ? p->pop[v] : 0);
            if (pp < p->pop_lo || pp > p->pop_hi) { pop_ok = 0; break; }
        }
        const uint32_t all = (FR_CON_CONTIG | FR_CON_POP | FR_CON_BOUNDARY | FR_CON_FIXED) & (con_valid | p->con_accept);
        const int bnd_ok = (all & FR_CON_BOUNDARY) ? boundary_ok_after(&c, v, T) : 1;
        const int fix_ok = (all & FR_CON_FIXED) ? fixed_ok_after(&c, v, T) : 1;
#define FR_PASS(M) ((!((M) & FR_CON_CONTIG) || contig_ok) && (!((M) & FR_CON_POP) || pop_ok) && \
                    (!((M) & FR_CON_BOUNDARY) || bnd_ok) && (!((M) & FR_CON_FIXED) || fix_ok))
        if (!FR_PASS(con_valid)) {
            if ((con_valid & FR_CON_CONTIG) && !contig_ok) { st->inv_contig += 1; flags = 4; }
            else { st->inv_pop += 1; flags = 8; }
        }
        if (flags) {
            if (o && o->trace && o->trace_len < o->trace_cap) {
                fr_record *r = &o->trace[o->trace_len++];
                r->draw = draw; r->v = v; r->flags = flags | (T << 8); r->cut = c.cut; r->nb = c.nb; r->wait = 0;
            }
            continue;
        }
        /* valid step: cut_accept (grid_chain_sec11.py:171-179) */
        st->steps += 1;
        int32_t same = 0, other = 0;
        for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1]; ++j) {
            int8_t aw = c.a[p->col_idx[j]];
            same += aw == A; other += aw == T;
        }
        const int32_t delta = same - other;                    /* cut(S') - cut(S)        */
        double bound;
        if (p->accept == FR_ACCEPT_UNIFORM) {          /* uniform_accept, :159-165 */
            bound = FR_PASS(p->con_accept) ? 1.0 : 0.0;
        } else if (p->accept == FR_ACCEPT_ANNEAL) {    /* annealing_cut_accept_backwards, :81-110 */
            bound = pow(p->base, p->beta * (double)(-delta)) * ((double)nb_after_flip(&c, v, T) / (double)c.nb);
            if (!FR_PASS(p->con_accept)) bound = 0.0;
        } else {
            bound = FR_PASS(p->con_accept) ? pow(p->base, (double)(-delta)) : 0.0;
        }
#undef FR_PASS
        const double U = u53(w[1], w[2]);
        const int acc = U < bound;
        if (acc) {
            int32_t before = nb_of(&c, v), after;
            for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1]; ++j) before += nb_of(&c, p->col_idx[j]);
            c.a[v] = T;
            c.pops[A] -= p->pop[v];
            c.pops[T] += p->pop[v];
            c.cut += delta;
            after = nb_of(&c, v);
            for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1]; ++j) after += nb_of(&c, p->col_idx[j]);
            c.nb += after - before;
            st->accepted += 1;
            st->last_flip = v;
            if (nf) {  /* v's and its neighbours' foreign-district counts, and the slot bound */
                for (int32_t j = p->row_ptr[v] - 1; j < p->row_ptr[v + 1]; ++j) {
                    const int32_t u = j < p->row_ptr[v] ? v : p->col_idx[j];
                    const int32_t f = n_foreign(&c, u);
                    nfh[nf[u]] -= 1; nfh[f] += 1; nf[u] = f;
                }
                if (dyn) {
                    wcap = 1;
                    for (int32_t j = 64; j >= 1; --j) if (nfh[j] > 0) { wcap = j; break; }
                    wthresh = (uint32_t)((0x100000000ull) % (uint64_t)wcap);
                }
            }
            if (ins) {  /* a neighbour entering b_nodes outside S: S is rebuilt from this state */
                int out = 0;
                for (int32_t j = p->row_ptr[v]; j < p->row_ptr[v + 1] && !out; ++j)
                    out = !ins[p->col_idx[j]] && in_boundary(&c, p->col_idx[j]);
                if (out) {
                    ns = band_build(&c, ins, slist);
                    sthresh = (uint32_t)((0x100000000ull) % (uint64_t)ns);
                }
            }
            st->wait_cur = geom_wait(p, draw, 1, c.nb);
            if (o && o->occupancy) { o->flip_count[v] += 1; o->last_accept[v] = st->steps; }
        }
        yield_state(&c, st, o, st->steps);
        if (o && o->trace && o->trace_len < o->trace_cap) {
            fr_record *r = &o->trace[o->trace_len++];
            r->draw = draw; r->v = v; r->flags = 1 | (acc ? 2 : 0) | (T << 8); r->cut = c.cut; r->nb = c.nb;
            r->wait = st->wait_cur;
        }
    }
    st->cut = c.cut;
    st->nb = c.nb;
    if (o) {
        if (o->final_assign) memcpy(o->final_assign, c.a, (size_t)n);
        /* finalisation, grid_chain_sec11.py:416-418 (t = number of yields) */
        if (o->num_flips) {
            const int64_t T = st->steps + 1;
            for (int32_t u = 0; u < n; ++u)
                if (o->last_flipped[u] == 0) o->part_sum[u] = T * p->labels[(int)c.a[u]];
        }
    }
done:
    free(nf);
    free(ins); free(slist);
    free(c.a); free(c.pops); free(c.stamp); free(c.queue); free(c.eu); free(c.ev);
    return rc;
}
