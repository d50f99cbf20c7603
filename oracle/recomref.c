/*
 * recomref.c -- TEST INFRASTRUCTURE ONLY (see recomref.h).  Plain restatement of the
 * ReCom proposal and gerrychain's chain loop: Kruskal maximum spanning tree, DFS subtree
 * populations, linear scans -- no cleverness, so that it can check the HIP kernel.
 */
#include "recomref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "flipref.h"

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t mulhi64(uint64_t r, uint64_t n) { return (uint64_t)(((unsigned __int128)r * n) >> 64); }

static double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

static void words(const rr_params *p, uint64_t d, uint32_t purpose, uint32_t w[4]) {
    const uint32_t ctr[4] = {(uint32_t)d, (uint32_t)(d >> 32), p->chain_id, purpose};
    const uint32_t key[2] = {(uint32_t)p->seed, (uint32_t)(p->seed >> 32)};
    fr_philox4x32_10(ctr, key, w);
}

typedef struct { uint32_t w; int32_t e; } wedge;

static int cmp_wedge(const void *x, const void *y) {  /* weight descending, then edge id ascending */
    const wedge *a = (const wedge *)x, *b = (const wedge *)y;
    if (a->w != b->w) return a->w > b->w ? -1 : 1;
    return a->e < b->e ? -1 : (a->e > b->e);
}

static int32_t uf_find(int32_t *par, int32_t x) {
    while (par[x] != x) { par[x] = par[par[x]]; x = par[x]; }
    return x;
}

int rr_run(const rr_params *p, const int8_t *init, rr_stats *st, int8_t *final_assign, rr_record *trace,
           int64_t trace_cap, int64_t *trace_len) {
    if (!p || !init || !st || p->n <= 1 || p->k < 2 || p->node_repeats < 1) return -2;
    const int32_t n = p->n;
    int32_t E = p->row_ptr[n] / 2;
    memset(st, 0, sizeof *st);
    if (trace_len) *trace_len = 0;
    int32_t *eu = malloc(sizeof(int32_t) * E), *ev = malloc(sizeof(int32_t) * E);
    int8_t *a = malloc(n), *na = malloc(n);
    int32_t *uf = malloc(sizeof(int32_t) * n), *tdeg = malloc(sizeof(int32_t) * n);
    int32_t *tadj = malloc(sizeof(int32_t) * 2 * n), *toff = malloc(sizeof(int32_t) * (n + 1));
    int32_t *parent = malloc(sizeof(int32_t) * n), *stack = malloc(sizeof(int32_t) * n);
    int32_t *orderv = malloc(sizeof(int32_t) * 2 * n);
    int64_t *spop = malloc(sizeof(int64_t) * n);
    int8_t *inM = malloc(n), *mark = malloc(n);
    wedge *we = malloc(sizeof(wedge) * (E + 1));
    int64_t *pops = calloc((size_t)p->k, sizeof(int64_t));
    int rc = 0;
    if (!eu || !ev || !a || !na || !uf || !tdeg || !tadj || !toff || !parent || !stack || !orderv || !spop || !inM ||
        !mark || !we || !pops) { rc = -2; goto done; }
    {
        int32_t e = 0;
        for (int32_t u = 0; u < n; ++u)
            for (int32_t j = p->row_ptr[u]; j < p->row_ptr[u + 1]; ++j)
                if (p->col_idx[j] > u) { eu[e] = u; ev[e] = p->col_idx[j]; ++e; }
    }
    memcpy(a, init, (size_t)n);
    for (int32_t u = 0; u < n; ++u) {
        if (a[u] < 0 || a[u] >= p->k) { rc = -2; goto done; }
        pops[a[u]] += p->pop[u];
    }
    for (int32_t d = 0; d < p->k; ++d)
        if (pops[d] < p->pop_lo || pops[d] > p->pop_hi) { rc = -1; goto done; }
    if (fr_districts_contiguous(n, p->row_ptr, p->col_idx, p->k, a) != 1) { rc = -1; goto done; }

#define CUT_OF(arr, out)                                                   \
    do {                                                                   \
        int32_t c_ = 0;                                                    \
        for (int32_t e_ = 0; e_ < E; ++e_) c_ += (arr)[eu[e_]] != (arr)[ev[e_]]; \
        (out) = c_;                                                        \
    } while (0)
#define NB_OF(arr, out)                                                              \
    do {                                                                             \
        int32_t b_ = 0;                                                              \
        for (int32_t u_ = 0; u_ < n; ++u_) {                                         \
            int f_ = 0;                                                              \
            for (int32_t j_ = p->row_ptr[u_]; j_ < p->row_ptr[u_ + 1]; ++j_)          \
                f_ |= (arr)[p->col_idx[j_]] != (arr)[u_];                            \
            b_ += f_;                                                                \
        }                                                                            \
        (out) = b_;                                                                  \
    } while (0)
    CUT_OF(a, st->cut);
    NB_OF(a, st->nb);
    st->sum_cut = st->cut;  /* yield #0 */
    st->sum_nb = st->nb;

    uint64_t d = 0;
    while (st->steps < p->n_steps) {
        if (p->max_draws > 0 && (int64_t)d >= p->max_draws) { st->stuck = 1; rc = 1; break; }
        uint32_t w[4];
        words(p, d, 0, w);
        const uint64_t draw = d++;
        /* recom: edge = random.choice(tuple(partition["cut_edges"])) */
        const uint64_t kk = mulhi64(((uint64_t)w[3] << 32) | w[0], (uint64_t)st->cut);
        int32_t e_sel = -1;
        for (int32_t e = 0, c = 0; e < E; ++e)
            if (a[eu[e]] != a[ev[e]]) { if ((uint64_t)c == kk) { e_sel = e; break; } ++c; }
        const int8_t d0 = a[eu[e_sel]], d1 = a[ev[e_sel]];
        int64_t popM = 0;
        for (int32_t u = 0; u < n; ++u) {
            inM[u] = a[u] == d0 || a[u] == d1;
            if (inM[u]) popM += p->pop[u];
        }
        st->proposals += 1;
        /* bipartition_tree */
        int32_t root = -1, child = -1, attempts = 0, tree = -1;
        for (;;) {
            if (attempts >= p->max_attempts) break;
            const int32_t t = attempts++;
            st->attempts += 1;
            if (t / p->node_repeats != tree) {  /* random_spanning_tree: max spanning tree of random weights */
                tree = t / p->node_repeats;
                st->trees += 1;
                uint32_t kw[4];
                words(p, draw, 0x80000000u | (uint32_t)tree, kw);
                const uint64_t key = ((uint64_t)kw[1] << 32) | kw[0];
                int32_t m = 0;
                for (int32_t e = 0; e < E; ++e)
                    if (inM[eu[e]] && inM[ev[e]]) { we[m].w = (uint32_t)(splitmix64(key + (uint64_t)e) >> 32); we[m].e = e; ++m; }
                qsort(we, (size_t)m, sizeof(wedge), cmp_wedge);
                for (int32_t u = 0; u < n; ++u) { uf[u] = u; tdeg[u] = 0; }
                int32_t nt = 0;
                for (int32_t i = 0; i < m; ++i) {
                    const int32_t x = uf_find(uf, eu[we[i].e]), y = uf_find(uf, ev[we[i].e]);
                    if (x == y) continue;
                    uf[x] = y;
                    tadj[2 * nt] = eu[we[i].e];
                    tadj[2 * nt + 1] = ev[we[i].e];
                    tdeg[eu[we[i].e]]++;
                    tdeg[ev[we[i].e]]++;
                    ++nt;
                }
                /* tree adjacency lists (toff / stack reused as the flat list) */
                memset(toff, 0, sizeof(int32_t) * (size_t)(n + 1));
                for (int32_t u = 0; u < n; ++u) toff[u + 1] = toff[u] + tdeg[u];
                for (int32_t u = 0; u < n; ++u) parent[u] = toff[u];  /* fill cursor */
                for (int32_t i = 0; i < nt; ++i) {
                    const int32_t x = tadj[2 * i], y = tadj[2 * i + 1];
                    orderv[parent[x]++] = y;
                    orderv[parent[y]++] = x;
                }
                memcpy(tadj, orderv, sizeof(int32_t) * (size_t)toff[n]);
            }
            uint32_t cw[4];
            words(p, draw, 0x40000000u | (uint32_t)t, cw);
            /* root = choice([x for x in h if h.degree(x) > 1]) */
            int32_t nr = 0;
            for (int32_t u = 0; u < n; ++u) nr += inM[u] && tdeg[u] > 1;
            if (nr == 0) continue;
            const uint64_t rk = mulhi64(((uint64_t)cw[1] << 32) | cw[0], (uint64_t)nr);
            root = -1;
            for (int32_t u = 0, c = 0; u < n; ++u)
                if (inM[u] && tdeg[u] > 1) { if ((uint64_t)c == rk) { root = u; break; } ++c; }
            /* subtree populations: DFS order from the root, then children before parents */
            int32_t sp = 0, no = 0;
            parent[root] = -1;
            stack[sp++] = root;
            while (sp) {
                const int32_t x = stack[--sp];
                orderv[no++] = x;
                for (int32_t j = toff[x]; j < toff[x + 1]; ++j)
                    if (tadj[j] != parent[x]) { parent[tadj[j]] = x; stack[sp++] = tadj[j]; }
            }
            for (int32_t i = 0; i < no; ++i) spop[orderv[i]] = p->pop[orderv[i]];
            for (int32_t i = no - 1; i > 0; --i) spop[parent[orderv[i]]] += spop[orderv[i]];
            /* cuts: |pop(subtree) - ideal| < epsilon * ideal, non-root nodes, ascending id */
            int32_t ncut = 0;
            for (int32_t u = 0; u < n; ++u)
                if (inM[u] && u != root && fabs((double)spop[u] - p->pop_target) < p->epsilon * p->pop_target) ++ncut;
            if (ncut == 0) continue;
            const uint64_t ck = mulhi64(((uint64_t)cw[3] << 32) | cw[2], (uint64_t)ncut);
            for (int32_t u = 0, c = 0; u < n; ++u)
                if (inM[u] && u != root && fabs((double)spop[u] - p->pop_target) < p->epsilon * p->pop_target) {
                    if ((uint64_t)c == ck) { child = u; break; }
                    ++c;
                }
            /* subset = subtree(child) */
            memset(mark, 0, (size_t)n);
            sp = 0;
            stack[sp++] = child;
            mark[child] = 1;
            while (sp) {
                const int32_t x = stack[--sp];
                for (int32_t j = toff[x]; j < toff[x + 1]; ++j)
                    if (tadj[j] != parent[x] && !mark[tadj[j]]) { mark[tadj[j]] = 1; stack[sp++] = tadj[j]; }
            }
            break;
        }
        if (child < 0) { st->stuck = 1; rc = 1; break; }
        for (int32_t u = 0; u < n; ++u) na[u] = inM[u] ? (mark[u] ? d0 : d1) : a[u];
        const int64_t p0 = spop[child], p1 = popM - spop[child];
        int32_t flags = 0, cut_new;
        CUT_OF(na, cut_new);
        if (p0 < p->pop_lo || p0 > p->pop_hi || p1 < p->pop_lo || p1 > p->pop_hi) {
            st->inv_pop += 1;
            flags = 8;
        } else {
            st->steps += 1;
            flags = 1;
            /* cut_accept: random() < base ** (cut - cut') */
            if (u53(w[1], w[2]) < pow(p->base, (double)(st->cut - cut_new))) {
                flags |= 2;
                st->accepted += 1;
                memcpy(a, na, (size_t)n);
                st->cut = cut_new;
                NB_OF(a, st->nb);
            }
            st->sum_cut += st->cut;
            st->sum_nb += st->nb;
        }
        if (trace && *trace_len < trace_cap) {
            rr_record *r = &trace[(*trace_len)++];
            r->draw = (int64_t)draw; r->edge = e_sel; r->root = root; r->child = child;
            r->attempts = attempts; r->flags = flags; r->cut = st->cut;
        }
    }
#undef CUT_OF
#undef NB_OF
    if (final_assign) memcpy(final_assign, a, (size_t)n);
done:
    free(eu); free(ev); free(a); free(na); free(uf); free(tdeg); free(tadj); free(toff); free(parent); free(stack);
    free(orderv); free(spop); free(inM); free(mark); free(we); free(pops);
    return rc;
}
