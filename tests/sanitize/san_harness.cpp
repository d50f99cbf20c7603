// Host sanitizer harness (SURVEY §5 "Race detection / sanitizers"): the native graph builder
// (flipcomplexityempirical_amd/csrc/fc_graph.cpp, fc_graph_create's body) and the plain-C
// oracle (oracle/flipref.c) built with -fsanitize=address,undefined and driven on one input
// file.  Test infrastructure only: tests/test_sanitize.py builds and runs it on the CPU.
//
// Input (little-endian): int32 n, int32 nnz, int32 row_ptr[n + 1], int32 col_idx[nnz],
// int32 pop[n], int32 has_pos, double pos[2 n] (if has_pos), uint32 flags, int32 k,
// int32 n_steps, int8 assign[n] (if n_steps > 0).  The header sizes are taken as given, so a
// malformed file must be rejected by the builder's checks, not by the harness.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../flipcomplexityempirical_amd/csrc/fc_internal.h"
#include "../../oracle/flipref.h"

template <typename T>
static bool rd(FILE *f, T *p, size_t cnt) {
    return cnt == 0 || std::fread(p, sizeof(T), cnt, f) == cnt;
}

int main(int argc, char **argv) {
    if (argc != 2) return 2;
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t n = 0, nnz = 0, has_pos = 0, k = 2, n_steps = 0;
    uint32_t flags = 0;
    if (!rd(f, &n, 1) || !rd(f, &nnz, 1) || n < 0 || nnz < 0) return 2;
    std::vector<int32_t> row((size_t)n + 1), col((size_t)nnz), pop((size_t)n);
    std::vector<double> pos;
    if (!rd(f, row.data(), row.size()) || !rd(f, col.data(), col.size()) || !rd(f, pop.data(), pop.size()) ||
        !rd(f, &has_pos, 1))
        return 2;
    if (has_pos) {
        pos.resize(2 * (size_t)n);
        if (!rd(f, pos.data(), pos.size())) return 2;
    }
    if (!rd(f, &flags, 1) || !rd(f, &k, 1) || !rd(f, &n_steps, 1)) return 2;
    std::vector<int8_t> assign((size_t)n);
    if (n_steps > 0 && !rd(f, assign.data(), assign.size())) return 2;
    std::fclose(f);
    // the builder reads row_ptr[n] entries of col_idx: hand it a buffer of exactly nnz
    // entries, so that a row_ptr claiming more is an ASan-visible overread unless rejected
    if (n > 0 && (row[n] < 0 || row[n] > nnz)) {
        std::printf("REJECTED harness: row_ptr[n] = %d outside the %d column entries given\n", row[n], nnz);
        return 0;
    }
    fc::HostGraph g;
    const std::string err = fc::build_host_graph(n, row.data(), n > 0 ? col.data() : nullptr, pop.data(),
                                                 has_pos ? pos.data() : nullptr, flags, g);
    if (!err.empty()) {
        std::printf("REJECTED %s\n", err.c_str());
        return 0;
    }
    int64_t exact = 0;
    for (int32_t v = 0; v < g.n; ++v) exact += (g.meta[v] >> 8) & 1u;
    std::printf("GRAPH n=%d E=%d ring_max=%d exact=%lld gamma=%d planar=%d\n", g.n, g.n_edges, g.ring_max,
                (long long)exact, g.n_gamma, (int)g.planar);
    if (n_steps <= 0) return 0;
    // the oracle on the same CSR: every output buffer and the trace on
    std::vector<int32_t> labels(k);
    for (int i = 0; i < k; ++i) labels[i] = i;
    std::vector<double> l1((size_t)n + 1);
    for (int32_t b = 0; b <= n; ++b) l1[b] = -(double)b / 1e6;
    fr_params p{};
    p.n = n;
    p.row_ptr = g.row_ptr.data();
    p.col_idx = g.col_idx.data();
    p.pop = g.pop.data();
    p.k = k;
    p.labels = labels.data();
    p.base = 1.5;
    p.pop_lo = 0;
    p.pop_hi = INT32_MAX;
    p.seed = 12345;
    p.chain_id = 3;
    p.n_steps = n_steps;
    p.max_draws = 64LL * 1024 * n_steps;
    p.log1mp = l1.data();
    p.proposal = k == 2 ? FR_PROPOSE_BI_SIGN : FR_PROPOSE_PAIR;
    const int64_t E = g.n_edges;
    std::vector<fr_record> trace(4096);
    std::vector<int64_t> cut_hist(E + 1), nb_hist((size_t)n + 1), cut_times(E), nf(n), ps(n), lf(n);
    std::vector<int8_t> fin(n);
    fr_outputs o{};
    o.trace = trace.data();
    o.trace_cap = (int64_t)trace.size();
    o.final_assign = fin.data();
    o.cut_hist = cut_hist.data();
    o.nb_hist = nb_hist.data();
    o.cut_times = cut_times.data();
    o.num_flips = nf.data();
    o.part_sum = ps.data();
    o.last_flipped = lf.data();
    fr_stats st{};
    const int rc = fr_run(&p, assign.data(), &st, &o);
    std::printf("ORACLE rc=%d steps=%lld proposals=%lld cut=%d nb=%d\n", rc, (long long)st.steps,
                (long long)st.proposals, st.cut, st.nb);
    return 0;
}
