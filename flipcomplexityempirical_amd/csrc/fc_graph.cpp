// Host graph builder: CSR + planar positions -> per-node link rings for the device.
//
// The reference checks contiguity of every proposal with single_flip_contiguous
// [gc-0.2] (imported grid_chain_sec11.py:22, used :340): one networkx Dijkstra per old
// neighbour through the old district.  The device replaces that search by a local test on
// the node's link ring (its neighbours and the far corners of its quadrilateral faces, in
// angular order): neighbours of the old district that lie on one linked run of the ring are
// connected around the node.  For k = 2 on a planar straight-line embedding the converse
// also holds (Jordan-curve argument, DESIGN.md "Contiguity"): at an interior node with a
// closed ring, two runs separated by gaps of the other district can never be joined, and on
// the outer face the same holds once we know whether the other district touches the outer
// boundary.  Nodes where that argument is proven by construction get kMetaExact; the rest
// fall back to the device BFS.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <unordered_map>

#include "fc_internal.h"

namespace fc {
namespace {

struct Dart {
    int32_t from, to;
};

inline double cross(double ax, double ay, double bx, double by) { return ax * by - ay * bx; }

// Proper or touching intersection test of segments p1p2 and p3p4 that share no endpoint.
bool segments_intersect(const double *p1, const double *p2, const double *p3, const double *p4) {
    auto orient = [](const double *a, const double *b, const double *c) {
        double v = cross(b[0] - a[0], b[1] - a[1], c[0] - a[0], c[1] - a[1]);
        return (v > 1e-12) - (v < -1e-12);
    };
    auto on_seg = [](const double *a, const double *b, const double *c) {  // c on ab (collinear)
        return std::min(a[0], b[0]) - 1e-12 <= c[0] && c[0] <= std::max(a[0], b[0]) + 1e-12 &&
               std::min(a[1], b[1]) - 1e-12 <= c[1] && c[1] <= std::max(a[1], b[1]) + 1e-12;
    };
    int o1 = orient(p1, p2, p3), o2 = orient(p1, p2, p4), o3 = orient(p3, p4, p1), o4 = orient(p3, p4, p2);
    if (o1 != o2 && o3 != o4 && o1 && o2 && o3 && o4) return true;
    if (!o1 && on_seg(p1, p2, p3)) return true;
    if (!o2 && on_seg(p1, p2, p4)) return true;
    if (!o3 && on_seg(p3, p4, p1)) return true;
    if (!o4 && on_seg(p3, p4, p2)) return true;
    return false;
}

// No two edges of the straight-line drawing meet except at a shared endpoint.
bool check_planar(const HostGraph &g) {
    const int32_t E = g.n_edges;
    if (E == 0) return true;
    double minx = 1e300, miny = 1e300, maxx = -1e300, maxy = -1e300, len = 0;
    for (int32_t i = 0; i < g.n; ++i) {
        minx = std::min(minx, g.pos[2 * i]); maxx = std::max(maxx, g.pos[2 * i]);
        miny = std::min(miny, g.pos[2 * i + 1]); maxy = std::max(maxy, g.pos[2 * i + 1]);
    }
    for (int32_t e = 0; e < E; ++e)
        len += std::hypot(g.pos[2 * g.eu[e]] - g.pos[2 * g.ev[e]], g.pos[2 * g.eu[e] + 1] - g.pos[2 * g.ev[e] + 1]);
    double cell = std::max(len / E, 1e-9);
    if (!std::isfinite(cell)) cell = 1e300;  // positions near DBL_MAX: one bucket, still exact
    // bucket coordinates are clamped in double before any integer conversion (a far-out or
    // overflowing ratio would otherwise be an undefined float -> int64 cast)
    auto bucket = [](double t, int64_t hi) -> int64_t {
        if (!(t > 0.0)) return 0;
        return t >= (double)(hi - 1) ? hi - 1 : (int64_t)t;
    };
    const int64_t nx = bucket((maxx - minx) / cell, 4096) + 1, ny = bucket((maxy - miny) / cell, 4096) + 1;
    std::unordered_map<int64_t, std::vector<int32_t>> buckets;
    auto cx = [&](double x) { return bucket((x - minx) / cell, nx); };
    auto cy = [&](double y) { return bucket((y - miny) / cell, ny); };
    for (int32_t e = 0; e < E; ++e) {
        const double *a = &g.pos[2 * g.eu[e]], *b = &g.pos[2 * g.ev[e]];
        for (int64_t x = cx(std::min(a[0], b[0])); x <= cx(std::max(a[0], b[0])); ++x)
            for (int64_t y = cy(std::min(a[1], b[1])); y <= cy(std::max(a[1], b[1])); ++y)
                buckets[x * ny + y].push_back(e);
    }
    for (auto &kv : buckets) {
        const auto &v = kv.second;
        for (size_t i = 0; i < v.size(); ++i)
            for (size_t j = i + 1; j < v.size(); ++j) {
                int32_t e = v[i], f = v[j];
                int32_t a = g.eu[e], b = g.ev[e], c = g.eu[f], d = g.ev[f];
                if (a == c || a == d || b == c || b == d) {
                    // shared endpoint: reject only collinear overlap
                    int32_t s = (a == c || a == d) ? a : b;
                    int32_t x = (s == a) ? b : a, y = (s == c) ? d : c;
                    double ux = g.pos[2 * x] - g.pos[2 * s], uy = g.pos[2 * x + 1] - g.pos[2 * s + 1];
                    double vx = g.pos[2 * y] - g.pos[2 * s], vy = g.pos[2 * y + 1] - g.pos[2 * s + 1];
                    if (std::fabs(cross(ux, uy, vx, vy)) < 1e-12 && ux * vx + uy * vy > 0) return false;
                    continue;
                }
                if (segments_intersect(&g.pos[2 * a], &g.pos[2 * b], &g.pos[2 * c], &g.pos[2 * d])) return false;
            }
    }
    return true;
}

bool check_connected(const HostGraph &g) {
    if (g.n == 0) return true;
    std::vector<uint8_t> seen(g.n, 0);
    std::vector<int32_t> q{0};
    seen[0] = 1;
    for (size_t h = 0; h < q.size(); ++h)
        for (int32_t j = g.row_ptr[q[h]]; j < g.row_ptr[q[h] + 1]; ++j)
            if (!seen[g.col_idx[j]]) { seen[g.col_idx[j]] = 1; q.push_back(g.col_idx[j]); }
    return (int32_t)q.size() == g.n;
}

}  // namespace

std::string build_host_graph(int32_t n, const int32_t *row_ptr, const int32_t *col_idx, const int32_t *pop,
                             const double *pos_xy, uint32_t flags, HostGraph &g) {
    if (n <= 0 || !row_ptr || !col_idx) return "graph: n must be positive and CSR arrays non-null";
    if (n > 32767) return "graph: round-1 kernels index nodes with int16 (n <= 32767)";
    g = HostGraph();
    g.n = n;
    g.row_ptr.assign(row_ptr, row_ptr + n + 1);
    if (g.row_ptr[0] != 0) return "graph: row_ptr[0] must be 0";
    for (int32_t i = 0; i < n; ++i)
        if (g.row_ptr[i + 1] < g.row_ptr[i]) return "graph: row_ptr must be non-decreasing";
    const int32_t nnz = g.row_ptr[n];
    if (nnz % 2) return "graph: CSR must be symmetric (odd number of entries)";
    g.col_idx.assign(col_idx, col_idx + nnz);
    g.pop.assign(n, 1);
    if (pop) g.pop.assign(pop, pop + n);
    for (int32_t i = 0; i < n; ++i) {
        auto b = g.col_idx.begin() + g.row_ptr[i], e = g.col_idx.begin() + g.row_ptr[i + 1];
        std::sort(b, e);
        for (auto it = b; it != e; ++it) {
            if (*it < 0 || *it >= n) return "graph: column index out of range";
            if (*it == i) return "graph: self loops are not allowed";
            if (it + 1 != e && *(it + 1) == *it) return "graph: duplicate edge";
        }
        g.max_degree = std::max(g.max_degree, g.row_ptr[i + 1] - g.row_ptr[i]);
    }
    auto adjacent = [&](int32_t u, int32_t w) {
        return std::binary_search(g.col_idx.begin() + g.row_ptr[u], g.col_idx.begin() + g.row_ptr[u + 1], w);
    };
    for (int32_t u = 0; u < n; ++u)
        for (int32_t j = g.row_ptr[u]; j < g.row_ptr[u + 1]; ++j)
            if (!adjacent(g.col_idx[j], u)) return "graph: CSR must be symmetric";
    for (int32_t u = 0; u < n; ++u)
        for (int32_t j = g.row_ptr[u]; j < g.row_ptr[u + 1]; ++j)
            if (g.col_idx[j] > u) { g.eu.push_back(u); g.ev.push_back(g.col_idx[j]); }
    g.n_edges = (int32_t)g.eu.size();
    if (g.max_degree > 16) return "graph: round-1 kernels support degree <= 16";
    g.connected = check_connected(g);

    // ---- rings ------------------------------------------------------------------------
    std::vector<std::vector<int32_t>> ring(n);
    std::vector<uint32_t> nbr(n, 0), link(n, 0);
    std::vector<uint8_t> exact(n, 0), gamma(n, 0);

    if (pos_xy) {
        for (size_t i = 0; i < 2 * (size_t)n; ++i)
            if (!std::isfinite(pos_xy[i])) return "graph: node positions must be finite";
        g.pos.assign(pos_xy, pos_xy + 2 * (size_t)n);
        g.planar = check_planar(g);
        // ccw neighbour order
        std::vector<std::vector<int32_t>> ccw(n);
        for (int32_t v = 0; v < n; ++v) {
            auto &c = ccw[v];
            c.assign(g.col_idx.begin() + g.row_ptr[v], g.col_idx.begin() + g.row_ptr[v + 1]);
            std::sort(c.begin(), c.end(), [&](int32_t a, int32_t b) {
                double ta = std::atan2(g.pos[2 * a + 1] - g.pos[2 * v + 1], g.pos[2 * a] - g.pos[2 * v]);
                double tb = std::atan2(g.pos[2 * b + 1] - g.pos[2 * v + 1], g.pos[2 * b] - g.pos[2 * v]);
                return ta < tb || (ta == tb && a < b);
            });
        }
        // dart index: position of w in ccw[v]
        auto idx_in = [&](int32_t v, int32_t w) {
            const auto &c = ccw[v];
            for (size_t i = 0; i < c.size(); ++i) if (c[i] == w) return (int32_t)i;
            return -1;
        };
        // face traversal: next(u->w) = w -> (cw successor of u around w) = ccw[w][idx-1]
        std::vector<int32_t> dart_off(n + 1, 0);
        for (int32_t v = 0; v < n; ++v) dart_off[v + 1] = dart_off[v] + (int32_t)ccw[v].size();
        const int32_t D = dart_off[n];
        std::vector<int32_t> face_of(D, -1);
        std::vector<std::vector<int32_t>> faces;   // vertex cycles
        std::vector<double> area;
        for (int32_t v = 0; v < n; ++v)
            for (int32_t i = 0; i < (int32_t)ccw[v].size(); ++i) {
                if (face_of[dart_off[v] + i] >= 0) continue;
                const int32_t fid = (int32_t)faces.size();
                faces.emplace_back();
                double a2 = 0;
                int32_t u = v, ui = i;
                for (int32_t guard = 0; guard <= D; ++guard) {
                    const int32_t d = dart_off[u] + ui;
                    if (face_of[d] >= 0) break;
                    face_of[d] = fid;
                    const int32_t w = ccw[u][ui];
                    faces.back().push_back(u);
                    a2 += cross(g.pos[2 * u], g.pos[2 * u + 1], g.pos[2 * w], g.pos[2 * w + 1]);
                    const int32_t k = idx_in(w, u);
                    const int32_t sz = (int32_t)ccw[w].size();
                    ui = (k - 1 + sz) % sz;
                    u = w;
                }
                area.push_back(0.5 * a2);
            }
        int32_t outer = -1;
        if (!faces.empty()) {
            outer = 0;
            for (int32_t f = 1; f < (int32_t)faces.size(); ++f) if (area[f] < area[outer]) outer = f;
        }
        if (outer >= 0 && g.connected) {
            std::vector<int32_t> cyc = faces[outer];
            std::vector<int32_t> srt = cyc;
            std::sort(srt.begin(), srt.end());
            g.outer_simple = std::adjacent_find(srt.begin(), srt.end()) == srt.end() && cyc.size() >= 3;
            for (int32_t x : cyc) gamma[x] = 1;
        }
        const bool global_ok = g.planar && g.connected && !(flags & FC_GRAPH_NO_EXACT);
        for (int32_t v = 0; v < n; ++v) {
            const auto &c = ccw[v];
            const int32_t d = (int32_t)c.size();
            // segments: for each wedge i (between c[i] and c[i+1]) the entries [c[i], (w)] and a
            // link flag for each step inside the wedge.
            std::vector<int32_t> ent;
            std::vector<uint8_t> lnk;      // lnk[j]: ent[j] linked to ent[j+1 mod L]
            std::vector<uint8_t> isn;
            int32_t n_breaks = 0, outer_pos = -1;
            if (d == 1) {
                ent.push_back(c[0]); isn.push_back(1); lnk.push_back(0);
                n_breaks = 1;
                if (face_of[dart_off[v]] == outer) outer_pos = 0;
            }
            for (int32_t i = 0; d >= 2 && i < d; ++i) {
                ent.push_back(c[i]); isn.push_back(1); lnk.push_back(0);
                const int32_t f = face_of[dart_off[v] + i];
                const auto &fv = faces[f];
                const int32_t un = c[(i + 1) % d];
                bool quad_ok = false, tri_ok = false;
                int32_t w = -1;
                if (f != outer && fv.size() == 3) {
                    tri_ok = adjacent(c[i], un);
                } else if (f != outer && fv.size() == 4) {
                    // face cycle v -> c[i] -> w -> un
                    int32_t s = 0;
                    while (fv[s] != v) ++s;
                    if (fv[(s + 1) % 4] == c[i] && fv[(s + 3) % 4] == un) {
                        w = fv[(s + 2) % 4];
                        if (w != v && w != c[i] && w != un) {
                            // diagonal v-w must run inside the face: c[i] and un strictly on opposite sides
                            const double *pv = &g.pos[2 * v], *pw = &g.pos[2 * w];
                            const double *pa = &g.pos[2 * c[i]], *pb = &g.pos[2 * un];
                            double sa = cross(pw[0] - pv[0], pw[1] - pv[1], pa[0] - pv[0], pa[1] - pv[1]);
                            double sb = cross(pw[0] - pv[0], pw[1] - pv[1], pb[0] - pv[0], pb[1] - pv[1]);
                            quad_ok = (sa > 1e-12 && sb < -1e-12) || (sa < -1e-12 && sb > 1e-12);
                        }
                    }
                }
                if (tri_ok) {
                    lnk.back() = 1;
                } else if (quad_ok) {
                    lnk.back() = 1;
                    ent.push_back(w); isn.push_back(0); lnk.push_back(1);
                } else {
                    ++n_breaks;
                    if (f == outer) outer_pos = (int32_t)ent.size() - 1;
                }
            }
            // rotate so that the ring starts right after a break (outer break preferred)
            const int32_t L = (int32_t)ent.size();
            int32_t start = 0;
            if (n_breaks > 0) {
                int32_t bpos = outer_pos;
                if (bpos < 0) for (int32_t j = 0; j < L; ++j) if (!lnk[j]) { bpos = j; break; }
                start = (bpos + 1) % L;
            }
            if (L > 16) return "graph: link ring longer than 16 entries";
            for (int32_t j = 0; j < L; ++j) {
                const int32_t s = (start + j) % L;
                ring[v].push_back(ent[s]);
                if (isn[s]) nbr[v] |= 1u << j;
                if (lnk[s]) link[v] |= 1u << j;
            }
            const bool closed = n_breaks == 0;
            const bool gamma_open = n_breaks == 1 && outer_pos >= 0 && gamma[v] && g.outer_simple;
            exact[v] = global_ok && L >= 2 && (closed || gamma_open);
        }
    } else {
        // no embedding: the ring is the neighbour list; consecutive adjacent neighbours link
        for (int32_t v = 0; v < n; ++v) {
            const int32_t d = g.row_ptr[v + 1] - g.row_ptr[v];
            for (int32_t j = 0; j < d; ++j) {
                ring[v].push_back(g.col_idx[g.row_ptr[v] + j]);
                nbr[v] |= 1u << j;
            }
            // link j joins entry j and entry j+1 (cyclically when the ring has >= 3 entries)
            const int32_t n_links = d >= 3 ? d : d - 1;
            for (int32_t j = 0; j < n_links; ++j)
                if (adjacent(ring[v][j], ring[v][(j + 1) % d])) link[v] |= 1u << j;
        }
    }

    // The device's conflict test relies on x in R(y) <=> y in R(x).  Neighbour entries are
    // symmetric by construction; a diagonal entry without its mirror is dropped (its node
    // then has a break and loses exactness).
    for (int32_t v = 0; v < n; ++v) {
        for (size_t j = 0; j < ring[v].size(); ++j) {
            if (nbr[v] >> j & 1u) continue;
            const int32_t x = ring[v][j];
            if (std::find(ring[x].begin(), ring[x].end(), v) != ring[x].end()) continue;
            const int32_t L = (int32_t)ring[v].size();
            std::vector<int32_t> ent;
            uint32_t nn = 0, ll = 0;
            for (int32_t q = 0, o = 0; q < L; ++q) {
                if (q == (int32_t)j) continue;
                ent.push_back(ring[v][q]);
                if (nbr[v] >> q & 1u) nn |= 1u << o;
                // the step out of the dropped entry's predecessor is now a break
                if ((link[v] >> q & 1u) && (q + 1) % L != (int32_t)j) ll |= 1u << o;
                ++o;
            }
            ring[v] = ent;
            nbr[v] = nn;
            link[v] = ll;
            exact[v] = 0;
            --j;
        }
    }

    int32_t rmax = 0;
    for (int32_t v = 0; v < n; ++v) rmax = std::max<int32_t>(rmax, (int32_t)ring[v].size());
    g.ring_max = rmax <= 8 ? 8 : 16;
    g.ring.assign((size_t)n * g.ring_max, 0);
    g.ring_eid.assign((size_t)n * g.ring_max, -1);
    g.meta.assign(n, 0);
    std::unordered_map<int64_t, int32_t> eid;
    eid.reserve(2 * (size_t)g.n_edges);
    for (int32_t e = 0; e < g.n_edges; ++e) eid[(int64_t)g.eu[e] * n + g.ev[e]] = e;
    for (int32_t v = 0; v < n; ++v) {
        const int32_t L = (int32_t)ring[v].size();
        for (int32_t j = 0; j < g.ring_max; ++j) {
            const int32_t x = j < L ? ring[v][j] : v;
            g.ring[(size_t)v * g.ring_max + j] = x;
            if (j < L && (nbr[v] >> j & 1u)) {
                int32_t a = std::min(v, x), b = std::max(v, x);
                g.ring_eid[(size_t)v * g.ring_max + j] = eid[(int64_t)a * n + b];
            }
        }
        uint64_t m = (uint64_t)L;
        if (exact[v]) m |= kMetaExact;
        if (gamma[v] && g.outer_simple) m |= kMetaGamma;
        m |= (uint64_t)nbr[v] << kMetaNbrShift;
        m |= (uint64_t)link[v] << kMetaLinkShift;
        g.meta[v] = m;
        g.n_exact += exact[v] ? 1 : 0;
        g.n_gamma += (gamma[v] && g.outer_simple) ? 1 : 0;
    }
    return "";
}

}  // namespace fc
