// Series diagnostics over the FC_DIAG_SERIES event logs: the per-yield |cut| list the
// reference driver builds (rce, grid_chain_sec11.py:367) expanded on the device, and its
// lag sums for the autocorrelation diagnostic of BASELINE config C4.
//
// Both kernels are HBM-bound streaming passes: expansion writes 2 B per yield (binary
// search of the chain's event log, which stays L2-resident); the lag pass reads the tile
// x[t0 .. t0+4095] once into LDS and x[t + L] once per lag from L2/HBM.
#include <hip/hip_runtime.h>

#include "fc_internal.h"

namespace fc {
namespace {

constexpr int kTile = 4096;
constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void series_expand_kernel(const fc_event *__restrict__ events, int64_t ev_cap,
                                                                 const int64_t *__restrict__ ev_len,
                                                                 const int64_t *__restrict__ t0,
                                                                 const int32_t *__restrict__ cut0,
                                                                 const int64_t *__restrict__ len, int32_t c0,
                                                                 int64_t stride, uint16_t *__restrict__ x) {
    const int32_t cl = (int32_t)blockIdx.y;
    const int32_t c = c0 + cl;
    const int64_t L = len[c];
    const int64_t base_t = (int64_t)blockIdx.x * kTile;
    if (base_t >= L) return;
    const fc_event *ev = events + (size_t)c * ev_cap;
    const int64_t ne = ev_len[c] < ev_cap ? ev_len[c] : ev_cap;
    const int64_t tw = t0[c];
    const int32_t x0 = cut0[c];
    // events are sorted by t: the value at yield tw + t is the cut of the last event with
    // ev.t <= tw + t (the window's initial |cut| before the first one)
    for (int i = threadIdx.x; i < kTile; i += kThreads) {
        const int64_t t = base_t + i;
        if (t >= L) break;
        const int64_t y = tw + t;
        int64_t lo = 0, hi = ne;  // first event with ev.t > y
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (ev[mid].t <= y) lo = mid + 1; else hi = mid;
        }
        x[(size_t)cl * stride + t] = lo ? ev[lo - 1].cut : (uint16_t)x0;
    }
}

__device__ inline int64_t block_sum(int64_t v, int64_t *red) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor((long long)v, off);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    int64_t s = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kThreads / 64; ++i) s += red[i];
    return s;
}

__global__ __launch_bounds__(kThreads) void series_lagsum_kernel(const uint16_t *__restrict__ x,
                                                                 const int64_t *__restrict__ len, int32_t c0,
                                                                 int64_t stride, const int32_t *__restrict__ lags,
                                                                 int32_t nlags, unsigned long long *__restrict__ sums) {
    __shared__ uint16_t tile[kTile];
    __shared__ int64_t red[kThreads / 64];
    const int32_t cl = (int32_t)blockIdx.y;
    const int32_t c = c0 + cl;
    const int64_t L = len[c];
    const int64_t base_t = (int64_t)blockIdx.x * kTile;
    if (base_t >= L) return;
    const uint16_t *xc = x + (size_t)cl * stride;
    for (int i = threadIdx.x; i < kTile; i += kThreads) tile[i] = base_t + i < L ? xc[base_t + i] : 0;
    __syncthreads();
    for (int j = 0; j < nlags; ++j) {
        const int64_t lag = lags[j];
        int64_t P = 0, H = 0, G = 0;
        for (int i = threadIdx.x; i < kTile; i += kThreads) {
            const int64_t t = base_t + i;
            if (t + lag >= L) break;
            const int64_t a = tile[i];
            const int64_t b = (i + lag < kTile) ? (int64_t)tile[i + lag] : (int64_t)xc[t + lag];
            P += a * b;
            H += a;
            G += b;
        }
        P = block_sum(P, red);
        H = block_sum(H, red);
        G = block_sum(G, red);
        if (threadIdx.x == 0 && (P | H | G)) {
            unsigned long long *o = sums + ((size_t)c * nlags + j) * 3;
            atomicAdd(o + 0, (unsigned long long)P);
            atomicAdd(o + 1, (unsigned long long)H);
            atomicAdd(o + 2, (unsigned long long)G);
        }
    }
}

// ---- frame-edge slope / angle series (boundary_slope + the driver's loop body,
// grid_chain_sec11.py:55-78,371-394; Frankenstein_chain.py:55-78,399-422), k = 2.
//
// One wavefront per chain.  Only frame edges matter, and for k = 2 an event at node v
// toggles the cut status of exactly the frame edges incident to v, so the frame-cut mask
// after event i is mask0 ^ (prefix-XOR of the toggle masks of events 0..i): each lane
// takes one event of a 64-event chunk and a wave XOR scan gives every lane its state.
constexpr int kFrameWords = 4;  // up to 256 frame edges

__device__ inline uint64_t shfl_up64(uint64_t x, int off) {
    return (uint64_t)__shfl_up((long long)x, off);
}

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_x(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}

// inclusive prefix XOR over the 64 lanes (whole wave active): row_shr steps inside each 16-lane
// row, then the row totals by the two row broadcasts (as fc_device.h wave_scan_incl)
__device__ __forceinline__ uint64_t wave_xscan64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo ^= dpp_x<0x111, 0xf>(lo); hi ^= dpp_x<0x111, 0xf>(hi);
    lo ^= dpp_x<0x112, 0xf>(lo); hi ^= dpp_x<0x112, 0xf>(hi);
    lo ^= dpp_x<0x114, 0xf>(lo); hi ^= dpp_x<0x114, 0xf>(hi);
    lo ^= dpp_x<0x118, 0xf>(lo); hi ^= dpp_x<0x118, 0xf>(hi);
    lo ^= dpp_x<0x142, 0xa>(lo); hi ^= dpp_x<0x142, 0xa>(hi);
    lo ^= dpp_x<0x143, 0xc>(lo); hi ^= dpp_x<0x143, 0xc>(hi);
    return ((uint64_t)hi << 32) | lo;
}

// The values depend on the frame-cut mask only through its first two cut edges (canonical
// order): the key j0 | j1 << 16, or kNoPair with fewer than two (NaN values)
constexpr uint32_t kNoPair = 0xffffffffu;

__device__ inline uint32_t frame_key(const uint64_t m[kFrameWords], int &cnt) {
    int j0 = -1, j1 = -1;
    cnt = 0;
#pragma unroll
    for (int w = 0; w < kFrameWords; ++w) {
        uint64_t x = m[w];
        cnt += __popcll(x);
        if (j1 < 0 && x) {
            if (j0 < 0) {
                j0 = 64 * w + __builtin_ctzll(x);
                x &= x - 1;
            }
            if (x) j1 = 64 * w + __builtin_ctzll(x);
        }
    }
    return cnt < 2 ? kNoPair : (uint32_t)j0 | ((uint32_t)j1 << 16);
}

// slope and angle of a key
__device__ inline void key_eval(uint32_t key, const double *__restrict__ mid, double cx, double cy, double &slope,
                                double &angle) {
#pragma clang fp contract(off)
    if (key == kNoPair) {  // the reference raises IndexError on temp[1] here
        slope = __builtin_nan("");
        angle = __builtin_nan("");
        return;
    }
    const int j0 = (int)(key & 0xffffu), j1 = (int)(key >> 16);
    const double ax = mid[2 * j0], ay = mid[2 * j0 + 1], bx = mid[2 * j1], by = mid[2 * j1 + 1];
    // slope = (endb[1]-enda[1])/(endb[0]-enda[0]) else np.Inf  (:378-382)
    slope = (bx != ax) ? (by - ay) / (bx - ax) : __builtin_inf();
    // arccos(clip(dot(a/|a|, b/|b|), -1, 1)) about (20, 20)  (:389-394)
    const double pax = ax - cx, pay = ay - cy, pbx = bx - cx, pby = by - cy;
    const double na = sqrt(pax * pax + pay * pay), nb = sqrt(pbx * pbx + pby * pby);
    double d = (pax / na) * (pbx / nb) + (pay / na) * (pby / nb);
    d = d < -1.0 ? -1.0 : (d > 1.0 ? 1.0 : d);
    angle = acos(d);
}

__device__ inline void frame_eval(const uint64_t m[kFrameWords], const double *__restrict__ mid, double cx,
                                  double cy, double &slope, double &angle, int &cnt) {
    key_eval(frame_key(m, cnt), mid, cx, cy, slope, angle);
}

// MODE 0: one (slope, angle, n_cut) entry per event, [cl * cap + i + 1] (entry 0: window start).
// MODE 1: count the change points of (slope, angle) -- the window start and every event whose
//         values differ bitwise from the previous entry's -- into cp_cnt[cl] (and per wave into
//         wcnt[cl * kFsWaves + w] for MODE 2).
// MODE 2: write them at cp_off[cl]: (yield t at which the values start, slope, angle); the
//         per-yield lists the reference plots (:476-484) are these values held to the next t.
// MODE 3: MODE 1 and 2 in one pass: each wave writes its change points to its own staging
//         range (t_out / slope_out / angle_out + cl * cap + w * (cap / kFsWaves)) and its count
//         to wcnt; frame_compact_kernel then packs them at the chain offsets.
// One workgroup of kFsWaves waves per chain: wave w takes a contiguous range of the chain's
// 64-event chunks; a first pass XORs the toggle masks of each range (one table lookup per
// event, no evaluation), so every wave knows the frame-cut mask at its range's start and the
// ranges are evaluated in parallel.  LT: the toggle tables (node -> row as int16, row ->
// frame-edge mask) and the midpoints are staged in LDS (sec11: 10.7 KB); the next chunk's events
// are loaded before the current one is evaluated.
constexpr int kFsWaves = kFrameWaves;

template <int MODE, bool LT>
__global__ __launch_bounds__(64 * kFsWaves) void frame_series_kernel(
    const int8_t *__restrict__ a0, int32_t npad, const fc_event *__restrict__ events, int64_t ev_cap,
    const int64_t *__restrict__ ev_len, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *__restrict__ fu,
    const int32_t *__restrict__ fv, const double *__restrict__ mid, double cx, double cy,
    const int32_t *__restrict__ tog_idx, const uint64_t *__restrict__ tog_mask, int32_t n_rows, int32_t n_nodes,
    int64_t cap, double *__restrict__ slope_out, double *__restrict__ angle_out, int32_t *__restrict__ cnt_out,
    const int64_t *__restrict__ t0, int64_t *__restrict__ cp_cnt, const int64_t *__restrict__ cp_off,
    int64_t *__restrict__ t_out, int64_t *__restrict__ wcnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint64_t sx[kFsWaves][kFrameWords];  // each range's XOR of toggle masks
    __shared__ int64_t sn[kFsWaves];                 // MODE 1: each range's change points
    const int lane = threadIdx.x & 63;
    const int w = (int)(threadIdx.x >> 6);
    const double *md = mid;
    const uint64_t *tm = tog_mask;
    const int16_t *ti16 = nullptr;
    if constexpr (LT) {
        double *smid = (double *)smem;                                     // [2 n_frame]
        uint64_t *stog = (uint64_t *)(smid + 2 * n_frame);                 // [n_rows][4]
        int16_t *sidx = (int16_t *)(stog + (size_t)n_rows * kFrameWords);  // [n_nodes]
        for (int i = threadIdx.x; i < 2 * n_frame; i += blockDim.x) smid[i] = mid[i];
        for (int i = threadIdx.x; i < n_rows * kFrameWords; i += blockDim.x) stog[i] = tog_mask[i];
        for (int i = threadIdx.x; i < n_nodes; i += blockDim.x) sidx[i] = (int16_t)tog_idx[i];
        __syncthreads();
        md = smid;
        tm = stog;
        ti16 = sidx;
    }
    const int32_t cl = (int32_t)blockIdx.x;
    const int32_t c = c0 + cl;
    const int8_t *a = a0 + (size_t)c * npad;
    const fc_event *ev = events + (size_t)c * ev_cap;
    const int64_t ne = ev_len[c];
    auto row_of = [&](int v) -> int32_t { return LT ? (int32_t)ti16[v] : tog_idx[v]; };
    // this wave's chunk range [k0, k1)
    const int64_t nk = (ne + 63) >> 6;
    const int64_t k0 = nk * w / kFsWaves, k1 = nk * (w + 1) / kFsWaves;
    // pass 1: the XOR of the range's toggle masks
    {
        uint64_t x[kFrameWords] = {0, 0, 0, 0};
        for (int64_t k = k0; k < k1; ++k) {
            const int64_t i = 64 * k + lane;
            if (i < ne) {
                const int32_t r = row_of((int)ev[i].v);
                if (r >= 0) {
#pragma unroll
                    for (int q = 0; q < kFrameWords; ++q) x[q] ^= tm[(size_t)r * kFrameWords + q];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < kFrameWords; ++q) {
            const uint64_t t = wave_xscan64(x[q]);
            if (lane == 63) sx[w][q] = t;
        }
    }
    // the window start's frame-cut mask, then this range's start
    uint64_t m[kFrameWords];
#pragma unroll
    for (int q = 0; q < kFrameWords; ++q) {
        const int j = 64 * q + lane;
        const bool cut = j < n_frame && a[fu[j]] != a[fv[j]];
        m[q] = __ballot(cut);
    }
    __syncthreads();
    for (int w2 = 0; w2 < w; ++w2)
#pragma unroll
        for (int q = 0; q < kFrameWords; ++q) m[q] ^= sx[w2][q];
    double *so = slope_out, *ao = angle_out;
    int32_t *co = cnt_out;
    int64_t *to = t_out;
    if constexpr (MODE == 0) {
        so += (size_t)cl * cap;
        ao += (size_t)cl * cap;
        co += (size_t)cl * cap;
    } else if constexpr (MODE == 2) {
        int64_t o = cp_off[cl];
        for (int w2 = 0; w2 < w; ++w2) o += wcnt[(size_t)cl * kFsWaves + w2];
        so += o;
        ao += o;
        to += o;
    } else if constexpr (MODE == 3) {
        const size_t o = (size_t)cl * (size_t)cap + (size_t)w * (size_t)(cap / kFsWaves);
        so += o;
        ao += o;
        to += o;
    }
    // the values before the range's first event (bit patterns: NaN == NaN), wave-uniform; the
    // window-start entry is wave 0's
    uint64_t prev_s, prev_a;
    uint32_t prev_key;  // MODE >= 1: the key of the event before this lane's (the range start's)
    int64_t pos = 0;  // change points this wave writes
    {
        double sl, an;
        int cnt;
        prev_key = frame_key(m, cnt);
        key_eval(prev_key, md, cx, cy, sl, an);
        prev_s = (uint64_t)__double_as_longlong(sl);
        prev_a = (uint64_t)__double_as_longlong(an);
        if (w == 0) {
            pos = 1;
            if (lane == 0) {
                if constexpr (MODE == 0) {
                    so[0] = sl;
                    ao[0] = an;
                    co[0] = cnt;
                } else if constexpr (MODE >= 2) {
                    so[0] = sl;
                    ao[0] = an;
                    to[0] = t0[c];
                }
            }
        }
    }
    // MODE >= 1: the queued candidate events (key, yield) of this wave, and their evaluation:
    // values against the previous entry's (the last evaluated one before them), change points
    // written / counted in order
    __shared__ uint32_t qk[kFsWaves][128];
    __shared__ int64_t qt[kFsWaves][128];
    int qn = 0;
    auto flush = [&](int nq) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the queue entries other lanes wrote
        const bool on = lane < nq;
        const uint32_t k = on ? qk[w][lane] : kNoPair;
        int64_t tq = 0;
        if constexpr (MODE >= 2) tq = on ? qt[w][lane] : 0;
        double sl, an;
        key_eval(k, md, cx, cy, sl, an);
        const uint64_t bs = (uint64_t)__double_as_longlong(sl), ba = (uint64_t)__double_as_longlong(an);
        uint64_t ps = shfl_up64(bs, 1), pa = shfl_up64(ba, 1);
        if (lane == 0) {
            ps = prev_s;
            pa = prev_a;
        }
        const bool chg = on && (bs != ps || ba != pa);
        const uint64_t cmk = __ballot(chg);
        if constexpr (MODE >= 2) {
            if (chg) {
                const int64_t o = pos + __popcll(cmk & ((1ull << lane) - 1ull));
                so[o] = sl;
                ao[o] = an;
                to[o] = tq;
            }
        }
        pos += __popcll(cmk);
        prev_s = (uint64_t)__shfl((long long)bs, nq - 1);
        prev_a = (uint64_t)__shfl((long long)ba, nq - 1);
        // the entries after the first nq move to the front (reads of [nq, qn), writes of [0, qn - nq):
        // disjoint when nq = 64, and the whole queue when nq = qn)
        const int rest = qn - nq;
        uint32_t k2 = 0;
        int64_t t2 = 0;
        if (lane < rest) {
            k2 = qk[w][nq + lane];
            if constexpr (MODE >= 2) t2 = qt[w][nq + lane];
        }
        if (lane < rest) {
            qk[w][lane] = k2;
            if constexpr (MODE >= 2) qt[w][lane] = t2;
        }
        qn = rest;
    };
    // this lane's event of the next chunk, loaded one chunk ahead
    int nv = 0;
    int64_t nt = 0;
    if (k0 < k1 && 64 * k0 + lane < ne) {
        nv = (int)ev[64 * k0 + lane].v;
        if (MODE >= 2) nt = ev[64 * k0 + lane].t;
    }
    for (int64_t k = k0; k < k1; ++k) {
        const int64_t b = 64 * k;
        const int64_t i = b + lane;
        const int vcur = nv;
        const int64_t tcur = nt;
        if (k + 1 < k1 && b + 64 + lane < ne) {
            nv = (int)ev[b + 64 + lane].v;
            if (MODE >= 2) nt = ev[b + 64 + lane].t;
        }
        uint64_t t[kFrameWords] = {0, 0, 0, 0};
        if (i < ne) {
            const int32_t r = row_of(vcur);
            if (r >= 0) {
#pragma unroll
                for (int q = 0; q < kFrameWords; ++q) t[q] = tm[(size_t)r * kFrameWords + q];
            }
        }
#pragma unroll
        for (int q = 0; q < kFrameWords; ++q) t[q] = wave_xscan64(t[q]) ^ m[q];
        if constexpr (MODE == 0) {
            double sl = 0.0, an = 0.0;
            int cnt = 0;
            if (i < ne) {
                frame_eval(t, md, cx, cy, sl, an, cnt);
                so[i + 1] = sl;
                ao[i + 1] = an;
                co[i + 1] = cnt;
            }
        } else {
            // only an event whose key differs from the previous event's can change the values: those
            // events are queued (in order) and evaluated 64 at a time
            int cnt;
            const uint32_t key = i < ne ? frame_key(t, cnt) : kNoPair;
            uint32_t pk = (uint32_t)__shfl_up((int)key, 1);
            if (lane == 0) pk = prev_key;
            const bool cand = i < ne && key != pk;
            const uint64_t qm = __ballot(cand);
            if (cand) {
                const int qi = qn + __popcll(qm & ((1ull << lane) - 1ull));
                qk[w][qi] = key;
                if constexpr (MODE >= 2) qt[w][qi] = tcur;
            }
            qn += __popcll(qm);
            const int last = (int)((ne - b < 64 ? ne - b : 64) - 1);  // the chunk's last event
            prev_key = (uint32_t)__shfl((int)key, last);
            if (qn >= 64) flush(64);
        }
#pragma unroll
        for (int q = 0; q < kFrameWords; ++q) m[q] = (uint64_t)__shfl((long long)t[q], 63);
    }
    if constexpr (MODE >= 1) {
        if (qn > 0) flush(qn);
    }
    if constexpr (MODE == 1 || MODE == 3) {
        if (lane == 0) {
            sn[w] = pos;
            wcnt[(size_t)cl * kFsWaves + w] = pos;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t tot = 0;
            for (int w2 = 0; w2 < kFsWaves; ++w2) tot += sn[w2];
            cp_cnt[cl] = tot;
        }
    }
}

// MODE 3's staging ranges packed at the chains' offsets: chain cl's wave w range (wcnt[cl][w]
// entries at cl * cap + w * (cap / kFsWaves)) goes to cp_off[cl] + the counts of waves < w.
__global__ __launch_bounds__(kThreads) void frame_compact_kernel(const int64_t *__restrict__ st_t,
                                                                 const double *__restrict__ st_s,
                                                                 const double *__restrict__ st_a, int64_t cap,
                                                                 const int64_t *__restrict__ wcnt,
                                                                 const int64_t *__restrict__ cp_off, int64_t *t_out,
                                                                 double *slope, double *angle) {
    const int32_t cl = (int32_t)blockIdx.x;
    int64_t dst = cp_off[cl];
    for (int w = 0; w < kFsWaves; ++w) {
        const int64_t n = wcnt[(size_t)cl * kFsWaves + w];
        const size_t src = (size_t)cl * (size_t)cap + (size_t)w * (size_t)(cap / kFsWaves);
        for (int64_t i = threadIdx.x; i < n; i += kThreads) {
            t_out[dst + i] = st_t[src + i];
            slope[dst + i] = st_s[src + i];
            angle[dst + i] = st_a[src + i];
        }
        dst += n;
    }
}

// LDS bytes of the staged tables, or 0 when they do not fit (then the kernel reads them from
// global memory)
inline size_t frame_lds_bytes(int32_t n_frame, int32_t n_rows, int32_t n_nodes) {
    const size_t b = 16 * (size_t)n_frame + 8 * kFrameWords * (size_t)n_rows + 2 * (size_t)n_nodes;
    return (b <= 48 * 1024 && n_nodes < 32768) ? (b + 15) & ~(size_t)15 : 0;
}

}  // namespace

int launch_series_expand(const fc_event *events, int64_t ev_cap, const int64_t *ev_len, const int64_t *t0,
                         const int32_t *cut0, const int64_t *len, int32_t c0, int32_t nc, int64_t stride,
                         int64_t max_len, uint16_t *x, void *stream) {
    if (nc <= 0 || max_len <= 0) return (int)hipSuccess;
    const dim3 grid((unsigned)((max_len + kTile - 1) / kTile), (unsigned)nc);
    hipLaunchKernelGGL(series_expand_kernel, grid, dim3(kThreads), 0, (hipStream_t)stream, events, ev_cap, ev_len,
                       t0, cut0, len, c0, stride, x);
    return (int)hipGetLastError();
}

int launch_series_lagsums(const uint16_t *x, const int64_t *len, int32_t c0, int32_t nc, int64_t stride,
                          int64_t max_len, const int32_t *lags, int32_t nlags, unsigned long long *sums,
                          void *stream) {
    if (nc <= 0 || max_len <= 0 || nlags <= 0) return (int)hipSuccess;
    const dim3 grid((unsigned)((max_len + kTile - 1) / kTile), (unsigned)nc);
    hipLaunchKernelGGL(series_lagsum_kernel, grid, dim3(kThreads), 0, (hipStream_t)stream, x, len, c0, stride, lags,
                       nlags, sums);
    return (int)hipGetLastError();
}

}  // namespace fc

namespace fc {

int launch_frame_series(const int8_t *a0, int32_t npad, const fc_event *events, int64_t ev_cap,
                        const int64_t *ev_len, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *fu,
                        const int32_t *fv, const double *mid, double cx, double cy, const int32_t *tog_idx,
                        const uint64_t *tog_mask, int32_t n_rows, int32_t n_nodes, int64_t cap, double *slope,
                        double *angle, int32_t *cnt, void *stream) {
    if (nc <= 0) return (int)hipSuccess;
    if (n_frame > 64 * kFrameWords) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)nc), block(64 * kFsWaves);
    const size_t lds = frame_lds_bytes(n_frame, n_rows, n_nodes);
#define FC_FS_ARGS a0, npad, events, ev_cap, ev_len, c0, nc, n_frame, fu, fv, mid, cx, cy, tog_idx, tog_mask, n_rows, n_nodes
    if (lds)
        hipLaunchKernelGGL((frame_series_kernel<0, true>), grid, block, lds, (hipStream_t)stream, FC_FS_ARGS,
                           cap, slope, angle, cnt, (const int64_t *)nullptr, (int64_t *)nullptr,
                           (const int64_t *)nullptr, (int64_t *)nullptr, (int64_t *)nullptr);
    else
        hipLaunchKernelGGL((frame_series_kernel<0, false>), grid, block, 0, (hipStream_t)stream, FC_FS_ARGS,
                           cap, slope, angle, cnt, (const int64_t *)nullptr, (int64_t *)nullptr,
                           (const int64_t *)nullptr, (int64_t *)nullptr, (int64_t *)nullptr);
    return (int)hipGetLastError();
}

int launch_frame_changes(const int8_t *a0, int32_t npad, const fc_event *events, int64_t ev_cap,
                         const int64_t *ev_len, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *fu,
                         const int32_t *fv, const double *mid, double cx, double cy, const int32_t *tog_idx,
                         const uint64_t *tog_mask, int32_t n_rows, int32_t n_nodes, const int64_t *t0,
                         int64_t *cp_cnt, const int64_t *cp_off, int64_t *t_out, double *slope, double *angle,
                         int64_t *wcnt, void *stream) {
    if (nc <= 0) return (int)hipSuccess;
    if (n_frame > 64 * kFrameWords) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)nc), block(64 * kFsWaves);
    const size_t lds = frame_lds_bytes(n_frame, n_rows, n_nodes);
    if (!cp_off) {
        if (lds)
            hipLaunchKernelGGL((frame_series_kernel<1, true>), grid, block, lds, (hipStream_t)stream, FC_FS_ARGS,
                               (int64_t)0, (double *)nullptr, (double *)nullptr, (int32_t *)nullptr, t0, cp_cnt, cp_off,
                               t_out, wcnt);
        else
            hipLaunchKernelGGL((frame_series_kernel<1, false>), grid, block, 0, (hipStream_t)stream, FC_FS_ARGS,
                               (int64_t)0, (double *)nullptr, (double *)nullptr, (int32_t *)nullptr, t0, cp_cnt, cp_off,
                               t_out, wcnt);
    } else {
        if (lds)
            hipLaunchKernelGGL((frame_series_kernel<2, true>), grid, block, lds, (hipStream_t)stream, FC_FS_ARGS,
                               (int64_t)0, slope, angle, (int32_t *)nullptr, t0, cp_cnt, cp_off, t_out, wcnt);
        else
            hipLaunchKernelGGL((frame_series_kernel<2, false>), grid, block, 0, (hipStream_t)stream, FC_FS_ARGS,
                               (int64_t)0, slope, angle, (int32_t *)nullptr, t0, cp_cnt, cp_off, t_out, wcnt);
    }
    return (int)hipGetLastError();
}

int launch_frame_stage(const int8_t *a0, int32_t npad, const fc_event *events, int64_t ev_cap,
                       const int64_t *ev_len, int32_t c0, int32_t nc, int32_t n_frame, const int32_t *fu,
                       const int32_t *fv, const double *mid, double cx, double cy, const int32_t *tog_idx,
                       const uint64_t *tog_mask, int32_t n_rows, int32_t n_nodes, const int64_t *t0,
                       int64_t *cp_cnt, int64_t stage_cap, int64_t *st_t, double *st_s, double *st_a,
                       int64_t *wcnt, void *stream) {
    if (nc <= 0) return (int)hipSuccess;
    if (n_frame > 64 * kFrameWords) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)nc), block(64 * kFsWaves);
    const size_t lds = frame_lds_bytes(n_frame, n_rows, n_nodes);
    if (lds)
        hipLaunchKernelGGL((frame_series_kernel<3, true>), grid, block, lds, (hipStream_t)stream, FC_FS_ARGS,
                           stage_cap, st_s, st_a, (int32_t *)nullptr, t0, cp_cnt, (const int64_t *)nullptr, st_t,
                           wcnt);
    else
        hipLaunchKernelGGL((frame_series_kernel<3, false>), grid, block, 0, (hipStream_t)stream, FC_FS_ARGS,
                           stage_cap, st_s, st_a, (int32_t *)nullptr, t0, cp_cnt, (const int64_t *)nullptr, st_t,
                           wcnt);
    return (int)hipGetLastError();
}

int launch_frame_compact(int32_t nc, int64_t stage_cap, const int64_t *st_t, const double *st_s,
                         const double *st_a, const int64_t *wcnt, const int64_t *cp_off, int64_t *t_out,
                         double *slope, double *angle, void *stream) {
    if (nc <= 0) return (int)hipSuccess;
    hipLaunchKernelGGL(frame_compact_kernel, dim3((unsigned)nc), dim3(kThreads), 0, (hipStream_t)stream, st_t, st_s,
                       st_a, stage_cap, wcnt, cp_off, t_out, slope, angle);
    return (int)hipGetLastError();
}
#undef FC_FS_ARGS

}  // namespace fc
