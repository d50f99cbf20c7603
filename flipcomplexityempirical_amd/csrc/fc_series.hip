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
