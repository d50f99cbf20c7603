// Chain dealing for the k = 2 flip launch (gfx950, MI355X).
//
// A launch lasts as long as its slowest chain, and a chain's pace is set by how many waves
// share its SIMD: on sec11, 1024 base-10 chains alone (one per SIMD) take 58 ms per 100,000
// steps, 2048 (two per SIMD) 61 ms and 4096 (four) 78 ms.  A launch that mixes bases is then
// set by the SIMDs the dispatcher hands the most short-boundary chains.  Dealing gives every
// SIMD one chain of each quarter of the previous launch's work (draws, most first; the
// chains' durations are stretched by their SIMD-mates and rank them poorly): this kernel
// sorts the chains by that key into `order` and zeroes the counters; each wave of the flip
// launch then reads its SIMD's arrival slot s (a counter per XCC_ID . HW_ID key) and claims
// the next chain of quarter s (dev::deal_chain).  Which wave runs which chain changes only
// the schedule: a chain's trajectory depends on its own state and stream alone.
//
// C2 (ten bases dealt c % 10) does not need it: the dispatcher's order already gives every
// SIMD one or two of the 1638 chains of bases 2.6-10 (tools/archive/deal_prof.sh), and dealing by
// draws measured 72.8-75.1 ms per launch against 74.4-74.5 without, so it is off by default
// (fc_params.tune_deal = 1 turns it on).
#include <hip/hip_runtime.h>

#include "fc_internal.h"

namespace fc {

namespace {

constexpr int kBins = 1024;
constexpr int kThreads = 1024;

// counting sort by descending key into kBins bins of [0, max]: order within a bin is
// arrival order (any order deals the same quarters up to the bin width)
__global__ __launch_bounds__(kThreads) void deal_order_kernel(const uint32_t *ctime, const ChainScalars *sc, int n,
                                                              int C, int timed, uint32_t *order, uint32_t *deal) {
    __shared__ uint32_t hist[kBins];
    __shared__ uint32_t maxk;
    const int t = (int)threadIdx.x;
    for (int i = t; i < kDealKeys + 4; i += kThreads) deal[i] = 0u;
    for (int i = t; i < kBins; i += kThreads) hist[i] = 0u;
    if (t == 0) maxk = 0u;
    __syncthreads();
    auto key = [&](int c) -> uint32_t { return timed ? ctime[c] : (uint32_t)max(n - sc[c].nb, 0); };
    uint32_t m = 0u;
    for (int c = t; c < C; c += kThreads) m = max(m, key(c));
    atomicMax(&maxk, m);
    __syncthreads();
    const uint64_t span = (uint64_t)maxk + 1u;
    auto bin = [&](int c) -> int { return kBins - 1 - (int)((uint64_t)key(c) * kBins / span); };
    for (int c = t; c < C; c += kThreads) atomicAdd(&hist[bin(c)], 1u);
    __syncthreads();
    // exclusive scan of the bins (Hillis-Steele over kBins = kThreads entries)
    uint32_t x = hist[t];
    for (int off = 1; off < kBins; off <<= 1) {
        __syncthreads();
        const uint32_t y = t >= off ? hist[t - off] : 0u;
        __syncthreads();
        hist[t] += y;
    }
    __syncthreads();
    hist[t] -= x;  // start of bin t
    __syncthreads();
    for (int c = t; c < C; c += kThreads) order[atomicAdd(&hist[bin(c)], 1u)] = (uint32_t)c;
}

}  // namespace

int launch_deal_order(const uint32_t *ctime, const ChainScalars *sc, int n, int n_chains, int timed, uint32_t *order,
                      uint32_t *deal, void *stream) {
    hipLaunchKernelGGL(deal_order_kernel, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, ctime, sc, n, n_chains,
                       timed, order, deal);
    return (int)hipGetLastError();
}

}  // namespace fc
