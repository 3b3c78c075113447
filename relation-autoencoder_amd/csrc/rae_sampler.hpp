// Negative-example sampling (learning/NegativeExampleGenerator.py:14-32):
//   ids = negSamplingCum.searchsorted(U(0, cum[-1]))   (numpy side='left', float64)
// Parity mode: the uniforms come from the caller (the model's MT19937 stream, drawn on the
// host exactly as the reference draws them) and only the search runs here -- the search is
// ~95 % of the host sampler's time (2.9 s of 3.0 s per 20 M draws at C3).
// Perf mode: the uniforms are generated in the kernel from a counter-based Philox4x32-10
// stream (seed, draw index), no host draw and no upload; not the reference's
// stream, so not bit-comparable with it.
// One thread per draw; the search is a branch-free lower bound over the float64 CDF
// (n <= 2^31), whose top levels stay in L2 / the Infinity Cache.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rae {

__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                             uint32_t k0, uint32_t k1) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
}

// Philox4x32-10 of counter (idx, 0, 0, 0) under key seed -> two 32-bit words -> a double in
// [0, 1) with 53 random bits, assembled like numpy's random_sample ((a>>5)*2^26 + (b>>6))/2^53
__device__ __forceinline__ double philox_uniform(uint64_t seed, uint64_t idx) {
    uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32), c2 = 0, c3 = 0;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        philox_round(c0, c1, c2, c3, k0, k1);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    const uint64_t a = c0 >> 5, b = c1 >> 6;
    return (double)(a * 67108864ull + b) * (1.0 / 9007199254740992.0);
}

// first i with cum[i] >= u  (numpy searchsorted, side='left')
__device__ __forceinline__ int32_t cdf_lower_bound(const double* __restrict__ cum, int64_t n, double u) {
    int64_t lo = 0, len = n;
    while (len > 0) {
        const int64_t half = len >> 1;
        const int64_t mid = lo + half;
        const bool right = cum[mid] < u;
        lo = right ? mid + 1 : lo;
        len = right ? len - half - 1 : half;
    }
    return (int32_t)lo;
}

template <bool PHILOX>
__global__ __launch_bounds__(256) void k_neg_sample(const double* __restrict__ cum, int64_t n,
                                                    const double* __restrict__ u, uint64_t seed,
                                                    uint64_t offset, int64_t count,
                                                    int32_t* __restrict__ out) {
    const double top = cum[n - 1];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double x = PHILOX ? philox_uniform(seed, offset + (uint64_t)i) * top : u[i];
        out[i] = cdf_lower_bound(cum, n, x);
    }
}

}  // namespace rae
