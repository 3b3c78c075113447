// Device helpers shared by the rae kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RAE_WAVE 64
#define RAE_FBT 512           // threads per workgroup of the forward kernel (8 waves)
#define RAE_BT 256            // threads per workgroup of the update kernels (4 waves)
#define RAE_NWAVE (RAE_BT / RAE_WAVE)
#define RAE_KCAP 8192         // LDS capacity (64-bit keys) of one row-index partition
#define RAE_PART 256          // target records per row-index partition

namespace rae {

// xor-butterfly all-reduce: every lane ends with the bitwise-identical sum (fp add is
// commutative, so partner lanes compute a+b and b+a identically).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// sum over the 16 lanes of a lane group (lane & ~15 fixed)
__device__ __forceinline__ float group16_sum(float v) {
    v += __shfl_xor(v, 8, 16);
    v += __shfl_xor(v, 4, 16);
    v += __shfl_xor(v, 2, 16);
    v += __shfl_xor(v, 1, 16);
    return v;
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
    const unsigned lo = __shfl_xor((unsigned)(v & 0xffffffffull), o, 64);
    const unsigned hi = __shfl_xor((unsigned)(v >> 32), o, 64);
    return ((unsigned long long)hi << 32) | lo;
}

// Block-wide sum / max for BT threads; `red` is >= BT/64 floats of LDS.
// Result broadcast to all threads; order fixed (wave order) -> deterministic.
template <int BT>
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x / RAE_WAVE;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < BT / RAE_WAVE; ++i) t += red[i];
    return t;
}
template <int BT>
__device__ __forceinline__ float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x / RAE_WAVE;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = red[0];
#pragma unroll
    for (int i = 1; i < BT / RAE_WAVE; ++i) t = fmaxf(t, red[i]);
    return t;
}

// Stable forms of Theano's rewritten log(sigmoid(x)) -> -softplus(-x) and sigmoid.
__device__ __forceinline__ float softplus(float x) {
    return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
}
__device__ __forceinline__ float log_sigmoid(float x) { return -softplus(-x); }
__device__ __forceinline__ float sigmoid(float x) {
    if (x >= 0.f) { const float z = expf(-x); return 1.f / (1.f + z); }
    const float z = expf(x);
    return z / (1.f + z);
}

// learning/Optimizers.py:30-31  acc <- acc + g^2 ; p <- p - lr*g/(sqrt(acc)+1e-6)
// learning/Optimizers.py:51     p <- p - lr*g                         (SGD)
template <int OPT>
__device__ __forceinline__ float opt_update(float p, float* acc, float g, float lr) {
    if (OPT == 0) {
        const float a = *acc + g * g;
        *acc = a;
        return p - (lr * g) / (sqrtf(a) + 1e-6f);
    } else {
        return p - lr * g;
    }
}

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) - (x < 0.f); }

// ---- float / float4 generic helpers -----------------------------------------------------
template <bool V4> struct VecT { typedef float T; };
template <> struct VecT<true> { typedef float4 T; };

__device__ __forceinline__ float vdot(float a, float b) { return a * b; }
__device__ __forceinline__ float vdot(float4 a, float4 b) {
    return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}
__device__ __forceinline__ void vzero(float& a) { a = 0.f; }
__device__ __forceinline__ void vzero(float4& a) { a = make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void vfma(float& acc, float s, float v) { acc += s * v; }
__device__ __forceinline__ void vfma(float4& acc, float s, float4 v) {
    acc.x += s * v.x; acc.y += s * v.y; acc.z += s * v.z; acc.w += s * v.w;
}
__device__ __forceinline__ void vadd(float& acc, float v) { acc += v; }
__device__ __forceinline__ void vadd(float4& acc, float4 v) {
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
}

}  // namespace rae
