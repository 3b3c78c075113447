// Device helpers shared by the rae kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RAE_WAVE 64
#define RAE_FBT 512           // threads per workgroup of the forward kernel (8 waves)
#ifndef RAE_BT
#define RAE_BT 256            // threads per workgroup of the update kernels (4 waves)
#endif
#define RAE_NWAVE (RAE_BT / RAE_WAVE)
#define RAE_KCAP 8192         // LDS capacity (64-bit keys) of one row-index partition
#define RAE_PART 256          // target records per row-index partition
#define RAE_HEAVY 4           // a parameter row with more records than this per step is "heavy"
#ifndef RAE_VHEAVY
#define RAE_VHEAVY 16         // ... than this: "very heavy", split over a workgroup's four waves
#endif

namespace rae {

// ---- cross-lane primitives (VALU DPP + gfx950 permlane swaps; no LDS round trip) -------
// DPP controls: quad_perm [1,0,3,2] = 0xB1 (lane^1), [2,3,0,1] = 0x4E (lane^2),
// row_half_mirror = 0x141 (within 8: i <-> 7-i), row_mirror = 0x140 (within 16: i <-> 15-i),
// row_shl:n = 0x100+n (lane i <- i+n), row_shr:n = 0x110+n (lane i <- i-n).
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
// float form for the quad_perm / row mirror patterns only (every lane has a source in its
// row): bound_ctrl lets the DPP-combine pass fold the move into its consumer
// (v_add_f32_dpp / v_max_f32_dpp -- one instruction per reduction step instead of three)
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// value of lane (lane ^ 16) / (lane ^ 32) via v_permlane16_swap / v_permlane32_swap
__device__ __forceinline__ unsigned xor16_u32(unsigned v) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? p[0] : p[1];
}
__device__ __forceinline__ unsigned xor32_u32(unsigned v) {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? p[0] : p[1];
}
// value of lane (lane ^ j) for j = 1..32 (j wave-uniform)
__device__ __forceinline__ unsigned xor_lane_u32(unsigned v, int j) {
    const int lane = threadIdx.x & 63;
    switch (j) {
        case 1: return dpp_u32<0xB1>(v);
        case 2: return dpp_u32<0x4E>(v);
        case 4: { const unsigned a = dpp_u32<0x104>(v), b = dpp_u32<0x114>(v);
                  return (lane & 4) ? b : a; }
        case 8: { const unsigned a = dpp_u32<0x108>(v), b = dpp_u32<0x118>(v);
                  return (lane & 8) ? b : a; }
        case 16: return xor16_u32(v);
        default: return xor32_u32(v);
    }
}
__device__ __forceinline__ unsigned long long xor_lane_u64(unsigned long long v, int j) {
    const unsigned lo = xor_lane_u32((unsigned)(v & 0xffffffffull), j);
    const unsigned hi = xor_lane_u32((unsigned)(v >> 32), j);
    return ((unsigned long long)hi << 32) | lo;
}

// sum over the 16 lanes of a lane group; every lane of the group gets the identical value
// (each step adds two commuted operands, so partner lanes compute bitwise-equal sums)
__device__ __forceinline__ float group16_sum(float v) {
    v += dpp_f32<0xB1>(v);
    v += dpp_f32<0x4E>(v);
    v += dpp_f32<0x141>(v);
    v += dpp_f32<0x140>(v);
    return v;
}
// wave-wide all-reduce sum, identical in every lane, fixed order -> deterministic
__device__ __forceinline__ float wave_sum(float v) {
    v = group16_sum(v);
    {
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v),
                                                        false, false);
        v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
    {
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v),
                                                        false, false);
        v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_f32<0xB1>(v));
    v = fmaxf(v, dpp_f32<0x4E>(v));
    v = fmaxf(v, dpp_f32<0x141>(v));
    v = fmaxf(v, dpp_f32<0x140>(v));
    v = fmaxf(v, __uint_as_float(xor16_u32(__float_as_uint(v))));
    v = fmaxf(v, __uint_as_float(xor32_u32(__float_as_uint(v))));
    return v;
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
    return xor_lane_u64(v, o);
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
// One exp shared by sigmoid(x) and softplus(x) = log(1 + e^x), hardware transcendental
// forms (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp): e = exp(-|x|),
//   sigmoid(x)  = x >= 0 ? 1/(1+e) : e/(1+e)
//   softplus(x) = max(x, 0) + log(1 + e)      (log_sigmoid(x) = -softplus(-x))
__device__ __forceinline__ void sigmoid_softplus(float x, float& sig, float& sp) {
    const float e = __expf(-fabsf(x));
    const float r = __builtin_amdgcn_rcpf(1.f + e);
    sig = x >= 0.f ? r : e * r;
    sp = fmaxf(x, 0.f) + __logf(1.f + e);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() carries a workgroup fence,
// for which the compiler drains vmcnt -- every global load and LDS-DMA the wave has in
// flight -- before the s_barrier.  Where a wave keeps bulk loads in flight across a
// barrier (decoder matrices, A-row DMA) that would put them on the critical path; this
// waits only for the wave's own LDS (and scalar) traffic.  Data a wave brought in by
// LDS-DMA becomes visible to the others only after that wave's s_waitcnt vmcnt(0) and a
// following barrier (dma_visible_barrier).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void dma_visible_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
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
        // one rounding, spelled out: left to fp-contract, the fused and the unfused forms of
        // p - lr g differ in the last bit near cancellation, and the two kernels that apply
        // SGD (k_update, the forward's private rows) must agree bit for bit
        return __builtin_fmaf(-lr, g, p);
    }
}

template <int OPT>
__device__ __forceinline__ void updv(float& p, float& ac, float g, float lr) {
    p = opt_update<OPT>(p, &ac, g, lr);
}
template <int OPT>
__device__ __forceinline__ void updv(float4& p, float4& ac, float4 g, float lr) {
    p.x = opt_update<OPT>(p.x, &ac.x, g.x, lr);
    p.y = opt_update<OPT>(p.y, &ac.y, g.y, lr);
    p.z = opt_update<OPT>(p.z, &ac.z, g.z, lr);
    p.w = opt_update<OPT>(p.w, &ac.w, g.w, lr);
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
// vectors of VW floats (1, 2, 4): the fast forward's m-vectors go two wide when m is even but
// not a multiple of 4 (C2: m = 30)
template <int VW> struct VecW { typedef float T; };
template <> struct VecW<2> { typedef float2 T; };
template <> struct VecW<4> { typedef float4 T; };
__device__ __forceinline__ float vdot(float2 a, float2 b) { return a.x * b.x + a.y * b.y; }
__device__ __forceinline__ void vzero(float2& a) { a = make_float2(0.f, 0.f); }
__device__ __forceinline__ void vfma(float2& acc, float s, float2 v) {
    acc.x += s * v.x; acc.y += s * v.y;
}
// Exchange-record loads through one buffer resource: the record's offset rides in the scalar
// soffset, the lane's column in a 32-bit voffset -- one SGPR per load instead of a 64-bit
// address pair, which is what lets the update's wide rounds fit its VGPR budget (RAE_UPD_WPE).
// (dword3 0x00020000: the gfx9-family raw-buffer format word.)
typedef unsigned rae_v4u __attribute__((ext_vector_type(4)));
struct RecBuf {
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ explicit RecBuf(const float* p)
        : rs(__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, -1, 0x00020000)) {}
    // element offsets (floats): soff wave-uniform, voff per lane
    __device__ __forceinline__ void load(float4& v, int voff, int soff) const {
        const rae_v4u u = __builtin_amdgcn_raw_buffer_load_b128(rs, voff * 4, soff * 4, 0);
        v = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                        __uint_as_float(u.w));
    }
    __device__ __forceinline__ void load(float& v, int voff, int soff) const {
        v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff * 4, soff * 4, 0));
    }
};

// non-temporal (streaming) row loads / stores, scalar or float4
typedef float rae_nt4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float ld_nt(const float* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ float4 ld_nt(const float4* p) {
    const rae_nt4 v = __builtin_nontemporal_load(reinterpret_cast<const rae_nt4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(float v, float* p) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_nt(float4 v, float4* p) {
    const rae_nt4 u = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(u, reinterpret_cast<rae_nt4*>(p));
}

__device__ __forceinline__ void vadd(float& acc, float v) { acc += v; }
__device__ __forceinline__ void vadd(float4& acc, float4 v) {
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
}

}  // namespace rae
