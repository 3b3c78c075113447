// func['label_<split>'] (learning/OieInduction.py:151-155 -> RelationClassifier.py:39-48):
//   S = X.W + Wb ; labels = argmax_k S (first maximum, numpy/Theano argmax) ; probs = softmax(S)
// over any row range of a CSR split with fixed weights.  HBM-streaming kernel: one wave per
// example (grid-strided), the example's feature ids loaded lane-parallel, then the W rows
// gathered RPW rows per wave instruction (LPR lanes per row, float4 columns when m % 4 == 0),
// U rounds of loads in flight before the FMAs; the RPW row partials are folded with
// permlane swaps, softmax / argmax over the lanes of group 0.
#pragma once
#include "rae_common.hpp"

namespace rae {

template <bool V4>
__device__ __forceinline__ void lbl_fold(typename VecT<V4>::T& v, int rpw) {
    float* e = reinterpret_cast<float*>(&v);
    constexpr int VW = V4 ? 4 : 1;
#pragma unroll
    for (int q = 0; q < VW; ++q) {
        if (rpw >= 4) e[q] += __uint_as_float(xor16_u32(__float_as_uint(e[q])));
        if (rpw >= 2) e[q] += __uint_as_float(xor32_u32(__float_as_uint(e[q])));
    }
}

// (v, k) before (best, bk) in numpy argmax order; k == INT_MAX marks "no candidate"
__device__ __forceinline__ bool lbl_better(float v, int k, float best, int bk) {
    if (k == 0x7fffffff) return false;
    if (bk == 0x7fffffff) return true;
    const bool vn = v != v, bn = best != best;
    if (bn) return vn && k < bk;
    if (vn) return true;
    return v > best || (v == best && k < bk);
}

template <bool V4>
__global__ __launch_bounds__(RAE_BT) void k_label(const int32_t* __restrict__ indptr,
                                                  const int32_t* __restrict__ indices,
                                                  const float* __restrict__ values,
                                                  const float* __restrict__ W,
                                                  const float* __restrict__ Wb, int m,
                                                  int64_t row0, int64_t nrows,
                                                  int64_t* __restrict__ labels,
                                                  float* __restrict__ probs) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    constexpr int U = 4;                         // load rounds in flight
    const int lane = threadIdx.x & 63;
    const int mv = m / VW;                       // vector columns (m % VW == 0)
    const int LPR = mv <= 16 ? 16 : (mv <= 32 ? 32 : 64);
    const int RPW = 64 / LPR;                    // rows per wave instruction
    const int NQ = (mv + 63) / 64;               // column chunks per lane (LPR == 64 only)
    const int grp = lane / LPR, col = lane - grp * LPR;
    const VT* Wv = reinterpret_cast<const VT*>(W);
    const VT* Wbv = reinterpret_cast<const VT*>(Wb);
    const int64_t nw = (int64_t)gridDim.x * RAE_NWAVE;
    for (int64_t e = blockIdx.x * (int64_t)RAE_NWAVE + (threadIdx.x >> 6); e < nrows; e += nw) {
        const int64_t ex = row0 + e;
        const int p0 = indptr[ex], p1 = indptr[ex + 1];
        VT acc[2];
        vzero(acc[0]);
        vzero(acc[1]);
        for (int pc = p0; pc < p1; pc += 64) {
            const int nf = min(64, p1 - pc);
            const int fid = lane < nf ? indices[pc + lane] : 0;
            const float fval = (lane < nf) ? (values ? values[pc + lane] : 1.f) : 0.f;
            for (int t0 = 0; t0 < nf; t0 += U * RPW) {
                VT x[U][2];
                float v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int t = t0 + u * RPW + grp;
                    const int tc = t < nf ? t : 0;
                    // both shuffles run on every lane: a ds_bpermute inside the t < nf branch
                    // reads source lanes that are inactive there (garbage), which dropped the
                    // last feature of rows with nnz = 17, 33, ... (LPR = 16 / 32)
                    const int f = __shfl(fid, tc, 64);
                    const float fv = __shfl(fval, tc, 64);
                    v[u] = t < nf ? fv : 0.f;
                    const VT* row = Wv + (int64_t)f * mv;
                    x[u][0] = row[col < mv ? col : 0];
                    if (NQ > 1) x[u][1] = row[col + 64 < mv ? col + 64 : 0];
                    else vzero(x[u][1]);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int q = 0; q < 2; ++q) vfma(acc[q], v[u], x[u][q]);
            }
        }
        lbl_fold<V4>(acc[0], RPW);
        // group 0 lanes hold S for columns col (+64): add Wb, argmax, softmax.  argmax has
        // numpy's semantics (Theano's MaxAndArgmax calls PyArray_ArgMax): the first maximum,
        // NaN counting as the maximum (first NaN wins) -- so a diverged row still gets a label
        // in [0, m), as the reference's does
        float best = -INFINITY;
        int bk = 0x7fffffff;                     // no candidate yet
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int c = col + 64 * q;
            const bool cv = grp == 0 && q < NQ && c < mv;
            VT sv = acc[q];
            if (cv) vadd(sv, Wbv[c]);
            acc[q] = sv;
            const float* se = reinterpret_cast<const float*>(&sv);
#pragma unroll
            for (int i = 0; i < VW; ++i)
                if (cv && lbl_better(se[i], c * VW + i, best, bk)) { best = se[i]; bk = c * VW + i; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ob = __shfl_xor(best, o, 64);
            const int ok = __shfl_xor(bk, o, 64);
            if (lbl_better(ob, ok, best, bk)) { best = ob; bk = ok; }
        }
        if (lane == 0) labels[e] = bk;
        if (probs) {
            float se = 0.f;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int c = col + 64 * q;
                if (grp == 0 && q < NQ && c < mv) {
                    const float* s = reinterpret_cast<const float*>(&acc[q]);
#pragma unroll
                    for (int i = 0; i < VW; ++i) se += expf(s[i] - best);
                }
            }
            se = wave_sum(se);
            VT* pr = reinterpret_cast<VT*>(probs + e * m);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int c = col + 64 * q;
                if (grp == 0 && q < NQ && c < mv) {
                    VT o = acc[q];
                    float* oe = reinterpret_cast<float*>(&o);
#pragma unroll
                    for (int i = 0; i < VW; ++i) oe[i] = expf(oe[i] - best) / se;
                    pr[c] = o;
                }
            }
        }
    }
}

}  // namespace rae
