// Per-example forward + backward of the encoder and the selectional-preference decoder.
//
// One RAE_FBT-thread workgroup per example b of this rank's slice of the global batch.
// Reference computation (file:line in /root/reference):
//   S = X.W + Wb ; P = softmax(S)                     RelationClassifier.py:35-36
//   H = alpha * -sum_k P log P                         OieModel.py:81
//   wC1 = P.C1^T ; wC2 = P.C2^T                        SelectionalPreferences.py:31-32
//   left = <wC1, A[e1]> ; right = <wC2, A[e1]>         :34-35  (A[args1] used twice)
//   u = [left+right+Ab[e1], left+right+Ab[e2]]         :36-38
//   g1_t = <wC1, A[n1_t]> + right + Ab[n1_t]           :41-48
//   g2_t = <wC2, A[n2_t]> + left  + Ab[n2_t]
//   scores = [logsig(u), H, H, logsig(-g)]             :39,49-50
//   cost = -mean(scores)                               OieModel.py:90
// and its analytic backward (the reference uses T.grad, Optimizers.py:27).
// Outputs: the exchange record (rae_step.hpp); nothing is scattered here -- the row
// gradients are formed deterministically in the update kernel from these records.
//
// Latency structure (the step is ~100 examples, so each example's dependent memory round
// trips ARE the kernel time): C1/C2 are loaded once into registers at kernel entry (both
// matvecs use them), the A-row gather is issued before the encoder and stored to LDS
// after it, and the encoder spreads the feature-row gathers over all threads.
#pragma once
#include "rae_common.hpp"
#include "rae_step.hpp"

namespace rae {

#define RAE_FNW (RAE_FBT / RAE_WAVE)     // waves per forward workgroup
#define RAE_NG (RAE_FBT / 16)            // 16-lane groups per forward workgroup
#define RAE_CRA 7                        // C rows cached per lane group (r <= 7*32 = 224)
#define RAE_CCC 2                        // C column vectors cached per lane (<= 32 vectors)

struct ExampleSmem {
    float *sP, *slogP, *sdP, *swC1, *swC2, *sdw1, *sdw2, *srows, *sdots, *sAbv, *scoef,
        *sred, *spart, *sfval, *sX, *sY, *sM;
    int *sfidx, *sids, *sint;
};

__host__ __device__ inline int example_smem_floats(int dec, int m, int r, int s) {
    const int m4 = align4(m), r4 = align4(r), NJ = 2 + 2 * s, NJ4 = align4(NJ);
    const int NR = (dec == 0) ? 1 + 2 * s : 2 + 2 * s;
    const int partf = (RAE_FNW * m4 > RAE_FBT * 4 + 4) ? RAE_FNW * m4 : RAE_FBT * 4 + 4;
    int f = 3 * m4 + 4 * r4 + NR * r4 + 2 * NJ4 + align4(3 * NJ) + 64 + partf +
            2 * RAE_FBT + NJ4 + 16;
    if (dec != 0) f += 3 * r4 + 4 * r4;
    return f;
}

__device__ inline ExampleSmem carve_example_smem(char* smem, int dec, int m, int r, int s) {
    ExampleSmem S;
    const int m4 = align4(m), r4 = align4(r), NJ = 2 + 2 * s, NJ4 = align4(NJ);
    const int NR = (dec == 0) ? 1 + 2 * s : 2 + 2 * s;
    const int partf = (RAE_FNW * m4 > RAE_FBT * 4 + 4) ? RAE_FNW * m4 : RAE_FBT * 4 + 4;
    float* p = reinterpret_cast<float*>(smem);
    S.sP = p; p += m4;
    S.slogP = p; p += m4;
    S.sdP = p; p += m4;
    S.swC1 = p; p += r4;
    S.swC2 = p; p += r4;
    S.sdw1 = p; p += r4;
    S.sdw2 = p; p += r4;
    S.srows = p; p += NR * r4;
    S.sdots = p; p += NJ4;
    S.sAbv = p; p += NJ4;
    S.scoef = p; p += align4(3 * NJ);
    S.sred = p; p += 64;
    S.spart = p; p += partf;
    S.sfval = p; p += RAE_FBT;
    S.sfidx = reinterpret_cast<int*>(p); p += RAE_FBT;
    S.sids = reinterpret_cast<int*>(p); p += NJ4;
    S.sint = reinterpret_cast<int*>(p); p += 16;
    if (dec != 0) {
        S.sX = p; p += r4;
        S.sY = p; p += r4;
        S.sM = p; p += 5 * r4;
    } else {
        S.sX = S.sY = S.sM = nullptr;
    }
    return S;
}

// ---- shared pieces of every decoder's example path --------------------------------------

// ids of the NJ records (e1, e2, neg1[t], neg2[t]), feature range; Ab after a barrier
__device__ __forceinline__ void load_ids(const StepArgs& a, int64_t ex, int64_t col,
                                         ExampleSmem& S) {
    const int NJ = 2 + 2 * a.s;
    for (int j = threadIdx.x; j < NJ; j += RAE_FBT) {
        int id;
        if (j == 0) id = a.args1[ex];
        else if (j == 1) id = a.args2[ex];
        else if (j < 2 + a.s) id = a.neg1[(int64_t)(j - 2) * a.neg_stride + col];
        else id = a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
        S.sids[j] = id;
    }
    if (threadIdx.x == 0) {
        S.sint[0] = a.indptr[ex];
        S.sint[1] = a.indptr[ex + 1];
    }
}

// A-row gather straight into LDS with LDS-DMA (global_load_lds: no VGPR staging, the
// copy proceeds asynchronously until the next barrier).  Row rho -> record j (SP skips e2:
// j = rho ? rho+1 : 0; bilinear j = rho).  One wave instruction moves 64 lanes x 16 B
// (V4) or 64 x 4 B; the LDS destination is the wave-uniform row base + lane*size.
typedef __attribute__((address_space(3))) void rae_lds_void;
typedef __attribute__((address_space(1))) void rae_glob_void;

template <bool V4>
__device__ __forceinline__ void gather_rows_dma(const StepArgs& a, ExampleSmem& S, int NR,
                                                int skip_e2) {
    constexpr int VW = V4 ? 4 : 1;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rv = a.r / VW, r4 = align4(a.r);
    const int nchunk = (rv + 63) / 64;
    for (int t = w; t < NR * nchunk; t += RAE_FNW) {
        const int rho = t / nchunk, ch = t - rho * nchunk;
        const int j = (rho == 0) ? 0 : rho + skip_e2;
        const int c = ch * 64 + lane;
        float* dst = S.srows + rho * r4 + ch * 64 * VW;
        if (c < rv) {
            const float* src = a.A + (int64_t)S.sids[j] * a.r + (int64_t)c * VW;
            if constexpr (V4)
                __builtin_amdgcn_global_load_lds((rae_glob_void*)src, (rae_lds_void*)dst, 16, 0, 0);
            else
                __builtin_amdgcn_global_load_lds((rae_glob_void*)src, (rae_lds_void*)dst, 4, 0, 0);
        }
    }
}

// S = X.W + Wb over all threads (slot = feature lane group), softmax, entropy.
// Returns H (alpha-scaled) in all threads.  V4 requires m % 4 == 0.
template <bool V4, bool V4R>
__device__ __forceinline__ float encoder_forward(const StepArgs& a, ExampleSmem& S, int NR,
                                                 int skip_e2) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int m = a.m, mv = m / VW;
    const int p0 = S.sint[0], p1 = S.sint[1];
    const int nslot = RAE_FBT / mv > 0 ? RAE_FBT / mv : 1;
    const int slot = threadIdx.x / mv, c = threadIdx.x - slot * mv;
    const VT* Wv = reinterpret_cast<const VT*>(a.W);
    VT acc;
    vzero(acc);
    for (int pc = p0; pc < p1; pc += RAE_FBT) {
        const int nf = min(RAE_FBT, p1 - pc);
        __syncthreads();
        if (threadIdx.x < nf) {
            S.sfidx[threadIdx.x] = a.indices[pc + threadIdx.x];
            S.sfval[threadIdx.x] = a.values ? a.values[pc + threadIdx.x] : 1.f;
        }
        __syncthreads();
        if (pc == p0) gather_rows_dma<V4R>(a, S, NR, skip_e2);   // overlaps the W-row loads
        if (slot < nslot) {
            for (int cc = c; cc < mv; cc += RAE_FBT) {      // mv > RAE_FBT only for huge m
                for (int f = slot; f < nf; f += nslot)
                    vfma(acc, S.sfval[f], Wv[(int64_t)S.sfidx[f] * mv + cc]);
            }
        }
    }
    if (p1 <= p0) gather_rows_dma<V4R>(a, S, NR, skip_e2);      // no features
    // combine slots in fixed order
    VT* part = reinterpret_cast<VT*>(S.spart);
    if (slot < nslot && mv <= RAE_FBT) part[slot * mv + c] = acc;
    __syncthreads();
    float* sS = S.sdP;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        float v = 0.f;
        for (int sl = 0; sl < nslot; ++sl) v += S.spart[sl * m + k];
        sS[k] = v + a.Wb[k];
    }
    __syncthreads();
    float mx = -INFINITY;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) mx = fmaxf(mx, sS[k]);
    mx = block_max<RAE_FBT>(mx, S.sred);
    float se = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) se += expf(sS[k] - mx);
    se = block_sum<RAE_FBT>(se, S.sred + 8);
    const float lse = logf(se);
    float hp = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        const float lp = (sS[k] - mx) - lse;
        const float p = expf(sS[k] - mx) / se;
        S.slogP[k] = lp;
        S.sP[k] = p;
        hp += p * lp;
    }
    hp = block_sum<RAE_FBT>(hp, S.sred + 16);
    return -a.alpha * hp;
}

// Register cache of C1, C2 (row-major (r, m)) in the lane-group layout:
// group gid (16 lanes) owns rows i = r0 + gid + NG*ra, lane q owns column vectors
// c = c0 + q + 16*cc.  When the whole matrix fits (r <= NG*RAE_CRA, m/VW <= 16*RAE_CCC) it is
// loaded once and serves both matvecs; otherwise chunks are (re)loaded from L2.
template <bool V4>
struct CCache {
    typedef typename VecT<V4>::T VT;
    VT c1[RAE_CRA][RAE_CCC], c2[RAE_CRA][RAE_CCC];

    __device__ __forceinline__ void load(const float* C1, const float* C2, int r, int mv, int r0,
                                         int c0) {
        const VT* C1v = reinterpret_cast<const VT*>(C1);
        const VT* C2v = reinterpret_cast<const VT*>(C2);
        const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
#pragma unroll
        for (int ra = 0; ra < RAE_CRA; ++ra) {
            const int i = r0 + gid + RAE_NG * ra;
#pragma unroll
            for (int cc = 0; cc < RAE_CCC; ++cc) {
                const int c = c0 + q + 16 * cc;
                if (i < r && c < mv) {
                    c1[ra][cc] = C1v[(int64_t)i * mv + c];
                    c2[ra][cc] = C2v[(int64_t)i * mv + c];
                } else {
                    vzero(c1[ra][cc]);
                    vzero(c2[ra][cc]);
                }
            }
        }
    }
};

__host__ __device__ inline bool ccache_fits(int r, int mv) {
    return r <= RAE_NG * RAE_CRA && mv <= 16 * RAE_CCC;
}

// wC1 = C1.P, wC2 = C2.P  -> S.swC1, S.swC2
template <bool V4>
__device__ __forceinline__ void sp_project(const StepArgs& a, ExampleSmem& S, CCache<V4>& cc_,
                                           bool fits) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int r = a.r, mv = a.m / VW;
    const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
    const VT* Pv = reinterpret_cast<const VT*>(S.sP);
    for (int r0 = 0; r0 < r; r0 += RAE_NG * RAE_CRA) {
        float s1[RAE_CRA], s2[RAE_CRA];
#pragma unroll
        for (int ra = 0; ra < RAE_CRA; ++ra) s1[ra] = s2[ra] = 0.f;
        for (int c0 = 0; c0 < mv; c0 += 16 * RAE_CCC) {
            if (!fits) cc_.load(a.C1, a.C2, r, mv, r0, c0);
#pragma unroll
            for (int cc = 0; cc < RAE_CCC; ++cc) {
                const int c = c0 + q + 16 * cc;
                if (c < mv) {
                    const VT p = Pv[c];
#pragma unroll
                    for (int ra = 0; ra < RAE_CRA; ++ra) {
                        s1[ra] += vdot(cc_.c1[ra][cc], p);
                        s2[ra] += vdot(cc_.c2[ra][cc], p);
                    }
                }
            }
        }
#pragma unroll
        for (int ra = 0; ra < RAE_CRA; ++ra) {
            const float t1 = group16_sum(s1[ra]);
            const float t2 = group16_sum(s2[ra]);
            const int i = r0 + gid + RAE_NG * ra;
            if (q == 0 && i < r) {
                S.swC1[i] = t1;
                S.swC2[i] = t2;
            }
        }
    }
}

// dP = C1^T.dw1 + C2^T.dw2 (+ S.sdP already holding other dP terms) + entropy term,
// then dS = softmax-backward; result in S.sdP.  has_c: C1/C2 terms present.
template <bool V4>
__device__ __forceinline__ void sp_project_back_and_softmax(const StepArgs& a, ExampleSmem& S,
                                                            CCache<V4>& cc_, bool fits,
                                                            bool has_c) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int m = a.m, r = a.r, m4 = align4(m), mv = m / VW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
    if (has_c) {
        for (int c0 = 0; c0 < mv; c0 += 16 * RAE_CCC) {
            VT acc[RAE_CCC];
#pragma unroll
            for (int cc = 0; cc < RAE_CCC; ++cc) vzero(acc[cc]);
            for (int r0 = 0; r0 < r; r0 += RAE_NG * RAE_CRA) {
                if (!fits) cc_.load(a.C1, a.C2, r, mv, r0, c0);
#pragma unroll
                for (int ra = 0; ra < RAE_CRA; ++ra) {
                    const int i = r0 + gid + RAE_NG * ra;
                    const float d1 = i < r ? S.sdw1[i] : 0.f;
                    const float d2 = i < r ? S.sdw2[i] : 0.f;
#pragma unroll
                    for (int cc = 0; cc < RAE_CCC; ++cc) {
                        vfma(acc[cc], d1, cc_.c1[ra][cc]);
                        vfma(acc[cc], d2, cc_.c2[ra][cc]);
                    }
                }
            }
            // reduce over the 4 lane groups of the wave, then waves through LDS
#pragma unroll
            for (int cc = 0; cc < RAE_CCC; ++cc) {
                float* v = reinterpret_cast<float*>(&acc[cc]);
#pragma unroll
                for (int e = 0; e < VW; ++e) {
                    v[e] += __shfl_xor(v[e], 16, 64);
                    v[e] += __shfl_xor(v[e], 32, 64);
                }
                const int c = c0 + q + 16 * cc;
                if (lane < 16 && c < mv)
                    reinterpret_cast<VT*>(S.spart + w * m4)[c] = acc[cc];
            }
            __syncthreads();
            for (int k = threadIdx.x; k < m; k += RAE_FBT) {
                const int cv = k / VW;
                if (cv >= c0 && cv < c0 + 16 * RAE_CCC) {
                    float dp = 0.f;
#pragma unroll
                    for (int ww = 0; ww < RAE_FNW; ++ww) dp += S.spart[ww * m4 + k];
                    S.sdP[k] += dp;
                }
            }
            __syncthreads();
        }
    }
    const float ce = 2.f * a.alpha * a.invD;   // d cost / dH_b = -2/D ; dH/dP = -alpha(logP+1)
    float sd = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        const float dp = S.sdP[k] + ce * (S.slogP[k] + 1.f);
        S.sdP[k] = dp;
        sd += S.sP[k] * dp;
    }
    sd = block_sum<RAE_FBT>(sd, S.sred + 24);
    for (int k = threadIdx.x; k < m; k += RAE_FBT) S.sdP[k] = S.sP[k] * (S.sdP[k] - sd);
    __syncthreads();
}

// write the common part of the exchange record
__device__ __forceinline__ void write_record(const StepArgs& a, ExampleSmem& S, float* rec) {
    const int m = a.m, r = a.r, NJ = 2 + 2 * a.s;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        rec[a.lay.oP + k] = S.sP[k];
        rec[a.lay.odS + k] = S.sdP[k];
    }
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        rec[a.lay.oV1 + i] = S.swC1[i];
        rec[a.lay.oV2 + i] = S.swC2[i];
        rec[a.lay.odw1 + i] = S.sdw1[i];
        rec[a.lay.odw2 + i] = S.sdw2[i];
    }
    for (int j = threadIdx.x; j < 3 * NJ; j += RAE_FBT) rec[a.lay.ocoef + j] = S.scoef[j];
    if (threadIdx.x == 0) rec[a.lay.oloss] = S.sred[32];
}

// ---- the SP example path ---------------------------------------------------------------
template <bool V4M, bool V4R>
__device__ void sp_example(const StepArgs& a, int64_t g, int bl, char* smem) {
    const int m = a.m, r = a.r, s = a.s, NR = 1 + 2 * s;
    const int r4 = align4(r);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int VWM = V4M ? 4 : 1;
    ExampleSmem S = carve_example_smem(smem, 0, m, r, s);
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;

    // round trip 1: ids + feature range; C1/C2 register cache (independent of everything)
    CCache<V4M> cc_;
    const bool fits = ccache_fits(r, m / VWM);
    if (fits) cc_.load(a.C1, a.C2, r, m / VWM, 0, 0);
    load_ids(a, ex, col, S);
    __syncthreads();
    // round trip 2: Ab values, A-row gather (prefetched into registers), features, W rows
    const int NJ = 2 + 2 * s;
    for (int j = threadIdx.x; j < NJ; j += RAE_FBT) S.sAbv[j] = a.Ab[S.sids[j]];
    const float H = encoder_forward<V4M, V4R>(a, S, NR, 1);
    __syncthreads();
    sp_project<V4M>(a, S, cc_, fits);
    __syncthreads();

    // dot products: row rho on wave rho % NW
    for (int rho = w; rho < NR; rho += RAE_FNW) {
        const float* row = S.srows + rho * r4;
        float d1 = 0.f, d2 = 0.f;
        const bool isn2 = rho > s;                // rows 1..s: neg1, s+1..2s: neg2
        const float* wv = isn2 ? S.swC2 : S.swC1;
        for (int i = lane; i < r; i += RAE_WAVE) {
            d1 += row[i] * wv[i];
            if (rho == 0) d2 += row[i] * S.swC2[i];
        }
        d1 = wave_sum(d1);
        if (rho == 0) d2 = wave_sum(d2);
        if (lane == 0) {
            if (rho == 0) {
                S.sdots[0] = d1;     // left  = <wC1, A[e1]>
                S.sdots[1] = d2;     // right = <wC2, A[e1]>
            } else {
                S.sdots[rho + 1] = d1;   // record j = rho + 1
            }
        }
    }
    __syncthreads();

    // scores, loss, coefficients (wave 0)
    if (w == 0) {
        const float left = S.sdots[0], right = S.sdots[1];
        float sdg1 = 0.f, sdg2 = 0.f, sls = 0.f;
        for (int t = lane; t < s; t += RAE_WAVE) {
            const float g1 = S.sdots[2 + t] + right + S.sAbv[2 + t];
            const float g2 = S.sdots[2 + s + t] + left + S.sAbv[2 + s + t];
            const float dg1 = sigmoid(g1) * a.invD;
            const float dg2 = sigmoid(g2) * a.invD;
            float* c1 = S.scoef + 3 * (2 + t);
            float* c2 = S.scoef + 3 * (2 + s + t);
            c1[0] = dg1; c1[1] = 0.f; c1[2] = dg1;
            c2[0] = 0.f; c2[1] = dg2; c2[2] = dg2;
            sdg1 += dg1;
            sdg2 += dg2;
            sls += log_sigmoid(-g1) + log_sigmoid(-g2);
        }
        sdg1 = wave_sum(sdg1);
        sdg2 = wave_sum(sdg2);
        sls = wave_sum(sls);
        if (lane == 0) {
            const float one = left + right;
            const float u1 = one + S.sAbv[0], u2 = one + S.sAbv[1];
            const float du1 = -sigmoid(-u1) * a.invD;
            const float du2 = -sigmoid(-u2) * a.invD;
            const float dl = du1 + du2 + sdg2;     // d cost / d left
            const float dr = du1 + du2 + sdg1;     // d cost / d right
            S.scoef[0] = dl; S.scoef[1] = dr; S.scoef[2] = du1;
            S.scoef[3] = 0.f; S.scoef[4] = 0.f; S.scoef[5] = du2;
            S.sred[32] = log_sigmoid(u1) + log_sigmoid(u2) + 2.f * H + sls;
        }
    }
    __syncthreads();

    // dwC1 = dl*a1 + sum_t dg1_t n1_t ; dwC2 = dr*a1 + sum_t dg2_t n2_t
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        const float a1 = S.srows[i];
        float v1 = S.scoef[0] * a1, v2 = S.scoef[1] * a1;
        for (int t = 0; t < s; ++t) {
            v1 += S.scoef[3 * (2 + t)] * S.srows[(1 + t) * r4 + i];
            v2 += S.scoef[3 * (2 + s + t) + 1] * S.srows[(1 + s + t) * r4 + i];
        }
        S.sdw1[i] = v1;
        S.sdw2[i] = v2;
    }
    for (int k = threadIdx.x; k < m; k += RAE_FBT) S.sdP[k] = 0.f;
    __syncthreads();
    sp_project_back_and_softmax<V4M>(a, S, cc_, fits, true);
    write_record(a, S, a.ex + (int64_t)bg * a.lay.rec);
}

}  // namespace rae
