// Per-example forward + backward of the encoder and the selectional-preference decoder.
//
// One 256-thread workgroup per example b of this rank's slice of the global batch.
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
#pragma once
#include "rae_common.hpp"
#include "rae_step.hpp"

namespace rae {

struct ExampleSmem {
    float *sP, *slogP, *sdP, *swC1, *swC2, *sdw1, *sdw2, *srows, *sdots, *sAbv, *scoef,
        *sred, *spart, *sfval, *sX, *sY, *sM;
    int *sfidx, *sids;
};

__host__ __device__ inline int example_smem_floats(int dec, int m, int r, int s) {
    const int m4 = align4(m), r4 = align4(r), NJ = 2 + 2 * s, NJ4 = align4(NJ);
    const int NR = (dec == 0) ? 1 + 2 * s : 2 + 2 * s;
    int f = 3 * m4 + 4 * r4 + NR * r4 + 2 * NJ4 + align4(3 * NJ) + 64 + RAE_NWAVE * m4 +
            2 * RAE_BT + NJ4;
    if (dec != 0) f += 3 * r4 + 4 * r4;   // bilinear: x, y, Ma2/MTa1 ... (rae_bilinear.hpp)
    return f;
}

__device__ inline ExampleSmem carve_example_smem(char* smem, int dec, int m, int r, int s) {
    ExampleSmem S;
    const int m4 = align4(m), r4 = align4(r), NJ = 2 + 2 * s, NJ4 = align4(NJ);
    const int NR = (dec == 0) ? 1 + 2 * s : 2 + 2 * s;
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
    S.spart = p; p += RAE_NWAVE * m4;
    S.sfval = p; p += RAE_BT;
    S.sfidx = reinterpret_cast<int*>(p); p += RAE_BT;
    S.sids = reinterpret_cast<int*>(p); p += NJ4;
    if (dec != 0) {
        S.sX = p; p += r4;
        S.sY = p; p += r4;
        S.sM = p; p += 4 * r4 + r4;
    } else {
        S.sX = S.sY = S.sM = nullptr;
    }
    return S;
}

// ---- shared pieces of every decoder's example path --------------------------------------

// ids of the NJ records (e1, e2, neg1[t], neg2[t]) and their Ab values
__device__ __forceinline__ void load_ids(const StepArgs& a, int64_t ex, int64_t col,
                                         ExampleSmem& S) {
    const int NJ = 2 + 2 * a.s;
    for (int j = threadIdx.x; j < NJ; j += RAE_BT) {
        int id;
        if (j == 0) id = a.args1[ex];
        else if (j == 1) id = a.args2[ex];
        else if (j < 2 + a.s) id = a.neg1[(int64_t)(j - 2) * a.neg_stride + col];
        else id = a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
        S.sids[j] = id;
        S.sAbv[j] = a.Ab[id];
    }
}

// gather A rows listed by `rowj` (record indices into sids) into srows (stride r4)
template <bool V4R>
__device__ __forceinline__ void gather_rows(const StepArgs& a, ExampleSmem& S, int NR,
                                            int rowj_skip_e2) {
    const int r = a.r, r4 = align4(r);
    // rho -> record j: rho 0 = e1; SP skips e2 (rowj_skip_e2), bilinear keeps it.
    if (V4R) {
        const int q = r >> 2, q4 = r4 >> 2;
        const float4* A4 = reinterpret_cast<const float4*>(a.A);
        float4* R4 = reinterpret_cast<float4*>(S.srows);
        for (int t = threadIdx.x; t < NR * q; t += RAE_BT) {
            const int rho = t / q, c = t - rho * q;
            const int j = (rho == 0) ? 0 : rho + rowj_skip_e2;
            R4[rho * q4 + c] = A4[(int64_t)S.sids[j] * q + c];
        }
    } else {
        for (int t = threadIdx.x; t < NR * r; t += RAE_BT) {
            const int rho = t / r, c = t - rho * r;
            const int j = (rho == 0) ? 0 : rho + rowj_skip_e2;
            S.srows[rho * r4 + c] = a.A[(int64_t)S.sids[j] * r + c];
        }
    }
}

// S = X.W + Wb, softmax, entropy.  Returns H (alpha-scaled) in all threads.
__device__ __forceinline__ float encoder_forward(const StepArgs& a, int64_t ex, ExampleSmem& S) {
    const int m = a.m;
    const int p0 = a.indptr[ex], p1 = a.indptr[ex + 1];
    float acc[2] = {0.f, 0.f};   // m <= 2*RAE_BT handled; larger m loops below
    float* sS = S.sdP;           // scratch for S
    for (int k0 = 0; k0 < m; k0 += 2 * RAE_BT) {
        acc[0] = acc[1] = 0.f;
        for (int pc = p0; pc < p1; pc += RAE_BT) {
            const int nf = min(RAE_BT, p1 - pc);
            __syncthreads();
            if (threadIdx.x < nf) {
                S.sfidx[threadIdx.x] = a.indices[pc + threadIdx.x];
                S.sfval[threadIdx.x] = a.values ? a.values[pc + threadIdx.x] : 1.f;
            }
            __syncthreads();
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = k0 + h * RAE_BT + threadIdx.x;
                if (k < m) {
                    float v = acc[h];
                    for (int f = 0; f < nf; ++f)
                        v += S.sfval[f] * a.W[(int64_t)S.sfidx[f] * m + k];
                    acc[h] = v;
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int k = k0 + h * RAE_BT + threadIdx.x;
            if (k < m) sS[k] = acc[h] + a.Wb[k];
        }
    }
    __syncthreads();
    float mx = -INFINITY;
    for (int k = threadIdx.x; k < m; k += RAE_BT) mx = fmaxf(mx, sS[k]);
    mx = block_max(mx, S.sred);
    float se = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_BT) se += expf(sS[k] - mx);
    se = block_sum(se, S.sred + 8);
    const float lse = logf(se);
    float hp = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_BT) {
        const float lp = (sS[k] - mx) - lse;
        const float p = expf(sS[k] - mx) / se;
        S.slogP[k] = lp;
        S.sP[k] = p;
        hp += p * lp;
    }
    hp = block_sum(hp, S.sred + 16);
    return -a.alpha * hp;
}

// wC1 = C1.P, wC2 = C2.P (C row-major (r,m)): 16-lane groups own rows, lanes own columns.
template <bool V4M>
__device__ __forceinline__ void sp_project(const StepArgs& a, ExampleSmem& S) {
    const int m = a.m, r = a.r;
    const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
    if (V4M) {
        const int mq = m >> 2;
        const float4* C14 = reinterpret_cast<const float4*>(a.C1);
        const float4* C24 = reinterpret_cast<const float4*>(a.C2);
        const float4* P4 = reinterpret_cast<const float4*>(S.sP);
        for (int i = gid; i < r; i += RAE_BT / 16) {
            float s1 = 0.f, s2 = 0.f;
            for (int c = q; c < mq; c += 16) {
                const float4 p = P4[c];
                const float4 x = C14[(int64_t)i * mq + c];
                const float4 y = C24[(int64_t)i * mq + c];
                s1 += x.x * p.x + x.y * p.y + x.z * p.z + x.w * p.w;
                s2 += y.x * p.x + y.y * p.y + y.z * p.z + y.w * p.w;
            }
            s1 = group16_sum(s1);
            s2 = group16_sum(s2);
            if (q == 0) {
                S.swC1[i] = s1;
                S.swC2[i] = s2;
            }
        }
    } else {
        for (int i = gid; i < r; i += RAE_BT / 16) {
            float s1 = 0.f, s2 = 0.f;
            for (int k = q; k < m; k += 16) {
                const float p = S.sP[k];
                s1 += a.C1[(int64_t)i * m + k] * p;
                s2 += a.C2[(int64_t)i * m + k] * p;
            }
            s1 = group16_sum(s1);
            s2 = group16_sum(s2);
            if (q == 0) {
                S.swC1[i] = s1;
                S.swC2[i] = s2;
            }
        }
    }
}

// dP = C1^T.dw1 + C2^T.dw2 (+ entropy term), then dS = softmax-backward; writes S.sdP.
#define RAE_MAXCC 8   // m <= 16*4*8 = 512 (V4) / 16*8*... handled by loop below
template <bool V4M>
__device__ __forceinline__ void sp_project_back_and_softmax(const StepArgs& a, ExampleSmem& S,
                                                            const float* C1, const float* C2,
                                                            bool has_sp) {
    const int m = a.m, r = a.r, m4 = align4(m);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
    // zero partials
    for (int k = threadIdx.x; k < RAE_NWAVE * m4; k += RAE_BT) S.spart[k] = 0.f;
    __syncthreads();
    if (has_sp) {
        if (V4M) {
            const int mq = m >> 2;
            const float4* C14 = reinterpret_cast<const float4*>(C1);
            const float4* C24 = reinterpret_cast<const float4*>(C2);
            for (int c0 = 0; c0 < mq; c0 += 16 * RAE_MAXCC) {
                float4 acc[RAE_MAXCC];
#pragma unroll
                for (int cc = 0; cc < RAE_MAXCC; ++cc) acc[cc] = make_float4(0.f, 0.f, 0.f, 0.f);
                for (int i = gid; i < r; i += RAE_BT / 16) {
                    const float d1 = S.sdw1[i], d2 = S.sdw2[i];
#pragma unroll
                    for (int cc = 0; cc < RAE_MAXCC; ++cc) {
                        const int c = c0 + q + 16 * cc;
                        if (c < mq) {
                            const float4 x = C14[(int64_t)i * mq + c];
                            const float4 y = C24[(int64_t)i * mq + c];
                            acc[cc].x += x.x * d1 + y.x * d2;
                            acc[cc].y += x.y * d1 + y.y * d2;
                            acc[cc].z += x.z * d1 + y.z * d2;
                            acc[cc].w += x.w * d1 + y.w * d2;
                        }
                    }
                }
#pragma unroll
                for (int cc = 0; cc < RAE_MAXCC; ++cc) {
                    float4 v = acc[cc];
                    v.x += __shfl_xor(v.x, 16, 64); v.x += __shfl_xor(v.x, 32, 64);
                    v.y += __shfl_xor(v.y, 16, 64); v.y += __shfl_xor(v.y, 32, 64);
                    v.z += __shfl_xor(v.z, 16, 64); v.z += __shfl_xor(v.z, 32, 64);
                    v.w += __shfl_xor(v.w, 16, 64); v.w += __shfl_xor(v.w, 32, 64);
                    const int c = c0 + q + 16 * cc;
                    if (lane < 16 && c < mq) {
                        float* dst = S.spart + w * m4 + 4 * c;
                        dst[0] += v.x; dst[1] += v.y; dst[2] += v.z; dst[3] += v.w;
                    }
                }
            }
        } else {
            for (int k0 = 0; k0 < m; k0 += 16 * RAE_MAXCC) {
                float acc[RAE_MAXCC];
#pragma unroll
                for (int cc = 0; cc < RAE_MAXCC; ++cc) acc[cc] = 0.f;
                for (int i = gid; i < r; i += RAE_BT / 16) {
                    const float d1 = S.sdw1[i], d2 = S.sdw2[i];
#pragma unroll
                    for (int cc = 0; cc < RAE_MAXCC; ++cc) {
                        const int k = k0 + q + 16 * cc;
                        if (k < m) acc[cc] += C1[(int64_t)i * m + k] * d1 + C2[(int64_t)i * m + k] * d2;
                    }
                }
#pragma unroll
                for (int cc = 0; cc < RAE_MAXCC; ++cc) {
                    float v = acc[cc];
                    v += __shfl_xor(v, 16, 64);
                    v += __shfl_xor(v, 32, 64);
                    const int k = k0 + q + 16 * cc;
                    if (lane < 16 && k < m) S.spart[w * m4 + k] += v;
                }
            }
        }
    }
    __syncthreads();
    // dP: + extra (already in sdP by caller for bilinear) + entropy term
    const float ce = 2.f * a.alpha * a.invD;   // d cost / dH_b = -2/D ; dH/dP = -alpha(logP+1)
    float sd = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_BT) {
        float dp = S.sdP[k];
#pragma unroll
        for (int ww = 0; ww < RAE_NWAVE; ++ww) dp += S.spart[ww * m4 + k];
        dp += ce * (S.slogP[k] + 1.f);
        S.sdP[k] = dp;
        sd += S.sP[k] * dp;
    }
    sd = block_sum(sd, S.sred + 24);
    for (int k = threadIdx.x; k < m; k += RAE_BT) S.sdP[k] = S.sP[k] * (S.sdP[k] - sd);
    __syncthreads();
}

// ---- the SP example path ---------------------------------------------------------------
template <bool V4M, bool V4R>
__device__ void sp_example(const StepArgs& a, int64_t g, int bl, char* smem) {
    const int m = a.m, r = a.r, s = a.s, NJ = 2 + 2 * s, NR = 1 + 2 * s;
    const int r4 = align4(r);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    ExampleSmem S = carve_example_smem(smem, 0, m, r, s);
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;

    load_ids(a, ex, col, S);
    __syncthreads();
    gather_rows<V4R>(a, S, NR, 1);        // rows: e1, n1[0..s), n2[0..s)
    const float H = encoder_forward(a, ex, S);
    __syncthreads();
    sp_project<V4M>(a, S);
    __syncthreads();

    // dot products: row rho on wave rho % 4
    for (int rho = w; rho < NR; rho += RAE_NWAVE) {
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
    for (int i = threadIdx.x; i < r; i += RAE_BT) {
        const float a1 = S.srows[i];
        float v1 = S.scoef[0] * a1, v2 = S.scoef[1] * a1;
        for (int t = 0; t < s; ++t) {
            v1 += S.scoef[3 * (2 + t)] * S.srows[(1 + t) * r4 + i];
            v2 += S.scoef[3 * (2 + s + t) + 1] * S.srows[(1 + s + t) * r4 + i];
        }
        S.sdw1[i] = v1;
        S.sdw2[i] = v2;
    }
    for (int k = threadIdx.x; k < m; k += RAE_BT) S.sdP[k] = 0.f;
    __syncthreads();
    sp_project_back_and_softmax<V4M>(a, S, a.C1, a.C2, true);

    // exchange record
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    for (int k = threadIdx.x; k < m; k += RAE_BT) {
        rec[a.lay.oP + k] = S.sP[k];
        rec[a.lay.odS + k] = S.sdP[k];
    }
    for (int i = threadIdx.x; i < r; i += RAE_BT) {
        rec[a.lay.oV1 + i] = S.swC1[i];
        rec[a.lay.oV2 + i] = S.swC2[i];
        rec[a.lay.odw1 + i] = S.sdw1[i];
        rec[a.lay.odw2 + i] = S.sdw2[i];
    }
    for (int j = threadIdx.x; j < 3 * NJ; j += RAE_BT) rec[a.lay.ocoef + j] = S.scoef[j];
    if (threadIdx.x == 0) rec[a.lay.oloss] = S.sred[32];
}

}  // namespace rae
