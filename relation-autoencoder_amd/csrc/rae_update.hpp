// Deterministic per-row gradient reduction + optimizer update over the global batch.
//
// Replaces the reference's dense T.grad + dense AdaGrad sweep (learning/Optimizers.py:27-33)
// by: one wavefront per distinct referenced row (from the per-step row index), which sums
// that row's contributions from the exchange records in (row, record) order and applies
// the update in place.  Rows not referenced by the batch have zero gradient in the
// reference and AdaGrad leaves them bit-unchanged (p - lr*0/(sqrt(acc)+1e-6) == p), so
// skipping them is exact.  With lambda1/lambda2 != 0 every W element has a non-zero
// regulariser gradient: then the W rows are only reduced into a dense scratch here and the
// dense sweep kernel (k_dense_w) applies the full update, as the reference does.
#pragma once
#include "rae_common.hpp"
#include "rae_index.hpp"
#include "rae_step.hpp"

namespace rae {

#define RAE_MAXQ 4   // float4 chunks per lane: rows up to 4*64*4 = 1024 floats

// update one contiguous parameter row held as float4 chunks g[] (lane-strided)
template <int OPT>
__device__ __forceinline__ void update_row4(float* p, float* acc, const float4* g, int nq,
                                            float lr, int lane) {
    float4* p4 = reinterpret_cast<float4*>(p);
    float4* a4 = reinterpret_cast<float4*>(acc);
#pragma unroll
    for (int cc = 0; cc < RAE_MAXQ; ++cc) {
        const int c = lane + RAE_WAVE * cc;
        if (c < nq) {
            float4 v = p4[c];
            float4 ac = (OPT == 0) ? a4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
            v.x = opt_update<OPT>(v.x, &ac.x, g[cc].x, lr);
            v.y = opt_update<OPT>(v.y, &ac.y, g[cc].y, lr);
            v.z = opt_update<OPT>(v.z, &ac.z, g[cc].z, lr);
            v.w = opt_update<OPT>(v.w, &ac.w, g[cc].w, lr);
            p4[c] = v;
            if (OPT == 0) a4[c] = ac;
        }
    }
}

template <int OPT>
__device__ __forceinline__ void update_row1(float* p, float* acc, const float* g, int n,
                                            float lr, int lane) {
#pragma unroll
    for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) {
        const int c = lane + RAE_WAVE * cc;
        if (c < n) {
            float ac = (OPT == 0) ? acc[c] : 0.f;
            p[c] = opt_update<OPT>(p[c], &ac, g[cc], lr);
            if (OPT == 0) acc[c] = ac;
        }
    }
}

__device__ __forceinline__ void fma4(float4& g, float s, const float4 v) {
    g.x += s * v.x; g.y += s * v.y; g.z += s * v.z; g.w += s * v.w;
}

// ---- A / Ab rows ---------------------------------------------------------------------
template <int OPT, bool V4>
__device__ void task_entity_row(const StepArgs& a, int h, int u, int lane) {
    const int r = a.r, NJ = 2 + 2 * a.s;
    const int32_t* hdr = a.hdrA + 2 * h;
    const int64_t base = (int64_t)h * a.RA;
    const int e = a.urowA[base + u];
    const int st = a.ustartA[base + u];
    const int en = (u + 1 < hdr[1]) ? a.ustartA[base + u + 1] : hdr[0];
    const bool xy = a.dec != 0;
    float gb = 0.f;
    if (V4) {
        const int nq = r >> 2;
        float4 g[RAE_MAXQ];
#pragma unroll
        for (int cc = 0; cc < RAE_MAXQ; ++cc) g[cc] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int i = st; i < en; ++i) {
            const int rec = a.srecA[base + i];
            const int b = rec / NJ, j = rec - b * NJ;
            const float* er = a.ex + (int64_t)b * a.lay.rec;
            const float al = er[a.lay.ocoef + 3 * j];
            const float be = er[a.lay.ocoef + 3 * j + 1];
            gb += er[a.lay.ocoef + 3 * j + 2];
            const float4* V1 = reinterpret_cast<const float4*>(er + a.lay.oV1);
            const float4* V2 = reinterpret_cast<const float4*>(er + a.lay.oV2);
#pragma unroll
            for (int cc = 0; cc < RAE_MAXQ; ++cc) {
                const int c = lane + RAE_WAVE * cc;
                if (c < nq) {
                    if (al != 0.f) fma4(g[cc], al, V1[c]);
                    if (be != 0.f) fma4(g[cc], be, V2[c]);
                    if (xy && j < 2) {
                        const float4* XY =
                            reinterpret_cast<const float4*>(er + (j == 0 ? a.lay.oX : a.lay.oY));
                        fma4(g[cc], 1.f, XY[c]);
                    }
                }
            }
        }
        update_row4<OPT>(a.A + (int64_t)e * r, a.aA ? a.aA + (int64_t)e * r : nullptr, g, nq,
                         a.lr, lane);
    } else {
        float g[4 * RAE_MAXQ];
#pragma unroll
        for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) g[cc] = 0.f;
        for (int i = st; i < en; ++i) {
            const int rec = a.srecA[base + i];
            const int b = rec / NJ, j = rec - b * NJ;
            const float* er = a.ex + (int64_t)b * a.lay.rec;
            const float al = er[a.lay.ocoef + 3 * j];
            const float be = er[a.lay.ocoef + 3 * j + 1];
            gb += er[a.lay.ocoef + 3 * j + 2];
#pragma unroll
            for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) {
                const int c = lane + RAE_WAVE * cc;
                if (c < r) {
                    if (al != 0.f) g[cc] += al * er[a.lay.oV1 + c];
                    if (be != 0.f) g[cc] += be * er[a.lay.oV2 + c];
                    if (xy && j < 2) g[cc] += er[(j == 0 ? a.lay.oX : a.lay.oY) + c];
                }
            }
        }
        update_row1<OPT>(a.A + (int64_t)e * r, a.aA ? a.aA + (int64_t)e * r : nullptr, g, r,
                         a.lr, lane);
    }
    if (lane == 0) {
        float ac = (OPT == 0) ? a.aAb[e] : 0.f;
        a.Ab[e] = opt_update<OPT>(a.Ab[e], &ac, gb, a.lr);
        if (OPT == 0) a.aAb[e] = ac;
    }
}

// ---- W rows ---------------------------------------------------------------------------
template <int OPT, bool V4>
__device__ void task_feature_row(const StepArgs& a, int64_t g0, int h, int u, int lane) {
    const int m = a.m;
    const int32_t* hdr = a.hdrW + 2 * h;
    const int64_t base = (int64_t)h * a.RW;
    const int f = a.urowW[base + u];
    const int st = a.ustartW[base + u];
    const int en = (u + 1 < hdr[1]) ? a.ustartW[base + u + 1] : hdr[0];
    const unsigned mask = (1u << a.posbits) - 1u;
    if (V4) {
        const int nq = m >> 2;
        float4 g[RAE_MAXQ];
#pragma unroll
        for (int cc = 0; cc < RAE_MAXQ; ++cc) g[cc] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int i = st; i < en; ++i) {
            const unsigned rec = (unsigned)a.srecW[base + i];
            const int b = (int)(rec >> a.posbits);
            float val = 1.f;
            if (a.values) val = a.values[a.indptr[g0 + b] + (int)(rec & mask)];
            const float4* dS =
                reinterpret_cast<const float4*>(a.ex + (int64_t)b * a.lay.rec + a.lay.odS);
#pragma unroll
            for (int cc = 0; cc < RAE_MAXQ; ++cc) {
                const int c = lane + RAE_WAVE * cc;
                if (c < nq) fma4(g[cc], val, dS[c]);
            }
        }
        if (a.reg_on) {
            float4* gs = reinterpret_cast<float4*>(a.gWs + (int64_t)f * m);
#pragma unroll
            for (int cc = 0; cc < RAE_MAXQ; ++cc) {
                const int c = lane + RAE_WAVE * cc;
                if (c < nq) gs[c] = g[cc];
            }
        } else {
            update_row4<OPT>(a.W + (int64_t)f * m, a.aW ? a.aW + (int64_t)f * m : nullptr, g, nq,
                             a.lr, lane);
        }
    } else {
        float g[4 * RAE_MAXQ];
#pragma unroll
        for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) g[cc] = 0.f;
        for (int i = st; i < en; ++i) {
            const unsigned rec = (unsigned)a.srecW[base + i];
            const int b = (int)(rec >> a.posbits);
            float val = 1.f;
            if (a.values) val = a.values[a.indptr[g0 + b] + (int)(rec & mask)];
            const float* dS = a.ex + (int64_t)b * a.lay.rec + a.lay.odS;
#pragma unroll
            for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) {
                const int c = lane + RAE_WAVE * cc;
                if (c < m) g[cc] += val * dS[c];
            }
        }
        if (a.reg_on) {
#pragma unroll
            for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) {
                const int c = lane + RAE_WAVE * cc;
                if (c < m) a.gWs[(int64_t)f * m + c] = g[cc];
            }
        } else {
            update_row1<OPT>(a.W + (int64_t)f * m, a.aW ? a.aW + (int64_t)f * m : nullptr, g, m,
                             a.lr, lane);
        }
    }
}

// ---- dense decoder rows (C1 / C2 rows of m): gC[i,:] = sum_b dw[b,i] P[b,:] -------------
template <int OPT>
__device__ void task_sp_matrix_row(const StepArgs& a, int which, int i, int slot, int lane) {
    const int m = a.m;
    float* C = which ? a.C2 : a.C1;
    float* aC = which ? a.aC2 : a.aC1;
    const int odw = which ? a.lay.odw2 : a.lay.odw1;
    float g[4 * RAE_MAXQ];
#pragma unroll
    for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) g[cc] = 0.f;
    for (int b = 0; b < a.L; ++b) {
        const float* er = a.ex + (int64_t)b * a.lay.rec;
        const float dw = er[odw + i];
#pragma unroll
        for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) {
            const int k = lane + RAE_WAVE * cc;
            if (k < m) g[cc] += dw * er[a.lay.oP + k];
        }
    }
    float* row = C + (int64_t)i * m;
    if (a.reg_on && a.ext_reg) {
        float l1 = 0.f, l2 = 0.f;
#pragma unroll
        for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) {
            const int k = lane + RAE_WAVE * cc;
            if (k < m) {
                const float w = row[k];
                g[cc] += a.l1adj * sgnf(w) + 2.f * a.l2adj * w;
                l1 += fabsf(w);
                l2 += w * w;
            }
        }
        const double L1 = wave_sum_d((double)l1), L2 = wave_sum_d((double)l2);
        if (lane == 0) {
            a.regpart[2 * slot] = L1;
            a.regpart[2 * slot + 1] = L2;
        }
    }
    update_row1<OPT>(row, aC ? aC + (int64_t)i * m : nullptr, g, m, a.lr, lane);
}

// ---- Wb + the batch cost --------------------------------------------------------------
template <int OPT>
__device__ void task_bias_and_cost(const StepArgs& a, int64_t g0, int lane) {
    const int m = a.m;
    float g[4 * RAE_MAXQ];
#pragma unroll
    for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) g[cc] = 0.f;
    double loss = 0.0;
    for (int b = 0; b < a.L; ++b) {
        const float* er = a.ex + (int64_t)b * a.lay.rec;
#pragma unroll
        for (int cc = 0; cc < 4 * RAE_MAXQ; ++cc) {
            const int k = lane + RAE_WAVE * cc;
            if (k < m) g[cc] += er[a.lay.odS + k];
        }
    }
    for (int b = lane; b < a.L; b += RAE_WAVE) loss += (double)a.ex[(int64_t)b * a.lay.rec + a.lay.oloss];
    loss = wave_sum_d(loss);
    update_row1<OPT>(a.Wb, a.aWb, g, m, a.lr, lane);
    if (lane == 0) {
        const double D = 4.0 * a.L + 2.0 * a.L * a.s;
        const float cost = (float)(-loss / D);        // -mean(all_scores), OieModel.py:90
        const int64_t batch = *a.cursor + a.step_offset;
        if (a.reg_on) *a.base_cost = cost;
        else a.costs[batch] = cost;
    }
}

}  // namespace rae
