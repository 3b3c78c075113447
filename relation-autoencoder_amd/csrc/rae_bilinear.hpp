// RESCAL ("rescal", learning/models/decoders/Bilinear.py) and RESCAL+SP ("rescal+sp",
// learning/models/decoders/BilinearPlusSP.py) decoders: forward + backward of this rank's
// examples, and the R/C tensor gradient + optimizer update of the global batch.
//
// Reference computation (R = the (r, r, m) tensor R or C):
//   M_b     = sum_k P_bk R[:,:,k]                                 Bilinear.py:33
//   one     = a1^T M_b a2            (+ <wC1,a1> + <wC2,a2>)      :58-59   (BPSP :70-72)
//   negOne_t= n1_t^T M_b a2          (+ <wC1,n1_t> + <wC2,a2>)    :68-69   (BPSP :85-87)
//   negTwo_t= a1^T M_b n2_t          (+ <wC1,a1> + <wC2,n2_t>)    :78-79   (BPSP :100-102)
//   u = [one + Ab[e1], one + Ab[e2]],  g = [negOne + Ab[n1]; negTwo + Ab[n2]]   :38-48
// Backward, with x = dOne a1 + sum_t dg1_t n1_t and y = sum_t dg2_t n2_t:
//   dCost/dM_b = x a2^T + a1 y^T                         (rank 2, never materialised)
//   dR[:,:,k]  = sum_b P_bk (x_b a2_b^T + a1_b y_b^T)    -> task_bilinear_rows (update)
//   dP_bk      = x^T R_k a2 + a1^T R_k y                  -> k_bil_dp + bil_finish
//   dA[e1] = dOne M a2 + M y,  dA[e2] = M^T x,  dA[n1_t] = dg1_t M a2,  dA[n2_t] = dg2_t M^T a1
//   (+ the SP terms for the hybrid).
//
// The forward phase of one step is five launches (all over this rank's l examples):
//   k_bil_enc  per example : encoder (P, log P, H), hybrid wC1/wC2, copies of A[e1], A[e2]
//   k_bil_m    MFMA GEMM   : M[b][i*r+j] = sum_k P[b][k] R[i][j][k]   (l x r^2, K = m)
//   k_bil_dec  per example : M a2, M^T a1 (one sweep of M_b), scores, loss, x, y,
//                            M y, M^T x (second sweep), the A-row gradient vectors
//   k_bil_dp   MFMA GEMM   : dP partials  sum_{i in block} sum_j U[b][i,j] R[i][j][k],
//                            U = x a2^T + a1 y^T generated on the fly (split over i-blocks)
//   k_bil_fin  per example : dP (+ hybrid C^T dw) -> entropy + softmax backward -> dS
// All GEMMs run on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation).
#pragma once
#include "rae_common.hpp"
#include "rae_sp.hpp"
#include "rae_step.hpp"

namespace rae {

typedef float rae_bf4 __attribute__((ext_vector_type(4)));
#define RAE_IB 8     // i rows per dP partial block (k_bil_dp)
#define RAE_KG 8     // 16-column tiles of m per pass of one R-row task (task_bilinear_rows)
#ifndef RAE_SWEEP_RB
#define RAE_SWEEP_RB 4   // M_b rows per wave whose loads are in flight together (bil_sweep)
#endif

// ---- k_bil_enc: encoder + hybrid SP projections --------------------------------------------
template <bool V4>
__device__ void bil_encode(const StepArgs& a, int64_t g, int bl, char* smem) {
    const DynDims Dm(a);
    const int m = Dm.m, r = Dm.r;
    ExampleSmem S = carve_example_smem(smem, a.dec, m, r, Dm.s);
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;
    load_ids(a, Dm, ex, col, S);
    __syncthreads();
    CCache<V4, DynDims> cc_;
    encoder_forward<V4, V4, false>(a, Dm, S, 0, 0, cc_);
    const bool hybrid = a.dec == 2;
    if (hybrid) {
        sp_project<V4>(a, Dm, S, cc_);
        __syncthreads();
    }
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        rec[a.lay.oP + k] = S.sP[k];
        rec[a.lay.oZ + k] = S.sZ[k];
    }
    const float* A1 = a.A + (int64_t)S.sids[0] * r;
    const float* A2 = a.A + (int64_t)S.sids[1] * r;
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        rec[a.lay.oA1 + i] = A1[i];
        rec[a.lay.oA2 + i] = A2[i];
        rec[a.lay.oV1 + i] = hybrid ? S.swC1[i] : 0.f;
        rec[a.lay.oV2 + i] = hybrid ? S.swC2[i] : 0.f;
    }
    if (threadIdx.x == 0) rec[a.lay.oloss] = S.sred[40];     // H until k_bil_dec
}

// ---- k_bil_m: M[b][ij] = sum_k P[b][k] R[ij][k]  (one wave = 16 examples x 64 ij) ----------
// MFMA 16x16x4: A[b][kk] = P, B[kk][ij] = R, D[b][ij]; with V4 the four K-slots of a lane
// take 4 consecutive k (one float4 per operand row per 4 MFMAs).
template <bool V4>
__device__ void bil_gemm_m(const StepArgs& a, int t, int lane) {
    const int l = a.l, m = a.m, r = a.r;
    const int nbt = (l + 15) / 16;
    const int64_t rr = (int64_t)r * r;
    const int bt = t % nbt;
    const int64_t ij0 = (int64_t)(t / nbt) * 64;
    const int li = lane & 15, kk = lane >> 4;
    const int b = bt * 16 + li;
    const bool bv = b < l;
    const float* Prow = a.ex + (int64_t)(a.rank * l + (bv ? b : 0)) * a.lay.rec + a.lay.oP;
    const float* Rrow[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int64_t ij = ij0 + 16 * n + li;
        Rrow[n] = a.R3 + (ij < rr ? ij : rr - 1) * m;
    }
    rae_bf4 acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = rae_bf4{0.f, 0.f, 0.f, 0.f};
    if constexpr (V4) {
        for (int k0 = 0; k0 < m; k0 += 16) {
            const int k = k0 + 4 * kk;
            const bool kv = k < m;                  // m % 4 == 0: the whole float4 is valid
            const int kc = kv ? k : 0;
            float4 p = *reinterpret_cast<const float4*>(Prow + kc);
            if (!kv || !bv) p = make_float4(0.f, 0.f, 0.f, 0.f);
            float4 rv[4];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                rv[n] = *reinterpret_cast<const float4*>(Rrow[n] + kc);
                if (!kv) rv[n] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.x, rv[n].x, acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.y, rv[n].y, acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.z, rv[n].z, acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.w, rv[n].w, acc[n], 0, 0, 0);
            }
        }
    } else {
        for (int k0 = 0; k0 < m; k0 += 4) {
            const int k = k0 + kk;
            const bool kv = k < m;
            const int kc = kv ? k : 0;
            const float p = (kv && bv) ? Prow[kc] : 0.f;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const float rv = kv ? Rrow[n][kc] : 0.f;
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(p, rv, acc[n], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int64_t ij = ij0 + 16 * n + li;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int bo = bt * 16 + kk * 4 + reg;
            if (bo < l && ij < rr) a.Mbuf[(int64_t)bo * rr + ij] = acc[n][reg];
        }
    }
}

// ---- bf16-operand forms (rae_config.mfma_bf16; BASELINE config 5) ------------------------
// v_mfma_f32_16x16x32_bf16: lane l holds A[l&15][8(l>>4) + e] and B[8(l>>4) + e][l&15],
// e = 0..7; fp32 values are rounded to bf16 (v_cvt_pk_bf16_f32, nearest even) as they enter
// the fragment, accumulation stays fp32.  K = 32 per instruction instead of 4.
typedef __bf16 rae_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ rae_bf16x8 to_bf16x8(float4 lo, float4 hi) {
    rae_bf16x8 v;
    v[0] = (__bf16)lo.x; v[1] = (__bf16)lo.y; v[2] = (__bf16)lo.z; v[3] = (__bf16)lo.w;
    v[4] = (__bf16)hi.x; v[5] = (__bf16)hi.y; v[6] = (__bf16)hi.z; v[7] = (__bf16)hi.w;
    return v;
}

// M[b][ij] (as bil_gemm_m) with bf16 operands; m % 4 == 0
__device__ void bil_gemm_m_bf16(const StepArgs& a, int t, int lane) {
    const int l = a.l, m = a.m, r = a.r;
    const int nbt = (l + 15) / 16;
    const int64_t rr = (int64_t)r * r;
    const int bt = t % nbt;
    const int64_t ij0 = (int64_t)(t / nbt) * 64;
    const int li = lane & 15, g = lane >> 4;
    const int b = bt * 16 + li;
    const bool bv = b < l;
    const float* Prow = a.ex + (int64_t)(a.rank * l + (bv ? b : 0)) * a.lay.rec + a.lay.oP;
    const float* Rrow[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int64_t ij = ij0 + 16 * n + li;
        Rrow[n] = a.R3 + (ij < rr ? ij : rr - 1) * m;
    }
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    rae_bf4 acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = rae_bf4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < m; k0 += 32) {
        const int ka = k0 + 8 * g, kb = ka + 4;
        const bool va = ka < m, vb = kb < m;
        float4 p0 = *reinterpret_cast<const float4*>(Prow + (va ? ka : 0));
        float4 p1 = *reinterpret_cast<const float4*>(Prow + (vb ? kb : 0));
        if (!va || !bv) p0 = z4;
        if (!vb || !bv) p1 = z4;
        const rae_bf16x8 pa = to_bf16x8(p0, p1);
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            float4 r0 = *reinterpret_cast<const float4*>(Rrow[n] + (va ? ka : 0));
            float4 r1 = *reinterpret_cast<const float4*>(Rrow[n] + (vb ? kb : 0));
            if (!va) r0 = z4;
            if (!vb) r1 = z4;
            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, to_bf16x8(r0, r1), acc[n], 0, 0, 0);
        }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int64_t ij = ij0 + 16 * n + li;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int bo = bt * 16 + g * 4 + reg;
            if (bo < l && ij < rr) a.Mbuf[(int64_t)bo * rr + ij] = acc[n][reg];
        }
    }
}

// dP partials (as bil_gemm_dp) with bf16 operands; K = j in steps of 32
__device__ void bil_gemm_dp_bf16(const StepArgs& a, int t, int lane) {
    const int l = a.l, m = a.m, r = a.r;
    const int nbt = (l + 15) / 16, nkt = (m + 15) / 16;
    const int bt = t % nbt, rest = t / nbt;
    const int kt = rest % nkt, ib = rest / nkt;
    const int li = lane & 15, g = lane >> 4;
    const int b = bt * 16 + li;
    const bool bv = b < l;
    const float* er = a.ex + (int64_t)(a.rank * l + (bv ? b : 0)) * a.lay.rec;
    const int k = kt * 16 + li;
    const bool kv = k < m;
    const int kc = kv ? k : 0;
    const int i0 = ib * RAE_IB;
    float xi[RAE_IB], ai[RAE_IB];
#pragma unroll
    for (int q = 0; q < RAE_IB; ++q) {
        const int i = min(i0 + q, r - 1);
        const bool use = bv && (i0 + q) < r;
        xi[q] = use ? er[a.lay.oX + i] : 0.f;
        ai[q] = use ? er[a.lay.oA1 + i] : 0.f;
    }
    rae_bf4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < r; j0 += 32) {
        const int jb = j0 + 8 * g;
        float a2j[8], yj[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const bool jv = jb + e < r;
            a2j[e] = jv ? er[a.lay.oA2 + jb + e] : 0.f;
            yj[e] = jv ? er[a.lay.oY + jb + e] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < RAE_IB; ++q) {
            const int i = min(i0 + q, r - 1);
            rae_bf16x8 ua, rb;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int j = jb + e;
                const bool jv = j < r;
                ua[e] = (__bf16)(xi[q] * a2j[e] + ai[q] * yj[e]);
                rb[e] = (__bf16)((jv && kv) ? a.R3[((int64_t)i * r + (jv ? j : 0)) * m + kc] : 0.f);
            }
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua, rb, acc, 0, 0, 0);
        }
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int bo = bt * 16 + g * 4 + reg;
        if (bo < l && kv) a.dPpart[((int64_t)ib * l + bo) * m + k] = acc[reg];
    }
}

// ---- k_bil_dp2: the bf16 dP contraction with the R slices staged in LDS -----------------------
// dP_b[k] = sum_i sum_j U_b[i,j] R[i][j][k],  U_b[i,j] = x_b[i] a2_b[j] + a1_b[i] y_b[j].
// One workgroup per block of RAE_IB2 rows i: the block's R[i] slices (r x m fp32, j-major)
// are staged ONCE into LDS as bf16 in (k, j) order -- the B fragment of
// v_mfma_f32_16x16x32_bf16 (8 consecutive j at one k) is then one ds_read_b128 -- and
// every (16 examples x 16 relations) tile of the rank's batch reads them from there, so R
// leaves HBM once per step instead of once per example tile through 4-byte strided loads
// (bil_gemm_dp_bf16).  A wave owns whole example tiles: it holds the tile's a2 / y for all
// j in registers (NJS x 8 per lane each) and runs all MT relation tiles, so U is built once
// per (i, 32-wide j step) and reused MT times.  Partial sums per i-block -> dPpart, summed
// in block order by bil_finish (deterministic).  Shapes: r <= 32 NJS, m <= 16 MT,
// r % 4 == m % 4 == 0.
#define RAE_IB2 2    // i rows per k_bil_dp2 workgroup (the q-loop selects x/a1 for q < 2)
template <int NJS, int MT>
constexpr size_t dp2_lds_bytes() { return (size_t)RAE_IB2 * MT * 16 * (NJS * 32 + 8) * 2; }
template <int NJS, int MT>
__device__ void bil_gemm_dp2(const StepArgs& a, int ib, char* smem) {
    // LDS row stride JS = JP + 8 bf16: 16-B aligned fragment reads, and the 16 rows k a
    // fragment read touches land on distinct bank groups
    constexpr int JP = NJS * 32, KP = MT * 16, JS = JP + 8;
    const int l = a.l, m = a.m, r = a.r;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, g = lane >> 4;
    __bf16* lds = reinterpret_cast<__bf16*>(smem);
    const int i0 = ib * RAE_IB2;
    const int ni = min(RAE_IB2, r - i0);
    // stage: R[i0+q][j][k] -> lds[q][k][j] (bf16, round to nearest even); the padding
    // (j >= r, k >= m) is zero.
    for (int e = tid; e < RAE_IB2 * KP * JS / 8; e += RAE_BT)
        reinterpret_cast<uint4*>(lds)[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    // A staging unit is 8 rows j x one float4 of k: its 8 loads are lanes' consecutive
    // 16-B chunks of whole rows (coalesced), and its 4 LDS stores are 16-B runs of 8 j at
    // one k (ds_write_b128).  All of a slice's loads are issued before its first store.
    const int m4 = m / 4, r8 = (r + 7) / 8, nunit = r8 * m4;
    constexpr int UU = ((JP / 8) * (KP / 4) + RAE_BT - 1) / RAE_BT;
    for (int q = 0; q < ni; ++q) {
        const float4* src = reinterpret_cast<const float4*>(a.R3 + (int64_t)(i0 + q) * r * m);
        __bf16* dst = lds + q * KP * JS;
        float4 v[UU][8];
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            const int e = tid + u * RAE_BT;
            const bool ok = e < nunit;
            const int jb = ok ? e / m4 : 0, kq = ok ? e - jb * m4 : 0;
#pragma unroll
            for (int h = 0; h < 8; ++h) {
                const int j = 8 * jb + h;
                v[u][h] = src[(j < r ? j : 0) * m4 + kq];
                if (j >= r) v[u][h] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            const int e = tid + u * RAE_BT;
            if (e < nunit) {
                const int jb = e / m4, kq = e - jb * m4;
                __bf16* d = dst + 4 * kq * JS + 8 * jb;
                rae_bf16x8 c0, c1, c2, c3;
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    c0[h] = (__bf16)v[u][h].x;
                    c1[h] = (__bf16)v[u][h].y;
                    c2[h] = (__bf16)v[u][h].z;
                    c3[h] = (__bf16)v[u][h].w;
                }
                *reinterpret_cast<rae_bf16x8*>(d) = c0;
                *reinterpret_cast<rae_bf16x8*>(d + JS) = c1;
                *reinterpret_cast<rae_bf16x8*>(d + 2 * JS) = c2;
                *reinterpret_cast<rae_bf16x8*>(d + 3 * JS) = c3;
            }
        }
    }
    __syncthreads();
    const int nbt = (l + 15) / 16;
    for (int bt = w; bt < nbt; bt += RAE_NWAVE) {
        const int b = bt * 16 + li;
        const bool bv = b < l;
        const float* er = a.ex + (int64_t)(a.rank * l + (bv ? b : 0)) * a.lay.rec;
        // a2 / y of the lane's example, all j (unconditional loads of clamped addresses,
        // then selects: no exec-masked branches)
        float4 a2v[NJS][2], yv[NJS][2];
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int js = 0; js < NJS; ++js) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int j = js * 32 + 8 * g + 4 * h;
                const bool ok = bv && j < r;
                const int jc = ok ? j : 0;
                const float4 va = *reinterpret_cast<const float4*>(er + a.lay.oA2 + jc);
                const float4 vy = *reinterpret_cast<const float4*>(er + a.lay.oY + jc);
                a2v[js][h] = ok ? va : z;
                yv[js][h] = ok ? vy : z;
            }
        }
        float xq[RAE_IB2], aq[RAE_IB2];
#pragma unroll
        for (int q = 0; q < RAE_IB2; ++q) {
            const bool ok = bv && q < ni;
            const int ic = i0 + (q < ni ? q : 0);
            const float xv = er[a.lay.oX + ic], av = er[a.lay.oA1 + ic];
            xq[q] = ok ? xv : 0.f;
            aq[q] = ok ? av : 0.f;
        }
        rae_bf4 acc[MT];
#pragma unroll
        for (int kt = 0; kt < MT; ++kt) acc[kt] = rae_bf4{0.f, 0.f, 0.f, 0.f};
        // software pipeline within each i: the next j step's MT B fragments are read from
        // LDS while the current step's MFMAs run
        rae_bf16x8 rb[2][MT];
#pragma unroll 1
        for (int q = 0; q < RAE_IB2; ++q) {
            const __bf16* lq = lds + q * KP * JS + 8 * g + li * JS;
#pragma unroll
            for (int kt = 0; kt < MT; ++kt)
                rb[0][kt] = *reinterpret_cast<const rae_bf16x8*>(lq + kt * 16 * JS);
            const float xv = xq[0] * (q == 0) + xq[RAE_IB2 - 1] * (q != 0);
            const float av = aq[0] * (q == 0) + aq[RAE_IB2 - 1] * (q != 0);
#pragma unroll
            for (int js = 0; js < NJS; ++js) {
                if (js + 1 < NJS) {
#pragma unroll
                    for (int kt = 0; kt < MT; ++kt)
                        rb[(js + 1) & 1][kt] =
                            *reinterpret_cast<const rae_bf16x8*>(lq + kt * 16 * JS + (js + 1) * 32);
                }
                const float* p2 = reinterpret_cast<const float*>(&a2v[js][0]);
                const float* py = reinterpret_cast<const float*>(&yv[js][0]);
                rae_bf16x8 ua;
#pragma unroll
                for (int e = 0; e < 8; ++e) ua[e] = (__bf16)(xv * p2[e] + av * py[e]);
#pragma unroll
                for (int kt = 0; kt < MT; ++kt)
                    acc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua, rb[js & 1][kt], acc[kt], 0, 0, 0);
            }
        }
#pragma unroll
        for (int kt = 0; kt < MT; ++kt) {
            const int k = kt * 16 + li;
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int bo = bt * 16 + g * 4 + reg;
                if (bo < l && k < m) a.dPpart[((int64_t)ib * l + bo) * m + k] = acc[kt][reg];
            }
        }
    }
}

// ---- k_bil_dec helpers ----------------------------------------------------------------------
// k_bil_dec runs 16 waves per example (RAE_DBT threads), twice the forward kernels' 8: the two
// M_b sweeps are bound by how many loads each CU has in flight (C5 forward 79.3 -> 73.8 us)
#ifndef RAE_DBT
#define RAE_DBT 1024
#endif
#define RAE_DNW (RAE_DBT / RAE_WAVE)
struct BilSmem {
    float *v, *w, *a1, *a2, *wC1, *wC2, *x, *y, *My, *Mtx, *dw1, *dw2, *rows, *part, *dots, *Abv,
        *coef, *red;
    int* ids;
};

__host__ __device__ inline int bil_dec_smem_floats(int r, int s) {
    const int r4 = align4(r), NJ4 = align4(2 + 2 * s);
    return 12 * r4 + 2 * s * r4 + RAE_DNW * r4 + align4(2 * s + 4) + NJ4 + align4(3 * (2 + 2 * s)) +
           64 + NJ4;
}

__device__ inline BilSmem carve_bil_smem(char* smem, int r, int s) {
    BilSmem S;
    const int r4 = align4(r), NJ4 = align4(2 + 2 * s);
    float* p = reinterpret_cast<float*>(smem);
    float** vecs[12] = {&S.v, &S.w, &S.a1, &S.a2, &S.wC1, &S.wC2, &S.x, &S.y, &S.My, &S.Mtx,
                        &S.dw1, &S.dw2};
    for (int q = 0; q < 12; ++q) { *vecs[q] = p; p += r4; }
    S.rows = p; p += 2 * s * r4;
    S.part = p; p += RAE_DNW * r4;
    S.dots = p; p += align4(2 * s + 4);
    S.Abv = p; p += NJ4;
    S.coef = p; p += align4(3 * (2 + 2 * s));
    S.red = p; p += 64;
    S.ids = reinterpret_cast<int*>(p);
    return S;
}

// One pass over M_b (r x r, row-major in HBM):
//   row_out[i] = sum_j M[i][j] vr[j]        col_out[j] = sum_i vl[i] M[i][j]
// wave w takes rows i = w, w + NW, ...; lanes hold column vectors; the column sums are
// per-wave partials combined in wave order (deterministic).
template <bool V4>
__device__ void bil_sweep(const float* M, int r, const float* vr, const float* vl, float* row_out,
                          float* col_out, float* part) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    constexpr int RB = RAE_SWEEP_RB;
    const int rv = r / VW, r4 = align4(r);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const VT* vrv = reinterpret_cast<const VT*>(vr);
    VT cacc[2], vrc[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        vzero(cacc[q]);
        const int c = lane + 64 * q;
        if (c < rv) vrc[q] = vrv[c]; else vzero(vrc[q]);
    }
    for (int i0 = w; i0 < r; i0 += RAE_DNW * RB) {
        VT x[RB][2];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const int i = min(i0 + RAE_DNW * u, r - 1);
            const VT* Mi = reinterpret_cast<const VT*>(M + (int64_t)i * r);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int c = lane + 64 * q;
                x[u][q] = Mi[c < rv ? c : 0];
            }
        }
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const int i = i0 + RAE_DNW * u;
            const bool iv = i < r;
            const float li = iv ? vl[i] : 0.f;
            float d = 0.f;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int c = lane + 64 * q;
                if (c < rv) {
                    d += vdot(x[u][q], vrc[q]);
                    vfma(cacc[q], li, x[u][q]);
                }
            }
            d = wave_sum(d);
            if (iv && lane == 0) row_out[i] = d;
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int c = lane + 64 * q;
        if (c < rv) reinterpret_cast<VT*>(part + w * r4)[c] = cacc[q];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < r; j += RAE_DBT) {
        float t = 0.f;
#pragma unroll
        for (int ww = 0; ww < RAE_DNW; ++ww) t += part[ww * r4 + j];
        col_out[j] = t;
    }
    __syncthreads();
}

// ---- k_bil_dec: scores, loss, coefficients, A-row gradient vectors -----------------------
template <bool V4>
__device__ void bil_decode(const StepArgs& a, int64_t g, int bl, char* smem) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int m = a.m, r = a.r, s = a.s, NJ = 2 + 2 * s;
    const int r4 = align4(r), rv = r / VW, r4v = r4 / VW;
    const bool hybrid = a.dec == 2;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    BilSmem S = carve_bil_smem(smem, r, s);
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    (void)m;
    RAE_STAMP(a, 0);

    if (threadIdx.x < NJ) {
        const int j = threadIdx.x;
        const int* src = (j == 0) ? a.args1 + ex
                       : (j == 1) ? a.args2 + ex
                       : (j < 2 + s) ? a.neg1 + (int64_t)(j - 2) * a.neg_stride + col
                                     : a.neg2 + (int64_t)(j - 2 - s) * a.neg_stride + col;
        const int id = *src;
        S.ids[j] = id;
        S.Abv[j] = a.Ab[id];
    }
    for (int i = threadIdx.x; i < r4; i += RAE_DBT) {
        const bool iv = i < r;
        S.a1[i] = iv ? rec[a.lay.oA1 + i] : 0.f;
        S.a2[i] = iv ? rec[a.lay.oA2 + i] : 0.f;
        S.wC1[i] = iv ? rec[a.lay.oV1 + i] : 0.f;
        S.wC2[i] = iv ? rec[a.lay.oV2 + i] : 0.f;
    }
    const float H = rec[a.lay.oloss];
    __syncthreads();
    RAE_STAMP(a, 1);
    // negative rows: rows[t] = A[n1_t], rows[s + t] = A[n2_t]
    for (int e = threadIdx.x; e < 2 * s * rv; e += RAE_DBT) {
        const int t = e / rv, c = e - t * rv;
        const VT* src = reinterpret_cast<const VT*>(a.A + (int64_t)S.ids[2 + t] * r);
        reinterpret_cast<VT*>(S.rows)[t * r4v + c] = src[c];
    }
    const float* Mb = a.Mbuf + (int64_t)bl * r * r;
    bil_sweep<V4>(Mb, r, S.a2, S.a1, S.v, S.w, S.part);     // v = M a2, w = M^T a1 (+ barrier)
    RAE_STAMP(a, 2);

    // dot products: rho < s: n1_t.(v [+ wC1]); s <= rho < 2s: n2_t.(w [+ wC2]);
    // 2s: a1.v; 2s+1: a1.wC1; 2s+2: a2.wC2
    {
        const VT* vv = reinterpret_cast<const VT*>(S.v);
        const VT* ww = reinterpret_cast<const VT*>(S.w);
        const VT* c1 = reinterpret_cast<const VT*>(S.wC1);
        const VT* c2 = reinterpret_cast<const VT*>(S.wC2);
        const VT* R = reinterpret_cast<const VT*>(S.rows);
        const VT* A1 = reinterpret_cast<const VT*>(S.a1);
        const VT* A2 = reinterpret_cast<const VT*>(S.a2);
        const int ntask = 2 * s + 3;
        for (int rho = w; rho < ntask; rho += RAE_DNW) {
            const VT* xa;
            const VT* xb;
            const VT* xc = nullptr;
            if (rho < s) { xa = R + rho * r4v; xb = vv; xc = c1; }
            else if (rho < 2 * s) { xa = R + rho * r4v; xb = ww; xc = c2; }
            else if (rho == 2 * s) { xa = A1; xb = vv; }
            else if (rho == 2 * s + 1) { xa = A1; xb = c1; }
            else { xa = A2; xb = c2; }
            float d = 0.f;
            for (int c = lane; c < rv; c += RAE_WAVE) {
                const VT xv = xa[c];
                d += vdot(xv, xb[c]);
                if (hybrid && xc) d += vdot(xv, xc[c]);
            }
            d = wave_sum(d);
            if (lane == 0) S.dots[rho] = d;
        }
    }
    __syncthreads();
    RAE_STAMP(a, 3);

    // scores, loss, coefficients (wave 0)
    if (w == 0) {
        const float sp1 = hybrid ? S.dots[2 * s + 1] : 0.f;
        const float sp2 = hybrid ? S.dots[2 * s + 2] : 0.f;
        float sdg1 = 0.f, sdg2 = 0.f, sls = 0.f;
        for (int t = lane; t < s; t += RAE_WAVE) {
            const float g1 = S.dots[t] + sp2 + S.Abv[2 + t];
            const float g2 = S.dots[s + t] + sp1 + S.Abv[2 + s + t];
            const float dg1 = sigmoid(g1) * a.invD;
            const float dg2 = sigmoid(g2) * a.invD;
            float* c1 = S.coef + 3 * (2 + t);
            float* c2 = S.coef + 3 * (2 + s + t);
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
            const float one = S.dots[2 * s] + sp1 + sp2;
            const float u1 = one + S.Abv[0], u2 = one + S.Abv[1];
            const float du1 = -sigmoid(-u1) * a.invD;
            const float du2 = -sigmoid(-u2) * a.invD;
            const float dOne = du1 + du2;
            S.coef[0] = 0.f; S.coef[1] = 0.f; S.coef[2] = du1;
            S.coef[3] = 0.f; S.coef[4] = 0.f; S.coef[5] = du2;
            S.red[0] = dOne;
            S.red[1] = dOne + sdg2;      // c_a1: <wC1,a1> sits in one and every negTwo
            S.red[2] = dOne + sdg1;      // c_a2: <wC2,a2> sits in one and every negOne
            S.red[32] = log_sigmoid(u1) + log_sigmoid(u2) + 2.f * H + sls;
        }
    }
    __syncthreads();

    // x = dOne a1 + sum_t dg1_t n1_t ; y = sum_t dg2_t n2_t ; hybrid dw1/dw2 (sums in t order)
    {
        const float dOne = S.red[0], ca1 = S.red[1], ca2 = S.red[2];
        for (int i = threadIdx.x; i < r4; i += RAE_DBT) {
            float n1 = 0.f, n2 = 0.f;
            for (int t = 0; t < s; ++t) {
                n1 += S.coef[3 * (2 + t)] * S.rows[t * r4 + i];
                n2 += S.coef[3 * (2 + s + t) + 1] * S.rows[(s + t) * r4 + i];
            }
            const bool iv = i < r;
            S.x[i] = iv ? dOne * S.a1[i] + n1 : 0.f;
            S.y[i] = iv ? n2 : 0.f;
            S.dw1[i] = iv ? ca1 * S.a1[i] + n1 : 0.f;
            S.dw2[i] = iv ? ca2 * S.a2[i] + n2 : 0.f;
        }
    }
    __syncthreads();
    RAE_STAMP(a, 4);
    bil_sweep<V4>(Mb, r, S.y, S.x, S.My, S.Mtx, S.part);    // M y, M^T x
    RAE_STAMP(a, 5);

    {
        const float dOne = S.red[0], ca1 = S.red[1], ca2 = S.red[2];
        for (int i = threadIdx.x; i < r; i += RAE_DBT) {
            const float c1 = hybrid ? S.wC1[i] : 0.f, c2 = hybrid ? S.wC2[i] : 0.f;
            rec[a.lay.oV1 + i] = S.v[i] + c1;
            rec[a.lay.oV2 + i] = S.w[i] + c2;
            rec[a.lay.oG1 + i] = dOne * S.v[i] + S.My[i] + ca1 * c1;
            rec[a.lay.oG2 + i] = S.Mtx[i] + ca2 * c2;
            rec[a.lay.oX + i] = S.x[i];
            rec[a.lay.oY + i] = S.y[i];
            rec[a.lay.odw1 + i] = hybrid ? S.dw1[i] : 0.f;
            rec[a.lay.odw2 + i] = hybrid ? S.dw2[i] : 0.f;
        }
        for (int j = threadIdx.x; j < NJ; j += RAE_DBT) {
            const float* c = S.coef + 3 * j;
            rec[a.lay.ocoef + 2 * j] = j < 2 ? 1.f : (j < 2 + s ? c[0] : c[1]);
            rec[a.lay.ocoef + 2 * j + 1] = c[2];
        }
        if (threadIdx.x == 0) rec[a.lay.oloss] = S.red[32];
    }
    RAE_STAMP(a, 6);
}

// ---- k_bil_dp: dP partials of one (16 examples) x (16 relations) tile over RAE_IB rows i ----
// A[b][kk] = U[b][i, j] = x_b[i] a2_b[j] + a1_b[i] y_b[j]  (j = j0 + kk), B[kk][k] = R[i][j][k]
__device__ void bil_gemm_dp(const StepArgs& a, int t, int lane) {
    const int l = a.l, m = a.m, r = a.r;
    const int nbt = (l + 15) / 16, nkt = (m + 15) / 16;
    const int bt = t % nbt, rest = t / nbt;
    const int kt = rest % nkt, ib = rest / nkt;
    const int li = lane & 15, kk = lane >> 4;
    const int b = bt * 16 + li;
    const bool bv = b < l;
    const float* er = a.ex + (int64_t)(a.rank * l + (bv ? b : 0)) * a.lay.rec;
    const int k = kt * 16 + li;
    const bool kv = k < m;
    const int kc = kv ? k : 0;
    const int i0 = ib * RAE_IB;
    float xi[RAE_IB], ai[RAE_IB];
#pragma unroll
    for (int q = 0; q < RAE_IB; ++q) {
        const int i = min(i0 + q, r - 1);
        const bool use = bv && (i0 + q) < r;
        xi[q] = use ? er[a.lay.oX + i] : 0.f;
        ai[q] = use ? er[a.lay.oA1 + i] : 0.f;
    }
    rae_bf4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < r; j0 += 4) {
        const int j = j0 + kk;
        const bool jv = j < r;
        const int jc = jv ? j : 0;
        const float a2j = jv ? er[a.lay.oA2 + jc] : 0.f;
        const float yj = jv ? er[a.lay.oY + jc] : 0.f;
        float rv[RAE_IB];
#pragma unroll
        for (int q = 0; q < RAE_IB; ++q) {
            const int i = min(i0 + q, r - 1);
            rv[q] = (jv && kv) ? a.R3[((int64_t)i * r + jc) * m + kc] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < RAE_IB; ++q) {
            const float u = xi[q] * a2j + ai[q] * yj;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(u, rv[q], acc, 0, 0, 0);
        }
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int bo = bt * 16 + kk * 4 + reg;
        if (bo < l && kv) a.dPpart[((int64_t)ib * l + bo) * m + k] = acc[reg];
    }
}

// ---- k_bil_fin: dP -> dS -------------------------------------------------------------------
__device__ void bil_finish(const StepArgs& a, int bl, float* sdp, float* red) {
    const int m = a.m, r = a.r, l = a.l;
    const bool hybrid = a.dec == 2;
    const int bg = a.rank * l + bl;
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    const float ce = 2.f * a.alpha * a.invD;      // entropy term, centred form (softmax_backward)
    float sd = 0.f, sz = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_BT) {
        float dp = 0.f;
#pragma unroll 10
        for (int ib = 0; ib < a.nib; ++ib) dp += a.dPpart[((int64_t)ib * l + bl) * m + k];
        if (hybrid) {
            float h = 0.f;
            for (int i = 0; i < r; ++i)
                h += rec[a.lay.odw1 + i] * a.C1[(int64_t)i * m + k] +
                     rec[a.lay.odw2 + i] * a.C2[(int64_t)i * m + k];
            dp += h;
        }
        sdp[k] = dp;
        const float p = rec[a.lay.oP + k];
        sd += p * dp;
        sz += p * rec[a.lay.oZ + k];
    }
    sd = block_sum<RAE_BT>(sd, red);
    sz = block_sum<RAE_BT>(sz, red + RAE_NWAVE);
    for (int k = threadIdx.x; k < m; k += RAE_BT)
        rec[a.lay.odS + k] = rec[a.lay.oP + k] * ((sdp[k] - sd) + ce * (rec[a.lay.oZ + k] - sz));
}

// ---- update: 16 rows ij of the R/C tensor (viewed as (r*r, m)) against all m columns ------
// gR[ij][k] = sum_b U_b[ij] P_b[k] over the global batch, then the optimizer in place.
// A[ij][kk] = U_{b0+kk}[ij], B[kk][k] = P_{b0+kk}[k], D[ij][k].
// k_bil_prep: lay out the bf16 R-gradient operands of the global batch (after the exchange).
// Blocks [0, 4*nit*nbs): one (factor, 64 rows i, 32 examples) tile, read along i (coalesced
// record runs), transposed through LDS, written along the examples.  The last nbs*nkt
// blocks: one (32 examples, 16 relations) P tile -> its 64 lanes' B fragments.
__device__ int bil_prep_blocks(const StepArgs& a) {
    return 4 * ((a.r + 63) / 64) * (a.Lp / 32) + (a.Lp / 32) * ((a.m + 15) / 16);
}
__device__ void bil_prep(const StepArgs& a) {
    __shared__ float tile[32][65];
    const int r = a.r, m = a.m, L = a.L, Lp = a.Lp, tid = threadIdx.x;
    const int nit = (r + 63) / 64, nbs = Lp / 32, nkt = (m + 15) / 16;
    const int nfacb = 4 * nit * nbs;
    const int blk = blockIdx.x;
    if (blk < nfacb) {
        const int bs = blk % nbs, rest = blk / nbs, it = rest % nit, f = rest / nit;
        const int off = f == 0 ? a.lay.oX : f == 1 ? a.lay.oA1 : f == 2 ? a.lay.oA2 : a.lay.oY;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int bb = (tid >> 6) + 4 * u, i = it * 64 + (tid & 63), b = bs * 32 + bb;
            tile[bb][tid & 63] = (b < L && i < r) ? a.ex[(int64_t)b * a.lay.rec + off + i] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int ii = (tid >> 5) + 8 * u, bb = tid & 31, i = it * 64 + ii;
            if (i < r) a.facT[((int64_t)f * r + i) * Lp + bs * 32 + bb] = tile[bb][ii];
        }
    } else if (blk < nfacb + nbs * nkt) {
        const int t = blk - nfacb, bs = t / nkt, kt = t - bs * nkt;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int bb = (tid >> 4) + 16 * u, k = kt * 16 + (tid & 15), b = bs * 32 + bb;
            tile[bb][tid & 15] = (b < L && k < m) ? a.ex[(int64_t)b * a.lay.rec + a.lay.oP + k] : 0.f;
        }
        __syncthreads();
        if (tid < 64) {
            const int g = tid >> 4, li = tid & 15;
            rae_bf16x8 v;
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = (__bf16)tile[8 * g + q][li];
            a.pfrag[(int64_t)t * 64 + tid] = *reinterpret_cast<const uint4*>(&v);
        }
    }
}

// bf16-operand gradient of 16 rows ij x 16 columns per tile: K = examples in steps of 32.
// The lane's 8 examples' factors are two float4 loads per factor (k_bil_prep's transposed
// copies) and each P fragment one 16-byte load.
__device__ __forceinline__ void bilinear_rows_acc_bf16(const StepArgs& a, int ijt, int kg0, int nk,
                                                       rae_bf4* acc, int lane) {
    const int r = a.r, L = a.L, Lp = a.Lp, nkt = (a.m + 15) / 16;
    const int64_t rr = (int64_t)r * r;
    const int li = lane & 15, g = lane >> 4;
    const int64_t ij = (int64_t)ijt * 16 + li;
    const bool ijv = ij < rr;
    const int ijc = (int)(ijv ? ij : 0);
    const int i = ijc / r, j = ijc - (ijc / r) * r;
    const float* xt = a.facT + (int64_t)i * Lp;
    const float* a1t = a.facT + (int64_t)(r + i) * Lp;
    const float* a2t = a.facT + (int64_t)(2 * r + j) * Lp;
    const float* yt = a.facT + (int64_t)(3 * r + j) * Lp;
    for (int b0 = 0; b0 < L; b0 += 32) {
        const int bb = b0 + 8 * g;
        float xv[8], a1v[8], a2v[8], yv[8];
        *reinterpret_cast<float4*>(xv) = *reinterpret_cast<const float4*>(xt + bb);
        *reinterpret_cast<float4*>(xv + 4) = *reinterpret_cast<const float4*>(xt + bb + 4);
        *reinterpret_cast<float4*>(a1v) = *reinterpret_cast<const float4*>(a1t + bb);
        *reinterpret_cast<float4*>(a1v + 4) = *reinterpret_cast<const float4*>(a1t + bb + 4);
        *reinterpret_cast<float4*>(a2v) = *reinterpret_cast<const float4*>(a2t + bb);
        *reinterpret_cast<float4*>(a2v + 4) = *reinterpret_cast<const float4*>(a2t + bb + 4);
        *reinterpret_cast<float4*>(yv) = *reinterpret_cast<const float4*>(yt + bb);
        *reinterpret_cast<float4*>(yv + 4) = *reinterpret_cast<const float4*>(yt + bb + 4);
        rae_bf16x8 pb[RAE_KG];
        const uint4* pf = a.pfrag + ((int64_t)(b0 / 32) * nkt + kg0) * 64 + lane;
#pragma unroll
        for (int q = 0; q < RAE_KG; ++q) {
            const uint4 u = pf[(q < nk ? q : 0) * 64];
            pb[q] = *reinterpret_cast<const rae_bf16x8*>(&u);
        }
        rae_bf16x8 ua;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float u = xv[e] * a2v[e] + a1v[e] * yv[e];    // zero past L (padded factors)
            ua[e] = (__bf16)(ijv ? u : 0.f);
        }
#pragma unroll
        for (int q = 0; q < RAE_KG; ++q) {
            if (q >= nk) continue;
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua, pb[q], acc[q], 0, 0, 0);
        }
    }
}

template <int OPT>
__device__ void task_bilinear_rows(const StepArgs& a, int ijt, int slot, int lane) {
    const int m = a.m, r = a.r, L = a.L;
    const int64_t rr = (int64_t)r * r;
    const int li = lane & 15, kk = lane >> 4;
    const int64_t ij = (int64_t)ijt * 16 + li;
    const bool ijv = ij < rr;
    const int ijc = (int)(ijv ? ij : 0);
    const int i = ijc / r, j = ijc - (ijc / r) * r;
    const int nkt = (m + 15) / 16;
    const bool reg = a.reg_on && a.ext_reg;
    float l1 = 0.f, l2 = 0.f;
    for (int kg0 = 0; kg0 < nkt; kg0 += RAE_KG) {
        const int nk = min(RAE_KG, nkt - kg0);
        rae_bf4 acc[RAE_KG];
#pragma unroll
        for (int q = 0; q < RAE_KG; ++q) acc[q] = rae_bf4{0.f, 0.f, 0.f, 0.f};
        if (a.bf16) bilinear_rows_acc_bf16(a, ijt, kg0, nk, acc, lane);
        else for (int b0 = 0; b0 < L; b0 += 4) {
            const int b = b0 + kk;
            const bool bv = b < L;
            const float* er = a.ex + (int64_t)(bv ? b : 0) * a.lay.rec;
            float u = er[a.lay.oX + i] * er[a.lay.oA2 + j] + er[a.lay.oA1 + i] * er[a.lay.oY + j];
            if (!bv || !ijv) u = 0.f;
            float pv[RAE_KG];
#pragma unroll
            for (int q = 0; q < RAE_KG; ++q) {
                const int k = (kg0 + q) * 16 + li;
                const bool ok = q < nk && k < m && bv;
                pv[q] = ok ? er[a.lay.oP + (k < m ? k : 0)] : 0.f;
            }
#pragma unroll
            for (int q = 0; q < RAE_KG; ++q)
                if (q < nk) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, pv[q], acc[q], 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < RAE_KG; ++q) {
            if (q >= nk) continue;
            const int k = (kg0 + q) * 16 + li;
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) {
                const int64_t row = (int64_t)ijt * 16 + kk * 4 + rg;
                if (row < rr && k < m) {
                    const int64_t o = row * m + k;
                    const float wv = a.R3[o];
                    float gg = acc[q][rg];
                    if (reg) {
                        gg += a.l1adj * sgnf(wv) + 2.f * a.l2adj * wv;
                        l1 += fabsf(wv);
                        l2 += wv * wv;
                    }
                    float ac = (OPT == 0) ? a.aR3[o] : 0.f;
                    a.R3[o] = opt_update<OPT>(wv, &ac, gg, a.lr);
                    if (OPT == 0) a.aR3[o] = ac;
                }
            }
        }
    }
    if (reg) {
        const double L1 = wave_sum_d((double)l1), L2 = wave_sum_d((double)l2);
        if (lane == 0) {
            a.regpart[2 * slot] = L1;
            a.regpart[2 * slot + 1] = L2;
        }
    }
}

}  // namespace rae
