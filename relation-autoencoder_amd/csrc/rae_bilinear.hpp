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
// The forward phase of one step is six launches (all over this rank's l examples); M_b is
// never materialised (SURVEY 7 hard part v):
//   k_bil_enc  per example : encoder (P, log P, H), hybrid wC1/wC2, copies of A[e1], A[e2]
//   k_bil_mt   MFMA pass   : one workgroup per 8 x 16 block of R's (i, j), staged in LDS; the
//                            block's M tiles M_b[i][j] = sum_k P_bk R[i][j][k] (K = m)
//                            contracted at once both ways: partials of M a2 and M^T a1
//   k_bil_dec  per example : v = M a2, w = M^T a1 (partials summed), scores, loss,
//                            coefficients, x, y (+ hybrid dw1, dw2)
//   k_bil_mt   again       : partials of M y, M^T x
//   k_bil_dp   MFMA GEMM   : dP partials  sum_{i in block} sum_j U[b][i,j] R[i][j][k],
//                            U = x a2^T + a1 y^T generated on the fly (split over i-blocks)
//   k_bil_fin  per example : dP (+ hybrid C^T dw) -> entropy + softmax backward -> dS; the
//                            A-row gradient vectors from v, w, M y, M^T x
// The GEMMs run on v_mfma_f32_16x16x4_f32 (exact fp32) or, with rae_config.mfma_bf16 (BASELINE
// config 5), on v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulation).
#pragma once
#include "rae_common.hpp"
#include "rae_sp.hpp"
#include "rae_step.hpp"

namespace rae {

typedef float rae_bf4 __attribute__((ext_vector_type(4)));
#define RAE_IB 8     // i rows per dP partial block (k_bil_dp)
#ifndef RAE_FAC_BF16
#define RAE_FAC_BF16 1     // R-gradient factor copies (facT) stored as bf16: half the operand loads
#endif
#ifndef RAE_RT_PAIR
#define RAE_RT_PAIR 1      // R-gradient: two K-steps' operand loads per round trip
#endif
#ifndef RAE_RT_STAGGER
#define RAE_RT_STAGGER 1   // k_bil_rows: odd workgroups compute before issuing their tile reads
#endif
#ifndef RAE_KG
#define RAE_KG 8     // 16-column tiles of m per pass of one R-row task (task_bilinear_rows)
#endif

// ---- k_bil_enc: encoder + hybrid SP projections --------------------------------------------

// factor f (0 X, 1 A1, 2 A2, 3 Y) of example b at row i of the transposed operand copy k_bil_rows
// reads (RAE_FAC_BF16: stored as bf16, the precision the R-gradient MFMA consumes it at)
__device__ __forceinline__ void put_fac(const StepArgs& a, int f, int i, int b, float v) {
    const int64_t o = ((int64_t)f * a.r + i) * a.Lp + b;
    if (RAE_FAC_BF16) reinterpret_cast<__bf16*>(a.facT)[o] = (__bf16)v;
    else a.facT[o] = v;
}

// P[b][k] of example b as its element of the bf16 B fragments k_bil_rows reads (k_bil_prep's
// pfrag layout: fragment (b / 32, k / 16), lane 16 ((b % 32) / 8) + k % 16, element b % 8)
__device__ __forceinline__ void prep_p_fragment(const StepArgs& a, int b, int k, float p) {
    const int nkt = (a.m + 15) / 16, bb = b & 31;
    const int64_t t = (int64_t)(b >> 5) * nkt + (k >> 4);
    const int lane = 16 * (bb >> 3) + (k & 15);
    reinterpret_cast<__bf16*>(a.pfrag)[(t * 64 + lane) * 8 + (bb & 7)] = (__bf16)p;
}

template <bool V4>
__device__ void bil_encode(const StepArgs& a, int64_t g, int bl, char* smem) {
    const DynDims Dm(a);
    const int m = Dm.m, r = Dm.r;
    ExampleSmem S = carve_example_smem(smem, a.dec, m, r, Dm.s);
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;
    load_desc(a, Dm, g, bl, S);
    __syncthreads();
    CCache<V4, DynDims> cc_;
    encoder_forward<V4, V4, false>(a, Dm, S, 0, 0, cc_, true);
    const bool hybrid = a.dec == 2;
    if (hybrid) {
        sp_project<V4>(a, Dm, S, cc_);
        __syncthreads();
    }
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        rec[a.lay.oP + k] = S.sP[k];
        rec[a.lay.oZ + k] = S.sZ[k];
        if (a.fuse_prep) prep_p_fragment(a, bg, k, S.sP[k]);
    }
    const float* A1 = a.A + (int64_t)S.sids[0] * r;
    const float* A2 = a.A + (int64_t)S.sids[1] * r;
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        const float v1 = A1[i], v2 = A2[i];
        rec[a.lay.oA1 + i] = v1;
        rec[a.lay.oA2 + i] = v2;
        rec[a.lay.oV1 + i] = hybrid ? S.swC1[i] : 0.f;
        rec[a.lay.oV2 + i] = hybrid ? S.swC2[i] : 0.f;
        if (a.fuse_prep) {
            put_fac(a, 1, i, bg, v1);
            put_fac(a, 2, i, bg, v2);
        }
    }
    if (threadIdx.x == 0) rec[a.lay.oloss] = S.sred[40];     // H until k_bil_dec
}

// k_bil_enc for compile-time shapes (C5: K = 100, r = 200), RESCAL: the SP fast path's encoder
// -- the example's descriptor in one read, the W rows on waves 0-3, the softmax in wave 0 behind
// an LDS arrival counter (no block barrier) -- while waves 4-5 copy A[e1] / A[e2] into the
// record (and their bf16 factor copies) and waves 6-7 zero V1 / V2.  Rows with more features
// than the W-row registers hold, and the hybrid (its C.P), take bil_encode.
template <class D>
__device__ void bil_encode_fast(const StepArgs& a, int64_t g, int bl, char* smem) {
    static_assert(D::fixed && D::m % 4 == 0 && D::r % 4 == 0 && D::r / 4 <= RAE_WAVE, "fast encoder");
    constexpr int m = D::m, r = D::r, s = D::s, NJ = 2 + 2 * s;
    constexpr int MV = m / 4, NSL = 256 / MV, KF = 3, RV = r / 4;
    constexpr int mp = ((m + 255) / 256) * 256, NI = mp / RAE_WAVE;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    ExampleSmem S = carve_example_smem(smem, a.dec, m, r, s);
    const int bg = a.rank * a.l + bl;
    {
        const int32_t* dsc = a.desc + ((g % a.index_window) * a.dnx + a.d0 + bl) * (int64_t)a.dstride;
        if (tid < a.dstride) {
            const int v = dsc[tid];
            if (tid == 0) S.sint[1] = v;                          // nf
            else if (tid == 1) S.sint[0] = v;                     // p0
            else if (tid < 2 + NJ) S.sids[tid - 2] = v;
            else if (tid - 2 - NJ < 256) S.sfidx[tid - 2 - NJ] = v;
        }
    }
    float wbk[NI];                           // wave 0: the bias entries it reduces
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int k = lane + RAE_WAVE * i;
        wbk[i] = (w == 0 && k < m) ? a.Wb[k] : 0.f;
    }
    if (tid == 0) S.sint[4] = 0;             // arrival counter of the W-row waves
    lds_barrier();
    const int p0 = S.sint[0], nf = S.sint[1];
    if (nf > a.dcap || nf > NSL * KF) {
        lds_barrier();
        bil_encode<true>(a, g, bl, smem);
        return;
    }
    if (a.values) {
        if (w < 4 && tid < nf) S.sfval[tid] = a.values[p0 + tid];
        lds_barrier();
    }
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (w < 4) {
        // W rows: slot = feature lane group, c = float4 column; the partial sums into LDS
        const float4* W4 = reinterpret_cast<const float4*>(a.W);
        const int slot = tid / MV, c = tid - slot * MV;
        float4 wv[KF];
        float fv[KF];
#pragma unroll
        for (int k = 0; k < KF; ++k) {
            const int f = slot + NSL * k;
            const bool ok = slot < NSL && f < nf;
            const int fi = S.sfidx[f < 256 ? f : 255];
            wv[k] = W4[(int64_t)(ok ? fi : 0) * MV + c];
            fv[k] = ok ? (a.values ? S.sfval[f < 256 ? f : 255] : 1.f) : 0.f;
        }
        float4 acc = z4;
#pragma unroll
        for (int k = 0; k < KF; ++k) vfma(acc, fv[k], wv[k]);
        if (slot < NSL) reinterpret_cast<float4*>(S.spart)[slot * MV + c] = acc;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) atomicAdd(&S.sint[4], 1);
    } else if (w < 6) {
        // copies of A[e1] (wave 4) / A[e2] (wave 5), taken before the update changes A
        if (lane < RV) {
            const float4 v = reinterpret_cast<const float4*>(a.A + (int64_t)S.sids[w - 4] * r)[lane];
            reinterpret_cast<float4*>(rec + (w == 4 ? a.lay.oA1 : a.lay.oA2))[lane] = v;
            if (a.fuse_prep) {
                put_fac(a, w - 3, 4 * lane + 0, bg, v.x);
                put_fac(a, w - 3, 4 * lane + 1, bg, v.y);
                put_fac(a, w - 3, 4 * lane + 2, bg, v.z);
                put_fac(a, w - 3, 4 * lane + 3, bg, v.w);
            }
        }
    } else if (lane < RV) {                  // V1 / V2 = 0 (no SP part)
        reinterpret_cast<float4*>(rec + (w == 6 ? a.lay.oV1 : a.lay.oV2))[lane] = z4;
    }
    if (w == 0) {
        while (__hip_atomic_load(&S.sint[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4)
            __builtin_amdgcn_s_sleep(1);
        float pz[NI], pp[NI];
        fast_softmax<m, NSL, NI>(a, S, wbk, lane, pz, pp);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int k = lane + RAE_WAVE * i;
            if (k < m) {
                rec[a.lay.oP + k] = pp[i];
                rec[a.lay.oZ + k] = pz[i];
                if (a.fuse_prep) prep_p_fragment(a, bg, k, pp[i]);
            }
        }
        if (lane == 0) rec[a.lay.oloss] = S.sred[40];       // H until k_bil_dec
    }
}

// ---- bf16 fragments -----------------------------------------------------------------------
// v_mfma_f32_16x16x32_bf16: lane l holds A[l&15][8(l>>4) + e] and B[8(l>>4) + e][l&15],
// e = 0..7; fp32 values are rounded to bf16 (nearest even) as they enter the fragment,
// accumulation stays fp32.  K = 32 per instruction instead of 4.
typedef __bf16 rae_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ rae_bf16x8 to_bf16x8(float4 lo, float4 hi) {
    rae_bf16x8 v;
    v[0] = (__bf16)lo.x; v[1] = (__bf16)lo.y; v[2] = (__bf16)lo.z; v[3] = (__bf16)lo.w;
    v[4] = (__bf16)hi.x; v[5] = (__bf16)hi.y; v[6] = (__bf16)hi.z; v[7] = (__bf16)hi.w;
    return v;
}

// ---- k_bil_mt: M-tile passes over R blocks, M never stored ---------------------------------
// Workgroup (it, jt) stages the block R[i0..i0+7][j0..j0+15][0..m) in LDS (fp32, or bf16 with
// K padded to 32: every (i, j) row of k is one fragment run).  Each wave takes 16-example
// tiles; for every i of the block one MFMA chain (K = m) gives the transposed M tile
//   D[j][b] = sum_k R[i][j][k] P_bk = M_b[i][j]        (A = the block's rows j at this i,
//                                                       B = P^T: lane (li, g) holds
//                                                       D[j0 + 4g + reg][b0 + li])
// which is contracted at once, both ways, with the example's vectors:
//   cv side:  vpart[jt][b][i] = sum_{j in block} D[j][b] cv_b[j]      (cv = a2, pass 1; y, pass 2)
//   cw side:  wpart[it][b][j] = sum_{i in block} cw_b[i] D[j][b]      (cw = a1, pass 1; x, pass 2)
// Partials per j-block / i-block are summed in block order by the consumer (k_bil_dec for
// pass 1: v = M a2, w = M^T a1; k_bil_fin for pass 2: M y, M^T x) -- deterministic.  R is read
// once per pass; (r/8)(r/16) workgroups (325 at r = 200: every block's staging in one round).
#ifndef RAE_MTI
#define RAE_MTI 8         // rows i per block (a multiple of 4)
#endif
#define RAE_MTJ 16        // columns j per block (one MFMA tile of rows)
#ifndef RAE_MTT
#define RAE_MTT RAE_FBT   // threads per k_bil_mt workgroup (8 waves)
#endif
#define RAE_MTW (RAE_MTT / RAE_WAVE)
#define RAE_MT_SB 8       // float4 staging loads per thread in flight per round
// bf16: the block image [(i,j)][KP + 8] and, for the dP contraction of the second pass, its
// transpose [k][pairs + 8] (every B fragment one ds_read_b128)
#define RAE_MT_TP (RAE_MTI * RAE_MTJ + 8)
#define RAE_MT_NKS (RAE_MTI * RAE_MTJ / 32)   // K steps of the dP contraction (32 pairs each)
static_assert(RAE_MTI % 4 == 0 && RAE_MTJ == 16, "M-tile blocks: 4k rows i x 16 columns j");
__host__ __device__ inline size_t bil_mt_lds_bytes(int m, bool bf16) {
    const int KP = (m + 31) / 32 * 32;
    return bf16 ? (size_t)RAE_MTI * RAE_MTJ * (KP + 8) * 2 + (size_t)KP * RAE_MT_TP * 2
                : (size_t)RAE_MTI * RAE_MTJ * m * 4;
}
// fp32 blocks are 512 m bytes: above m = 320 they exceed the 160 KiB of LDS, and the block's
// MFMA chains read R straight from global memory (L2) instead (bil_mt<false, true>)
#define RAE_MT_LDS_MAX (160 * 1024)
#ifndef RAE_MT_STAMP_PASS
#define RAE_MT_STAMP_PASS 0
#endif
#ifdef RAE_STAMPS      // one pass only, past the per-example stamp region (l <= 1024)
#define RAE_MT_STAMP(slot)                                                                      \
    do {                                                                                        \
        if (a.stamps && pass == RAE_MT_STAMP_PASS && threadIdx.x == 0)                          \
            a.stamps[16384 + (size_t)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define RAE_MT_STAMP(slot) do { } while (0)
#endif

// DP: the instantiation that may carry the dP contraction (the second pass); the first pass's
// instantiation has none of its registers (occupancy)
template <bool BF16, bool DIRECT = false, bool DP = true>
__device__ void bil_mt(const StepArgs& a, int pass, char* smem) {
    static_assert(!(BF16 && DIRECT), "bf16 blocks are always staged (m <= 128)");
    const int r = a.r, m = a.m, l = a.l;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, g = lane >> 4;
    const int nbj = (r + RAE_MTJ - 1) / RAE_MTJ;
    const int it = blockIdx.x / nbj, jt = blockIdx.x - it * nbj;
    const int i0 = it * RAE_MTI, j0 = jt * RAE_MTJ;
    const int KP = (m + 31) / 32 * 32, ST = BF16 ? KP + 8 : m;   // row (i, j) stride in LDS
    const bool tr = DP && BF16 && pass == 1 && a.mtP != nullptr;  // stage the transpose too
    __bf16* sT = reinterpret_cast<__bf16*>(smem) + RAE_MTI * RAE_MTJ * ST;
    RAE_MT_STAMP(0);
    // ---- stage: LDS row (ii, jj) = R[i0+ii][j0+jj][0..m); rows past r are zero
    if (DIRECT) {
        // no staging: the MFMA chains read the block's rows from global memory
    } else if ((m & 3) == 0) {
        const int m4 = m / 4, nv = RAE_MTI * RAE_MTJ * m4;
        for (int e0 = 0; e0 < nv; e0 += RAE_MTT * RAE_MT_SB) {
            float4 v[RAE_MT_SB];
#pragma unroll
            for (int u = 0; u < RAE_MT_SB; ++u) {
                const int e = e0 + u * RAE_MTT + tid;
                const int row = e / m4, kq = e - row * m4;
                const int i = i0 + row / RAE_MTJ, j = j0 + row % RAE_MTJ;
                const bool ok = e < nv && i < r && j < r;
                const float4 x = *reinterpret_cast<const float4*>(
                    a.R3 + ((int64_t)(ok ? i : 0) * r + (ok ? j : 0)) * m + 4 * kq);
                v[u] = ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < RAE_MT_SB; ++u) {
                const int e = e0 + u * RAE_MTT + tid;
                if (e < nv) {
                    const int row = e / m4, kq = e - row * m4;
                    if constexpr (BF16) {
                        typedef __bf16 bf4_t __attribute__((ext_vector_type(4)));
                        bf4_t q;
                        q[0] = (__bf16)v[u].x; q[1] = (__bf16)v[u].y;
                        q[2] = (__bf16)v[u].z; q[3] = (__bf16)v[u].w;
                        *reinterpret_cast<bf4_t*>(reinterpret_cast<__bf16*>(smem) + row * ST + 4 * kq) = q;
                        if (tr) {
#pragma unroll
                            for (int c = 0; c < 4; ++c) sT[(4 * kq + c) * RAE_MT_TP + row] = q[c];
                        }
                    } else {
                        *reinterpret_cast<float4*>(reinterpret_cast<float*>(smem) + row * ST + 4 * kq) = v[u];
                    }
                }
            }
        }
    } else {
        for (int e = tid; e < RAE_MTI * RAE_MTJ * m; e += RAE_MTT) {
            const int row = e / m, k = e - row * m;
            const int i = i0 + row / RAE_MTJ, j = j0 + row % RAE_MTJ;
            const float x = (i < r && j < r) ? a.R3[((int64_t)i * r + j) * m + k] : 0.f;
            if constexpr (BF16) {
                reinterpret_cast<__bf16*>(smem)[row * ST + k] = (__bf16)x;
                if (tr) sT[k * RAE_MT_TP + row] = (__bf16)x;
            } else {
                reinterpret_cast<float*>(smem)[row * ST + k] = x;
            }
        }
    }
    if constexpr (BF16) {                      // zero K padding [m, KP)
        for (int e = tid; e < RAE_MTI * RAE_MTJ * (KP - m); e += RAE_MTT) {
            const int row = e / (KP - m), k = m + (e - row * (KP - m));
            reinterpret_cast<__bf16*>(smem)[row * ST + k] = (__bf16)0.f;
            if (tr) sT[k * RAE_MT_TP + row] = (__bf16)0.f;
        }
    }
    RAE_MT_STAMP(1);
    const int ov = pass == 0 ? a.lay.oA2 : a.lay.oY;      // cv: contracted over j
    const int ow = pass == 0 ? a.lay.oA1 : a.lay.oX;      // cw: contracted over i
    const int nbt = (l + 15) / 16;
    // dP operands of the second pass (bf16), for lane (li, g) of an example tile: a2 / y at
    // j0 + 8 (g&1) .. +7 and x / a1 at rows i0 + 2 ks + g/2, ks < RAE_MT_NKS (unconditional loads of
    // clamped addresses, then selects: a conditional load becomes a flat load through a zeroed
    // scratch slot)
    const bool dpass = DP && BF16 && pass == 1 && a.mtP != nullptr;
    struct DpOps { float a2v[8], yv[8], xq[RAE_MT_NKS], cq[RAE_MT_NKS]; };
    auto load_dp = [&](DpOps& o, const float* erb, bool bv) {
        const int jh = j0 + 8 * (g & 1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = jh + 4 * h;                // r4 padding of the record is zero
            const bool ok = bv && j < r;
            const int jc = j < r ? j : 0;
            const float4 va = *reinterpret_cast<const float4*>(erb + a.lay.oA2 + jc);
            const float4 vy = *reinterpret_cast<const float4*>(erb + a.lay.oY + jc);
            o.a2v[4 * h + 0] = ok ? va.x : 0.f; o.a2v[4 * h + 1] = ok ? va.y : 0.f;
            o.a2v[4 * h + 2] = ok ? va.z : 0.f; o.a2v[4 * h + 3] = ok ? va.w : 0.f;
            o.yv[4 * h + 0] = ok ? vy.x : 0.f; o.yv[4 * h + 1] = ok ? vy.y : 0.f;
            o.yv[4 * h + 2] = ok ? vy.z : 0.f; o.yv[4 * h + 3] = ok ? vy.w : 0.f;
        }
        const int ib = i0 + (g >> 1);
#pragma unroll
        for (int ks = 0; ks < RAE_MT_NKS; ++ks) {
            const int q = min(ib + 2 * ks, r - 1);
            const float lx = erb[a.lay.oX + q], lc = erb[a.lay.oA1 + q];
            const bool ok = bv && ib + 2 * ks < r;
            o.xq[ks] = ok ? lx : 0.f;
            o.cq[ks] = ok ? lc : 0.f;
        }
    };
    bool first = true;
    for (int bt = w; bt < nbt || first; bt += RAE_MTW) {
        const bool has = bt < nbt;
        // operands of this lane's example b0 + li, loaded before the barrier (in flight with
        // the staging): P (the B fragments), cv at j0 + 4g .. +3, cw at i0 .. i0 + 7
        const int bb = bt * 16 + li;
        const bool bv = has && bb < l;
        const float* erb = a.ex + (int64_t)(a.rank * l + (bv ? bb : 0)) * a.lay.rec;
        const float* Pa = erb + a.lay.oP;
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        // masked by a multiply, not a select: the compiler turns "load, then zero" into a load
        // through a zeroed scratch slot when registers are tight (the address is always valid)
        const float okv = (bv && j0 + 4 * g < r) ? 1.f : 0.f;
        float4 cv = *reinterpret_cast<const float4*>(erb + ov + (j0 + 4 * g < r ? j0 + 4 * g : 0));
        cv.x *= okv; cv.y *= okv; cv.z *= okv; cv.w *= okv;
        float cw[RAE_MTI];
#pragma unroll
        for (int q = 0; q < RAE_MTI / 4; ++q) {
            const int i = i0 + 4 * q;
            const float4 c = *reinterpret_cast<const float4*>(erb + ow + (i < r ? i : 0));
            const bool ok = bv && i < r;
            cw[4 * q + 0] = ok ? c.x : 0.f; cw[4 * q + 1] = ok ? c.y : 0.f;
            cw[4 * q + 2] = ok ? c.z : 0.f; cw[4 * q + 3] = ok ? c.w : 0.f;
        }
        rae_bf16x8 pf[4];                            // bf16: K <= 128 (m <= 128)
        if constexpr (BF16) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int k0 = ks * 32 + 8 * g;
                const float4 lo = *reinterpret_cast<const float4*>(Pa + (k0 < m ? k0 : 0));
                const float4 hi = *reinterpret_cast<const float4*>(Pa + (k0 + 4 < m ? k0 + 4 : 0));
                pf[ks] = to_bf16x8((bv && k0 < m) ? lo : z4, (bv && k0 + 4 < m) ? hi : z4);
            }
        }
        if (first) {
            RAE_MT_STAMP(2);
            __syncthreads();                         // the block is staged
            RAE_MT_STAMP(3);
            first = false;
        }
        if (!has) break;
        float vp[RAE_MTI];                           // cv side, per i of the block
        float4 wacc = z4;                            // cw side: j0 + 4g + reg
#pragma unroll
        for (int ii = 0; ii < RAE_MTI; ++ii) {
            rae_bf4 acc = {0.f, 0.f, 0.f, 0.f};
            if constexpr (BF16) {
                const __bf16* srow = reinterpret_cast<const __bf16*>(smem) + (ii * RAE_MTJ + li) * ST + 8 * g;
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    if (ks * 32 < KP) {
                        const rae_bf16x8 sf = *reinterpret_cast<const rae_bf16x8*>(srow + ks * 32);
                        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sf, pf[ks], acc, 0, 0, 0);
                    }
                }
            } else if (DIRECT) {
                const int i = i0 + ii, j = j0 + li;
                const bool rv = i < r && j < r;
                const float* grow = a.R3 + ((int64_t)(rv ? i : 0) * r + (rv ? j : 0)) * m;
                for (int k0 = 0; k0 < m; k0 += 4) {
                    const int k = k0 + g;
                    const float sa = (rv && k < m) ? grow[k] : 0.f;
                    const float pb = (bv && k < m) ? Pa[k] : 0.f;
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(sa, pb, acc, 0, 0, 0);
                }
            } else {
                const float* srow = reinterpret_cast<const float*>(smem) + (ii * RAE_MTJ + li) * ST;
                for (int k0 = 0; k0 < m; k0 += 4) {
                    const int k = k0 + g;
                    const float sa = k < m ? srow[k] : 0.f;
                    const float pb = (bv && k < m) ? Pa[k] : 0.f;
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(sa, pb, acc, 0, 0, 0);
                }
            }
            vp[ii] = acc[0] * cv.x + acc[1] * cv.y + acc[2] * cv.z + acc[3] * cv.w;
            wacc.x += cw[ii] * acc[0];
            wacc.y += cw[ii] * acc[1];
            wacc.z += cw[ii] * acc[2];
            wacc.w += cw[ii] * acc[3];
        }
        RAE_MT_STAMP(4);
        // cv side: sum over the four lane groups g (fixed order); groups g < RAE_MTI / 4 write
        // i0 + 4g .. +3
#pragma unroll
        for (int ii = 0; ii < RAE_MTI; ++ii) {
            vp[ii] += __uint_as_float(xor16_u32(__float_as_uint(vp[ii])));
            vp[ii] += __uint_as_float(xor32_u32(__float_as_uint(vp[ii])));
        }
        if (bv) {
            float* vo = a.mtV + ((int64_t)jt * l + bb) * a.r4 + i0 + 4 * g;
            if (4 * g < RAE_MTI && i0 + 4 * g < r) {
                float4 o = make_float4(vp[0], vp[1], vp[2], vp[3]);
#pragma unroll
                for (int q = 1; q < RAE_MTI / 4; ++q)
                    if (g == q) o = make_float4(vp[4 * q], vp[4 * q + 1], vp[4 * q + 2], vp[4 * q + 3]);
                *reinterpret_cast<float4*>(vo) = o;
            }
            if (j0 + 4 * g < r)
                *reinterpret_cast<float4*>(a.mtW + ((int64_t)it * l + bb) * a.r4 + j0 + 4 * g) = wacc;
        }
        RAE_MT_STAMP(5);
        if constexpr (BF16 && DP) {
            if (dpass) {
                // the block's share of dP_b[k] = sum_ij U_b[i][j] R[i][j][k], U = x a2^T + a1 y^T,
                // from the same staged block (k_bil_dp2's contraction without another read of
                // R): D[b][k] over K = the block's 16 RAE_MTI (i, j) pairs = its LDS rows; A = U (lane
                // (li, g): example bb, pairs 32 ks + 8g .. +7 = row i0 + 2 ks + g/2, columns
                // j0 + 8 (g&1) .. +7), B = 8 rows of the LDS image at column k
                DpOps dop;
                load_dp(dop, erb, bv);
                const int nkt = (m + 15) / 16;               // <= 8 (m <= 128)
                rae_bf4 dacc[8];
#pragma unroll
                for (int kt = 0; kt < 8; ++kt) dacc[kt] = rae_bf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
                for (int ks = 0; ks < RAE_MT_NKS; ++ks) {    // rolled: one K step's fragments live
                    float xk = dop.xq[0], ak = dop.cq[0];    // selects, not a dynamic index
#pragma unroll
                    for (int t = 1; t < RAE_MT_NKS; ++t)
                        if (ks == t) { xk = dop.xq[t]; ak = dop.cq[t]; }
                    rae_bf16x8 ua;
#pragma unroll
                    for (int e = 0; e < 8; ++e) ua[e] = (__bf16)(xk * dop.a2v[e] + ak * dop.yv[e]);
                    // B[pair][k]: the transposed image, 8 consecutive pairs at column k
                    const __bf16* lt = sT + li * RAE_MT_TP + ks * 32 + 8 * g;
#pragma unroll
                    for (int kt = 0; kt < 8; ++kt) {
                        if (kt >= nkt) break;
                        const rae_bf16x8 rb =
                            *reinterpret_cast<const rae_bf16x8*>(lt + kt * 16 * RAE_MT_TP);
                        dacc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua, rb, dacc[kt], 0, 0, 0);
                    }
                }
                RAE_MT_STAMP(6);
#pragma unroll
                for (int kt = 0; kt < 8; ++kt) {
                    if (kt >= nkt) break;
                    const int k = kt * 16 + li;
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) {     // D[b = 4g + reg][k = li]
                        const int bo = bt * 16 + 4 * g + reg;
                        if (bo < l && k < m)
                            a.mtP[((int64_t)blockIdx.x * l + bo) * m + k] = dacc[kt][reg];
                    }
                }
                RAE_MT_STAMP(7);
            }
        }
    }
}

// sum of the per-block partials [q0, q1) of one example's M-tile output (four interleaved
// chains, a fixed order: the loads are independent)
__device__ __forceinline__ float mt_sum(const float* part, int q0, int q1, int l, int r4, int b, int i) {
    const float* p = part + (int64_t)b * r4 + i;
    const int64_t st = (int64_t)l * r4;
    float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
    int q = q0;
    for (; q + 4 <= q1; q += 4) {
        t0 += p[q * st];
        t1 += p[(q + 1) * st];
        t2 += p[(q + 2) * st];
        t3 += p[(q + 3) * st];
    }
    for (; q < q1; ++q) t0 += p[q * st];
    return (t0 + t1) + (t2 + t3);
}
// One example's M-tile sums with four threads per element i: quarter qd of the workgroup's
// index space sums half the partials of one output -- qd 0/1: the j-block partials (mtV),
// qd 2/3: the i-block partials (mtW) -- into q0v / q1v / q0w / q1w; the caller combines the
// halves in order (after a barrier).
template <int T>
__device__ __forceinline__ void mt_sums_split(const StepArgs& a, int b, float* q0v, float* q1v,
                                              float* q0w, float* q1w) {
    const int r = a.r, r4 = a.r4;
    const int nbi = (r + RAE_MTI - 1) / RAE_MTI, nbj = (r + RAE_MTJ - 1) / RAE_MTJ;
    for (int e = threadIdx.x; e < 4 * r4; e += T) {
        const int qd = e / r4, i = e - qd * r4;
        const int n = qd < 2 ? nbj : nbi, h = n / 2;
        const float t = i < r ? mt_sum(qd < 2 ? a.mtV : a.mtW, (qd & 1) ? h : 0, (qd & 1) ? n : h,
                                       a.l, r4, b, i) : 0.f;
        (qd == 0 ? q0v : qd == 1 ? q1v : qd == 2 ? q0w : q1w)[i] = t;
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
#ifndef RAE_IB2
#define RAE_IB2 2    // i rows per k_bil_dp2 workgroup (the q-loop selects x/a1 for q < 2)
#endif
// threads per k_bil_dp2 workgroup: 512 for C5's <7, 7> (its 7 example tiles in one round);
// <8, 8> needs more than the 256 VGPRs an 8-wave workgroup allows, so it keeps 4 waves
template <int NJS, int MT>
constexpr int dp2_threads() { return (NJS >= 8 || MT >= 8) ? 256 : 512; }
template <int NJS, int MT>
constexpr size_t dp2_lds_bytes() { return (size_t)RAE_IB2 * MT * 16 * (NJS * 32 + 8) * 2; }
template <int NJS, int MT>
__device__ void bil_gemm_dp2(const StepArgs& a, int ib, char* smem) {
    constexpr int RAE_DP2T = dp2_threads<NJS, MT>();
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
    for (int e = tid; e < RAE_IB2 * KP * JS / 8; e += RAE_DP2T)
        reinterpret_cast<uint4*>(lds)[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    // A staging unit is 8 rows j x one float4 of k: its 8 loads are lanes' consecutive
    // 16-B chunks of whole rows (coalesced), and its 4 LDS stores are 16-B runs of 8 j at
    // one k (ds_write_b128).  All of a slice's loads are issued before its first store.
    const int m4 = m / 4, r8 = (r + 7) / 8, nunit = r8 * m4;
    constexpr int UU = ((JP / 8) * (KP / 4) + RAE_DP2T - 1) / RAE_DP2T;
    for (int q = 0; q < ni; ++q) {
        const float4* src = reinterpret_cast<const float4*>(a.R3 + (int64_t)(i0 + q) * r * m);
        __bf16* dst = lds + q * KP * JS;
        float4 v[UU][8];
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            const int e = tid + u * RAE_DP2T;
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
            const int e = tid + u * RAE_DP2T;
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
    for (int bt = w; bt < nbt; bt += RAE_DP2T / RAE_WAVE) {
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
// k_bil_dec runs 16 waves per example (RAE_DBT threads): the 2s negative rows' gathers and dots
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

// ---- k_bil_dec: scores, loss, coefficients, x, y -----------------------
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
    // negative rows: rows[t] = A[n1_t], rows[s + t] = A[n2_t]; v = M a2, w = M^T a1: the
    // first k_bil_mt pass's block partials, summed in block order
    for (int e = threadIdx.x; e < 2 * s * rv; e += RAE_DBT) {
        const int t = e / rv, c = e - t * rv;
        const VT* src = reinterpret_cast<const VT*>(a.A + (int64_t)S.ids[2 + t] * r);
        reinterpret_cast<VT*>(S.rows)[t * r4v + c] = src[c];
    }
    mt_sums_split<RAE_DBT>(a, bl, S.v, S.My, S.w, S.Mtx);    // My / Mtx: scratch halves here
    __syncthreads();
    for (int i = threadIdx.x; i < r4; i += RAE_DBT) {
        const float v = S.v[i] + S.My[i], w = S.w[i] + S.Mtx[i];
        S.v[i] = v;
        S.w[i] = w;
        if (i < r) {
            rec[a.lay.oG1 + i] = v;                       // for k_bil_fin
            rec[a.lay.oG2 + i] = w;
        }
    }
    __syncthreads();
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
            float sg1, spl1, sg2, spl2;           // hardware exp/log (rae_common.hpp)
            sigmoid_softplus(g1, sg1, spl1);
            sigmoid_softplus(g2, sg2, spl2);
            const float dg1 = sg1 * a.invD;
            const float dg2 = sg2 * a.invD;
            float* c1 = S.coef + 3 * (2 + t);
            float* c2 = S.coef + 3 * (2 + s + t);
            c1[0] = dg1; c1[1] = 0.f; c1[2] = dg1;
            c2[0] = 0.f; c2[1] = dg2; c2[2] = dg2;
            sdg1 += dg1;
            sdg2 += dg2;
            sls -= spl1 + spl2;                   // log sigmoid(-g) = -softplus(g)
        }
        sdg1 = wave_sum(sdg1);
        sdg2 = wave_sum(sdg2);
        sls = wave_sum(sls);
        if (lane == 0) {
            const float one = S.dots[2 * s] + sp1 + sp2;
            const float u1 = one + S.Abv[0], u2 = one + S.Abv[1];
            float su1, pu1, su2, pu2;             // sigmoid(-u), softplus(-u)
            sigmoid_softplus(-u1, su1, pu1);
            sigmoid_softplus(-u2, su2, pu2);
            const float du1 = -su1 * a.invD;
            const float du2 = -su2 * a.invD;
            const float dOne = du1 + du2;
            S.coef[0] = 0.f; S.coef[1] = 0.f; S.coef[2] = du1;
            S.coef[3] = 0.f; S.coef[4] = 0.f; S.coef[5] = du2;
            S.red[0] = dOne;
            S.red[1] = dOne + sdg2;      // c_a1: <wC1,a1> sits in one and every negTwo
            S.red[2] = dOne + sdg1;      // c_a2: <wC2,a2> sits in one and every negOne
            S.red[32] = -pu1 - pu2 + 2.f * H + sls;   // log sigmoid(u) = -softplus(-u)
        }
    }
    __syncthreads();

    // x = dOne a1 + sum_t dg1_t n1_t ; y = sum_t dg2_t n2_t ; hybrid dw1/dw2 (sums in t order),
    // straight into the record (the second k_bil_vw pass and k_bil_dp read x, y from there)
    {
        const float dOne = S.red[0], ca1 = S.red[1], ca2 = S.red[2];
        for (int i = threadIdx.x; i < r; i += RAE_DBT) {
            float n1 = 0.f, n2 = 0.f;
            for (int t = 0; t < s; ++t) {
                n1 += S.coef[3 * (2 + t)] * S.rows[t * r4 + i];
                n2 += S.coef[3 * (2 + s + t) + 1] * S.rows[(s + t) * r4 + i];
            }
            const float xv = dOne * S.a1[i] + n1;
            rec[a.lay.oX + i] = xv;
            rec[a.lay.oY + i] = n2;
            if (a.fuse_prep) {
                put_fac(a, 0, i, bg, xv);
                put_fac(a, 3, i, bg, n2);
            }
            rec[a.lay.odw1 + i] = hybrid ? ca1 * S.a1[i] + n1 : 0.f;
            rec[a.lay.odw2 + i] = hybrid ? ca2 * S.a2[i] + n2 : 0.f;
        }
        for (int j = threadIdx.x; j < NJ; j += RAE_DBT) {
            const float* c = S.coef + 3 * j;
            rec[a.lay.ocoef + 2 * j] = j < 2 ? 1.f : (j < 2 + s ? c[0] : c[1]);
            rec[a.lay.ocoef + 2 * j + 1] = c[2];
        }
        if (threadIdx.x == 0) {
            rec[a.lay.oloss] = S.red[32];
            rec[a.lay.oAux + 0] = dOne;
            rec[a.lay.oAux + 1] = ca1;
            rec[a.lay.oAux + 2] = ca2;
        }
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
// RAE_FINT threads (16 waves): the dP partial sums are split NS = RAE_FINT / m ways (each
// split sums every NS-th i-block partial in order; the splits are combined in order), so a
// thread has ~nib / NS independent loads instead of nib.
#define RAE_FINT 1024
#define RAE_FINW (RAE_FINT / RAE_WAVE)
__device__ void bil_finish(const StepArgs& a, int bl, float* sdp, float* smt, float* red) {
    const int m = a.m, r = a.r, l = a.l;
    const bool hybrid = a.dec == 2;
    const int bg = a.rank * l + bl;
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    const float ce = 2.f * a.alpha * a.invD;      // entropy term, centred form (softmax_backward)
    const int NS = max(1, RAE_FINT / m);
    // dP partials: per M-tile block of the second k_bil_mt pass (mtP), or per row block of
    // k_bil_dp / k_bil_dp2 (dPpart)
    const float* pbase = a.mtP ? a.mtP : a.dPpart;
    const int npart = a.mtP ? a.nmtp : a.nib;
    for (int e = threadIdx.x; e < NS * m; e += RAE_FINT) {
        const int sp = e / m, k = e - sp * m;
        const float* pp = pbase + (int64_t)bl * m + k;
        const int64_t st = (int64_t)l * m;
        // eight independent chains (fixed order): the loads of eight partials issue together
        float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int ib = sp;
        for (; ib + 7 * NS < npart; ib += 8 * NS) {
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] += pp[(ib + u * NS) * st];
        }
        for (int u = 0; ib < npart; ib += NS, ++u) t[u] += pp[ib * st];
        sdp[e] = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
    }
    mt_sums_split<RAE_FINT>(a, bl, smt, smt + 1024, smt + 2048, smt + 3072);
    __syncthreads();
    float sd = 0.f, sz = 0.f;
    for (int k = threadIdx.x; k < m; k += RAE_FINT) {
        float dp = 0.f;
        for (int sp = 0; sp < NS; ++sp) dp += sdp[sp * m + k];
        if (hybrid) {
            float h = 0.f;
            for (int i = 0; i < r; ++i)
                h += rec[a.lay.odw1 + i] * a.C1[(int64_t)i * m + k] +
                     rec[a.lay.odw2 + i] * a.C2[(int64_t)i * m + k];
            dp += h;
        }
        const float p = rec[a.lay.oP + k];
        sd += p * dp;
        sz += p * rec[a.lay.oZ + k];
        rec[a.lay.odS + k] = dp;                      // dP, scaled below
    }
    sd = block_sum<RAE_FINT>(sd, red);
    sz = block_sum<RAE_FINT>(sz, red + RAE_FINW);
    for (int k = threadIdx.x; k < m; k += RAE_FINT)
        rec[a.lay.odS + k] = rec[a.lay.oP + k] * ((rec[a.lay.odS + k] - sd) + ce * (rec[a.lay.oZ + k] - sz));
    // the A-row gradient vectors (rae_step.hpp), from v = M a2, w = M^T a1 (record G1 / G2),
    // M y, M^T x (My / MtX) and the hybrid's wC1 / wC2 (V1 / V2):
    //   V1 = v + wC1,  V2 = w + wC2,  G1 = dOne v + M y + c_a1 wC1,  G2 = M^T x + c_a2 wC2
    const float dOne = rec[a.lay.oAux + 0], ca1 = rec[a.lay.oAux + 1], ca2 = rec[a.lay.oAux + 2];
    for (int i = threadIdx.x; i < r; i += RAE_FINT) {
        const float v = rec[a.lay.oG1 + i], w = rec[a.lay.oG2 + i];
        const float my = smt[i] + smt[1024 + i];                   // second k_bil_mt pass
        const float mx = smt[2048 + i] + smt[3072 + i];
        const float c1 = hybrid ? rec[a.lay.oV1 + i] : 0.f, c2 = hybrid ? rec[a.lay.oV2 + i] : 0.f;
        rec[a.lay.oV1 + i] = v + c1;
        rec[a.lay.oV2 + i] = w + c2;
        rec[a.lay.oG1 + i] = dOne * v + my + ca1 * c1;
        rec[a.lay.oG2 + i] = mx + ca2 * c2;
    }
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
            if (i < r) put_fac(a, f, i, bs * 32 + bb, tile[bb][ii]);
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
// (row (i, j) of this lane's column li; ijv false: a padding row, zero contributions)
template <bool PAIR = (RAE_RT_PAIR != 0)>
__device__ __forceinline__ void bilinear_rows_acc_bf16_ij(const StepArgs& a, int i, int j, bool ijv,
                                                          int kg0, int nk, rae_bf4* acc, int lane) {
    const int r = a.r, L = a.L, Lp = a.Lp, nkt = (a.m + 15) / 16;
    const int g = lane >> 4;
    const float* xt = a.facT + (int64_t)i * Lp;
    const float* a1t = a.facT + (int64_t)(r + i) * Lp;
    const float* a2t = a.facT + (int64_t)(2 * r + j) * Lp;
    const float* yt = a.facT + (int64_t)(3 * r + j) * Lp;
    const __bf16* fb = reinterpret_cast<const __bf16*>(a.facT);
    const __bf16* xb = fb + (int64_t)i * Lp;
    const __bf16* a1b = fb + (int64_t)(r + i) * Lp;
    const __bf16* a2b = fb + (int64_t)(2 * r + j) * Lp;
    const __bf16* yb = fb + (int64_t)(3 * r + j) * Lp;
    // one K-step (32 examples): the lane's 8 examples of each factor and the P fragments
    struct Step {
        float xv[8], a1v[8], a2v[8], yv[8];
        rae_bf16x8 pb[RAE_KG];
    };
    auto load = [&](Step& st, int b0) {
        const int bb = b0 + 8 * g;
        if (RAE_FAC_BF16) {                              // 8 examples of a factor: one 16-B load
            const rae_bf16x8 vx = *reinterpret_cast<const rae_bf16x8*>(xb + bb);
            const rae_bf16x8 v1 = *reinterpret_cast<const rae_bf16x8*>(a1b + bb);
            const rae_bf16x8 v2 = *reinterpret_cast<const rae_bf16x8*>(a2b + bb);
            const rae_bf16x8 vy = *reinterpret_cast<const rae_bf16x8*>(yb + bb);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                st.xv[e] = (float)vx[e];
                st.a1v[e] = (float)v1[e];
                st.a2v[e] = (float)v2[e];
                st.yv[e] = (float)vy[e];
            }
        } else {
        *reinterpret_cast<float4*>(st.xv) = *reinterpret_cast<const float4*>(xt + bb);
        *reinterpret_cast<float4*>(st.xv + 4) = *reinterpret_cast<const float4*>(xt + bb + 4);
        *reinterpret_cast<float4*>(st.a1v) = *reinterpret_cast<const float4*>(a1t + bb);
        *reinterpret_cast<float4*>(st.a1v + 4) = *reinterpret_cast<const float4*>(a1t + bb + 4);
        *reinterpret_cast<float4*>(st.a2v) = *reinterpret_cast<const float4*>(a2t + bb);
        *reinterpret_cast<float4*>(st.a2v + 4) = *reinterpret_cast<const float4*>(a2t + bb + 4);
        *reinterpret_cast<float4*>(st.yv) = *reinterpret_cast<const float4*>(yt + bb);
        *reinterpret_cast<float4*>(st.yv + 4) = *reinterpret_cast<const float4*>(yt + bb + 4);
        }
        const uint4* pf = a.pfrag + ((int64_t)(b0 / 32) * nkt + kg0) * 64 + lane;
#pragma unroll
        for (int q = 0; q < RAE_KG; ++q) {
            const uint4 u = pf[(q < nk ? q : 0) * 64];
            st.pb[q] = *reinterpret_cast<const rae_bf16x8*>(&u);
        }
    };
    auto mfma = [&](const Step& st) {
        rae_bf16x8 ua;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float u = st.xv[e] * st.a2v[e] + st.a1v[e] * st.yv[e];   // zero past L (padded)
            ua[e] = (__bf16)(ijv ? u : 0.f);
        }
#pragma unroll
        for (int q = 0; q < RAE_KG; ++q) {          // D[k][ij]: P^T as A, U as B
            if (q >= nk) continue;
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st.pb[q], ua, acc[q], 0, 0, 0);
        }
    };
    if constexpr (PAIR) {
        // two K-steps' loads issued before either step's MFMAs: half the dependent round trips
        int b0 = 0;
        for (; b0 + 32 < L; b0 += 64) {
            Step s0, s1;
            load(s0, b0);
            load(s1, b0 + 32);
            __builtin_amdgcn_sched_barrier(0);
            mfma(s0);
            mfma(s1);
        }
        if (b0 < L) {
            Step s0;
            load(s0, b0);
            mfma(s0);
        }
    } else {
        for (int b0 = 0; b0 < L; b0 += 32) {
            Step s0;
            load(s0, b0);
            mfma(s0);
        }
    }
}

__device__ __forceinline__ void bilinear_rows_acc_bf16(const StepArgs& a, int ijt, int kg0, int nk,
                                                       rae_bf4* acc, int lane) {
    const int r = a.r;
    const int64_t ij = (int64_t)ijt * 16 + (lane & 15);
    const bool ijv = ij < (int64_t)r * r;
    const int ijc = (int)(ijv ? ij : 0);
    bilinear_rows_acc_bf16_ij(a, ijc / r, ijc - (ijc / r) * r, ijv, kg0, nk, acc, lane);
}

// One wave: 16 rows ij x all m columns.  The gradient tile comes out transposed (D[k][ij]:
// lane (li, kk) holds k = 16q + 4kk + rg of row ij = 16 ijt + li), so each lane updates four
// consecutive parameters of one row: float4 read-modify-write, every load of the tile issued
// before its first store (one memory round trip per column group instead of one per element).
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
    const bool vec = (m & 3) == 0;
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
                if (q < nk) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(pv[q], u, acc[q], 0, 0, 0);
        }
        auto apply = [&](float wv, float& ac, float gg) {
            if (reg) {
                gg += a.l1adj * sgnf(wv) + 2.f * a.l2adj * wv;
                l1 += fabsf(wv);
                l2 += wv * wv;
            }
            return opt_update<OPT>(wv, &ac, gg, a.lr);
        };
        if (vec) {
            float4 wv[RAE_KG], av[RAE_KG];
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int q = 0; q < RAE_KG; ++q) {
                const int k0 = (kg0 + q) * 16 + 4 * kk;
                const bool ok = q < nk && ijv && k0 < m;
                const int64_t o = ok ? ij * m + k0 : 0;
                wv[q] = ok ? *reinterpret_cast<const float4*>(a.R3 + o) : z4;
                av[q] = (OPT == 0 && ok) ? *reinterpret_cast<const float4*>(a.aR3 + o) : z4;
            }
#pragma unroll
            for (int q = 0; q < RAE_KG; ++q) {
                const int k0 = (kg0 + q) * 16 + 4 * kk;
                if (!(q < nk && ijv && k0 < m)) continue;
                const int64_t o = ij * m + k0;
                float4 w = wv[q], ac = av[q];
                w.x = apply(w.x, ac.x, acc[q][0]);
                w.y = apply(w.y, ac.y, acc[q][1]);
                w.z = apply(w.z, ac.z, acc[q][2]);
                w.w = apply(w.w, ac.w, acc[q][3]);
                *reinterpret_cast<float4*>(a.R3 + o) = w;
                if (OPT == 0) *reinterpret_cast<float4*>(a.aR3 + o) = ac;
            }
        } else {
#pragma unroll
            for (int q = 0; q < RAE_KG; ++q) {
                if (q >= nk || !ijv) continue;
#pragma unroll
                for (int rg = 0; rg < 4; ++rg) {
                    const int k = (kg0 + q) * 16 + 4 * kk + rg;
                    if (k >= m) continue;
                    const int64_t o = ij * m + k;
                    float ac = (OPT == 0) ? a.aR3[o] : 0.f;
                    a.R3[o] = apply(a.R3[o], ac, acc[q][rg]);
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

// k_bil_rows' fast path (bf16 operands, m % 4 == 0, m <= RAE_RT_LDS_M): the wave's 16 rows
// of R and of the optimizer state are one contiguous 64m-byte run each; they are copied into
// the wave's LDS slice by direct global->LDS loads (global_load_lds_dwordx4: lane-linear
// 1 KB per instruction) issued BEFORE the gradient, so the parameter reads are in flight
// during it -- all waves of the launch start together, and with loads after the gradient
// the latency-bound gradient phase and the HBM-bound read-modify-write phase never overlap
// (measured at C5: 8.2 + 16.7 us sequential).  Then float4 read-modify-write from LDS,
// float4 stores to HBM.
#define RAE_RT_LDS_M 128
__host__ __device__ inline size_t bil_rows_lds_bytes(int m, bool bf16, bool adagrad) {
    return (bf16 && (m & 3) == 0 && m <= RAE_RT_LDS_M) ? (size_t)RAE_NWAVE * (adagrad ? 2 : 1) * 16 * m * 4 : 0;
}
template <int OPT>
__device__ void task_bilinear_rows_lds(const StepArgs& a, int ijt, int slot, int lane, float* sw) {
    typedef __attribute__((address_space(3))) void lds_void_t;
    typedef __attribute__((address_space(1))) void glb_void_t;
    const int m = a.m, r = a.r;
    const int64_t rr = (int64_t)r * r;
    const int li = lane & 15, kk = lane >> 4;
    const int64_t ij = (int64_t)ijt * 16 + li;
    const bool ijv = ij < rr;
    const int64_t base = (int64_t)ijt * 16 * m;
    const int nrow = (int)min((int64_t)16, rr - (int64_t)ijt * 16);
    const int nv = nrow * m / 4;                          // float4s of the tile
    float* sR = sw;
    float* sA = sw + 16 * m;
    rae_bf4 acc[RAE_KG];
#pragma unroll
    for (int q = 0; q < RAE_KG; ++q) acc[q] = rae_bf4{0.f, 0.f, 0.f, 0.f};
    const int nk = (m + 15) / 16;                         // <= RAE_KG: one column group
    // RAE_RT_STAGGER: every other workgroup runs its gradient before its tile reads are issued,
    // so half of the launch's read-modify-write traffic meets the other half's gradient phase
    const bool pre = RAE_RT_STAGGER && (blockIdx.x & 1);
    if (pre) bilinear_rows_acc_bf16(a, ijt, 0, nk, acc, lane);
    for (int n = 0; n * 64 < nv; ++n) {
        const int idx = n * 64 + lane;
        if (idx < nv) {
            __builtin_amdgcn_global_load_lds((glb_void_t*)(a.R3 + base + 4 * idx),
                                             (lds_void_t*)(sR + n * 256), 16, 0, 0);
            if constexpr (OPT == 0)
                __builtin_amdgcn_global_load_lds((glb_void_t*)(a.aR3 + base + 4 * idx),
                                                 (lds_void_t*)(sA + n * 256), 16, 0, 0);
        }
    }
    const bool reg = a.reg_on && a.ext_reg;
    float l1 = 0.f, l2 = 0.f;
    if (!pre) bilinear_rows_acc_bf16(a, ijt, 0, nk, acc, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the tile has landed in LDS
#pragma unroll
    for (int q = 0; q < RAE_KG; ++q) {
        const int k0 = q * 16 + 4 * kk;
        if (!(q < nk && ijv && k0 < m)) continue;
        const int lo = li * m + k0;
        float4 w = *reinterpret_cast<const float4*>(sR + lo);
        float4 ac = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (OPT == 0) ac = *reinterpret_cast<const float4*>(sA + lo);
        float* wp = &w.x;
        float* ap = &ac.x;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float gg = acc[q][e];
            if (reg) {
                gg += a.l1adj * sgnf(wp[e]) + 2.f * a.l2adj * wp[e];
                l1 += fabsf(wp[e]);
                l2 += wp[e] * wp[e];
            }
            wp[e] = opt_update<OPT>(wp[e], &ap[e], gg, a.lr);
        }
        *reinterpret_cast<float4*>(a.R3 + base + lo) = w;
        if constexpr (OPT == 0) *reinterpret_cast<float4*>(a.aR3 + base + lo) = ac;
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
