// Split SP forward for large runtime shapes (C4: r x m = 90 k floats per decoder matrix).
//
// The fused example kernel (rae_sp.hpp sp_example) streams C1 and C2 through every example's
// workgroup twice (C.P, then C^T.dw): 1.4 MB per example at C4, so the forward is bound by
// each CU's fill rate from L2.  Here the two matrix products run once for the rank's whole
// batch as fp32-MFMA GEMMs, and the per-example work is split around them:
//   k_sp_enc   per example : S = X.W + Wb, P = softmax(S), H          -> record P; z, H parked
//   k_sp_cp    GEMM        : V1 = P C1^T, V2 = P C2^T  (l x r, K = m)  -> record V1, V2
//   k_sp_dec   two workgroups per example, one per negative side (h = 0: neg1, 1: neg2): A[e1]
//              and that side's s rows, dots, the side's coefficients and its weighted row sum
//              N_h = sum_t dg_t A[neg_h,t]  -> scratch (N_h, A[e1], per-example scalars)
//   k_sp_ctdw  GEMM        : dP = dw1 C1 + dw2 C2      (l x m, K = 2r), the operand assembled as it
//                            loads (dw1 = dl A[e1] + N1, dw2 = dr A[e1] + N2: dl, dr need both
//                            sides' sums), and in its epilogue the centred softmax backward,
//                            element-wise -> record dS; the tiles also store dw1, dw2, G1 (or dl,
//                            dr for the wire record) and the loss
// The softmax backward's two sums per example come from k_sp_enc / k_sp_dec, not from dP:
// sum_k P_k dP_k = <dw1, C1.P> + <dw2, C2.P> = dl left + <N1, V1> + dr right + <N2, V2> (V = k_sp_cp's
// vectors, left / right = <V1, A[e1]>, <V2, A[e1]>) and sum_k P_k z_k -- so
// dS_bk = P_bk ((dP_bk - sd_b) + ce (z_bk - sz_b)) needs nothing outside the tile (round 5: the
// fifth launch, k_sp_fin, is gone, and the decoder's 121 KB A-row gather per example at C4 is
// split over two workgroups).
// Same arithmetic as sp_example (SelectionalPreferences.py:30-51, RelationClassifier.py:35-36,
// OieModel.py:81); only the fp32 summation order of the products and row sums differs.  Until
// k_sp_ctdw the record's dS slot holds z = S - max S and its loss slot holds H.
#pragma once
#include "rae_sp.hpp"

namespace rae {

typedef float rae_f32x4 __attribute__((ext_vector_type(4)));

// k_sp_dec pieces: each negative side is split into RAE_SPD_NQ ranges of negatives, one
// workgroup each (2 RAE_SPD_NQ workgroups per example)
#ifndef RAE_SPD_NQ
#define RAE_SPD_NQ 1   // measured (C4 forward, events): 1 -> 28.6 us, 2 -> 30.8, 3 -> 38.0
#endif
#define RAE_SPD_NP (2 * RAE_SPD_NQ)
static_assert(RAE_SPD_NQ >= 1 && 8 + 3 * RAE_SPD_NP <= 32, "pieces' scalars fit the 32-float block");
// per-example scratch of the split forward (a.sps, stride a.spss = sps_stride(r)):
// [N_{h,q} (r4 each, piece p = h NQ + q) | A[e1] (r4) | scalars (32)]
enum {
    SPS_SZ = 0,      // sum_k P_k z_k (k_sp_enc)
    SPS_LEFT,        // <V1, A[e1]>, <V2, A[e1]>      (k_sp_dec piece 0)
    SPS_RIGHT,
    SPS_DU1,         // d cost / d u1, u2 (positive scores)
    SPS_DU2,
    SPS_LBASE,       // -softplus(-u1) - softplus(-u2) + 2 H
    SPS_PIECE = 8    // + 3 p: piece p's sum of coefficients, of log sigmoids, <N_p, V_h>
};
__host__ __device__ inline int sps_stride(int r) { return (RAE_SPD_NP + 1) * align4(r) + 32; }
__host__ __device__ inline int sps_oa(int r4) { return RAE_SPD_NP * r4; }          // A[e1]
__host__ __device__ inline int sps_os(int r4) { return (RAE_SPD_NP + 1) * r4; }    // scalars
__host__ __device__ inline int spd_neg_per_piece(int s) { return (s + RAE_SPD_NQ - 1) / RAE_SPD_NQ; }
// LDS of one k_sp_dec piece: V1, V2, its 1 + ns rows, dots / ids / Ab / coefficients, the row-sum
// partials (<= 8 groups) and the block-sum scratch
__host__ __device__ inline int sp_dec_side_smem_floats(int r, int s) {
    const int ns = spd_neg_per_piece(s), r4 = align4(r), s4 = align4(ns + 2);
    return 2 * r4 + (1 + ns) * r4 + 4 * s4 + 8 * r4 + 64;
}

template <bool V4>
__device__ void sp_split_enc(const StepArgs& a, int64_t g, int bl, char* smem) {
    const DynDims Dm(a);
    const int m = Dm.m;
    ExampleSmem S = carve_example_smem(smem, 0, m, Dm.r, 0);      // no A rows here
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    RAE_STAMP(a, 8);
    load_desc(a, Dm, g, bl, S, false);
    __syncthreads();
    RAE_STAMP(a, 9);
    CCache<V4, DynDims> cc_;                                       // unused: no C here
    encoder_forward<V4, V4, false, DynDims, CCache<V4, DynDims>, true>(a, Dm, S, 0, 1, cc_, true);
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        rec[a.lay.oP + k] = S.sP[k];
        rec[a.lay.odS + k] = S.sZ[k];
    }
    if (threadIdx.x == 0) {
        rec[a.lay.oloss] = S.sred[40];
        // sz = sum_k P_k z_k for k_sp_ctdw's epilogue (the encoder's wave 0 for m <= 512)
        float x = S.sred[41];
        if (m > 8 * RAE_WAVE) {
            x = 0.f;
            for (int k = 0; k < m; ++k) x += S.sP[k] * S.sZ[k];
        }
        a.sps[(int64_t)bl * a.spss + sps_os(align4(Dm.r)) + SPS_SZ] = x;
    }
    RAE_STAMP(a, 14);
}

// four fp32 MFMAs over a 16-deep K chunk: lane (li, g) supplies K = k0 + 4g + j for MFMA j
__device__ __forceinline__ rae_f32x4 mfma4_f32(const float4 x, const float4 y, rae_f32x4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.w, acc, 0, 0, 0);
    return acc;
}
// branch-free: the load always issues (clamped to element 0, always valid) and the value is
// selected after -- a guarded load compiles to an exec-masked branch per load, and the branches
// serialised every operand load of the GEMM tiles behind its own wait
template <bool VEC>
__device__ __forceinline__ float4 load4_guard(const float* p, int k, int n, bool ok) {
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (VEC) {                                       // n % 4 == 0: k < n covers k + 3
        const bool in = ok && k < n;
        const float4 v = *reinterpret_cast<const float4*>(p + (in ? k : 0));
        return in ? v : z4;
    }
    float4 v;
    const float x0 = p[(ok && k < n) ? k : 0], x1 = p[(ok && k + 1 < n) ? k + 1 : 0];
    const float x2 = p[(ok && k + 2 < n) ? k + 2 : 0], x3 = p[(ok && k + 3 < n) ? k + 3 : 0];
    v.x = (ok && k < n) ? x0 : 0.f;
    v.y = (ok && k + 1 < n) ? x1 : 0.f;
    v.z = (ok && k + 2 < n) ? x2 : 0.f;
    v.w = (ok && k + 3 < n) ? x3 : 0.f;
    return v;
}

__host__ __device__ inline int sp_cp_tasks(int l, int r) { return 2 * ((l + 15) / 16) * ((r + 15) / 16); }
__host__ __device__ inline int sp_ctdw_tasks(int l, int m) { return ((l + 15) / 16) * ((m + 15) / 16); }

// The two GEMMs: one workgroup per 16 x 16 output tile (k_sp_cp 4 waves, k_sp_ctdw RAE_DW_NW);
// wave w takes the K chunks c = w, w + NW, ... (16 deep each), RAE_SPG_U* chunks' loads issued
// before their MFMAs, and the waves' accumulators are combined in LDS in wave order
// (deterministic; k_vrec repeats k_sp_cp's order).
#ifndef RAE_SPG_UCP
#define RAE_SPG_UCP 5   // k_sp_cp: 16-deep K chunks per wave per round (C4: m = 300, 19
                        // chunks over 4 waves -- all in one round)
#endif
#ifndef RAE_DW_NW
#define RAE_DW_NW 8     // k_sp_ctdw: waves per tile workgroup (K split over them; C4 forward
                        // 27.2 us at 4, 26.5 at 8, 26.9-27.3 at 16 -- profiles/r05_ab.txt)
#endif
#define RAE_DW_BT (RAE_DW_NW * RAE_WAVE)
#ifndef RAE_SPG_UDW
#define RAE_SPG_UDW 3   // k_sp_ctdw (C4: 2r = 600, 38 chunks over 8 waves, two rounds: 26.5 us,
                        // as at 2; at 4 waves rounds of 5 measured 28.0, 10 28.7, 4 28.8)
#endif
template <int NW = RAE_NWAVE>
__device__ __forceinline__ void sp_gemm_combine(rae_f32x4 acc, float* red, int lane, int w,
                                                float out[4]) {
    float4* r4 = reinterpret_cast<float4*>(red);
    r4[w * 64 + lane] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    if (w == 0) {
        float4 t = r4[lane];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) {
            const float4 u = r4[ww * 64 + lane];
            t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        out[0] = t.x; out[1] = t.y; out[2] = t.z; out[3] = t.w;
    }
}

// k_sp_cp: tile (example, i) of V1 or V2.  A = P (rows b, K = k), B = C^T (K = k, columns i):
// both K-contiguous, one float4 per lane per 16-deep chunk.
template <bool VEC>
__device__ void sp_split_cp(const StepArgs& a, int task, float* red) {
    const int l = a.l, m = a.m, r = a.r;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nbt = (l + 15) / 16, nit = (r + 15) / 16;
    const int which = task / (nbt * nit), t2 = task - which * nbt * nit;
    const int bt = t2 / nit, it = t2 - bt * nit;
    const int li = lane & 15, g = lane >> 4;
    const int b = bt * 16 + li, i = it * 16 + li;
    const bool bv = b < l, iv = i < r;
    const float* Pr = a.ex + (int64_t)(a.rank * l + (bv ? b : 0)) * a.lay.rec + a.lay.oP;
    const float* Cr = (which ? a.C2 : a.C1) + (int64_t)(iv ? i : 0) * m;
    rae_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nch = (m + 15) / 16;
    for (int c0 = w; c0 < nch; c0 += RAE_NWAVE * RAE_SPG_UCP) {
        float4 x[RAE_SPG_UCP], y[RAE_SPG_UCP];
#pragma unroll
        for (int u = 0; u < RAE_SPG_UCP; ++u) {
            const int k = (c0 + u * RAE_NWAVE) * 16 + 4 * g;     // >= m past the last chunk
            x[u] = load4_guard<VEC>(Pr, k, m, bv);
            y[u] = load4_guard<VEC>(Cr, k, m, iv);
        }
#pragma unroll
        for (int u = 0; u < RAE_SPG_UCP; ++u) acc = mfma4_f32(x[u], y[u], acc);
    }
    float o[4];
    sp_gemm_combine(acc, red, lane, w, o);
    if (w != 0) return;
    // into the vectors the update reads (the record, or the wire record's vector buffer)
    float* vb = const_cast<float*>(a.vb);
    const int oV = which ? a.vV2 : a.vV1;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {                   // D[b = 4g + reg][i = li]
        const int bo = bt * 16 + 4 * g + reg;
        if (bo < l && iv) vb[(int64_t)(a.rank * l + bo) * a.vbs + oV + i] = o[reg];
    }
}

// k_vrec (SP wire record, world_size > 1, after the exchange): V1 = P C1^T, V2 = P C2^T and
// G1 = dl V1 + dr V2 for every example of the global batch into the vector buffer -- the
// vectors the wire record leaves out.  One WAVE per 16 x 16 tile of V1 and V2 at once (no LDS, no
// barrier: every operand load of the tile issued up front), yet per output element the same
// arithmetic as k_sp_cp: chunk c (16 deep) goes to accumulator c % 4 (k_sp_cp's wave c % 4), the
// four summed in order -- so the split forward's own vectors and every rank's are bit-identical.
// task = (example tile, embedding tile).
#ifndef RAE_VR_KC
#define RAE_VR_KC 4          // 16-deep K chunks whose operand loads one round issues (4: 128
                             // registers, 4 waves per SIMD; 8: 168, 3)
#endif
static_assert(RAE_VR_KC % 4 == 0, "chunk u of a round feeds accumulator u % 4");
__host__ __device__ inline int vrec_tasks(int L, int r) { return ((L + 15) / 16) * ((r + 15) / 16); }
template <bool VEC>
__device__ void sp_vrec(const StepArgs& a, int task, int lane) {
    const int L = a.L, m = a.m, r = a.r;
    const int nit = (r + 15) / 16;
    const int bt = task / nit, it = task - bt * nit;
    const int li = lane & 15, g = lane >> 4;
    const int b = bt * 16 + li, i = it * 16 + li;
    const bool bv = b < L, iv = i < r;
    const float* Pr = a.ex + (int64_t)(bv ? b : 0) * a.lay.rec + a.lay.oP;
    const float* C1r = a.C1 + (int64_t)(iv ? i : 0) * m;
    const float* C2r = a.C2 + (int64_t)(iv ? i : 0) * m;
    const int nch = (m + 15) / 16;
    // the coefficients of the tile's four output rows first: independent of the products
    float dlv[4], drv[4];
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int bo = bt * 16 + 4 * g + reg;
        const float* rec = a.ex + (int64_t)(bo < L ? bo : 0) * a.lay.rec + a.lay.oAux;
        dlv[reg] = rec[0];
        drv[reg] = rec[1];
    }
    rae_f32x4 acc1[4], acc2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc1[q] = acc2[q] = rae_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nch; c0 += RAE_VR_KC) {          // one round at m <= 16 RAE_VR_KC
        // V1's operands (P and C1) in one round trip, then C2's into the same registers: the
        // P fragments serve both products (fewer live registers: more resident waves)
        float4 x[RAE_VR_KC], y[RAE_VR_KC];
#pragma unroll
        for (int u = 0; u < RAE_VR_KC; ++u) {
            const int k = (c0 + u) * 16 + 4 * g;           // >= m past the last chunk
            const bool cv = c0 + u < nch;
            x[u] = load4_guard<VEC>(Pr, k, m, bv && cv);
            y[u] = load4_guard<VEC>(C1r, k, m, iv && cv);
        }
#pragma unroll
        for (int u = 0; u < RAE_VR_KC; ++u)                // RAE_VR_KC % 4 == 0: chunk c0 + u
            if (c0 + u < nch) acc1[u & 3] = mfma4_f32(x[u], y[u], acc1[u & 3]);   // -> acc u % 4
#pragma unroll
        for (int u = 0; u < RAE_VR_KC; ++u) {
            const int k = (c0 + u) * 16 + 4 * g;
            y[u] = load4_guard<VEC>(C2r, k, m, iv && c0 + u < nch);
        }
#pragma unroll
        for (int u = 0; u < RAE_VR_KC; ++u)
            if (c0 + u < nch) acc2[u & 3] = mfma4_f32(x[u], y[u], acc2[u & 3]);
    }
    // sp_gemm_combine's order: wave 0's accumulator, + wave 1's, + wave 2's, + wave 3's
    rae_f32x4 o1 = acc1[0], o2 = acc2[0];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
        o1 += acc1[q];
        o2 += acc2[q];
    }
    float* vb = const_cast<float*>(a.vb);
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {                   // D[b = 4g + reg][i = li]
        const int bo = bt * 16 + 4 * g + reg;
        if (bo < L && iv) {
            float* v = vb + (int64_t)bo * a.vbs;
            v[a.vV1 + i] = o1[reg];
            v[a.vV2 + i] = o2[reg];
            v[a.vG1 + i] = fmaf(dlv[reg], o1[reg], drv[reg] * o2[reg]);   // as k_sp_dec
        }
    }
}

// the sums of an example's pieces (in piece order): side h's row sum N_h at column i, and the
// scalars of side h (f = 0: coefficients, 1: log sigmoids, 2: <N, V_h>)
__device__ __forceinline__ float sps_side(const float* scl, int h, int f) {
    float v = scl[SPS_PIECE + 3 * (h * RAE_SPD_NQ) + f];
#pragma unroll
    for (int q = 1; q < RAE_SPD_NQ; ++q) v += scl[SPS_PIECE + 3 * (h * RAE_SPD_NQ + q) + f];
    return v;
}
template <bool VEC>
__device__ __forceinline__ float4 sps_rowsum4(const float* sp, int h, int i, int r, bool ok) {
    const int r4 = align4(r);
    float4 v = load4_guard<VEC>(sp + (h * RAE_SPD_NQ) * r4, i, r, ok);
#pragma unroll
    for (int q = 1; q < RAE_SPD_NQ; ++q) {
        const float4 u = load4_guard<VEC>(sp + (h * RAE_SPD_NQ + q) * r4, i, r, ok);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    return v;
}
__device__ __forceinline__ float sps_rowsum(const float* sp, int h, int i, int r4) {
    float v = sp[(h * RAE_SPD_NQ) * r4 + i];
#pragma unroll
    for (int q = 1; q < RAE_SPD_NQ; ++q) v += sp[(h * RAE_SPD_NQ + q) * r4 + i];
    return v;
}

// k_sp_ctdw: tile (example, k) of dP.  A = dw (rows b, K = i: one float4 per lane per chunk,
// assembled as it loads: dl A[e1] + N1 / dr A[e1] + N2, N_h the sum of the side's pieces), B = C
// (K = i rows, columns k: four strided scalars per lane); K runs over C1's then C2's i.  Besides
// dS the tile stores, for its 16 examples and the embedding columns i = 16 kt + (0..15)
// (+ 16 nkt q), dw1, dw2 (what the update's dense tiles read) and G1 = dl V1 + dr V2 (or dl, dr
// for the wire record), and tile kt = 0 the loss -- their loads issued before the GEMM, their
// stores after it.
template <bool VEC>
__device__ void sp_split_ctdw(const StepArgs& a, int task, float* red) {
    const int l = a.l, m = a.m, r = a.r, r4 = align4(r);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nkt = (m + 15) / 16;
    const int bt = task / nkt, kt = task - bt * nkt;
    const int li = lane & 15, g = lane >> 4;
    const int b = bt * 16 + li, k = kt * 16 + li;
    const bool bv = b < l, kv = k < m;
    const int oS = sps_os(r4);
    float* sdl = red + RAE_DW_BT * 4;                     // [16]: sd of the tile's examples
    // this lane's GEMM row (example b): dl, dr from both sides' sums
    const float* spb = a.sps + (int64_t)(bv ? b : 0) * a.spss;
    const float* scb = spb + oS;
    const float du1b = scb[SPS_DU1], du2b = scb[SPS_DU2];
    const float dlb = du1b + du2b + sps_side(scb, 1, 0);  // as sp_coefficients: d cost / d left
    const float drb = du1b + du2b + sps_side(scb, 0, 0);
    float lft = 0.f, rgt = 0.f, nv1 = 0.f, nv2 = 0.f;
    if (w == 0 && g == 0) {
        lft = scb[SPS_LEFT]; rgt = scb[SPS_RIGHT];
        nv1 = sps_side(scb, 0, 2); nv2 = sps_side(scb, 1, 2);
    }
    // the tile's stores of dw1, dw2, G1: pair (example eo, column ii) per thread
    const int pr = threadIdx.x & 255, eo = pr >> 4, ii = pr & 15;   // waves >= 4 repeat 0-3's
    const int bo_s = bt * 16 + eo;
    const bool sv = bo_s < l;
    const int bs = sv ? bo_s : 0;
    const float* sps_s = a.sps + (int64_t)bs * a.spss;
    const float* scs = sps_s + oS;
    const int is0 = kt * 16 + ii;
    const bool iv0 = sv && is0 < r;
    const int ic0 = iv0 ? is0 : 0;
    const float s_du1 = scs[SPS_DU1], s_du2 = scs[SPS_DU2];
    const float s_sdg1 = sps_side(scs, 0, 0), s_sdg2 = sps_side(scs, 1, 0);
    const float* vrow = a.vb + (int64_t)(a.rank * l + bs) * a.vbs;
    const float sa0 = sps_s[sps_oa(r4) + ic0];
    const float sn10 = sps_rowsum(sps_s, 0, ic0, r4), sn20 = sps_rowsum(sps_s, 1, ic0, r4);
    const float sv10 = vrow[a.vV1 + ic0], sv20 = vrow[a.vV2 + ic0];
    const bool lossl = kt == 0 && ii == 0 && sv;
    const float lbase = lossl ? scs[SPS_LBASE] : 0.f;
    const float sls = lossl ? sps_side(scs, 0, 1) + sps_side(scs, 1, 1) : 0.f;
    // the epilogue's operands (wave 0): P, z and sz of its four output rows
    const int kc = kv ? k : 0;
    float pk[4], zk[4], sz[4];
    if (w == 0) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int bo = min(bt * 16 + 4 * g + reg, l - 1);
            const float* rec = a.ex + (int64_t)(a.rank * l + bo) * a.lay.rec;
            pk[reg] = rec[a.lay.oP + kc];
            zk[reg] = rec[a.lay.odS + kc];
            sz[reg] = a.sps[(int64_t)bo * a.spss + oS + SPS_SZ];
        }
    }
    rae_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nci = (r + 15) / 16, nch = 2 * nci;
    for (int c0 = w; c0 < nch; c0 += RAE_DW_NW * RAE_SPG_UDW) {
        float4 x[RAE_SPG_UDW], y[RAE_SPG_UDW];
#pragma unroll
        for (int u = 0; u < RAE_SPG_UDW; ++u) {
            const int c = c0 + u * RAE_DW_NW;
            const bool cv = c < nch;
            const int which = c >= nci, i = (c - which * nci) * 16 + 4 * g;
            const float* Cm = which ? a.C2 : a.C1;
            const float4 nn = sps_rowsum4<VEC>(spb, which, i, r, bv && cv);
            const float4 ae = load4_guard<VEC>(spb + sps_oa(r4), i, r, bv && cv);
            const float dd = which ? drb : dlb;
            x[u] = make_float4(fmaf(dd, ae.x, nn.x), fmaf(dd, ae.y, nn.y),
                               fmaf(dd, ae.z, nn.z), fmaf(dd, ae.w, nn.w));
            // branch-free strided column loads (clamped row, select after)
            const bool o0 = cv && kv && i < r, o1 = cv && kv && i + 1 < r;
            const bool o2 = cv && kv && i + 2 < r, o3 = cv && kv && i + 3 < r;
            const float c0 = Cm[(int64_t)(o0 ? i : 0) * m + kc], c1 = Cm[(int64_t)(o1 ? i + 1 : 0) * m + kc];
            const float c2 = Cm[(int64_t)(o2 ? i + 2 : 0) * m + kc], c3 = Cm[(int64_t)(o3 ? i + 3 : 0) * m + kc];
            y[u].x = o0 ? c0 : 0.f;
            y[u].y = o1 ? c1 : 0.f;
            y[u].z = o2 ? c2 : 0.f;
            y[u].w = o3 ? c3 : 0.f;
        }
#pragma unroll
        for (int u = 0; u < RAE_SPG_UDW; ++u) acc = mfma4_f32(x[u], y[u], acc);
    }
    // dw1, dw2 and G1 (the same fmaf forms as the GEMM operand and as k_vrec)
    {
        const float dl = s_du1 + s_du2 + s_sdg2, dr = s_du1 + s_du2 + s_sdg1;
        float* dwr = a.dwb + (int64_t)(a.rank * l + bs) * a.dws;
        float* rec = a.ex + (int64_t)(a.rank * l + bs) * a.lay.rec;
        const bool st = threadIdx.x < 256;
        if (iv0 && st) {
            dwr[a.dw1o + is0] = fmaf(dl, sa0, sn10);
            dwr[a.dw2o + is0] = fmaf(dr, sa0, sn20);
            if (!a.lay.wire) rec[a.lay.oG1 + is0] = fmaf(dl, sv10, dr * sv20);
        }
        for (int is = is0 + 16 * nkt; st && sv && is < r; is += 16 * nkt) {    // r > 16 nkt only
            const float ae = sps_s[sps_oa(r4) + is];
            dwr[a.dw1o + is] = fmaf(dl, ae, sps_rowsum(sps_s, 0, is, r4));
            dwr[a.dw2o + is] = fmaf(dr, ae, sps_rowsum(sps_s, 1, is, r4));
            if (!a.lay.wire) rec[a.lay.oG1 + is] = fmaf(dl, vrow[a.vV1 + is], dr * vrow[a.vV2 + is]);
        }
        if (lossl && st) {
            rec[a.lay.oloss] = lbase + sls;
            if (a.lay.wire) {                             // k_vrec rebuilds G1 from (dl, dr)
                rec[a.lay.oAux + 0] = dl;
                rec[a.lay.oAux + 1] = dr;
            }
        }
    }
    if (w == 0 && g == 0) sdl[li] = fmaf(dlb, lft, nv1) + fmaf(drb, rgt, nv2);
    float o[4];
    sp_gemm_combine<RAE_DW_NW>(acc, red, lane, w, o);     // its barrier also publishes sdl
    if (w != 0) return;
    // epilogue: dS_bk = P_bk ((dP_bk - sd_b) + ce (z_bk - sz_b))   (softmax_backward's centred
    // form)
    const float ce = 2.f * a.alpha * a.invD;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {                   // D[b = 4g + reg][k = li]
        const int bo = bt * 16 + 4 * g + reg;
        if (bo < l && kv) {
            float* rec = a.ex + (int64_t)(a.rank * l + bo) * a.lay.rec;
            rec[a.lay.odS + k] = pk[reg] * ((o[reg] - sdl[4 * g + reg]) + ce * (zk[reg] - sz[reg]));
        }
    }
}

// k_sp_dec, piece q of side h of example bl: the A rows of e1 and of the piece's negatives of
// that side by LDS-DMA, the dots <V1, A[e1]>, <V2, A[e1]> and <V_h, A[neg_h,t]>, the piece's
// coefficients (its record entries written here), its weighted row sum N = sum_t dg_t A[neg_h,t]
// and <N, V_h>; piece 0 of side 0 also the positive scores' terms and a copy of A[e1].  The
// assembly dw = d A[e1] + N waits for every piece: k_sp_ctdw.
// phase stamps (diagnostic builds): piece 0 of each example, at the example's slot
#ifdef RAE_STAMPS
#define SPD_STAMP(slot)                                                                     \
    do {                                                                                    \
        if (a.stamps && threadIdx.x == 0 && pc == 0)                                        \
            a.stamps[(size_t)bl * 16 + (slot)] = __builtin_amdgcn_s_memrealtime();          \
    } while (0)
#else
#define SPD_STAMP(slot) do { } while (0)
#endif
template <bool V4>
__device__ void sp_split_dec(const StepArgs& a, int64_t g, int bl, int pc, char* smem) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int r = a.r, s = a.s, r4 = align4(r), rv = r / VW, r4v = r4 / VW;
    const int h = pc / RAE_SPD_NQ, q = pc - h * RAE_SPD_NQ;
    const int nsp = spd_neg_per_piece(s), t0 = q * nsp;
    const int nt = max(0, min(s - t0, nsp));                  // this piece's negatives
    const int s4 = align4(nsp + 2), NR = 1 + nt;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float* p = reinterpret_cast<float*>(smem);
    float* sV1 = p; p += r4;
    float* sV2 = p; p += r4;
    float* srows = p; p += (1 + nsp) * r4;
    float* sdots = p; p += s4;            // [0] left, [1] right, [2 + u] negative t0 + u
    float* sAb = p; p += s4;              // [0] e1, [1] e2, [2 + u] negative t0 + u
    float* scf = p; p += s4;              // coefficient of negative t0 + u
    int* sid = reinterpret_cast<int*>(p); p += s4;
    float* spart = p; p += 8 * r4;
    float* sred = p;
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    float* sp = a.sps + (int64_t)bl * a.spss;
    float* scl = sp + sps_os(r4);
    const bool lead = pc == 0;                                // the positive terms, A[e1]
    SPD_STAMP(0);
    if (threadIdx.x < nt + 2) {
        const int j = threadIdx.x;
        const int* src = j == 0 ? a.args1 + ex : j == 1 ? a.args2 + ex
                       : (h ? a.neg2 : a.neg1) + (int64_t)(t0 + j - 2) * a.neg_stride + col;
        sid[j] = *src;
    }
    const float H = (lead && threadIdx.x == 0) ? rec[a.lay.oloss] : 0.f;
    __syncthreads();
    SPD_STAMP(1);
    if (threadIdx.x < nt + 2) sAb[threadIdx.x] = a.Ab[sid[threadIdx.x]];
    {   // rho 0: A[e1]; rho >= 1: negative t0 + rho - 1 (id slot rho + 1)
        const int nchunk = (rv + 63) / 64;
        for (int t = w; t < NR * nchunk; t += RAE_FNW) {
            const int rho = t / nchunk, ch = t - rho * nchunk;
            const int c = ch * 64 + lane;
            float* dst = srows + rho * r4 + ch * 64 * VW;
            if (c < rv) {
                const float* src = a.A + (int64_t)sid[rho ? rho + 1 : 0] * r + (int64_t)c * VW;
                if constexpr (V4)
                    __builtin_amdgcn_global_load_lds((rae_glob_void*)src, (rae_lds_void*)dst, 16, 0, 0);
                else
                    __builtin_amdgcn_global_load_lds((rae_glob_void*)src, (rae_lds_void*)dst, 4, 0, 0);
            }
        }
    }
    const float* vrow = a.vb + (int64_t)bg * a.vbs;          // k_sp_cp's V1, V2
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        sV1[i] = vrow[a.vV1 + i];
        sV2[i] = vrow[a.vV2 + i];
    }
    __syncthreads();                                          // the A-row DMA has landed
    SPD_STAMP(2);
    {   // dots, 16 lanes each (sp_dots' arithmetic): t = 0 left, 1 right, 2 + u negative
        const VT* Rv = reinterpret_cast<const VT*>(srows);
        const VT* W1 = reinterpret_cast<const VT*>(sV1);
        const VT* W2 = reinterpret_cast<const VT*>(sV2);
        const VT* Wh = h ? W2 : W1;
        const int ndot = nt + 2;
        for (int base = 0; base < ndot * 16; base += RAE_FBT) {
            const int idx = base + threadIdx.x, t = idx >> 4, qq = idx & 15;
            float d = 0.f;
            if (t < ndot) {
                const VT* wv = t == 0 ? W1 : (t == 1 ? W2 : Wh);
                const VT* x = Rv + (t < 2 ? 0 : t - 1) * r4v;
                for (int c = qq; c < rv; c += 16) d += vdot(x[c], wv[c]);
            }
            d = group16_sum(d);
            if (t < ndot && qq == 0) sdots[t] = d;
        }
    }
    __syncthreads();
    SPD_STAMP(3);
    if (w == 0) {   // the piece's coefficients (sp_coefficients' arithmetic), one wave
        const float left = sdots[0], right = sdots[1], oth = h ? left : right;
        float sdg = 0.f, sls = 0.f;
        for (int u = lane; u < nt; u += RAE_WAVE) {
            const float gg = sdots[2 + u] + oth + sAb[2 + u];
            float sg, spl;
            sigmoid_softplus(gg, sg, spl);
            const float dg = sg * a.invD;
            scf[u] = dg;
            const int j = 2 + h * s + t0 + u;
            rec[a.lay.ocoef + 2 * j] = dg;
            rec[a.lay.ocoef + 2 * j + 1] = dg;
            sdg += dg;
            sls -= spl;                                       // log sigmoid(-g) = -softplus(g)
        }
        sdg = wave_sum(sdg);
        sls = wave_sum(sls);
        if (lane == 0) {
            scl[SPS_PIECE + 3 * pc + 0] = sdg;
            scl[SPS_PIECE + 3 * pc + 1] = sls;
            if (lead) {
                const float one = left + right;
                const float u1 = one + sAb[0], u2 = one + sAb[1];
                float su1, pu1, su2, pu2;                     // sigmoid(-u), softplus(-u)
                sigmoid_softplus(-u1, su1, pu1);
                sigmoid_softplus(-u2, su2, pu2);
                const float du1 = -su1 * a.invD, du2 = -su2 * a.invD;
                scl[SPS_LEFT] = left;
                scl[SPS_RIGHT] = right;
                scl[SPS_DU1] = du1;
                scl[SPS_DU2] = du2;
                scl[SPS_LBASE] = -pu1 - pu2 + 2.f * H;        // log sigmoid(u) = -softplus(-u)
                rec[a.lay.ocoef + 0] = 1.f;                   // e1: left / right carry it
                rec[a.lay.ocoef + 1] = du1;
                rec[a.lay.ocoef + 2] = 0.f;
                rec[a.lay.ocoef + 3] = du2;
            }
        }
    }
    __syncthreads();
    SPD_STAMP(4);
    // N = sum_t dg_t A[neg_h,t]: thread owns (vector column, row group), groups in fixed order
    const int ngrp = RAE_FBT / rv > 8 ? 8 : (RAE_FBT / rv > 0 ? RAE_FBT / rv : 1);
    {
        const int grp = threadIdx.x / rv, c = threadIdx.x - grp * rv;
        if (grp < ngrp && rv <= RAE_FBT) {
            const VT* R = reinterpret_cast<const VT*>(srows);
            VT v;
            vzero(v);
            for (int u = grp; u < nt; u += ngrp) vfma(v, scf[u], R[(1 + u) * r4v + c]);
            reinterpret_cast<VT*>(spart)[grp * rv + c] = v;
        }
    }
    __syncthreads();
    SPD_STAMP(5);
    const float* sVh = h ? sV2 : sV1;
    float x1 = 0.f;
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        float v = 0.f;
        for (int gg = 0; gg < ngrp; ++gg) v += spart[gg * r + i];
        sp[pc * r4 + i] = v;
        x1 += v * sVh[i];
        if (lead) sp[sps_oa(r4) + i] = srows[i];              // A[e1] for the assembly
    }
    const float nv = block_sum<RAE_FBT>(x1, sred);
    if (threadIdx.x == 0) scl[SPS_PIECE + 3 * pc + 2] = nv;
    SPD_STAMP(6);
    SPD_STAMP(7);
}

}  // namespace rae
