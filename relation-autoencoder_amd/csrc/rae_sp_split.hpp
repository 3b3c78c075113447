// Split SP forward for large runtime shapes (C4: r x m = 90 k floats per decoder matrix).
//
// The fused example kernel (rae_sp.hpp sp_example) streams C1 and C2 through every example's
// workgroup twice (C.P, then C^T.dw): 1.4 MB per example at C4, so the forward is bound by
// each CU's fill rate from L2.  Here the two matrix products run once for the rank's whole
// batch as fp32-MFMA GEMMs, and the per-example work is split around them:
//   k_sp_enc   per example : S = X.W + Wb, P = softmax(S), H          -> record P; z, H parked
//   k_sp_cp    GEMM        : V1 = P C1^T, V2 = P C2^T  (l x r, K = m)  -> record V1, V2
//   k_sp_dec   per example : A rows, dots, scores, loss, coefficients, dw1, dw2, G1
//   k_sp_ctdw  GEMM        : dP = dw1 C1 + dw2 C2      (l x m, K = 2r), and in its epilogue the
//                            centred softmax backward, element-wise    -> record dS
// The softmax backward's two sums per example come from k_sp_enc / k_sp_dec, not from dP:
// sum_k P_k dP_k = <dw1, C1.P> + <dw2, C2.P> = <dw1, V1> + <dw2, V2> (V = k_sp_cp's vectors) and
// sum_k P_k z_k -- so dS_bk = P_bk ((dP_bk - sd_b) + ce (z_bk - sz_b)) needs nothing outside the
// tile (round 5: the fifth launch, k_sp_fin, is gone; C4 forward 36 -> ~32 us).
// Same arithmetic as sp_example (SelectionalPreferences.py:30-51, RelationClassifier.py:35-36,
// OieModel.py:81); only the fp32 summation order of the two products differs.  Until k_sp_ctdw
// the record's dS slot holds z = S - max S and, until k_sp_dec, its loss slot holds H.
#pragma once
#include "rae_sp.hpp"

namespace rae {

typedef float rae_f32x4 __attribute__((ext_vector_type(4)));

template <bool V4>
__device__ void sp_split_enc(const StepArgs& a, int64_t g, int bl, char* smem) {
    const DynDims Dm(a);
    const int m = Dm.m;
    ExampleSmem S = carve_example_smem(smem, 0, m, Dm.r, 0);      // no A rows here
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    load_desc(a, Dm, g, bl, S, false);
    __syncthreads();
    CCache<V4, DynDims> cc_;                                       // unused: no C here
    encoder_forward<V4, V4, false>(a, Dm, S, 0, 1, cc_, true);
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    for (int k = threadIdx.x; k < m; k += RAE_FBT) {
        rec[a.lay.oP + k] = S.sP[k];
        rec[a.lay.odS + k] = S.sZ[k];
    }
    if (threadIdx.x == 0) rec[a.lay.oloss] = S.sred[40];
    if (threadIdx.x < RAE_WAVE) {                // sz = sum_k P_k z_k for k_sp_ctdw's epilogue
        float x = 0.f;
        for (int k = threadIdx.x; k < m; k += RAE_WAVE) x += S.sP[k] * S.sZ[k];
        x = wave_sum(x);
        if (threadIdx.x == 0) a.dPs[2 * bl + 1] = x;
    }
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

// The two GEMMs: one 4-wave workgroup per 16 x 16 output tile; wave w takes the K chunks
// c = w, w + 4, ... (16 deep each), four chunks' loads issued before their MFMAs, and the
// four waves' accumulators are combined in LDS in wave order (deterministic).
#define RAE_SPG_U 4
__device__ __forceinline__ void sp_gemm_combine(rae_f32x4 acc, float* red, int lane, int w,
                                                float out[4]) {
    float4* r4 = reinterpret_cast<float4*>(red);
    r4[w * 64 + lane] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    if (w == 0) {
        float4 t = r4[lane];
#pragma unroll
        for (int ww = 1; ww < RAE_NWAVE; ++ww) {
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
    for (int c0 = w; c0 < nch; c0 += RAE_NWAVE * RAE_SPG_U) {
        float4 x[RAE_SPG_U], y[RAE_SPG_U];
#pragma unroll
        for (int u = 0; u < RAE_SPG_U; ++u) {
            const int k = (c0 + u * RAE_NWAVE) * 16 + 4 * g;     // >= m past the last chunk
            x[u] = load4_guard<VEC>(Pr, k, m, bv);
            y[u] = load4_guard<VEC>(Cr, k, m, iv);
        }
#pragma unroll
        for (int u = 0; u < RAE_SPG_U; ++u) acc = mfma4_f32(x[u], y[u], acc);
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

// k_sp_ctdw: tile (example, k) of dP.  A = dw (rows b, K = i: one float4 per lane per chunk),
// B = C (K = i rows, columns k: four strided scalars per lane); K runs over C1's then C2's i.
template <bool VEC>
__device__ void sp_split_ctdw(const StepArgs& a, int task, float* red) {
    const int l = a.l, m = a.m, r = a.r;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nkt = (m + 15) / 16;
    const int bt = task / nkt, kt = task - bt * nkt;
    const int li = lane & 15, g = lane >> 4;
    const int b = bt * 16 + li, k = kt * 16 + li;
    const bool bv = b < l, kv = k < m;
    const float* dwr = a.dwb + (int64_t)(a.rank * l + (bv ? b : 0)) * a.dws;
    const int kc = kv ? k : 0;
    // the epilogue's operands (wave 0): P, z and the example's two sums of its four output rows,
    // loaded before the GEMM so they are not a dependent round trip after it
    float pk[4], zk[4], sd[4], sz[4];
    if (w == 0) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int bo = min(bt * 16 + 4 * g + reg, l - 1);
            const float* rec = a.ex + (int64_t)(a.rank * l + bo) * a.lay.rec;
            pk[reg] = rec[a.lay.oP + kc];
            zk[reg] = rec[a.lay.odS + kc];
            sd[reg] = a.dPs[2 * bo];
            sz[reg] = a.dPs[2 * bo + 1];
        }
    }
    rae_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nci = (r + 15) / 16, nch = 2 * nci;
    for (int c0 = w; c0 < nch; c0 += RAE_NWAVE * RAE_SPG_U) {
        float4 x[RAE_SPG_U], y[RAE_SPG_U];
#pragma unroll
        for (int u = 0; u < RAE_SPG_U; ++u) {
            const int c = c0 + u * RAE_NWAVE;
            const bool cv = c < nch;
            const int which = c >= nci, i = (c - which * nci) * 16 + 4 * g;
            const float* Dw = dwr + (which ? a.dw2o : a.dw1o);
            const float* Cm = which ? a.C2 : a.C1;
            x[u] = load4_guard<VEC>(Dw, i, r, bv && cv);
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
        for (int u = 0; u < RAE_SPG_U; ++u) acc = mfma4_f32(x[u], y[u], acc);
    }
    float o[4];
    sp_gemm_combine(acc, red, lane, w, o);
    if (w != 0) return;
    // epilogue: dS_bk = P_bk ((dP_bk - sd_b) + ce (z_bk - sz_b))   (softmax_backward's centred
    // form; sd, sz per example from k_sp_dec)
    const float ce = 2.f * a.alpha * a.invD;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {                   // D[b = 4g + reg][k = li]
        const int bo = bt * 16 + 4 * g + reg;
        if (bo < l && kv) {
            float* rec = a.ex + (int64_t)(a.rank * l + bo) * a.lay.rec;
            rec[a.lay.odS + k] = pk[reg] * ((o[reg] - sd[reg]) + ce * (zk[reg] - sz[reg]));
        }
    }
}

template <bool V4>
__device__ void sp_split_dec(const StepArgs& a, int64_t g, int bl, char* smem) {
    const DynDims Dm(a);
    const int m = Dm.m, r = Dm.r, s = Dm.s, NR = 1 + 2 * s, NJ = 2 + 2 * s;
    ExampleSmem S = carve_example_smem(smem, 0, m, r, s);
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    RAE_STAMP(a, 0);
    load_ids(a, Dm, ex, col, S);
    const float H = rec[a.lay.oloss];
    __syncthreads();
    RAE_STAMP(a, 1);
    if (threadIdx.x < NJ) S.sAbv[threadIdx.x] = a.Ab[S.sids[threadIdx.x]];
    gather_rows_dma<V4>(a, Dm, S, NR, 1);
    const float* vrow = a.vb + (int64_t)bg * a.vbs;          // k_sp_cp's V1, V2
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        S.swC1[i] = vrow[a.vV1 + i];
        S.swC2[i] = vrow[a.vV2 + i];
    }
    __syncthreads();                                      // the A-row DMA has landed
    RAE_STAMP(a, 2);
    sp_dots<V4>(Dm, S);
    __syncthreads();
    RAE_STAMP(a, 3);
    sp_coefficients(a, Dm, S, H);
    __syncthreads();
    RAE_STAMP(a, 4);
    sp_weighted_rows<V4>(Dm, S);
    __syncthreads();
    RAE_STAMP(a, 5);
    const float dl = S.scoef[0], dr = S.scoef[1];
    float* dwr = a.dwb + (int64_t)bg * a.dws;
    for (int i = threadIdx.x; i < r; i += RAE_FBT) {
        dwr[a.dw1o + i] = S.sdw1[i];
        dwr[a.dw2o + i] = S.sdw2[i];
        // A[e1]'s vector, one explicit fma (k_vrec forms it the same way: bit-identical)
        if (!a.lay.wire) rec[a.lay.oG1 + i] = fmaf(dl, S.swC1[i], dr * S.swC2[i]);
    }
    if (a.lay.wire && threadIdx.x == 0) {                 // k_vrec rebuilds G1 from (dl, dr)
        rec[a.lay.oAux + 0] = dl;
        rec[a.lay.oAux + 1] = dr;
    }
    for (int j = threadIdx.x; j < NJ; j += RAE_FBT) {
        const float* c = S.scoef + 3 * j;
        const float cj = j == 0 ? 1.f : (j == 1 ? 0.f : (j < 2 + s ? c[0] : c[1]));
        rec[a.lay.ocoef + 2 * j] = cj;
        rec[a.lay.ocoef + 2 * j + 1] = c[2];
    }
    if (threadIdx.x == 0) rec[a.lay.oloss] = S.sred[32];
    // the softmax backward's sum for k_sp_ctdw's epilogue: sd = sum_k P_k dP_k
    // = <dw1, V1> + <dw2, V2> (k_sp_enc left sz = sum_k P_k z_k)
    float x1 = 0.f;
    for (int i = threadIdx.x; i < r; i += RAE_FBT) x1 += S.sdw1[i] * S.swC1[i] + S.sdw2[i] * S.swC2[i];
    const float sd = block_sum<RAE_FBT>(x1, S.sred + 48);
    if (threadIdx.x == 0) a.dPs[2 * bl] = sd;
    RAE_STAMP(a, 6);
    RAE_STAMP(a, 7);
}

}  // namespace rae
