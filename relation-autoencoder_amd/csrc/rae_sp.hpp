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
// Output: the exchange record (rae_step.hpp); nothing is scattered here -- the row
// gradients are formed deterministically in the update kernel from these records.
//
// The step is ~100 examples, so one example's dependent memory round trips and its
// instruction issue ARE the kernel time.  Hence: dimensions are compile-time for the
// BASELINE shapes (FixDims; DynDims is the runtime-shape fallback), C1/C2 are held in
// registers and serve both matvecs, the A rows arrive by LDS-DMA while the W rows load,
// softmax / coefficient work runs in one wave without barriers, and every cross-lane
// reduction is DPP / permlane (VALU), not LDS.
#pragma once
#include "rae_common.hpp"
#include "rae_step.hpp"

namespace rae {

#define RAE_FNW (RAE_FBT / RAE_WAVE)     // waves per forward workgroup
#define RAE_NG (RAE_FBT / 16)            // 16-lane groups per forward workgroup
#ifndef RAE_CEARLY
#define RAE_CEARLY 0   // measured: C loads first delay the id chain (vmcnt is in order)
#endif

// ---- compile-time or runtime shapes ------------------------------------------------------
struct DynDims {
    int m, r, s;
    __device__ explicit DynDims(const StepArgs& a) : m(a.m), r(a.r), s(a.s) {}
    static constexpr bool fixed = false;
};
template <int M, int R, int S>
struct FixDims {
    static constexpr int m = M, r = R, s = S;
    __device__ explicit FixDims(const StepArgs&) {}
    static constexpr bool fixed = true;
};

// compile-time extents (0 for runtime shapes)
template <class D> struct DimT { static constexpr int m = 0, r = 0; };
template <int M, int R, int S> struct DimT<FixDims<M, R, S>> { static constexpr int m = M, r = R; };

struct ExampleSmem {
    float *sP, *sZ, *sdP, *swC1, *swC2, *sdw1, *sdw2, *srows, *sdots, *sAbv, *scoef,
        *sred, *spart, *sfval, *sX, *sY, *sM;
    int *sfidx, *sids, *sint;
};

// P / logP / dP regions are padded to a multiple of 64 vectors so the register-cache
// matvecs may read past m (the padding holds zeros)
__host__ __device__ inline int pad_m(int m) { return ((m + 255) / 256) * 256; }

__host__ __device__ inline int example_smem_floats(int dec, int m, int r, int s) {
    const int mp = pad_m(m), r4 = align4(r), NJ = 2 + 2 * s, NJ4 = align4(NJ);
    const int NR = (dec == 0) ? 1 + 2 * s : 2 + 2 * s;
    int partf = (RAE_FNW * mp > RAE_FBT * 4) ? RAE_FNW * mp : RAE_FBT * 4;
    if (16 * r4 > partf) partf = 16 * r4;
    int f = 3 * mp + 4 * r4 + NR * r4 + 2 * NJ4 + align4(3 * NJ) + 64 + partf +
            2 * RAE_FBT + NJ4 + 16;
    if (dec != 0) f += 3 * r4 + 4 * r4;
    return f;
}

__device__ inline ExampleSmem carve_example_smem(char* smem, int dec, int m, int r, int s) {
    ExampleSmem S;
    const int mp = pad_m(m), r4 = align4(r), NJ = 2 + 2 * s, NJ4 = align4(NJ);
    const int NR = (dec == 0) ? 1 + 2 * s : 2 + 2 * s;
    int partf = (RAE_FNW * mp > RAE_FBT * 4) ? RAE_FNW * mp : RAE_FBT * 4;
    if (16 * r4 > partf) partf = 16 * r4;
    float* p = reinterpret_cast<float*>(smem);
    S.sP = p; p += mp;
    S.sZ = p; p += mp;            // shifted scores z = S - max S (encoder_forward)
    S.sdP = p; p += mp;
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

// ids of the NJ records (e1, e2, neg1[t], neg2[t]) and the feature range
template <class D>
__device__ __forceinline__ void load_ids(const StepArgs& a, const D& Dm, int64_t ex, int64_t col,
                                         ExampleSmem& S) {
    const int NJ = 2 + 2 * Dm.s;
    const int j = threadIdx.x;
    if (j < NJ) {
        const int* src = (j == 0) ? a.args1 + ex
                       : (j == 1) ? a.args2 + ex
                       : (j < 2 + Dm.s) ? a.neg1 + (int64_t)(j - 2) * a.neg_stride + col
                                        : a.neg2 + (int64_t)(j - 2 - Dm.s) * a.neg_stride + col;
        S.sids[j] = *src;
    }
    if (threadIdx.x == RAE_FBT - 1) {
        S.sint[0] = a.indptr[ex];
        S.sint[1] = a.indptr[ex + 1];
    }
}

// The example's descriptor (rae_index.hpp build_batch_desc, built with the row index): the NJ
// entity ids, the CSR start, the feature count and the first dcap feature ids in one coalesced
// read -- load_ids plus the encoder's feature-id read, one dependent round trip less before the
// W-row gather.  S.sint[0] = first CSR position, S.sint[2] = feature count.
template <class D>
__device__ __forceinline__ void load_desc(const StepArgs& a, const D& Dm, int64_t g, int bl,
                                          ExampleSmem& S, bool ids = true) {
    const int NJ = 2 + 2 * Dm.s;                     // ids = false: S has no room for them
    const int32_t* dsc = a.desc + ((g % a.index_window) * a.dnx + a.d0 + bl) * (int64_t)a.dstride;
    for (int t = threadIdx.x; t < a.dstride; t += RAE_FBT) {
        const int v = dsc[t];
        if (t == 0) S.sint[2] = v;
        else if (t == 1) S.sint[0] = v;
        else if (t < 2 + NJ) { if (ids) S.sids[t - 2] = v; }
        else if (t - 2 - NJ < a.dcap) S.sfidx[t - 2 - NJ] = v;
    }
}

// A-row gather straight into LDS with LDS-DMA (global_load_lds: no VGPR staging; the copy
// lands while the W rows load).  Row rho -> record j (SP skips e2: j = rho ? rho+1 : 0;
// bilinear j = rho).  One wave instruction moves 64 lanes x 16 B (V4) or 64 x 4 B; the LDS
// destination is the wave-uniform row base + lane*size.
typedef __attribute__((address_space(3))) void rae_lds_void;
typedef __attribute__((address_space(1))) void rae_glob_void;

template <bool V4, class D>
__device__ __forceinline__ void gather_rows_dma(const StepArgs& a, const D& Dm, ExampleSmem& S,
                                                int NR, int skip_e2, int w0 = 0,
                                                int nw = RAE_FNW) {
    constexpr int VW = V4 ? 4 : 1;
    const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) - w0;
    const int rv = Dm.r / VW, r4 = align4(Dm.r);
    const int nchunk = (rv + 63) / 64;
    for (int t = w; t < NR * nchunk; t += nw) {
        const int rho = t / nchunk, ch = t - rho * nchunk;
        const int j = (rho == 0) ? 0 : rho + skip_e2;
        const int c = ch * 64 + lane;
        float* dst = S.srows + rho * r4 + ch * 64 * VW;
        if (c < rv) {
            const float* src = a.A + (int64_t)S.sids[j] * Dm.r + (int64_t)c * VW;
            if constexpr (V4)
                __builtin_amdgcn_global_load_lds((rae_glob_void*)src, (rae_lds_void*)dst, 16, 0, 0);
            else
                __builtin_amdgcn_global_load_lds((rae_glob_void*)src, (rae_lds_void*)dst, 4, 0, 0);
        }
    }
}

// diagnostic knockouts of the C3 forward's data movement (variant builds only, wrong results:
// timing of the chain without the decoder-matrix ingest / W-row gather / A-row gather)
#ifndef RAE_KO_C
#define RAE_KO_C 0
#endif
#ifndef RAE_KO_W
#define RAE_KO_W 0
#endif
#ifndef RAE_KO_A
#define RAE_KO_A 0
#endif
#if (RAE_KO_C || RAE_KO_W || RAE_KO_A) && !defined(RAE_DIAG)
#error "RAE_KO_C / RAE_KO_W / RAE_KO_A are timing knockouts with wrong results: a diagnostic build (-DRAE_DIAG)"
#endif

// ---- decoder weight matrices C1, C2 (r, m) in registers ----------------------------------
// group gid (16 lanes) owns rows i = gid + NG*ra, lane q owns column vectors c = q + 16*cc.
// Fixed shapes that fit keep the whole pair resident for both matvecs; otherwise the
// matrices stream through the same registers chunk by chunk.
template <int VW_, class D>
struct CCacheW {
    typedef typename VecW<VW_>::T VT;
    static constexpr int VW = VW_;
    static constexpr int RA0 = D::fixed ? (DimT<D>::r + RAE_NG - 1) / RAE_NG : 7;
    static constexpr int CC0 = D::fixed ? (DimT<D>::m / VW + 15) / 16 : 2;
    static constexpr bool FITS = D::fixed && RA0 <= 7 && CC0 <= 2;
    static constexpr int RA = FITS ? RA0 : 7;
    static constexpr int CC = FITS ? CC0 : 2;
    VT c1[RA][CC], c2[RA][CC];

    // branch-free: out-of-range rows/columns load a clamped (valid) element; their
    // contributions are multiplied by zero-padded P / zeroed dw
    __device__ __forceinline__ void load(const StepArgs& a, const D& Dm, int r0, int c0) {
        const VT* C1v = reinterpret_cast<const VT*>(a.C1);
        const VT* C2v = reinterpret_cast<const VT*>(a.C2);
        const int mv = Dm.m / VW;
        const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
#pragma unroll
        for (int ra = 0; ra < RA; ++ra) {
#if RAE_KO_C     // diagnostic knockout (wrong results): every lane reads row 0 (L1-hot C)
            const int i = 0;
#else
            const int i = min(r0 + gid + RAE_NG * ra, Dm.r - 1);
#endif
#pragma unroll
            for (int cc = 0; cc < CC; ++cc) {
                const int c = min(c0 + q + 16 * cc, mv - 1);
                c1[ra][cc] = C1v[i * mv + c];
                c2[ra][cc] = C2v[i * mv + c];
            }
        }
    }
};
template <bool V4, class D> using CCache = CCacheW<V4 ? 4 : 1, D>;

// wC1 = C1.P, wC2 = C2.P  -> S.swC1, S.swC2
template <bool V4, class D>
__device__ __forceinline__ void sp_project(const StepArgs& a, const D& Dm, ExampleSmem& S,
                                           CCache<V4, D>& cc_) {
    typedef typename VecT<V4>::T VT;
    typedef CCache<V4, D> CC_;
    const int mv = Dm.m / CC_::VW;
    const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
    const VT* Pv = reinterpret_cast<const VT*>(S.sP);
    for (int r0 = 0; r0 < Dm.r; r0 += RAE_NG * CC_::RA) {
        float s1[CC_::RA], s2[CC_::RA];
#pragma unroll
        for (int ra = 0; ra < CC_::RA; ++ra) s1[ra] = s2[ra] = 0.f;
        for (int c0 = 0; c0 < mv; c0 += 16 * CC_::CC) {
            if (!CC_::FITS) cc_.load(a, Dm, r0, c0);
#pragma unroll
            for (int cc = 0; cc < CC_::CC; ++cc) {
                const VT p = Pv[c0 + q + 16 * cc];          // zero beyond m (padded)
#pragma unroll
                for (int ra = 0; ra < CC_::RA; ++ra) {
                    s1[ra] += vdot(cc_.c1[ra][cc], p);
                    s2[ra] += vdot(cc_.c2[ra][cc], p);
                }
            }
        }
#pragma unroll
        for (int ra = 0; ra < CC_::RA; ++ra) {
            const float t1 = group16_sum(s1[ra]);
            const float t2 = group16_sum(s2[ra]);
            const int i = r0 + gid + RAE_NG * ra;
            if (q == 0 && i < Dm.r) {
                S.swC1[i] = t1;
                S.swC2[i] = t2;
            }
        }
    }
}

// dP += C1^T.dw1 + C2^T.dw2 into S.sdP (which holds any other dP terms)
template <bool V4, class D>
__device__ __forceinline__ void sp_project_back(const StepArgs& a, const D& Dm, ExampleSmem& S,
                                                CCache<V4, D>& cc_) {
    typedef typename VecT<V4>::T VT;
    typedef CCache<V4, D> CC_;
    constexpr int VW = CC_::VW;
    const int mp = pad_m(Dm.m), mv = Dm.m / VW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int gid = threadIdx.x >> 4, q = threadIdx.x & 15;
    for (int c0 = 0; c0 < mv; c0 += 16 * CC_::CC) {
        VT acc[CC_::CC];
#pragma unroll
        for (int cc = 0; cc < CC_::CC; ++cc) vzero(acc[cc]);
        for (int r0 = 0; r0 < Dm.r; r0 += RAE_NG * CC_::RA) {
            if (!CC_::FITS) cc_.load(a, Dm, r0, c0);
#pragma unroll
            for (int ra = 0; ra < CC_::RA; ++ra) {
                const int i = r0 + gid + RAE_NG * ra;
                const float d1 = i < Dm.r ? S.sdw1[i] : 0.f;
                const float d2 = i < Dm.r ? S.sdw2[i] : 0.f;
#pragma unroll
                for (int cc = 0; cc < CC_::CC; ++cc) {
                    vfma(acc[cc], d1, cc_.c1[ra][cc]);
                    vfma(acc[cc], d2, cc_.c2[ra][cc]);
                }
            }
        }
        // reduce over the 4 lane groups of the wave (permlane swaps), then waves via LDS
#pragma unroll
        for (int cc = 0; cc < CC_::CC; ++cc) {
            float* v = reinterpret_cast<float*>(&acc[cc]);
#pragma unroll
            for (int e = 0; e < VW; ++e) {
                v[e] += __uint_as_float(xor16_u32(__float_as_uint(v[e])));
                v[e] += __uint_as_float(xor32_u32(__float_as_uint(v[e])));
            }
            if (lane < 16) reinterpret_cast<VT*>(S.spart + w * mp)[c0 + q + 16 * cc] = acc[cc];
        }
        __syncthreads();
        for (int k = threadIdx.x; k < Dm.m; k += RAE_FBT) {
            const int cv = k / VW;
            if (cv >= c0 && cv < c0 + 16 * CC_::CC) {
                float dp = 0.f;
#pragma unroll
                for (int ww = 0; ww < RAE_FNW; ++ww) dp += S.spart[ww * mp + k];
                S.sdP[k] += dp;
            }
        }
        __syncthreads();
    }
}

// S = X.W + Wb spread over all threads (slot = feature lane group), then, in wave 0 (no
// barriers) for m <= 512: softmax, entropy.  Issues the A-row LDS-DMA and the decoder
// register cache behind the W-row loads.  Leaves H (alpha-scaled) in S.sred[40] and the
// shifted scores z = S - max(S) in S.sZ (log P = z - lse; see softmax_backward).
#ifndef RAE_ENC_KF
#define RAE_ENC_KF 4
#endif
// encoder phase stamps (diagnostic builds, slots 10-13): only the split forward's k_sp_enc
// records them (RAE_ENC_STAMPS there), the fused paths keep those slots for their own
#if defined(RAE_STAMPS)
#define RAE_ESTAMP(a, slot) do { if (ESTAMP) RAE_STAMP(a, slot); } while (0)
#else
#define RAE_ESTAMP(a, slot) do { } while (0)
#endif
template <bool V4, bool V4R, bool LOADC, class D, class Cache, bool ESTAMP = false>
__device__ __forceinline__ void encoder_forward(const StepArgs& a, const D& Dm, ExampleSmem& S,
                                                int NR, int skip_e2, Cache& cc_,
                                                bool desc = false) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int m = Dm.m, mv = m / VW, mp = pad_m(m);
    // desc: ids and features came with the example's descriptor (load_desc)
    const int p0 = S.sint[0], p1 = desc ? p0 + S.sint[2] : S.sint[1];
    const bool have = desc && p1 - p0 <= a.dcap;     // the feature ids are in S.sfidx already
    const int nslot = RAE_FBT / mv > 0 ? RAE_FBT / mv : 1;
    const int slot = threadIdx.x / mv, c = threadIdx.x - slot * mv;
    const VT* Wv = reinterpret_cast<const VT*>(a.W);
    VT acc;
    vzero(acc);
    const int lane = threadIdx.x & 63;
    const bool w0 = threadIdx.x < RAE_WAVE;
    // S = the slots' partial sums + Wb: for m <= 128 wave 0 forms its (<= 2 per lane) entries
    // itself, right before the softmax (no barrier); larger m all threads, one entry each (wave
    // 0 alone measured slower at m = 300).  The bias entries are loaded now, so they are not a
    // dependent round trip behind the W rows' barrier.
    const bool wS = m <= 2 * RAE_WAVE;
    float wbk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int k = lane + RAE_WAVE * i;
        wbk[i] = (wS && w0 && k < m) ? a.Wb[k] : 0.f;
    }
    const float wb0 = (!wS && threadIdx.x < m) ? a.Wb[threadIdx.x] : 0.f;
    const bool vals = a.values != nullptr;
    bool issued = false;
    for (int pc = p0; pc < p1; pc += RAE_FBT) {
        const int nf = min(RAE_FBT, p1 - pc);
        // binary features whose ids came with the descriptor: nothing to stage, no barrier
        if (!have || vals) {
            if (threadIdx.x < nf) {
                if (!have) S.sfidx[threadIdx.x] = a.indices[pc + threadIdx.x];
                S.sfval[threadIdx.x] = vals ? a.values[pc + threadIdx.x] : 1.f;
            }
            __syncthreads();
        }
        RAE_ESTAMP(a, 10);
        if (!issued) gather_rows_dma<V4R>(a, Dm, S, NR, skip_e2);
        if (slot < nslot) {
            // RAE_ENC_KF rows' loads in flight per round (the feature order of the sum is kept):
            // W is a random-row gather from HBM, and one dependent load per feature had put
            // nf / nslot full round trips on the chain (C4: m = 300, 6 slots, ~14 features)
            for (int cc = c; cc < mv; cc += RAE_FBT)          // mv > RAE_FBT only for huge m
                for (int f0 = slot; f0 < nf; f0 += nslot * RAE_ENC_KF) {
                    VT wv[RAE_ENC_KF];
                    float fv[RAE_ENC_KF];
#pragma unroll
                    for (int u = 0; u < RAE_ENC_KF; ++u) {
                        const int f = f0 + u * nslot;
                        const bool ok = f < nf;
                        wv[u] = Wv[(int64_t)S.sfidx[ok ? f : f0] * mv + cc];
                        fv[u] = ok ? (vals ? S.sfval[f] : 1.f) : 0.f;
                    }
#pragma unroll
                    for (int u = 0; u < RAE_ENC_KF; ++u)
                        if (f0 + u * nslot < nf) vfma(acc, fv[u], wv[u]);
                }
        }
        if (LOADC && !issued) cc_.load(a, Dm, 0, 0);         // behind the W-row loads
        issued = true;
        if (pc + RAE_FBT < p1) __syncthreads();             // the next chunk restages
    }
    if (!issued) {
        gather_rows_dma<V4R>(a, Dm, S, NR, skip_e2);
        if (LOADC) cc_.load(a, Dm, 0, 0);
    }
    VT* part = reinterpret_cast<VT*>(S.spart);
    if (slot < nslot && mv <= RAE_FBT) part[slot * mv + c] = acc;
    __syncthreads();
    RAE_ESTAMP(a, 11);
    float* sS = S.sdP;
    if (!wS) {
        for (int k = threadIdx.x; k < mp; k += RAE_FBT) {
            float v = 0.f;
            if (k < m) {
                for (int sl = 0; sl < nslot; ++sl) v += S.spart[sl * m + k];
                v += k == (int)threadIdx.x ? wb0 : a.Wb[k];
            }
            sS[k] = v;
        }
        __syncthreads();
    }
    RAE_ESTAMP(a, 12);
    if (m <= 8 * RAE_WAVE) {
        if (w0) {                                          // wave 0: no block barriers
            // S = the slots' partial sums + Wb (slot order) and the softmax, the lane's scores in
            // registers, one exp each (fast_softmax's form: P = e / sum e as e * (1 / sum e));
            // also sum_k P_k z_k (S.sred[41], the split forward's sz)
            float sv[8], ev[8];
            float mx = -INFINITY;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int k = lane + RAE_WAVE * i;
                float v = 0.f;
                if (k < m) {
                    if (wS) {
                        for (int sl = 0; sl < nslot; ++sl) v += S.spart[sl * m + k];
                        v += wbk[i < 2 ? i : 0];
                    } else {
                        v = sS[k];
                    }
                    mx = fmaxf(mx, v);
                }
                sv[i] = v;
            }
            mx = wave_max(mx);
            float se = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int k = lane + RAE_WAVE * i;
                ev[i] = k < m ? __expf(sv[i] - mx) : 0.f;
                se += ev[i];
            }
            se = wave_sum(se);
            const float inv = 1.f / se, lse = __logf(se);
            float hp = 0.f, zp = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int k = lane + RAE_WAVE * i;
                const float z = k < m ? sv[i] - mx : 0.f;
                const float p = ev[i] * inv;
                if (k < mp) {
                    S.sZ[k] = z;
                    S.sP[k] = p;
                }
                hp += p * (z - lse);
                zp += p * z;
            }
            hp = wave_sum(hp);
            zp = wave_sum(zp);
            if (lane == 0) {
                S.sred[40] = -a.alpha * hp;
                S.sred[41] = zp;
            }
        }
    } else {
        float mx = -INFINITY;
        for (int k = threadIdx.x; k < m; k += RAE_FBT) mx = fmaxf(mx, sS[k]);
        mx = block_max<RAE_FBT>(mx, S.sred);
        float se = 0.f;
        for (int k = threadIdx.x; k < m; k += RAE_FBT) se += __expf(sS[k] - mx);
        se = block_sum<RAE_FBT>(se, S.sred + 8);
        const float lse = __logf(se);
        float hp = 0.f;
        for (int k = threadIdx.x; k < mp; k += RAE_FBT) {
            float z = 0.f, p = 0.f;
            if (k < m) {
                z = sS[k] - mx;
                p = __expf(z) / se;
            }
            S.sZ[k] = z;
            S.sP[k] = p;
            hp += p * (z - lse);
        }
        hp = block_sum<RAE_FBT>(hp, S.sred + 16);
        if (threadIdx.x == 0) S.sred[40] = -a.alpha * hp;
    }
    __syncthreads();
    RAE_ESTAMP(a, 13);
}

// entropy term + softmax backward.  With d = the decoder's dCost/dP and the entropy's
// dCost/dP_k = ce (log P_k + 1), ce = 2 alpha / D (cost has -2H/D, dH/dP = -alpha(logP+1)):
//   dS_k = P_k (dP_k - sum_j P_j dP_j) = P_k ((d_k - sum_j P_j d_j) + ce (z_k - sum_j P_j z_j))
// with z = S - max S (log P - sum P log P is shift invariant).  The centred form avoids the
// cancellation of the large constant log P + 1 against its mean, which in fp32 costs ~1e-7
// relative to log m -- more than the whole signal when P is near uniform.  Wave 0 for
// m <= 512.
template <class D>
__device__ __forceinline__ void softmax_backward(const StepArgs& a, const D& Dm, ExampleSmem& S) {
    const int m = Dm.m;
    const float ce = 2.f * a.alpha * a.invD;
    const int lane = threadIdx.x & 63;
    if (m <= 8 * RAE_WAVE) {
        if (threadIdx.x < RAE_WAVE) {                  // the lane's entries in registers
            float pk[8], dk[8], zk[8];
            float sd = 0.f, sz = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int k = lane + RAE_WAVE * i;
                const bool in = k < m;
                pk[i] = in ? S.sP[k] : 0.f;
                dk[i] = in ? S.sdP[k] : 0.f;
                zk[i] = in ? S.sZ[k] : 0.f;
                sd += pk[i] * dk[i];
                sz += pk[i] * zk[i];
            }
            sd = wave_sum(sd);
            sz = wave_sum(sz);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int k = lane + RAE_WAVE * i;
                if (k < m) S.sdP[k] = pk[i] * ((dk[i] - sd) + ce * (zk[i] - sz));
            }
        }
    } else {
        float sd = 0.f, sz = 0.f;
        for (int k = threadIdx.x; k < m; k += RAE_FBT) {
            sd += S.sP[k] * S.sdP[k];
            sz += S.sP[k] * S.sZ[k];
        }
        sd = block_sum<RAE_FBT>(sd, S.sred + 24);
        sz = block_sum<RAE_FBT>(sz, S.sred + 48);
        for (int k = threadIdx.x; k < m; k += RAE_FBT)
            S.sdP[k] = S.sP[k] * ((S.sdP[k] - sd) + ce * (S.sZ[k] - sz));
    }
    __syncthreads();
}

// write the common part of the exchange record
// t0 / nt: the threads that write (thread t0 + u strides by nt); with_p: also P and dS
template <class D>
__device__ __forceinline__ void write_record(const StepArgs& a, const D& Dm, ExampleSmem& S,
                                             int bg, int t0 = 0, int nt = RAE_FBT,
                                             bool with_p = true) {
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    float* dwr = a.dwb + (int64_t)bg * a.dws;
    const int m = Dm.m, r = Dm.r, NJ = 2 + 2 * Dm.s;
    const int tid = (int)threadIdx.x - t0;
    if (with_p)
        for (int k = tid; k < m; k += nt) {
            rec[a.lay.oP + k] = S.sP[k];
            rec[a.lay.odS + k] = S.sdP[k];
        }
    const float dl = S.scoef[0], dr = S.scoef[1];
    for (int i = tid; i < r; i += nt) {
        const float w1 = S.swC1[i], w2 = S.swC2[i];
        dwr[a.dw1o + i] = S.sdw1[i];
        dwr[a.dw2o + i] = S.sdw2[i];
        if (!a.lay.wire) {                             // wire record: k_vrec rebuilds these
            rec[a.lay.oV1 + i] = w1;
            rec[a.lay.oV2 + i] = w2;
            rec[a.lay.oG1 + i] = dl * w1 + dr * w2;    // A[e1]: left and right both read it
        }
    }
    if (a.lay.wire && tid == 0) {
        rec[a.lay.oAux + 0] = dl;
        rec[a.lay.oAux + 1] = dr;
    }
    for (int j = tid; j < NJ; j += nt) {
        const float* c = S.scoef + 3 * j;
        const float cj = j == 0 ? 1.f : (j == 1 ? 0.f : (j < 2 + Dm.s ? c[0] : c[1]));
        rec[a.lay.ocoef + 2 * j] = cj;
        rec[a.lay.ocoef + 2 * j + 1] = c[2];
    }
    if (tid == 0) rec[a.lay.oloss] = S.sred[32];
}

// softmax backward and the record, overlapped (m <= 512): wave 0 computes dS from registers and
// stores P and dS straight into the record while waves 1.. write the rest of it
template <class D>
__device__ __forceinline__ void softmax_backward_record(const StepArgs& a, const D& Dm,
                                                        ExampleSmem& S, int bg) {
    const int m = Dm.m;
    if (m > 8 * RAE_WAVE) {
        softmax_backward(a, Dm, S);
        write_record(a, Dm, S, bg);
        return;
    }
    if (threadIdx.x >= RAE_WAVE) {
        write_record(a, Dm, S, bg, RAE_WAVE, RAE_FBT - RAE_WAVE, false);
        return;
    }
    const int lane = threadIdx.x;
    const float ce = 2.f * a.alpha * a.invD;
    float* rec = a.ex + (int64_t)bg * a.lay.rec;
    float pk[8], dk[8], zk[8];
    float sd = 0.f, sz = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {                      // softmax_backward's arithmetic
        const int k = lane + RAE_WAVE * i;
        const bool in = k < m;
        pk[i] = in ? S.sP[k] : 0.f;
        dk[i] = in ? S.sdP[k] : 0.f;
        zk[i] = in ? S.sZ[k] : 0.f;
        sd += pk[i] * dk[i];
        sz += pk[i] * zk[i];
    }
    sd = wave_sum(sd);
    sz = wave_sum(sz);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int k = lane + RAE_WAVE * i;
        if (k < m) {
            rec[a.lay.oP + k] = pk[i];
            rec[a.lay.odS + k] = pk[i] * ((dk[i] - sd) + ce * (zk[i] - sz));
        }
    }
}

// v1[i] = c_a * row0[i] + sum_t coef1_t * rowsA_t[i],  v2 likewise (sums in t order):
// thread owns (vector column, row group); groups combined in LDS in fixed order.
template <bool V4, class D>
__device__ __forceinline__ void sp_weighted_rows(const D& Dm, ExampleSmem& S) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int s = Dm.s, r4 = align4(Dm.r), rv = Dm.r / VW;
    const int ngrp = RAE_FBT / rv > 8 ? 8 : (RAE_FBT / rv > 0 ? RAE_FBT / rv : 1);
    const int grp = threadIdx.x / rv, c = threadIdx.x - grp * rv;
    VT* part = reinterpret_cast<VT*>(S.spart);                 // [2][ngrp][rv]
    if (grp < ngrp && rv <= RAE_FBT) {
        const VT* R = reinterpret_cast<const VT*>(S.srows);
        const int r4v = r4 / VW;
        VT v1, v2;
        vzero(v1);
        vzero(v2);
        if (grp == 0) {
            const VT a1 = R[c];
            vfma(v1, S.scoef[0], a1);
            vfma(v2, S.scoef[1], a1);
        }
        for (int t = grp; t < s; t += ngrp) {
            vfma(v1, S.scoef[3 * (2 + t)], R[(1 + t) * r4v + c]);
            vfma(v2, S.scoef[3 * (2 + s + t) + 1], R[(1 + s + t) * r4v + c]);
        }
        part[grp * rv + c] = v1;
        part[(ngrp + grp) * rv + c] = v2;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < Dm.r; i += RAE_FBT) {
        float v1 = 0.f, v2 = 0.f;
        for (int gg = 0; gg < ngrp; ++gg) {
            v1 += S.spart[gg * Dm.r + i];
            v2 += S.spart[(ngrp + gg) * Dm.r + i];
        }
        S.sdw1[i] = v1;
        S.sdw2[i] = v2;
    }
}

// dot products of the example's A rows with wC1 / wC2 (S.srows, S.swC1, S.swC2 -> S.sdots):
// 16 lanes per dot (strided columns, then one 16-lane DPP sum), every dot at once -- one
// wave_sum per row serialised ~13 reductions per wave at C4, one thread per dot serialised
// r LDS reads per thread at C2 (fp32 rows)
template <bool V4, class D>
__device__ __forceinline__ void sp_dots(const D& Dm, ExampleSmem& S) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int r = Dm.r, s = Dm.s, NR = 1 + 2 * s, r4 = align4(r);
    const int rv = r / VW, r4v = r4 / VW;
    const VT* Rv = reinterpret_cast<const VT*>(S.srows);
    const VT* W1 = reinterpret_cast<const VT*>(S.swC1);
    const VT* W2 = reinterpret_cast<const VT*>(S.swC2);
    const int ndot = NR + 1;
    for (int base = 0; base < ndot * 16; base += RAE_FBT) {     // uniform trip count
        const int idx = base + threadIdx.x, t = idx >> 4, q = idx & 15;
        float d = 0.f;
        if (t < ndot) {
            // t = 0: <wC1, A[e1]> (left); t = NR: <wC2, A[e1]> (right); else row t with wC1
            // (rows 1..s: neg1) or wC2 (rows s+1..2s: neg2)
            const int rho = t == NR ? 0 : t;
            const VT* wv = (t == NR || rho > s) ? W2 : W1;
            const VT* x = Rv + rho * r4v;
            for (int c = q; c < rv; c += 16) d += vdot(x[c], wv[c]);
        }
        d = group16_sum(d);
        if (t < ndot && q == 0) {
            if (t == 0) S.sdots[0] = d;             // left  = <wC1, A[e1]>
            else if (t == NR) S.sdots[1] = d;       // right = <wC2, A[e1]>
            else S.sdots[t + 1] = d;                // record j = rho + 1
        }
    }
}

// scores, loss, coefficients (wave 0): S.sdots, S.sAbv, H -> S.scoef, loss in S.sred[32]
template <class D>
__device__ __forceinline__ void sp_coefficients(const StepArgs& a, const D& Dm, ExampleSmem& S,
                                                float H) {
    const int s = Dm.s;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (w == 0) {
        const float left = S.sdots[0], right = S.sdots[1];
        float sdg1 = 0.f, sdg2 = 0.f, sls = 0.f;
        for (int t = lane; t < s; t += RAE_WAVE) {
            const float g1 = S.sdots[2 + t] + right + S.sAbv[2 + t];
            const float g2 = S.sdots[2 + s + t] + left + S.sAbv[2 + s + t];
            // hardware transcendental forms (one exp per score; the fast path's): a single
            // wave runs this block, so the libm sequences were its whole 1.7 us at C4
            float sg1, sp1, sg2, sp2;
            sigmoid_softplus(g1, sg1, sp1);
            sigmoid_softplus(g2, sg2, sp2);
            const float dg1 = sg1 * a.invD;
            const float dg2 = sg2 * a.invD;
            float* c1 = S.scoef + 3 * (2 + t);
            float* c2 = S.scoef + 3 * (2 + s + t);
            c1[0] = dg1; c1[1] = 0.f; c1[2] = dg1;
            c2[0] = 0.f; c2[1] = dg2; c2[2] = dg2;
            sdg1 += dg1;
            sdg2 += dg2;
            sls -= sp1 + sp2;                   // log sigmoid(-g) = -softplus(g)
        }
        sdg1 = wave_sum(sdg1);
        sdg2 = wave_sum(sdg2);
        sls = wave_sum(sls);
        if (lane == 0) {
            const float one = left + right;
            const float u1 = one + S.sAbv[0], u2 = one + S.sAbv[1];
            float su1, pu1, su2, pu2;               // sigmoid(-u), softplus(-u)
            sigmoid_softplus(-u1, su1, pu1);
            sigmoid_softplus(-u2, su2, pu2);
            const float du1 = -su1 * a.invD;
            const float du2 = -su2 * a.invD;
            const float dl = du1 + du2 + sdg2;     // d cost / d left
            const float dr = du1 + du2 + sdg1;     // d cost / d right
            S.scoef[0] = dl; S.scoef[1] = dr; S.scoef[2] = du1;
            S.scoef[3] = 0.f; S.scoef[4] = 0.f; S.scoef[5] = du2;
            S.sred[32] = -pu1 - pu2 + 2.f * H + sls;   // log sigmoid(u) = -softplus(-u)
        }
    }
}

// sp_coefficients + sp_weighted_rows for s <= 32 and r-vectors of <= 64 columns, without their
// two barriers and LDS hand-offs (the fast path's form): every wave computes the scores'
// coefficients in registers (lanes t: neg1[t], lanes 32 + t: neg2[t]); wave 0 also leaves them
// in S.scoef / S.sred[32] for the record; waves 0 / 1 sum dw1 / dw2 one vector column per lane,
// the coefficients broadcast by readlane, in record order; the other waves clear S.sdP.  Ends
// with the block barrier.
template <bool VR, class D>
__device__ __forceinline__ void sp_coef_rows_regs(const StepArgs& a, const D& Dm, ExampleSmem& S,
                                                  float H) {
    typedef typename VecT<VR>::T VT;
    constexpr int VW = VR ? 4 : 1;
    const int s = Dm.s, r4v = align4(Dm.r) / VW, rv = Dm.r / VW, mp = pad_m(Dm.m);
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float left = S.sdots[0], right = S.sdots[1];
    const int tq = lane & 31;
    const bool hi = lane >= 32;
    float dg = 0.f, ls = 0.f;
    if (tq < s) {
        const int j = 2 + (hi ? s : 0) + tq;
        const float gg = S.sdots[j] + (hi ? left : right) + S.sAbv[j];
        float sg, spl;
        sigmoid_softplus(gg, sg, spl);
        dg = sg * a.invD;
        ls = -spl;                                     // log sigmoid(-g) = -softplus(g)
    }
    float hs = group16_sum(dg);
    hs += __uint_as_float(xor16_u32(__float_as_uint(hs)));
    const float other = __uint_as_float(xor32_u32(__float_as_uint(hs)));
    const float sdg1 = hi ? other : hs, sdg2 = hi ? hs : other;
    const float one = left + right;
    const float u1 = one + S.sAbv[0], u2 = one + S.sAbv[1];
    float su1, spu1, su2, spu2;                        // sigmoid(-u), softplus(-u)
    sigmoid_softplus(-u1, su1, spu1);
    sigmoid_softplus(-u2, su2, spu2);
    const float du1 = -su1 * a.invD, du2 = -su2 * a.invD;
    const float dl = du1 + du2 + sdg2;                 // d cost / d left
    const float dr = du1 + du2 + sdg1;                 // d cost / d right
    if (w < 2) {
        const VT* R = reinterpret_cast<const VT*>(S.srows);
        const float c0 = w == 0 ? dl : dr;
        const int off = w == 0 ? 0 : s;
        if (w == 0) {                                  // the record's coefficients and loss
            if (tq < s) {
                float* c = S.scoef + 3 * (2 + (hi ? s : 0) + tq);
                c[0] = hi ? 0.f : dg;
                c[1] = hi ? dg : 0.f;
                c[2] = dg;
            }
            const float sls = wave_sum(ls);
            if (lane == 0) {
                S.scoef[0] = dl; S.scoef[1] = dr; S.scoef[2] = du1;
                S.scoef[3] = 0.f; S.scoef[4] = 0.f; S.scoef[5] = du2;
                S.sred[32] = -spu1 - spu2 + 2.f * H + sls;
            }
        }
        // branch-free (lanes past the row work on column 0, not stored): every readlane runs
        // with the whole wave active -- a source lane outside EXEC has no defined value
        const int lc = lane < rv ? lane : 0;
        VT v;
        vzero(v);
        vfma(v, c0, R[lc]);
        for (int t = 0; t < s; ++t) {
            const float ct = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dg),
                                                                       (w == 0 ? 0 : 32) + t));
            vfma(v, ct, R[(1 + off + t) * r4v + lc]);
        }
        if (lane < rv) reinterpret_cast<VT*>(w == 0 ? S.sdw1 : S.sdw2)[lane] = v;
    } else {
        for (int k = threadIdx.x - 2 * RAE_WAVE; k < mp; k += RAE_FBT - 2 * RAE_WAVE) S.sdP[k] = 0.f;
    }
    __syncthreads();
}

// ---- the SP example path ---------------------------------------------------------------
#ifndef RAE_FWD_PFLAG
#define RAE_FWD_PFLAG 1      // fast path: P published by an LDS flag, not a block barrier
#endif
#ifndef RAE_FWD_CWAIT
#define RAE_FWD_CWAIT 1      // fast path: C loads last on every wave, C.P in load order
#endif
#ifndef RAE_FWD_CEARLY47
#define RAE_FWD_CEARLY47 0   // fast path: waves 4-7 issue their C share at kernel start
#endif
template <bool V4, class D>
__device__ void sp_example(const StepArgs& a, int64_t g, int bl, char* smem) {
    const D Dm(a);
    const int m = Dm.m, r = Dm.r, s = Dm.s, NR = 1 + 2 * s;
    // the r-vectors (A rows, V, dw) go four wide whenever r allows, independent of m (C2:
    // m = 30, r = 100)
    constexpr bool VR = V4 || (D::fixed && DimT<D>::r % 4 == 0);
    const int r4 = align4(r), mp = pad_m(m);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    ExampleSmem S = carve_example_smem(smem, 0, m, r, s);
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;

    RAE_STAMP(a, 0);
#ifdef RAE_STAMPS
    if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 16 + 14] = __builtin_amdgcn_s_memtime();
#endif
    CCache<V4, D> cc_;
#if RAE_CEARLY
    // the decoder matrices do not depend on the batch: their loads go out first and land
    // while the id -> feature -> W-row chain runs
    if (CCache<V4, D>::FITS) cc_.load(a, Dm, 0, 0);
    constexpr bool kLoadC = false;
#else
    constexpr bool kLoadC = CCache<V4, D>::FITS;
#endif
    load_desc(a, Dm, g, bl, S);
    __syncthreads();
    RAE_STAMP(a, 1);
    const int NJ = 2 + 2 * s;
    if (threadIdx.x < NJ) S.sAbv[threadIdx.x] = a.Ab[S.sids[threadIdx.x]];
    encoder_forward<V4, VR, kLoadC>(a, Dm, S, NR, 1, cc_, true);
    const float H = S.sred[40];
    RAE_STAMP(a, 2);
    sp_project<V4>(a, Dm, S, cc_);
    __syncthreads();
    RAE_STAMP(a, 3);

    sp_dots<VR>(Dm, S);
    __syncthreads();
    RAE_STAMP(a, 4);

    // scores, loss, coefficients (wave 0)
    if (s <= 32 && r / (VR ? 4 : 1) <= RAE_WAVE) {
        // coefficients in every wave's registers and dw1 / dw2 by waves 0 / 1 (one barrier)
        sp_coef_rows_regs<VR>(a, Dm, S, H);
        RAE_STAMP(a, 8);
    } else {
        sp_coefficients(a, Dm, S, H);
        __syncthreads();
        RAE_STAMP(a, 8);
        // dwC1 = dl*a1 + sum_t dg1_t n1_t ; dwC2 = dr*a1 + sum_t dg2_t n2_t
        sp_weighted_rows<VR>(Dm, S);
        for (int k = threadIdx.x; k < mp; k += RAE_FBT) S.sdP[k] = 0.f;
        __syncthreads();
    }
    RAE_STAMP(a, 5);
    sp_project_back<V4>(a, Dm, S, cc_);
    RAE_STAMP(a, 9);
    softmax_backward_record(a, Dm, S, bg);
    RAE_STAMP(a, 6);
    RAE_STAMP(a, 7);
#ifdef RAE_STAMPS
    if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 16 + 15] = __builtin_amdgcn_s_memtime();
#endif
}

// One 16-B-per-lane LDS-DMA (global_load_lds_dwordx4; M0 = the wave-uniform LDS row base) as
// inline asm: the compiler's wait-count pass treats every LDS access behind an LDS-DMA it can
// see as a possible alias and puts a vmcnt(0) -- every outstanding load -- in front of it, which
// in the fast path serialised the W-row partial sums, the P hand-off and C.P behind the whole
// 160 KB of decoder-matrix loads.  Issued before those loads, an LDS-DMA the pass cannot see
// only ever makes its counted waits wait for more (vmcnt retires in issue order); the rows are
// read after dma_visible_barrier (vmcnt(0) + barrier).
// M0 is a reserved register the compiler cannot take as a clobber: the asm saves it into a
// scratch SGPR and restores it behind the load (the instruction reads M0 at issue), so any M0
// value the compiler keeps live across the block -- e.g. for its own global_load_lds -- is
// unchanged.  tests/test_isa.py checks every LDS-DMA of the C3 forward in the code object.
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}
__device__ __forceinline__ void dma_row16(const float* gsrc, uint32_t lds) {
    uint32_t saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved) : "v"(gsrc), "s"(lds) : "memory");
}

// record stores of the fast path
template <class T>
__device__ __forceinline__ void rec_st(T* p, T v) { *p = v; }

// Wave 0 of a fast path, once the W-row partial sums of the NSL feature slots are in S.spart:
// S = X.W + Wb, softmax and entropy -- z = S - max S and P into S.sZ / S.sP (and pz / pp: the
// lane's entries k = lane + 64 i), H (alpha-scaled) into S.sred[40].
template <int m, int NSL, int NI>
__device__ __forceinline__ void fast_softmax(const StepArgs& a, ExampleSmem& S, const float (&wbk)[NI],
                                             int lane, float (&pz)[NI], float (&pp)[NI]) {
    float sv[NI];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int k = lane + RAE_WAVE * i;
        float v = 0.f;
        if (k < m) {
#pragma unroll
            for (int sl = 0; sl < NSL; ++sl) v += S.spart[sl * m + k];
            v += wbk[i];
            mx = fmaxf(mx, v);
        }
        sv[i] = v;
    }
    mx = wave_max(mx);
    float ev[NI];
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int k = lane + RAE_WAVE * i;
        ev[i] = k < m ? __expf(sv[i] - mx) : 0.f;
        se += ev[i];
    }
    se = wave_sum(se);
    const float inv = 1.f / se, lse = __logf(se);
    float hp = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int k = lane + RAE_WAVE * i;
        const float z = k < m ? sv[i] - mx : 0.f;
        const float p = ev[i] * inv;
        S.sZ[k] = z;
        S.sP[k] = p;
        pz[i] = z;
        pp[i] = p;
        hp += p * (z - lse);
    }
    hp = wave_sum(hp);
    if (lane == 0) S.sred[40] = -a.alpha * hp;
}

// ---- the SP example path for compile-time shapes (BASELINE configs) ---------------------
// Same arithmetic as sp_example, re-timed for a 100-example step where the kernel is a
// dependent chain: waves 0-3 run the critical chain (ids -> feature ids -> W rows -> S ->
// softmax) while waves 4-7 issue the A-row LDS-DMA and the Ab loads, and every wave
// then issues its share of the decoder-matrix loads.  No barrier drains vmcnt until the
// decoder matrices are needed (lds_barrier), so the ~200 KB of bulk loads per CU overlap
// the chain instead of sitting in front of it.  Softmax and the score coefficients use
// hardware exp/log/rcp; the coefficient work is spread over 2s lanes.
template <class D> struct FastSP { static constexpr int VM = 4; static constexpr bool ok = false; };
template <int M, int R, int S> struct FastSP<FixDims<M, R, S>> {
    // the m-vectors (W rows, C1 / C2 columns, P) four wide, or two wide for an even m that is
    // not a multiple of 4 (C2: m = 30, 120-B rows at 8-B alignment)
    static constexpr int VM = M % 4 == 0 ? 4 : 2;
    static constexpr bool ok = M % 2 == 0 && R % 4 == 0 && S <= 32 && M / VM <= 32 &&
                               R / 4 <= RAE_WAVE;
};
template <class D>
__device__ void sp_example_fast(const StepArgs& a, int64_t g, int bl, char* smem) {
    static_assert(FastSP<D>::ok, "fast SP path");
    constexpr int m = D::m, r = D::r, s = D::s, NR = 1 + 2 * s, NJ = 2 + 2 * s;
    constexpr int VM = FastSP<D>::VM;
    typedef typename VecW<VM>::T MT;
    typedef CCacheW<VM, D> CCF;
    constexpr int MV = m / VM, NSL = 256 / MV, KF = 3;
    constexpr int r4 = r, mp = ((m + 255) / 256) * 256;
    const D Dm(a);
    // wave index as a scalar: role branches are then uniform control flow (s_cbranch on an
    // SGPR), not exec-masked linearised code whose register reuse forces vmcnt(0) waits
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    ExampleSmem S = carve_example_smem(smem, 0, m, r, s);
    float* const arows = S.srows;
    const int bg = a.rank * a.l + bl;
    const int64_t ex = g * (int64_t)a.L + bg;
    const int64_t col = a.neg_mode ? ex : (int64_t)bg;

    RAE_STAMP(a, 0);
#ifdef RAE_STAMPS
    if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 16 + 14] = __builtin_amdgcn_s_memtime();
#endif
    CCF cc_;
#if RAE_FWD_CWAIT && RAE_FWD_CEARLY47
    // waves 4-7 have no load on the chain: their half of C goes out at once (the other half
    // follows the W rows of waves 0-3), so C's ingest starts ~1 us earlier
    if (w >= 4) cc_.load(a, Dm, 0, 0);
#endif
    // the example's descriptor (rae_index.hpp build_batch_desc): feature count, CSR start,
    // entity ids and feature ids in one coalesced read
    {
        const int32_t* dsc = a.desc + ((g % a.index_window) * a.dnx + a.d0 + bl) * (int64_t)a.dstride;
        if (tid < a.dstride) {
            const int v = dsc[tid];
            if (tid == 0) S.sint[1] = v;                          // nf
            else if (tid == 1) S.sint[0] = v;                     // p0
            else if (tid < 2 + NJ) S.sids[tid - 2] = v;
            else if (tid - 2 - NJ < 256) {
                S.sfidx[tid - 2 - NJ] = v;
                S.sfval[tid - 2 - NJ] = 1.f;
            }
        }
    }
    constexpr int NI = mp / RAE_WAVE;
    float wbk[NI];                           // wave 0: the bias entries it reduces
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int k = lane + RAE_WAVE * i;
        wbk[i] = (w == 0 && k < m) ? a.Wb[k] : 0.f;
    }
    if (tid == 0) {
        S.sint[4] = 0;                       // arrival counter of the W-row waves
        S.sint[5] = 0;                       // P ready (RAE_FWD_PFLAG)
    }
    lds_barrier();
    RAE_STAMP(a, 1);
    const int p0 = S.sint[0], nf = S.sint[1];
#if RAE_FWD_CWAIT
    // rows with more features than the W-row registers hold (NSL*KF = 30 at C3; the synthetic
    // C3 rows have 9..39, P(nf > 30) ~ 1e-6) take the general path: then the decoder-matrix
    // loads are the LAST vector-memory ops of every wave, so C.P waits for each C load by a
    // counted vmcnt and runs while the rest of C lands
    if (nf > a.dcap || nf > NSL * KF) {
#else
    if (nf > a.dcap) {                       // longer than the descriptor holds: general path
#endif
        lds_barrier();
        sp_example<VM == 4, D>(a, g, bl, smem);
        return;
    }
    if (a.values) {                          // non-binary features: their values
        if (w < 4 && tid < nf) S.sfval[tid] = a.values[p0 + tid];
        lds_barrier();
    }
    RAE_STAMP(a, 10);

    // Per-CU issue order W rows -> A rows -> decoder matrices: vmcnt and the CU's memory
    // queue are in issue order, so the 5 KB of W rows the chain waits on go out first, the
    // A rows (needed after C.P) next, and the 160 KB of decoder matrices last.
    // W rows (waves 0-3): slot = feature lane group, c = float4 column.
    const MT* Wm = reinterpret_cast<const MT*>(a.W);
    const int slot = tid / MV, c = tid - slot * MV;
    MT wv[KF];
    float fv[KF];
    if (w < 4) {
#pragma unroll
        for (int k = 0; k < KF; ++k) {
            const int f = slot + NSL * k;
            const bool ok = slot < NSL && f < nf;
            const int fi = RAE_KO_W ? 0 : S.sfidx[f < 256 ? f : 255];   // knockout: row 0
            wv[k] = Wm[(int64_t)(ok ? fi : 0) * MV + c];
            fv[k] = ok ? S.sfval[f < 256 ? f : 255] : 0.f;
        }
    }
    lds_barrier();                           // every W-row load is issued
    RAE_STAMP(a, 11);
    // Each role is one uniform branch, so the compiler's vmcnt bookkeeping for the W-row
    // FMAs sees only the 28 decoder-matrix loads behind them (not the DMA loop).
    float abv = 0.f;
#if RAE_FWD_CWAIT
    // the decoder-matrix loads are issued by common code after the role branch: issued in one
    // place, their registers need no copies where the role paths merge (copies of a loaded
    // register wait for it, which had put a vmcnt(0) -- all of C -- in front of C.P)
    if (w >= 4) {
        // A rows by LDS-DMA, one row per wave instruction (r / 4 = 50 lanes x 16 B), rows
        // w-4, w, w+4, ...: a fixed unrolled count (no loop, so the vmcnt bookkeeping of the
        // C loads behind it stays exact)
        static_assert(r / 4 <= RAE_WAVE, "one DMA instruction per A row");
        constexpr int RPW4 = (NR + 3) / 4;
        const int ln = lane < r / 4 ? lane : 0;
#pragma unroll
        for (int k = 0; k < RPW4; ++k) {
            const int rho = (w - 4) + 4 * k;
            if (rho < NR && lane < r / 4) {
                const int j = rho == 0 ? 0 : rho + 1;            // SP: e2's row is not read
                const float* src = a.A + (int64_t)(RAE_KO_A ? 0 : S.sids[j]) * r + (int64_t)ln * 4;
                dma_row16(src, lds_addr(arows + rho * r4));
            }
        }
        if (tid - 256 < NJ) abv = a.Ab[S.sids[tid - 256]];
    }
    asm volatile("" ::: "memory");
    if (!RAE_FWD_CEARLY47 || w < 4) cc_.load(a, Dm, 0, 0);
    if (w < 4) {
        MT acc;
        vzero(acc);
#pragma unroll
        for (int k = 0; k < KF; ++k) vfma(acc, fv[k], wv[k]);
        if (slot < NSL) reinterpret_cast<MT*>(S.spart)[slot * MV + c] = acc;
    }
    if (false) {
#else
    if (w < 4) {
#endif
        asm volatile("" ::: "memory");
        cc_.load(a, Dm, 0, 0);
        MT acc;
        vzero(acc);
#pragma unroll
        for (int k = 0; k < KF; ++k) vfma(acc, fv[k], wv[k]);
        if (slot < NSL) {
#if !RAE_FWD_CWAIT
            for (int f = slot + NSL * KF; f < nf; f += NSL)      // rows with > NSL*KF features
                vfma(acc, S.sfval[f], Wm[(int64_t)S.sfidx[f] * MV + c]);
#endif
            reinterpret_cast<MT*>(S.spart)[slot * MV + c] = acc;
        }
    } else if (!RAE_FWD_CWAIT) {
        gather_rows_dma<true>(a, Dm, S, NR, 1, 4, 4);
        if (tid - 256 < NJ) abv = a.Ab[S.sids[tid - 256]];
        asm volatile("" ::: "memory");
        cc_.load(a, Dm, 0, 0);
    }
    RAE_STAMP(a, 12);
    // S = X.W + Wb and the softmax run in wave 0 as soon as waves 0-3 have their partial
    // sums in LDS (LDS arrival counter) -- not behind a block barrier, which would also
    // wait for waves 4-7, still issuing (and back-pressured on) the bulk loads.
    if (w < 4) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) atomicAdd(&S.sint[4], 1);
    }
    if (w == 0) {
        while (__hip_atomic_load(&S.sint[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4)
            __builtin_amdgcn_s_sleep(1);
        RAE_STAMP(a, 13);
        float pz[NI], pp[NI];
        fast_softmax<m, NSL, NI>(a, S, wbk, lane, pz, pp);
        if (RAE_FWD_PFLAG) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(&S.sint[5], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    if (RAE_FWD_PFLAG) {
        // P / Z / H ready: an LDS flag instead of a block barrier, so the waves that run the
        // chain do not wait for waves 4-7 still issuing their bulk loads
        if (w != 0)
            while (__hip_atomic_load(&S.sint[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
    } else {
        lds_barrier();
    }
    const float H = S.sred[40];
    RAE_STAMP(a, 2);
#if RAE_FWD_CWAIT
    {
        // wC1 = C1.P, wC2 = C2.P: the 2*RA partial dots in C's load order (each waits for its
        // own loads only), then the 2*RA group reductions as independent interleaved DPP
        // chains, then one masked store block
        typedef CCF CC_;
        static_assert(CC_::FITS && CC_::CC <= 2, "fast path keeps C1/C2 in registers");
        const int gid = tid >> 4, q = tid & 15;
        const MT* Pv = reinterpret_cast<const MT*>(S.sP);
        MT pv[CC_::CC];
#pragma unroll
        for (int cc = 0; cc < CC_::CC; ++cc) pv[cc] = Pv[q + 16 * cc];   // zero beyond m (padded)
        float s1[CC_::RA], s2[CC_::RA];
#pragma unroll
        for (int ra = 0; ra < CC_::RA; ++ra) {
            s1[ra] = vdot(cc_.c1[ra][0], pv[0]);
            s2[ra] = vdot(cc_.c2[ra][0], pv[0]);
#pragma unroll
            for (int cc = 1; cc < CC_::CC; ++cc) {
                s1[ra] += vdot(cc_.c1[ra][cc], pv[cc]);
                s2[ra] += vdot(cc_.c2[ra][cc], pv[cc]);
            }
        }
#pragma unroll
        for (int ra = 0; ra < CC_::RA; ++ra) {
            s1[ra] = group16_sum(s1[ra]);
            s2[ra] = group16_sum(s2[ra]);
        }
        if (q == 0) {
#pragma unroll
            for (int ra = 0; ra < CC_::RA; ++ra) {
                const int i = gid + RAE_NG * ra;
                if (i < r) {
                    S.swC1[i] = s1[ra];
                    S.swC2[i] = s2[ra];
                }
            }
        }
    }
#else
    sp_project<true>(a, Dm, S, cc_);
#endif
    if (w >= 4 && tid - 256 < NJ) S.sAbv[tid - 256] = abv;
    dma_visible_barrier();                   // A rows (LDS-DMA) and Ab landed
    RAE_STAMP(a, 3);

    // dot products: wave w takes rows w, w+8, ...; all LDS reads first, then the
    // independent wave reductions interleave
    constexpr int RV = r / 4;
    static_assert(RV <= RAE_WAVE, "one float4 column per lane");
    const bool lv = lane < RV;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* Rv = reinterpret_cast<const float4*>(arows);
    // branch-free: every lane reads a valid LDS float4 (lanes past the row re-read column 0)
    // and is zeroed through wc, so all the wave's LDS reads issue back to back
    const int lc = lv ? lane : 0;
    float4 wc1 = reinterpret_cast<const float4*>(S.swC1)[lc];
    float4 wc2 = reinterpret_cast<const float4*>(S.swC2)[lc];
    if (!lv) wc1 = wc2 = z4;
    {
        constexpr int RPW = (NR + RAE_FNW - 1) / RAE_FNW;
        float d[RPW];
        float4 xr[RPW];
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int rho = w + RAE_FNW * q;            // wave-uniform
            xr[q] = Rv[(rho < NR ? rho : 0) * RV + lc];
        }
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int rho = w + RAE_FNW * q;
            const float v = vdot(xr[q], rho > s ? wc2 : wc1);   // rows 1..s: neg1, s+1..2s: neg2
            d[q] = rho < NR ? v : 0.f;
        }
        float d0b = (w == 0) ? vdot(xr[0], wc2) : 0.f;
#pragma unroll
        for (int q = 0; q < RPW; ++q) d[q] = wave_sum(d[q]);
        if (w == 0) d0b = wave_sum(d0b);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < RPW; ++q) {
                const int rho = w + RAE_FNW * q;
                if (rho == 0) {
                    S.sdots[0] = d[q];       // left  = <wC1, A[e1]>
                    S.sdots[1] = d0b;        // right = <wC2, A[e1]>
                } else if (rho < NR) {
                    S.sdots[rho + 1] = d[q];
                }
            }
        }
    }
    lds_barrier();
    RAE_STAMP(a, 4);

    // scores, loss and coefficients -- computed by EVERY wave (identical values; no barrier
    // to broadcast them): lanes 0..s-1 neg1[t], lanes 32..32+s-1 neg2[t]
    const float left = S.sdots[0], right = S.sdots[1];
    const int tq = lane & 31;
    const bool hi = lane >= 32;
    float dg = 0.f, ls = 0.f;
    if (tq < s) {
        const int j = 2 + (hi ? s : 0) + tq;
        const float gg = S.sdots[j] + (hi ? left : right) + S.sAbv[j];
        float sg, spl;
        sigmoid_softplus(gg, sg, spl);
        dg = sg * a.invD;
        ls = -spl;                           // log_sigmoid(-g)
    }
    float hs = group16_sum(dg);
    hs += __uint_as_float(xor16_u32(__float_as_uint(hs)));
    const float other = __uint_as_float(xor32_u32(__float_as_uint(hs)));
    const float sdg1 = hi ? other : hs, sdg2 = hi ? hs : other;
    const float one = left + right;
    const float u1 = one + S.sAbv[0], u2 = one + S.sAbv[1];
    float su1, spu1, su2, spu2;
    sigmoid_softplus(-u1, su1, spu1);
    sigmoid_softplus(-u2, su2, spu2);
    const float du1 = -su1 * a.invD, du2 = -su2 * a.invD;
    const float dl = du1 + du2 + sdg2;       // d cost / d left
    const float dr = du1 + du2 + sdg1;       // d cost / d right
    float* rec = a.ex + (int64_t)bg * a.lay.rec;

    // dw1 = dl a1 + sum_t dg1_t n1_t (wave 0), dw2 = dr a1 + sum_t dg2_t n2_t (wave 1):
    // one float4 column per lane, the t-sum in order, coefficients broadcast by readlane
    if (w < 2) {
        const float c0 = w == 0 ? dl : dr;
        float4 v = z4;
        // the coefficients broadcast (readlane) with the whole wave active -- a source lane
        // outside EXEC has no defined value -- into scalars, then the row sum on the row's lanes
        float ct[s];
#pragma unroll
        for (int t = 0; t < s; ++t)
            ct[t] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dg), (w == 0 ? 0 : 32) + t));
        if (lv) {
            vfma(v, c0, Rv[lane]);
#pragma unroll
            for (int t = 0; t < s; ++t) vfma(v, ct[t], Rv[(1 + (w == 0 ? 0 : s) + t) * RV + lane]);
            reinterpret_cast<float4*>(w == 0 ? S.sdw1 : S.sdw2)[lane] = v;
            rec_st(reinterpret_cast<float4*>(a.dwb + (int64_t)bg * a.dws + (w == 0 ? a.dw1o : a.dw2o)) + lane, v);
        }
    } else if (w == 2) {                     // V1 = wC1, V2 = wC2 (wire record: k_vrec's)
        if (lv && !a.lay.wire) {
            rec_st(reinterpret_cast<float4*>(rec + a.lay.oV1) + lane, wc1);
            rec_st(reinterpret_cast<float4*>(rec + a.lay.oV2) + lane, wc2);
        }
    } else if (w == 3) {                     // G1 = dl wC1 + dr wC2 (A[e1]'s gradient)
        if (a.lay.wire) {                    // wire record: (dl, dr) for k_vrec's G1
            if (lane == 0) {
                rec_st(rec + a.lay.oAux + 0, dl);
                rec_st(rec + a.lay.oAux + 1, dr);
            }
        } else if (lv) {
            float4 gv;
            gv.x = dl * wc1.x + dr * wc2.x;
            gv.y = dl * wc1.y + dr * wc2.y;
            gv.z = dl * wc1.z + dr * wc2.z;
            gv.w = dl * wc1.w + dr * wc2.w;
            rec_st(reinterpret_cast<float4*>(rec + a.lay.oG1) + lane, gv);
        }
    } else if (w == 4) {                     // coefficients (c_j, gamma_j) and the loss
        if (tq < s) {
            const int j = 2 + (hi ? s : 0) + tq;
            rec_st(rec + a.lay.ocoef + 2 * j, dg);
            rec_st(rec + a.lay.ocoef + 2 * j + 1, dg);
        }
        const float sls = wave_sum(ls);
        if (lane == 0) {
            rec_st(rec + a.lay.ocoef + 0, 1.f);
            rec_st(rec + a.lay.ocoef + 1, du1);
            rec_st(rec + a.lay.ocoef + 2, 0.f);
            rec_st(rec + a.lay.ocoef + 3, du2);
            rec_st(rec + a.lay.oloss, -spu1 - spu2 + 2.f * H + sls);
        }
    }
    lds_barrier();
    RAE_STAMP(a, 8);
    RAE_STAMP(a, 5);

    // dP = C1^T dw1 + C2^T dw2: per-wave partials (rows held in registers), reduced over the
    // wave's 4 lane groups; the 8 wave partials are summed by wave 0 below
    {
        typedef CCF CC_;
        const int gid = tid >> 4, q = tid & 15;
        MT acc[CC_::CC];
#pragma unroll
        for (int cc = 0; cc < CC_::CC; ++cc) vzero(acc[cc]);
        float d1[CC_::RA], d2[CC_::RA];              // branch-free: all LDS reads issue at once
#pragma unroll
        for (int ra = 0; ra < CC_::RA; ++ra) {
            const int i = gid + RAE_NG * ra;
            d1[ra] = S.sdw1[i < r ? i : r - 1];
            d2[ra] = S.sdw2[i < r ? i : r - 1];
        }
#pragma unroll
        for (int ra = 0; ra < CC_::RA; ++ra) {
            const bool iv = gid + RAE_NG * ra < r;
            const float e1 = iv ? d1[ra] : 0.f, e2 = iv ? d2[ra] : 0.f;
#pragma unroll
            for (int cc = 0; cc < CC_::CC; ++cc) {
                vfma(acc[cc], e1, cc_.c1[ra][cc]);
                vfma(acc[cc], e2, cc_.c2[ra][cc]);
            }
        }
        if constexpr (VM == 4 && CC_::CC == 2) {
            // transpose-reduce the 8 partials over the wave's 4 lane groups with permlane
            // swaps: each swap + add halves two values at once (6 swaps instead of 16), and
            // leaves lane group G holding value {0,2,1,3}[G] of each float4
            float* v0 = reinterpret_cast<float*>(&acc[0]);
            float* v1 = reinterpret_cast<float*>(&acc[1]);
            const float x[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
            float h[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {                 // xor-32 halves
                const auto p = __builtin_amdgcn_permlane32_swap(
                    __float_as_uint(x[2 * k]), __float_as_uint(x[2 * k + 1]), false, false);
                h[k] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
            }
            float t[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {                 // xor-16 halves
                const auto p = __builtin_amdgcn_permlane16_swap(
                    __float_as_uint(h[2 * k]), __float_as_uint(h[2 * k + 1]), false, false);
                t[k] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
            }
            const int G = lane >> 4;
            const int e = (G == 1) ? 2 : (G == 2 ? 1 : G);   // {0,2,1,3}[G]
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const int col = q + 16 * cc;
                if (col < MV) S.spart[w * mp + 4 * col + e] = t[cc];
            }
        } else {
#pragma unroll
            for (int cc = 0; cc < CC_::CC; ++cc) {
                float* v = reinterpret_cast<float*>(&acc[cc]);
#pragma unroll
                for (int e = 0; e < VM; ++e) {
                    v[e] += __uint_as_float(xor16_u32(__float_as_uint(v[e])));
                    v[e] += __uint_as_float(xor32_u32(__float_as_uint(v[e])));
                }
                const int col = q + 16 * cc;
                if (lane < 16 && col < MV) reinterpret_cast<MT*>(S.spart + w * mp)[col] = acc[cc];
            }
        }
    }
    lds_barrier();
    RAE_STAMP(a, 9);

    // softmax backward (wave 0) straight into the record:
    //   dS_k = P_k ((dP_k - sum_j P_j dP_j) + ce (z_k - sum_j P_j z_j))   (softmax_backward)
    if (w == 0) {
        const float ce = 2.f * a.alpha * a.invD;
        float pk[NI], zk[NI], dp[NI];
        float sd = 0.f, sz = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int k = lane + RAE_WAVE * i;
            float v = 0.f;
            if (k < m) {
#pragma unroll
                for (int ww = 0; ww < RAE_FNW; ++ww) v += S.spart[ww * mp + k];
            }
            dp[i] = v;
            pk[i] = k < m ? S.sP[k] : 0.f;
            zk[i] = k < m ? S.sZ[k] : 0.f;
            sd += pk[i] * dp[i];
            sz += pk[i] * zk[i];
        }
        sd = wave_sum(sd);
        sz = wave_sum(sz);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int k = lane + RAE_WAVE * i;
            if (k < m) {
                rec_st(rec + a.lay.oP + k, pk[i]);
                rec_st(rec + a.lay.odS + k, pk[i] * ((dp[i] - sd) + ce * (zk[i] - sz)));
            }
        }
    }
    RAE_STAMP(a, 6);
    RAE_STAMP(a, 7);
#ifdef RAE_STAMPS
    if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 16 + 15] = __builtin_amdgcn_s_memtime();
#endif
}


}  // namespace rae
