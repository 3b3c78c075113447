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
//
// Work items of k_update:
//   one workgroup (four waves, the batch split four ways) per dense decoder-matrix tile
//   (16x16, MFMA) and Wb tile, and per very heavy A / W row (> RAE_VHEAVY records);
//   one wavefront for the batch cost, for each bilinear R-row block, and for every other
//   referenced A row and W row.
#pragma once
#include "rae_common.hpp"
#include "rae_index.hpp"
#include "rae_p2p.hpp"
#include "rae_step.hpp"

namespace rae {


// ---- dense decoder-matrix tiles on MFMA ---------------------------------------------
// Gradient of a 16x16 tile of a matrix M (nrows x m) whose gradient is
//   G[i][k] = sum_b coef(b, i) * P_b[k]      (a batch-contracted outer-product sum)
// computed with v_mfma_f32_16x16x4_f32 (exact fp32, k-ordered fma chain -> deterministic):
//   A[i][b] = coef(b, i)   lane l holds A[l&15][b0 + (l>>4)]
//   B[b][k] = P_b[k]       lane l holds B[b0 + (l>>4)][l&15]
//   D[row][col]            col = lane&15, row = (lane>>4)*4 + reg
// SP/hybrid C1, C2: coef(b, i) = dw1_b[i] / dw2_b[i]; Wb (ones): one row of ones times dS_b.
typedef float rae_f4 __attribute__((ext_vector_type(4)));
#ifndef RAE_TU
#define RAE_TU 13    // k-steps (x4 examples) whose operands are loaded before the MFMA chain
#endif
#ifndef RAE_UNR1
#define RAE_UNR1 4   // record vectors per round on light rows (Q = 1)
#endif
#ifndef RAE_UNRH
#define RAE_UNRH 8   // record vectors per round on heavy rows (> RAE_UNR1 records; Q = 1)
#endif
template <int N> struct IntC { static constexpr int value = N; };
#ifndef RAE_UPD_NT
#define RAE_UPD_NT 3 // row parameter traffic: bit 0 non-temporal loads, bit 1 non-temporal stores
                     // (both: C3 step 19.8 -> 18.5 us, C5 89.3 -> 86.8; profiles/r03_ab.txt)
#endif

// parameters + accumulators of the tile elements this lane updates (lanes >= 16 of a Wb tile
// own nothing): loaded up front, in flight with the records
template <int OPT>
__device__ __forceinline__ void tile_params(const StepArgs& a, const float* M, const float* aM,
                                            int nrows, bool ones, int i0, int k0, int lane,
                                            float pw[4], float pa[4]) {
    const int li = lane & 15, lk = lane >> 4, col = k0 + li;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int row = i0 + lk * 4 + reg;
        const bool ok = row < nrows && col < a.m && (!ones || row == i0);
        const int o = ok ? (ones ? col : row * a.m + col) : 0;
        pw[reg] = M[o];
        pa[reg] = (OPT == 0) ? aM[o] : 0.f;
    }
}

// the tile's MFMA chain over examples [b0, b1) of the global batch (b0 a multiple of 4)
__device__ __forceinline__ rae_f4 tile_accum(const StepArgs& a, int nrows, int odw, bool ones,
                                             int i0, int k0, int b0, int b1, int lane) {
    const int li = lane & 15, lk = lane >> 4;
    const int m = a.m, L = a.L;
    const int i = i0 + li, k = k0 + li;
    const bool iv = i < nrows, kv = k < m;
    const int ic = iv ? i : 0, kc = kv ? k : 0;
    rae_f4 acc = {0.f, 0.f, 0.f, 0.f};
    const int ox = odw + ic, oy = (ones ? a.lay.odS : a.lay.oP) + kc;   // Wb: sum_b dS_b
    // L % 4 == 0 (every k-step's 4 examples exist): the k-step's first record offset is
    // wave-uniform and rides in the buffer load's soffset, the lane's (example, column) in
    // one voffset VGPR for all TU loads
    const RecBuf rb_(a.ex);
    const bool whole = (L & 3) == 0;
    const int rec = a.lay.rec, vx = lk * rec + ox, vy = lk * rec + oy;
    for (int bb = b0; bb < b1; bb += 4 * RAE_TU) {
        float av[RAE_TU], bv[RAE_TU];
        // every operand load goes out before the first MFMA: the sched_barrier keeps the
        // scheduler from sinking each load next to its MFMA (which serialised 32 round trips)
#pragma unroll
        for (int u = 0; u < RAE_TU; ++u) {
            const int bs = bb + 4 * u;
            if (whole) {
                const int so = (bs < b1 ? bs : 0) * rec;
                if (ones) av[u] = 1.f; else rb_.load(av[u], vx, so);
                rb_.load(bv[u], vy, so);
            } else {
                const int b = bs + lk;
                const int rb = (b < b1 ? b : 0) * rec;
                av[u] = ones ? 1.f : a.ex[rb + ox];
                bv[u] = a.ex[rb + oy];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < RAE_TU; ++u) {
            const bool bvld = bb + 4 * u + lk < b1;
            const float x = (bvld && iv && (!ones || li == 0)) ? av[u] : 0.f;
            const float y = (bvld && kv) ? bv[u] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc, 0, 0, 0);
        }
    }
    return acc;
}

template <int OPT>
__device__ __forceinline__ void tile_apply(const StepArgs& a, float* M, float* aM, int nrows,
                                           bool ones, int i0, int k0, int slot, rae_f4 acc,
                                           const float pw[4], const float pa[4], int lane) {
    const int li = lane & 15, lk = lane >> 4, col = k0 + li, m = a.m;
    float l1 = 0.f, l2 = 0.f;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int row = i0 + lk * 4 + reg;
        if (row < nrows && col < m && (!ones || row == i0)) {
            const int o = ones ? col : row * m + col;
            const float w = pw[reg];
            float g = acc[reg];
            if (!ones && a.reg_on && a.ext_reg) {
                g += a.l1adj * sgnf(w) + 2.f * a.l2adj * w;
                l1 += fabsf(w);
                l2 += w * w;
            }
            float ac = pa[reg];
            M[o] = opt_update<OPT>(w, &ac, g, a.lr);
            if (OPT == 0) aM[o] = ac;
        }
    }
    if (!ones && a.reg_on && a.ext_reg) {
        const double L1 = wave_sum_d((double)l1), L2 = wave_sum_d((double)l2);
        if (lane == 0) {
            a.regpart[2 * slot] = L1;
            a.regpart[2 * slot + 1] = L2;
        }
    }
}

// One 16x16 tile per workgroup: the batch (K) split into four contiguous quarters, one per
// wave, the four partial accumulators summed in wave order (deterministic) by wave 0, which
// applies the update -- a K = L chain becomes four K = L/4 chains in parallel.
template <int OPT>
__device__ void wg_tile(const StepArgs& a, float* M, float* aM, int nrows, int odw, bool ones,
                        int i0, int k0, int slot, int w, int lane, rae_f4* sacc) {
    const int q = ((a.L + 15) / 16) * 4;                   // examples per wave, multiple of 4
    const int b0 = min(w * q, a.L), b1 = min(b0 + q, a.L);
    float pw[4], pa[4];
    if (w == 0) tile_params<OPT>(a, M, aM, nrows, ones, i0, k0, lane, pw, pa);
    const rae_f4 acc = tile_accum(a, nrows, odw, ones, i0, k0, b0, b1, lane);
    sacc[w * RAE_WAVE + lane] = acc;
    __syncthreads();
    if (w == 0) {
        rae_f4 t = sacc[lane];
#pragma unroll
        for (int ww = 1; ww < RAE_NWAVE; ++ww) t += sacc[ww * RAE_WAVE + lane];
        tile_apply<OPT>(a, M, aM, nrows, ones, i0, k0, slot, t, pw, pa, lane);
    }
}

// ---- dense partials (data parallel, SP: RecLayout wire 2) ----------------------------------
// Each rank reduces the decoder-matrix gradients of its OWN l examples before the exchange
// (k_dpart: dC1, dC2 = sum_b dw_b P_b^T and dWb = sum_b dS_b, the same MFMA tile chain as wg_tile
// with K = l split over four waves) into a partial block that rides in its records; the update
// sums the G blocks in rank order -- K = l + G instead of a K = L chain per tile (which at
// L = 8192 was the partitioned update's tail).  Element e of rank k's block: dpart_off.
__device__ __forceinline__ int64_t dpart_off(const StepArgs& a, int k, int e) {
    const int q = e / a.lay.pc;
    return (int64_t)(k * a.l + q) * a.lay.rec + a.lay.oPart + (e - q * a.lay.pc);
}
__host__ __device__ inline int dpart_tasks(int r, int m) {
    return 2 * ((r + 15) / 16) * ((m + 15) / 16) + (m + 15) / 16;
}
// tile t of this rank's partial block: C1 tiles, C2 tiles, Wb tiles (one workgroup each)
__device__ void dpart_tile(const StepArgs& a, int t, int w, int lane, rae_f4* sacc) {
    const int m = a.m, l = a.l, mt = (m + 15) / 16, nC = ((a.r + 15) / 16) * mt;
    const int which = t < nC ? 0 : (t < 2 * nC ? 1 : 2);
    const bool ones = which == 2;
    const int ti = t - which * nC;
    const int i0 = ones ? 0 : (ti / mt) * 16, k0 = (ones ? ti : ti % mt) * 16;
    const int nrows = ones ? 1 : a.r;
    const int li = lane & 15, lk = lane >> 4;
    const int i = i0 + li, k = k0 + li;
    const bool iv = i < nrows, kv = k < m;
    const int q = ((l + 15) / 16) * 4;                   // examples per wave, multiple of 4
    const int b0 = min(w * q, l), b1 = min(b0 + q, l);
    const int64_t e0 = (int64_t)a.rank * l;
    const float* Ar = a.dwb + (which == 1 ? a.dw2o : a.dw1o) + (iv ? i : 0);
    const float* Br = a.ex + (ones ? a.lay.odS : a.lay.oP) + (kv ? k : 0);
    rae_f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int bb = b0; bb < b1; bb += 4 * RAE_TU) {
        float av[RAE_TU], bv[RAE_TU];
#pragma unroll
        for (int u = 0; u < RAE_TU; ++u) {               // every operand load before the chain
            const int b = bb + 4 * u + lk;
            const int64_t ex = e0 + (b < b1 ? b : b0);
            av[u] = ones ? 1.f : Ar[ex * a.dws];
            bv[u] = Br[ex * a.lay.rec];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < RAE_TU; ++u) {
            const bool ok = bb + 4 * u + lk < b1;
            const float x = (ok && iv && (!ones || li == 0)) ? av[u] : 0.f;
            const float y = (ok && kv) ? bv[u] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc, 0, 0, 0);
        }
    }
    sacc[w * RAE_WAVE + lane] = acc;
    __syncthreads();
    if (w != 0) return;
    rae_f4 ts = sacc[lane];
#pragma unroll
    for (int ww = 1; ww < RAE_NWAVE; ++ww) ts += sacc[ww * RAE_WAVE + lane];
    const int base = which * a.r * m;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {                  // D[row = 4 lk + reg][col = li]
        const int row = i0 + lk * 4 + reg, col = k0 + li;
        if (row < nrows && col < m && (!ones || row == i0))
            a.ex[dpart_off(a, a.rank, base + (ones ? col : row * m + col))] = ts[reg];
    }
}

// the update's tile task with dense partials: the G ranks' partial sums in rank order, then
// the optimizer (one wave)
template <int OPT>
__device__ void tile_from_partials(const StepArgs& a, float* M, float* aM, int nrows, bool ones,
                                   int base, int i0, int k0, int slot, int lane) {
    float pw[4], pa[4];
    tile_params<OPT>(a, M, aM, nrows, ones, i0, k0, lane, pw, pa);
    const int li = lane & 15, lk = lane >> 4, col = k0 + li, m = a.m;
    float v[4][8];
    rae_f4 acc;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int row = i0 + lk * 4 + reg;
        const bool ok = row < nrows && col < m && (!ones || row == i0);
        const int e = ok ? base + (ones ? col : row * m + col) : 0;
        float g = 0.f;
        for (int k0g = 0; k0g < a.G; k0g += 8) {         // loads of 8 ranks in flight
#pragma unroll
            for (int k = 0; k < 8; ++k) v[reg][k] = k0g + k < a.G ? a.ex[dpart_off(a, k0g + k, e)] : 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) if (k0g + k < a.G) g += v[reg][k];
        }
        acc[reg] = g;
    }
    tile_apply<OPT>(a, M, aM, nrows, ones, i0, k0, slot, acc, pw, pa, lane);
}

// ---- the batch cost: -mean(all_scores) = -(sum_b loss_b) / (4L + 2Ls)  (OieModel.py:90)
// One workgroup: wave w sums examples [w q, (w + 1) q) of the global batch with eight loads in
// flight per lane (eight chains, combined in a fixed order), the four wave sums combined in wave
// order -- a fixed summation order; at L = 8192 a single lane-strided chain was 128 dependent
// round trips, the partitioned update's tail.
__device__ void task_cost(const StepArgs& a, int w, int lane, double* sred) {
    const int q = (a.L + RAE_NWAVE - 1) / RAE_NWAVE;
    const int b0 = min(w * q, a.L), b1 = min(b0 + q, a.L);
    double t[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int c = b0 + lane; c < b1; c += 8 * RAE_WAVE) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int b = c + u * RAE_WAVE;
            v[u] = a.ex[(int64_t)(b < b1 ? b : b0) * a.lay.rec + a.lay.oloss];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] += c + u * RAE_WAVE < b1 ? (double)v[u] : 0.0;
    }
    double loss = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
    loss = wave_sum_d(loss);
    if (lane == 0) sred[w] = loss;
    __syncthreads();
    if (w != 0) return;
    loss = sred[0];
#pragma unroll
    for (int ww = 1; ww < RAE_NWAVE; ++ww) loss += sred[ww];
    if (lane == 0) {
        const double D = 4.0 * a.L + 2.0 * a.L * a.s;
        const float cost = (float)(-loss / D);
        const int64_t batch = step_batch(a);
        if (a.reg_on) *a.base_cost = cost;
        else a.costs[batch] = cost;
    }
}

// ---- one parameter row held as lane-strided vectors (Q per lane) ----------------------
template <bool V4, int Q>
struct RowVec {
    typedef typename VecT<V4>::T VT;
    VT v[Q];
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int q = 0; q < Q; ++q) vzero(v[q]);
    }
    // parameter / accumulator rows stream through once per step: RAE_UPD_NT reads (and
    // apply_row writes) them non-temporally, so they do not push the exchange records -- read
    // by many row tasks each -- out of L2
    __device__ __forceinline__ void load(const float* p, int nv, int lane) {
        const VT* pv = reinterpret_cast<const VT*>(p);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int c = lane + RAE_WAVE * q;
            if (RAE_UPD_NT & 1) v[q] = ld_nt(pv + (c < nv ? c : 0));
            else v[q] = pv[c < nv ? c : 0];
        }
    }
};


template <int OPT, bool V4, int Q>
__device__ __forceinline__ void apply_row(float* p, float* acc, RowVec<V4, Q>& pv,
                                          RowVec<V4, Q>& av, const RowVec<V4, Q>& g, int nv,
                                          float lr, int lane) {
    typedef typename VecT<V4>::T VT;
    VT* pp = reinterpret_cast<VT*>(p);
    VT* aa = reinterpret_cast<VT*>(acc);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int c = lane + RAE_WAVE * q;
        if (c < nv) {
            updv<OPT>(pv.v[q], av.v[q], g.v[q], lr);
            if (RAE_UPD_NT & 2) {
                st_nt(pv.v[q], pp + c);
                if (OPT == 0) st_nt(av.v[q], aa + c);
            } else {
                pp[c] = pv.v[q];
                if (OPT == 0) aa[c] = av.v[q];
            }
        }
    }
}

// ---- A / Ab rows -------------------------------------------------------------------------
// g(A[e]) = sum over the row's records (in sorted order) of c_j * vec_j (rae_step.hpp: one
// r-vector per record: G1 for e1, G2 for e2 on the bilinear decoders, V1 for neg1, V2 for
// neg2), g(Ab[e]) = sum gamma_j.  Record metadata is loaded lane-parallel (one lane per
// record) and broadcast with v_readlane (wave-uniform -> scalar addressing); the record
// vectors are loaded UNR at a time with every load issued before the first FMA.
// entity_accum: records [st, en) of the slot's sorted list into g (lane-strided row) and gb
// (this lane's share of the Ab gradient); rec0 = the record of a one-record row.
// VS: where the record vectors are -- 0: SP records, 1: bilinear records (e2 has its own G2),
// 2: the SP wire record's vector buffer (StepArgs::vb; data parallel).  0 / 1 address them with
// the record offsets at compile-time-known fields (the single-rank hot path's code).
template <bool V4, int Q, int VS>
__device__ __forceinline__ void entity_accum(const StepArgs& a, int64_t base, int st, int en,
                                             int rec0, RowVec<V4, Q>& g, float& gb, int lane) {
    constexpr int VW = V4 ? 4 : 1;
    constexpr int UNR = Q == 1 ? RAE_UNR1 : 2;
    constexpr int UNRH = Q == 1 ? RAE_UNRH : RAE_UNRH / 2;
    constexpr bool XY = VS == 1, EXT = VS == 2;
    typedef typename VecT<V4>::T VT;
    const int nv = a.r / VW, s = a.s, NJ = 2 + 2 * s;
    const int oG1 = EXT ? a.vG1 : a.lay.oG1, oV1 = EXT ? a.vV1 : a.lay.oV1;
    const int oV2 = EXT ? a.vV2 : a.lay.oV2;
    const int vo1 = XY ? a.lay.oG2 : oV1;         // SP: e2 has no A gradient (c = 0)
    const RecBuf rb_(EXT ? a.vb : a.ex);          // the record vectors (rae_step.hpp vb)
    for (int c0 = st; c0 < en; c0 += RAE_WAVE) {
        const int n = min(RAE_WAVE, en - c0);
        // a one-record row's record rides in its segment: no srec round trip (rec0 < 0: a chunk
        // of a split row, whose records are always read from the list)
        const int rec = (en - st == 1 && rec0 >= 0) ? rec0 : a.srecA[base + c0 + (lane < n ? lane : 0)];
        const int b = rec / NJ, j = rec - b * NJ;
        const int rb = b * a.lay.rec;
        const float* er = a.ex + rb + a.lay.ocoef + 2 * j;
        const float cj = er[0];
        const float ga = er[1];
        const int vo = (EXT ? b * a.vbs : rb) + (j == 0 ? oG1 : (j == 1 ? vo1 : (j < 2 + s ? oV1 : oV2)));
        // one round: U record vectors loaded (all issued before the first FMA), then summed
        // in record order -- the same order for every U, so the round width is free.  The
        // vectors' offsets need only the record ids: their loads are issued before the first
        // use of the coefficients (c_j, gamma_j), whose round trip then overlaps theirs instead
        // of preceding them (the compiler waits at a value's first use)
        auto round = [&](auto Uc, int k0) {
            constexpr int U = decltype(Uc)::value;
            VT v[U][Q];
            float ck[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int ok = __builtin_amdgcn_readlane(vo, min(k0 + k, n - 1));
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const int c = lane + RAE_WAVE * q;
                    rb_.load(v[k][q], (c < nv ? c : 0) * VW, ok);
                }
            }
#pragma unroll
            for (int k = 0; k < U; ++k)
                ck[k] = (k0 + k < n)
                    ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cj), min(k0 + k, n - 1)))
                    : 0.f;
#pragma unroll
            for (int k = 0; k < U; ++k)
#pragma unroll
                for (int q = 0; q < Q; ++q) vfma(g.v[q], ck[k], v[k][q]);
        };
        // Zipf-frequent entities carry tens of records per step: wide rounds keep their
        // dependent round trips (the update's tail) few
        if (n <= RAE_HEAVY && n <= UNR) {
            round(IntC<UNR>{}, 0);
        } else {
#pragma clang loop unroll(disable)
            for (int k0 = 0; k0 < n; k0 += UNRH) round(IntC<UNRH>{}, k0);
        }
        gb += lane < n ? ga : 0.f;
    }
}

// (pipelined peer-to-peer form: the new Ab also into the peers mk that read row e next batch)
template <int OPT>
__device__ __forceinline__ void ab_update(const StepArgs& a, int e, float ab0, float aab0, float gb,
                                          unsigned mk = 0u) {
    float ac = aab0;
    const float v = opt_update<OPT>(ab0, &ac, gb, a.lr);
    a.Ab[e] = v;
    if (OPT == 0) a.aAb[e] = ac;
    if (mk) pipe_push_ab(a, e, mk, v);
}

template <int OPT, bool V4, int Q, int VS, bool PP = false>
__device__ void task_entity_row(const StepArgs& a, int64_t slot, int4 seg, int lane) {
    constexpr int VW = V4 ? 4 : 1;
    const int r = a.r, nv = r / VW;
    const int64_t base = slot * a.RA;
    const int e = seg.x;
    float* prow = a.A + (int64_t)e * r;
    float* arow = (OPT == 0) ? a.aA + (int64_t)e * r : nullptr;
    RowVec<V4, Q> pv, av, g;
    pv.load(prow, nv, lane);                     // parameters in flight with the records
    if (OPT == 0) av.load(arow, nv, lane); else av.zero();
#ifdef RAE_STAMPS
    if (a.stamps && lane == 0) {   // diagnostic: the row's segment has arrived (prow issued)
        const int gw_ = __builtin_amdgcn_readfirstlane(blockIdx.x * RAE_NWAVE + (threadIdx.x >> 6));
        a.stamps[(size_t)gw_ * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const float ab0 = a.Ab[e];
    const float aab0 = (OPT == 0) ? a.aAb[e] : 0.f;
    const unsigned mk = pipe_mark<PP>(a, 0, e);
    g.zero();
    float gb = 0.f;
    if (seg.z - seg.y > RAE_VHEAVY) {
        // a very heavy row the workgroup slots (NVC) could not take: wg_entity_row's arithmetic
        // in one wave -- four contiguous quarters summed separately, combined in quarter order
        // -- so the row's update is bit-identical whichever task runs it (the slots differ
        // between the replicated and the partitioned data-parallel plans)
        const int st = seg.y, en = seg.z, ch = (en - st + RAE_NWAVE - 1) / RAE_NWAVE;
#pragma unroll 1
        for (int w = 0; w < RAE_NWAVE; ++w) {
            const int c0 = min(st + w * ch, en), c1 = min(c0 + ch, en);
            RowVec<V4, Q> gw;
            gw.zero();
            float gbw = 0.f;
            if (c0 < c1) entity_accum<V4, Q, VS>(a, base, c0, c1, seg.w, gw, gbw, lane);
            gbw = wave_sum(gbw);
            if (w == 0) {
                g = gw;
                gb = gbw;
            } else {
#pragma unroll
                for (int q = 0; q < Q; ++q) vadd(g.v[q], gw.v[q]);
                gb += gbw;
            }
        }
    } else {
        entity_accum<V4, Q, VS>(a, base, seg.y, seg.z, seg.w, g, gb, lane);
        gb = wave_sum(gb);
    }
    apply_row<OPT, V4, Q>(prow, arow, pv, av, g, nv, a.lr, lane);
    pipe_push_row(a, 0, e, mk, pv.v, nv, lane);
    if (lane == 0) ab_update<OPT>(a, e, ab0, aab0, gb, mk);
}

// A very heavy row (> RAE_VHEAVY records) per workgroup: its sorted record list split into
// four contiguous chunks, one per wave; wave 0 sums the partial rows in wave order and applies
// the update (its parameter loads in flight meanwhile).  spart: RAE_NWAVE * 64 * Q vectors.
template <int OPT, bool V4, int Q, int VS, bool PP = false>
__device__ void wg_entity_row(const StepArgs& a, int64_t slot, int4 seg, int w, int lane,
                              typename VecT<V4>::T* spart, float* sgb) {
    constexpr int VW = V4 ? 4 : 1;
    const int r = a.r, nv = r / VW;
    const int64_t base = slot * a.RA;
    const int e = seg.x, st = seg.y, en = seg.z;
    const bool chunk = seg.w < 0;                // a chunk of a split row: partial sum only
    const int ch = (en - st + RAE_NWAVE - 1) / RAE_NWAVE;
    const int c0 = min(st + w * ch, en), c1 = min(c0 + ch, en);
    float* prow = a.A + (int64_t)e * r;
    float* arow = (OPT == 0) ? a.aA + (int64_t)e * r : nullptr;
    RowVec<V4, Q> pv, av, g;
    float ab0 = 0.f, aab0 = 0.f;
    unsigned mk = 0u;
    if (w == 0 && !chunk) {
        pv.load(prow, nv, lane);
        if (OPT == 0) av.load(arow, nv, lane); else av.zero();
        ab0 = a.Ab[e];
        aab0 = (OPT == 0) ? a.aAb[e] : 0.f;
        mk = pipe_mark<PP>(a, 0, e);
    }
    g.zero();
    float gb = 0.f;
    if (c0 < c1) entity_accum<V4, Q, VS>(a, base, c0, c1, seg.w, g, gb, lane);
    gb = wave_sum(gb);
#pragma unroll
    for (int q = 0; q < Q; ++q) spart[(w * Q + q) * RAE_WAVE + lane] = g.v[q];
    if (lane == 0) sgb[w] = gb;
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            g.v[q] = spart[q * RAE_WAVE + lane];
#pragma unroll
            for (int ww = 1; ww < RAE_NWAVE; ++ww) vadd(g.v[q], spart[(ww * Q + q) * RAE_WAVE + lane]);
        }
        float gt = sgb[0];
#pragma unroll
        for (int ww = 1; ww < RAE_NWAVE; ++ww) gt += sgb[ww];
        if (chunk) {                             // k_heavy_fin combines the row's chunks
            typedef typename VecT<V4>::T VT;
            float* hp = a.hpart + (int64_t)(-1 - seg.w) * a.hps;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int c = lane + RAE_WAVE * q;
                if (c < nv) reinterpret_cast<VT*>(hp)[c] = g.v[q];
            }
            if (lane == 0) hp[align4(r)] = gt;
            return;
        }
        apply_row<OPT, V4, Q>(prow, arow, pv, av, g, nv, a.lr, lane);
        pipe_push_row(a, 0, e, mk, pv.v, nv, lane);
        if (lane == 0) ab_update<OPT>(a, e, ab0, aab0, gt, mk);
    }
}

// ---- W rows: g(W[f]) = sum over the row's CSR records of x_bf * dS_b ----------------------
template <bool V4, int Q>
__device__ __forceinline__ void feature_accum(const StepArgs& a, int64_t ex0, int64_t base,
                                              int st, int en, int rec0, RowVec<V4, Q>& g,
                                              int lane) {
    constexpr int VW = V4 ? 4 : 1;
    constexpr int UNR = Q == 1 ? RAE_UNR1 : 2;
    constexpr int UNRH = Q == 1 ? RAE_UNRH : RAE_UNRH / 2;
    typedef typename VecT<V4>::T VT;
    const int nv = a.m / VW;
    const unsigned mask = (1u << a.posbits) - 1u;
    const RecBuf rb_(a.ex);
    for (int c0 = st; c0 < en; c0 += RAE_WAVE) {
        const int n = min(RAE_WAVE, en - c0);
        const unsigned rec = (unsigned)((en - st == 1 && rec0 >= 0) ? rec0
                                                                      : a.srecW[base + c0 + (lane < n ? lane : 0)]);
        const int b = (int)(rec >> a.posbits);
        float val = 1.f;
        if (a.values) val = a.values[a.indptr[ex0 + b] + (int)(rec & mask)];
        if (lane >= n) val = 0.f;
        auto round = [&](auto Uc, int k0) {
            constexpr int U = decltype(Uc)::value;
            VT v[U][Q];
            float cv[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int src = min(k0 + k, n - 1);
                const int bk = __builtin_amdgcn_readlane(b, src);
                cv[k] = (k0 + k < n) ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(val), src))
                                     : 0.f;
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const int c = lane + RAE_WAVE * q;
                    rb_.load(v[k][q], (c < nv ? c : 0) * VW, bk * a.lay.rec + a.lay.odS);
                }
            }
#pragma unroll
            for (int k = 0; k < U; ++k)
#pragma unroll
                for (int q = 0; q < Q; ++q) vfma(g.v[q], cv[k], v[k][q]);
        };
        if (n <= RAE_HEAVY && n <= UNR) {
            round(IntC<UNR>{}, 0);
        } else {                                    // Zipf-frequent features: wide rounds
#pragma clang loop unroll(disable)
            for (int k0 = 0; k0 < n; k0 += UNRH) round(IntC<UNRH>{}, k0);
        }
    }
}

// W row f with gradient g: applied, or (lambda != 0) left in the dense scratch for k_dense_w
template <int OPT, bool V4, int Q, bool PP = false>
__device__ __forceinline__ void feature_finish(const StepArgs& a, int f, RowVec<V4, Q>& pv,
                                               RowVec<V4, Q>& av, RowVec<V4, Q>& g, int lane,
                                               unsigned mk = 0u) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int m = a.m, nv = m / VW;
    if (a.reg_on) {
        VT* gs = reinterpret_cast<VT*>(a.gWs + (int64_t)f * m);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int c = lane + RAE_WAVE * q;
            if (c < nv) gs[c] = g.v[q];
        }
    } else {
        float* arow = (OPT == 0 && a.aW) ? a.aW + (int64_t)f * m : nullptr;
        apply_row<OPT, V4, Q>(a.W + (int64_t)f * m, arow, pv, av, g, nv, a.lr, lane);
        pipe_push_row(a, 1, f, mk, pv.v, nv, lane);
    }
}

template <int OPT, bool V4, int Q, bool PP = false>
__device__ void task_feature_row(const StepArgs& a, int64_t ex0, int64_t slot, int4 seg, int lane) {
    constexpr int VW = V4 ? 4 : 1;
    const int m = a.m, nv = m / VW;
    const int64_t base = slot * a.RW;
    const int f = seg.x;
    RowVec<V4, Q> pv, av, g;
    if (!a.reg_on) {
        pv.load(a.W + (int64_t)f * m, nv, lane);
        if (OPT == 0) av.load(a.aW + (int64_t)f * m, nv, lane); else av.zero();
    }
    const unsigned mk = pipe_mark<PP>(a, 1, f);
#ifdef RAE_STAMPS
    if (a.stamps && lane == 0) {   // diagnostic: the row's segment has arrived (prow issued)
        const int gw_ = __builtin_amdgcn_readfirstlane(blockIdx.x * RAE_NWAVE + (threadIdx.x >> 6));
        a.stamps[(size_t)gw_ * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    g.zero();
    if (seg.z - seg.y > RAE_VHEAVY) {
        // an overflowed very heavy row: wg_feature_row's four-quarter arithmetic in one wave
        // (bit-identical to the workgroup task; see task_entity_row)
        const int st = seg.y, en = seg.z, ch = (en - st + RAE_NWAVE - 1) / RAE_NWAVE;
#pragma unroll 1
        for (int w = 0; w < RAE_NWAVE; ++w) {
            const int c0 = min(st + w * ch, en), c1 = min(c0 + ch, en);
            RowVec<V4, Q> gw;
            gw.zero();
            if (c0 < c1) feature_accum<V4, Q>(a, ex0, base, c0, c1, seg.w, gw, lane);
            if (w == 0) {
                g = gw;
            } else {
#pragma unroll
                for (int q = 0; q < Q; ++q) vadd(g.v[q], gw.v[q]);
            }
        }
    } else {
        feature_accum<V4, Q>(a, ex0, base, seg.y, seg.z, seg.w, g, lane);
    }
    feature_finish<OPT, V4, Q, PP>(a, f, pv, av, g, lane, mk);
}

// a very heavy W row per workgroup (as wg_entity_row)
template <int OPT, bool V4, int Q, bool PP = false>
__device__ void wg_feature_row(const StepArgs& a, int64_t ex0, int64_t slot, int4 seg, int w,
                               int lane, typename VecT<V4>::T* spart) {
    constexpr int VW = V4 ? 4 : 1;
    const int m = a.m, nv = m / VW;
    const int64_t base = slot * a.RW;
    const int f = seg.x, st = seg.y, en = seg.z;
    const bool chunk = seg.w < 0;                // a chunk of a split row: partial sum only
    const int ch = (en - st + RAE_NWAVE - 1) / RAE_NWAVE;
    const int c0 = min(st + w * ch, en), c1 = min(c0 + ch, en);
    RowVec<V4, Q> pv, av, g;
    unsigned mk = 0u;
    if (w == 0 && !a.reg_on && !chunk) {
        pv.load(a.W + (int64_t)f * m, nv, lane);
        if (OPT == 0) av.load(a.aW + (int64_t)f * m, nv, lane); else av.zero();
        mk = pipe_mark<PP>(a, 1, f);
    }
    g.zero();
    if (c0 < c1) feature_accum<V4, Q>(a, ex0, base, c0, c1, seg.w, g, lane);
#pragma unroll
    for (int q = 0; q < Q; ++q) spart[(w * Q + q) * RAE_WAVE + lane] = g.v[q];
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            g.v[q] = spart[q * RAE_WAVE + lane];
#pragma unroll
            for (int ww = 1; ww < RAE_NWAVE; ++ww) vadd(g.v[q], spart[(ww * Q + q) * RAE_WAVE + lane]);
        }
        if (chunk) {                             // k_heavy_fin combines the row's chunks
            typedef typename VecT<V4>::T VT;
            float* hp = a.hpart + (int64_t)(-1 - seg.w) * a.hps;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int c = lane + RAE_WAVE * q;
                if (c < nv) reinterpret_cast<VT*>(hp)[c] = g.v[q];
            }
            return;
        }
        feature_finish<OPT, V4, Q, PP>(a, f, pv, av, g, lane, mk);
    }
}

// k_heavy_fin: entry e of the slot's combine list -- a row split into chunks: the chunks'
// partial sums in chunk order (chunk k = records [st + k hch, ...) of the row's sorted list),
// then the update, as the unsplit row task would apply it (one wave per row)
template <int OPT, bool V4, int Q, bool PP = false>
__device__ void heavy_fin(const StepArgs& a, int e, int lane) {
    typedef typename VecT<V4>::T VT;
    constexpr int VW = V4 ? 4 : 1;
    const int64_t g = step_batch(a);
    const int64_t slot = g % a.index_window;
    const int4 th = reinterpret_cast<const int4*>(a.thdr)[slot];
    if (e >= th.z) return;
    const int4 f = reinterpret_cast<const int4*>(a.hfin)[slot * a.HF + e];
    const bool isA = f.x >= 0;
    const int row = isA ? f.x : ~f.x;
    const int w = isA ? a.r : a.m, nv = w / VW;
    RowVec<V4, Q> pv, av, gs;
    float* prow = (isA ? a.A : a.W) + (int64_t)row * w;
    float* arow = (OPT == 0) ? (isA ? a.aA : a.aW) + (int64_t)row * w : nullptr;
    const bool ld = isA || !a.reg_on;
    if (ld) {
        pv.load(prow, nv, lane);
        if (OPT == 0) av.load(arow, nv, lane); else av.zero();
    }
    float ab0 = 0.f, aab0 = 0.f;
    if (isA) {
        ab0 = a.Ab[row];
        aab0 = (OPT == 0) ? a.aAb[row] : 0.f;
    }
    const unsigned mk = pipe_mark<PP>(a, isA ? 0 : 1, row);
    gs.zero();
    float gb = 0.f;
    const float* hp0 = a.hpart + (int64_t)f.y * a.hps;
    for (int k0 = 0; k0 < f.z; k0 += 8) {              // eight chunks' loads in flight
        VT v[8][Q];
        float b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = min(k0 + u, f.z - 1);
            const float* hp = hp0 + (int64_t)k * a.hps;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int c = lane + RAE_WAVE * q;
                v[u][q] = reinterpret_cast<const VT*>(hp)[c < nv ? c : 0];
            }
            b[u] = isA ? hp[align4(a.r)] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (k0 + u < f.z) {
#pragma unroll
                for (int q = 0; q < Q; ++q) vadd(gs.v[q], v[u][q]);
                gb += b[u];
            }
        }
    }
    if (isA) {
        apply_row<OPT, V4, Q>(prow, arow, pv, av, gs, nv, a.lr, lane);
        pipe_push_row(a, 0, row, mk, pv.v, nv, lane);
        if (lane == 0) ab_update<OPT>(a, row, ab0, aab0, gb, mk);
    } else {
        feature_finish<OPT, V4, Q, PP>(a, row, pv, av, gs, lane, mk);
    }
}

// ---- private rows (StepArgs::priv): per example, the rows only its own records reference ----
// The row index (rae_index.hpp) marks a row that exactly one record of the global batch
// references -- ~95 % of the A rows and ~90 % of the W rows at C3 -- in the example's pmask and
// leaves it out of the dispatch table.  RAE_PRA + 1 workgroups per example take them: the first
// RAE_PRA its A / Ab rows (wave i of them the marked rows i, i + 4 RAE_PRA, ...), the last its W
// rows (wave w: marked features w, w + 4, ...).  A row j's gradient is its one
// record's c_j vec_j (Ab: gamma_j), a W row's x_f dS_b: k_update's one-record row task, the same
// arithmetic and stores, so the parameters are bit-identical to the per-row tasks these replace.
// The loads are batched: one round trip for the example's descriptor ids, coefficients and
// record vectors (no task entry, no segment), one for a round of up to PRMAX rows.
#ifndef RAE_PRMAX
#define RAE_PRMAX 4          // rows per round of one wave (within the update kernel's VGPR budget)
#endif
#ifndef RAE_PRA
#define RAE_PRA 3            // workgroups per example for its A rows (+ 1 for its W rows)
#endif
// Partitioned data-parallel plans (StepArgs::privc): a rank owns ~1/G of each example's private
// rows, so one WAVE per example takes them (its A rows, then its W rows): L / 4 workgroups.
__host__ __device__ inline int priv_workgroups(int compact, int L) {
    return compact ? (L + RAE_NWAVE - 1) / RAE_NWAVE : (RAE_PRA + 1) * L;
}
// the example's marked A / Ab rows wa0, wa0 + na, ... (bits of pmask words 0, 1)
template <int OPT, bool V4, int Q, int VS>
__device__ __forceinline__ void priv_A_rows(const StepArgs& a, int b, int4 pm, const int32_t* dsc,
                                            const float* rec, int wa0, int na, int lane) {
    constexpr int VW = V4 ? 4 : 1;
    constexpr int PRM = Q == 1 ? RAE_PRMAX : RAE_PRMAX / 2;
    constexpr bool XY = VS == 1, EXT = VS == 2;
    const int s = a.s, NJ = 2 + 2 * s, r = a.r, nv = r / VW;
    // record j's entity id and coefficients (c_j, gamma_j) in lane j (NJ <= 64: plan)
    const int sid = dsc[2 + (lane < NJ ? lane : 0)];
    const float2 cg = reinterpret_cast<const float2*>(rec + a.lay.ocoef)[lane < NJ ? lane : 0];
    // record vector of slot j: vec_0 = G1, vec_1 = G2 (bilinear) / V1, neg1 V1, neg2 V2
    const int oG1 = EXT ? a.vG1 : a.lay.oG1, oV1 = EXT ? a.vV1 : a.lay.oV1;
    const int oV2 = EXT ? a.vV2 : a.lay.oV2;
    const int vo1 = XY ? a.lay.oG2 : oV1;
    const RecBuf rb_(EXT ? a.vb : a.ex);
    const int rb0 = b * (EXT ? a.vbs : a.lay.rec);
    uint64_t M = ((uint64_t)(uint32_t)pm.y << 32) | (uint32_t)pm.x;
    for (int i = 0; i < wa0; ++i) M &= M - 1;
    while (M) {
        int jr[PRM];
        RowVec<V4, Q> pv[PRM], av[PRM], vv[PRM];
        float ab[PRM], aab[PRM];
#pragma unroll
        for (int k = 0; k < PRM; ++k) {                   // a round: every load issued first
            jr[k] = M ? __builtin_ctzll(M) : -1;
            for (int i = 0; i < na; ++i) M &= M - 1;
            if (jr[k] < 0) continue;
            const int j = jr[k];
            const int64_t e = __builtin_amdgcn_readlane(sid, j);
            pv[k].load(a.A + e * r, nv, lane);
            if (OPT == 0) av[k].load(a.aA + e * r, nv, lane); else av[k].zero();
            const int vo = rb0 + (j == 0 ? oG1 : (j == 1 ? vo1 : (j < 2 + s ? oV1 : oV2)));
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int c = lane + RAE_WAVE * q;
                rb_.load(vv[k].v[q], (c < nv ? c : 0) * VW, vo);
            }
            ab[k] = a.Ab[e];
            aab[k] = (OPT == 0) ? a.aAb[e] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < PRM; ++k) {
            const int j = jr[k];
            if (j < 0) continue;
            const int64_t e = __builtin_amdgcn_readlane(sid, j);
            const float cj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cg.x), j));
            const float gj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cg.y), j));
            RowVec<V4, Q> gr;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                vzero(gr.v[q]);
                vfma(gr.v[q], cj, vv[k].v[q]);
            }
            apply_row<OPT, V4, Q>(a.A + e * r, (OPT == 0) ? a.aA + e * r : nullptr, pv[k], av[k],
                                  gr, nv, a.lr, lane);
            if (lane == 0) ab_update<OPT>(a, (int)e, ab[k], aab[k], gj);
        }
    }
}
// the example's marked W rows wf0, wf0 + nfw, ... (bits of pmask word 2)
template <int OPT, bool V4, int Q>
__device__ __forceinline__ void priv_W_rows(const StepArgs& a, int4 pm, const int32_t* dsc,
                                            const float* rec, int wf0, int nfw, int lane) {
    constexpr int VW = V4 ? 4 : 1;
    constexpr int PRM = Q == 1 ? RAE_PRMAX : RAE_PRMAX / 2;
    const int NJ = 2 + 2 * a.s, m = a.m, nv = m / VW;
    const int p0 = dsc[1];
    const int fid = dsc[2 + NJ + (lane < 32 ? lane : 0)];   // features 0..31 (privnf <= dcap)
    typedef typename VecT<V4>::T VT;
    const VT* rv = reinterpret_cast<const VT*>(rec);
    VT ds[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int c = lane + RAE_WAVE * q;
        ds[q] = rv[a.lay.odS / VW + (c < nv ? c : 0)];
    }
    unsigned M = (unsigned)pm.z;
    for (int i = 0; i < wf0; ++i) M &= M - 1;
    while (M) {
        int fr[PRM];
        RowVec<V4, Q> pv[PRM], av[PRM];
        float xv[PRM];
#pragma unroll
        for (int k = 0; k < PRM; ++k) {
            fr[k] = M ? __builtin_ctz(M) : -1;
            for (int i = 0; i < nfw; ++i) M &= M - 1;
            if (fr[k] < 0) continue;
            const int64_t f = __builtin_amdgcn_readlane(fid, fr[k]);
            pv[k].load(a.W + f * m, nv, lane);
            if (OPT == 0) av[k].load(a.aW + f * m, nv, lane); else av[k].zero();
            xv[k] = a.values ? a.values[p0 + fr[k]] : 1.f;
        }
#pragma unroll
        for (int k = 0; k < PRM; ++k) {
            if (fr[k] < 0) continue;
            const int64_t f = __builtin_amdgcn_readlane(fid, fr[k]);
            RowVec<V4, Q> gr;
#pragma unroll
            for (int q = 0; q < Q; ++q) { vzero(gr.v[q]); vfma(gr.v[q], xv[k], ds[q]); }
            apply_row<OPT, V4, Q>(a.W + f * m, (OPT == 0) ? a.aW + f * m : nullptr, pv[k], av[k],
                                  gr, nv, a.lr, lane);
        }
    }
}
// private-row workgroup t, wave w: RAE_PRA workgroups per example for its A rows (wave i of them
// the marked rows i, i + 4 RAE_PRA, ...) + one for its W rows (wave w: w, w + 4, ...); compact:
// wave w of workgroup t takes every owned private row of example 4 t + w
template <int OPT, bool V4, int Q, int VS>
__device__ void task_private_rows(const StepArgs& a, int64_t g, int t, int w, int lane) {
    int b, sub;
    const bool compact = VS != 0 && a.privc;       // VS 0: the single-rank SP plan, never compact
    if (compact) {
        b = t * RAE_NWAVE + w;
        sub = 0;
        if (b >= a.L) return;
    } else {
        b = t / (RAE_PRA + 1);
        sub = t - b * (RAE_PRA + 1);
    }
    const int64_t slot = g % a.index_window;
    const int4 pm = reinterpret_cast<const int4*>(a.pmask)[slot * a.L + b];
    const int32_t* dsc = a.desc + (slot * a.dnx + b) * (int64_t)a.dstride;    // priv: dnx == L
    const float* rec = a.ex + (int64_t)b * a.lay.rec;
    if (compact) {
        priv_A_rows<OPT, V4, Q, VS>(a, b, pm, dsc, rec, 0, 1, lane);
        priv_W_rows<OPT, V4, Q>(a, pm, dsc, rec, 0, 1, lane);
    } else if (sub < RAE_PRA) {
        priv_A_rows<OPT, V4, Q, VS>(a, b, pm, dsc, rec, sub * RAE_NWAVE + w, RAE_NWAVE * RAE_PRA, lane);
    } else {
        priv_W_rows<OPT, V4, Q>(a, pm, dsc, rec, w, RAE_NWAVE, lane);
    }
}

}  // namespace rae
