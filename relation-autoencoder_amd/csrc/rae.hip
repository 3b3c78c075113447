// MI355X (gfx950) relation-autoencoder training path: kernels + C ABI (include/rae.h).
//
// Per training step (one func['train'] call of learning/OieInduction.py:189):
//   SP:        k_forward  one workgroup per example: encoder + decoder forward/backward
//                         (rae_sp.hpp) -> exchange record
//   bilinear:  k_bil_enc -> k_bil_mt (MFMA) -> k_bil_dec -> k_bil_mt (MFMA) -> k_bil_dp (MFMA)
//              -> k_bil_fin
//                         (rae_bilinear.hpp) -> exchange record
//   (the per-batch row index is built ahead, a window of batches at a time: k_idx_count ->
//    k_idx_scatter -> k_idx_sort -> k_build_tasks, rae_index.hpp)
//   [caller all-gathers the exchange records across data-parallel ranks]
//   k_update   one wavefront per distinct referenced row / dense decoder row / bias:
//              deterministic gradient sums + AdaGrad/SGD in place (rae_update.hpp)
//   k_dense_w + k_finalize_cost   only when lambda1/lambda2 != 0 (dense W regulariser)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/rae.h"
#include "rae_bilinear.hpp"
#include "rae_sp_split.hpp"
#include "rae_common.hpp"
#include "rae_dp.hpp"
#include "rae_index.hpp"
#include "rae_label.hpp"
#include "rae_p2p.hpp"
#include "rae_sampler.hpp"
#include "rae_sp.hpp"
#include "rae_step.hpp"
#include "rae_update.hpp"

using namespace rae;

#define RAE_VERSION 1
#ifndef RAE_UPD_WPE
#define RAE_UPD_WPE 5   // SP update: <= 102 VGPRs -> 20 waves per CU (6: 85 VGPRs spilled the
                        // Q = 2 rows of C4 -- 23.8 vs 20.2 us update; r03_ab.txt)
#endif

// ======================================================================================
// kernels
// ======================================================================================
template <bool V4, class D>
__global__ __launch_bounds__(RAE_FBT) __attribute__((amdgpu_waves_per_eu(1, 2)))
void k_forward(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t g = step_batch(a);
    if constexpr (FastSP<D>::ok) sp_example_fast<D>(a, g, blockIdx.x, smem);
    else sp_example<V4, D>(a, g, blockIdx.x, smem);
}

// ---- split SP forward for large runtime shapes (rae_sp_split.hpp) ----
template <bool V4>
__global__ __launch_bounds__(RAE_FBT) void k_sp_enc(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    sp_split_enc<V4>(a, step_batch(a), blockIdx.x, smem);
}
template <bool VEC>
__global__ __launch_bounds__(RAE_BT) void k_sp_cp(StepArgs a) {
    __shared__ __attribute__((aligned(16))) float red[RAE_BT * 4];
    sp_split_cp<VEC>(a, blockIdx.x, red);
}
template <bool V4>
__global__ __launch_bounds__(RAE_FBT) void k_sp_dec(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    sp_split_dec<V4>(a, step_batch(a), blockIdx.x / RAE_SPD_NP, blockIdx.x % RAE_SPD_NP, smem);
}
template <bool VEC>
__global__ __launch_bounds__(RAE_DW_BT) void k_sp_ctdw(StepArgs a) {
    __shared__ __attribute__((aligned(16))) float red[RAE_DW_BT * 4 + 16];
    sp_split_ctdw<VEC>(a, blockIdx.x, red);
}
// SP dense partials (data parallel): this rank's dC1 / dC2 / dWb into its records, before the exchange
__global__ __launch_bounds__(RAE_BT) void k_dpart(StepArgs a) {
    __shared__ __attribute__((aligned(16))) rae_f4 sacc[RAE_BT];
    dpart_tile(a, blockIdx.x, threadIdx.x >> 6, threadIdx.x & 63, sacc);
}
// SP wire record (data parallel): V1, V2, G1 of the whole global batch after the exchange
template <bool VEC>
__global__ __launch_bounds__(RAE_BT) void k_vrec(StepArgs a) {
    const int t = blockIdx.x * RAE_NWAVE + (threadIdx.x >> 6);
    if (t < vrec_tasks(a.L, a.r)) sp_vrec<VEC>(a, t, threadIdx.x & 63);
}

// ---- RESCAL / RESCAL+SP forward phase (rae_bilinear.hpp) ----
template <bool V4>
__global__ __launch_bounds__(RAE_FBT) void k_bil_enc(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bil_encode<V4>(a, step_batch(a), blockIdx.x, smem);
}
template <class D>
__global__ __launch_bounds__(RAE_FBT) void k_bil_enc_fast(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bil_encode_fast<D>(a, step_batch(a), blockIdx.x, smem);
}
#ifdef RAE_MT_WPE      // A/B: occupancy target of the M-tile passes (waves per SIMD)
#define RAE_MT_ATTR __attribute__((amdgpu_waves_per_eu(RAE_MT_WPE)))
#else
#define RAE_MT_ATTR
#endif
template <bool BF16, bool DIRECT = false, bool DP = true>
__global__ __launch_bounds__(RAE_MTT) RAE_MT_ATTR void k_bil_mt(StepArgs a, int pass) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bil_mt<BF16, DIRECT, DP>(a, pass, smem);
}
template <bool V4>
__global__ __launch_bounds__(RAE_DBT) void k_bil_dec(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bil_decode<V4>(a, step_batch(a), blockIdx.x, smem);
}
__host__ __device__ inline int bil_dp_tasks(int l, int m, int nib) {
    return ((l + 15) / 16) * ((m + 15) / 16) * nib;
}
template <bool BF16>
__global__ __launch_bounds__(RAE_BT) void k_bil_dp(StepArgs a) {
    const int t = blockIdx.x * RAE_NWAVE + (threadIdx.x >> 6);
    if (t >= bil_dp_tasks(a.l, a.m, a.nib)) return;
    if constexpr (BF16) bil_gemm_dp_bf16(a, t, threadIdx.x & 63);
    else bil_gemm_dp(a, t, threadIdx.x & 63);
}
template <int NJS, int MT>
__global__ __launch_bounds__((dp2_threads<NJS, MT>())) void k_bil_dp2(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bil_gemm_dp2<NJS, MT>(a, blockIdx.x, smem);
}
__global__ __launch_bounds__(RAE_BT) void k_bil_prep(StepArgs a) { bil_prep(a); }
// the R-tensor update: one wave per 16 rows (i, j) of R x all m relations (slot nCt + tile)
__host__ __device__ inline int n_ctiles(int dec, int r, int m);
__host__ __device__ inline int n_rtiles(int dec, int r, int m);
template <int OPT, bool LDS>
__global__ __launch_bounds__(RAE_BT) void k_bil_rows(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int t = blockIdx.x * RAE_NWAVE + w;
    if (t >= n_rtiles(a.dec, a.r, a.m)) return;
    const int slot = n_ctiles(a.dec, a.r, a.m) + t;
    if constexpr (LDS)
        task_bilinear_rows_lds<OPT>(a, t, slot, threadIdx.x & 63,
                                    reinterpret_cast<float*>(smem) + (size_t)w * (OPT == 0 ? 2 : 1) * 16 * a.m);
    else
        task_bilinear_rows<OPT>(a, t, slot, threadIdx.x & 63);
}
__global__ __launch_bounds__(RAE_FINT) void k_bil_fin(StepArgs a) {
    __shared__ float sdp[1024];          // NS * m <= max(RAE_FINT, m) <= 1024
    __shared__ float smt[4 * 1024];      // M-tile half sums, r <= 1024
    __shared__ float red[2 * RAE_FINW];
    bil_finish(a, blockIdx.x, sdp, smt, red);
}

// shapes with compile-time specialisations of the forward kernel (BASELINE.json configs
// C3/C5: K=100 r=200 s=20; C2: K=30 r=100 s=10); every other shape runs the runtime-shape
// instantiation of the same code
typedef FixDims<100, 200, 20> DimsC3;
typedef FixDims<30, 100, 10> DimsC2;

// row index of global batches [first, first + gridDim.x) (rae_index.hpp): blockIdx.y = table
// (0 A / Ab, 1 W; 2: the example descriptors), blockIdx.z = slice of RAE_IDX_EPS examples or
// hash partition
__global__ __launch_bounds__(RAE_BT) void k_idx_count(StepArgs a, int64_t first) {
    __shared__ int sh[RAE_IDX_HMAX + RAE_IDX_EPS + 1];
    const int64_t g = first + blockIdx.x;
    if (blockIdx.y == 2) {
        build_batch_desc<RAE_BT>(a, g, g % a.index_window, blockIdx.z);
        return;
    }
    index_count<RAE_BT>(a, g, g % a.index_window, blockIdx.y, blockIdx.z, sh);
}
__global__ __launch_bounds__(RAE_BT) void k_idx_scatter(StepArgs a, int64_t first) {
    __shared__ int sh[2 * RAE_IDX_HMAX + RAE_IDX_EPS + 1 + 32];
    const int64_t g = first + blockIdx.x;
    index_scatter<RAE_BT>(a, g, g % a.index_window, blockIdx.y, blockIdx.z, sh);
}
template <bool BIG>
__global__ __launch_bounds__(RAE_FBT) void k_idx_sort(StepArgs a, int64_t first) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t g = first + blockIdx.x;
    index_sort<RAE_FBT, BIG>(a, g, g % a.index_window, blockIdx.y, blockIdx.z, smem);
}
// the update's dispatch tables of the same batches (after k_idx_sort): blockIdx.y = range of
// RAE_TASK_PER table entries
__global__ __launch_bounds__(RAE_BT) void k_build_tasks(StepArgs a, int64_t first) {
    __shared__ int sh[6 * (RAE_IDX_HMAX + 1)];
    const int64_t g = first + blockIdx.x;
    build_batch_tasks<RAE_BT>(a, g, g % a.index_window, blockIdx.y, sh);
}

// partitioned data-parallel update (rae_dp.hpp): the peers' row lists of global batches
// [first, first + gridDim.x); blockIdx.y = peer, blockIdx.z = direction * 2 + table
__global__ __launch_bounds__(RAE_FBT) void k_build_dplists(StepArgs a, int64_t first) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t g = first + blockIdx.x;
    build_dp_list<RAE_FBT>(a, g, g % a.index_window, blockIdx.z >> 1, blockIdx.y, blockIdx.z & 1,
                           smem);
}
// peer-to-peer exchange (rae_p2p.hpp)
__global__ __launch_bounds__(RAE_BT) void k_p2p_recs(StepArgs a) { p2p_push_records(a); }
__global__ __launch_bounds__(RAE_BT) void k_p2p_rows(StepArgs a) { p2p_push_rows(a); }
__global__ __launch_bounds__(RAE_BT) void k_p2p_pre(StepArgs a, int prologue, int nmb) {
    p2p_pre(a, prologue, nmb);
}
__global__ __launch_bounds__(64) void k_p2p_signal(StepArgs a, int kind) { p2p_signal(a, kind); }
__global__ __launch_bounds__(64) void k_p2p_wait(StepArgs a, int kind, unsigned per) {
    p2p_wait(a, kind, per);
}
template <bool PACK>
__global__ __launch_bounds__(RAE_BT) void k_dp_move(StepArgs a) {
    const int64_t t = (int64_t)blockIdx.x * RAE_NWAVE + (threadIdx.x >> 6);
    dp_move<PACK>(a, t, threadIdx.x & 63);
}

__host__ __device__ inline int n_ctiles(int dec, int r, int m) {
    return dec != RAE_DEC_RESCAL ? 2 * ((r + 15) / 16) * ((m + 15) / 16) : 0;
}
__host__ __device__ inline int n_rtiles(int dec, int r, int m) {
    return dec != RAE_DEC_SP ? (r * r + 15) / 16 : 0;    // 16 rows of R/C x all m each
}

#ifdef RAE_STAMPS
#define RAE_WAVE_END()                                                                      \
    do {                                                                                    \
        if (a.stamps && lane == 0)      /* end of the wave's LAST task */                    \
            a.stamps[(size_t)gw * 4 + 2] = __builtin_amdgcn_s_memrealtime();                 \
    } while (0)
#else
#define RAE_WAVE_END() do { } while (0)
#endif

// Update launch layout (workgroups of RAE_NWAVE = 4 waves), in dispatch order:
//   [0, nT)              one dense 16x16 tile per workgroup: C1/C2 tiles, then Wb tiles
//                        (no row index needed: they start at once; K = batch split 4 ways)
//   [nT, nT + nP)        one wave task each, no row index needed: the cost
//   then, after the batch's index header: one workgroup per very heavy A row, per very heavy
//   W row, and the remaining workgroups' waves grid-stride over the heavy A rows, heavy W
//   rows, light A rows, light W rows (one row per wave)
__host__ __device__ inline int update_wave_free_tasks(int dec, int r, int m) {
    return 1;                                            // the cost (R rows: k_bil_rows)
}
#ifndef RAE_SPLIT_RM
#define RAE_SPLIT_RM 32768    // r*m above which the SP forward runs split (rae_sp_split.hpp)
#endif
#ifndef RAE_ROWS_FIRST
#define RAE_ROWS_FIRST 0      // update: dispatch the row tasks ahead of the dense tiles
#endif
#ifndef RAE_ROWPCT
#define RAE_ROWPCT 100        // row-task waves per 100 dispatch-table capacity entries
#endif
#ifndef RAE_HCH
#define RAE_HCH 128           // very heavy rows above this many records are split into chunks
#endif
#ifndef RAE_PRIV_MAXL
#define RAE_PRIV_MAXL 4096    // private rows (auto) below this global batch (equal at 4096)
#endif
#ifndef RAE_HCH_MINL
#define RAE_HCH_MINL 2048     // ... in plans with a global batch of at least this many examples
#endif
#ifndef RAE_NVC_MIN
#define RAE_NVC_MIN 32
#endif
#ifndef RAE_NVC_DIV
#define RAE_NVC_DIV 2         // very heavy row workgroup slots: max(32, L / RAE_NVC_DIV)
#endif
#ifndef RAE_UPD_WGCAP
#define RAE_UPD_WGCAP 6144    // row-task workgroups (grid-stride beyond; 1536 = one resident round)
#endif
#ifndef RAE_PRIV_LAST
#define RAE_PRIV_LAST 1       // private-row workgroups dispatched after every other update task
#endif
#ifndef RAE_PRIV_ROWW
#define RAE_PRIV_ROWW 4       // private rows: row-task waves per example of the global batch
#endif
// own: the share of the global batch's rows this rank updates (1 / G for the partitioned
// data-parallel update: the row grid and the very heavy slots are sized from it)
__host__ __device__ inline int64_t update_grid(int dec, int r, int m, int TC, int NVC, int L,
                                               int priv, int privc, int own) {
    const int nT = n_ctiles(dec, r, m) + (m + 15) / 16;
    const int nP = (update_wave_free_tasks(dec, r, m) + RAE_NWAVE - 1) / RAE_NWAVE;
    int64_t rows = ((int64_t)TC * RAE_ROWPCT / 100 / own + RAE_NWAVE - 1) / RAE_NWAVE;
    // with the private rows (StepArgs::priv) taken per example by leading workgroups, the
    // dispatch table keeps ~5 % of the rows: a smaller row grid, grid-striding when a batch has more
    if (priv) {
        const int64_t pr = ((int64_t)L * RAE_PRIV_ROWW / own + RAE_NWAVE - 1) / RAE_NWAVE;
        if (pr < rows) rows = pr;
    }
    if (RAE_UPD_WGCAP > 0 && rows > RAE_UPD_WGCAP) rows = RAE_UPD_WGCAP;
    return (int64_t)nT + nP + NVC + rows + (priv ? (int64_t)priv_workgroups(privc, L) : 0);
}

// LDS of one update workgroup: workgroup tasks' partials (a row: Q vectors per lane, or a tile:
// 4 floats per lane, per wave) + the Ab partials
template <bool V4, int Q>
__host__ __device__ constexpr int update_lds_floats() {
    return (RAE_NWAVE * Q * RAE_WAVE * (V4 ? 4 : 1) > RAE_NWAVE * RAE_WAVE * 4
                ? RAE_NWAVE * Q * RAE_WAVE * (V4 ? 4 : 1) : RAE_NWAVE * RAE_WAVE * 4) + RAE_NWAVE;
}

// wg0 / ngrid: this workgroup's index and the number of workgroups of the update's own grid
// (the fused bilinear kernel puts the update's workgroups in front of the R-tile ones)
// VS: where the A-row tasks find the record vectors (rae_update.hpp entity_accum): 0 SP records
// (single rank), 1 bilinear records, 2 the SP wire record's vector buffer (data parallel)
template <int OPT, bool V4, int Q, int VS, bool PP = false>
__device__ __forceinline__ void update_body(const StepArgs& a, int wg0, int ngrid, float* lds) {
    typedef typename VecT<V4>::T VT;
    constexpr int kF = update_lds_floats<V4, Q>() - RAE_NWAVE;
    float* sgb = lds + kF;
    VT* spart = reinterpret_cast<VT*>(lds);
    const int lane = threadIdx.x & 63;
    // wave / workgroup indices as provably uniform values: every task index, row id and
    // record offset derived from them is then scalar (s_load of the segment, SGPR soffsets,
    // scalar branches) instead of VGPR-resident and exec-masked
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int wgp = __builtin_amdgcn_readfirstlane(wg0);
    const int gw = wgp * RAE_NWAVE + w;
    const int64_t g = step_batch(a);
    if (a.priv) {                 // private rows: (RAE_PRA + 1) L workgroups (1 per example when
                                  // compact), dispatched first (RAE_PRIV_LAST 0) or last
        const int nX = priv_workgroups(a.privc, a.L);
        const int x = RAE_PRIV_LAST ? wgp - (ngrid - nX) : wgp;
        if (x >= 0 && x < nX) {
            task_private_rows<OPT, V4, Q, VS>(a, g, x, w, lane);
            return;
        }
        if (!RAE_PRIV_LAST) wgp -= nX;
        ngrid -= nX;
    }
    const int64_t ex0 = g * (int64_t)a.L;
    const int mt = (a.m + 15) / 16, rt = (a.r + 15) / 16;
    const int nCt = n_ctiles(a.dec, a.r, a.m);
    const int nT = nCt + mt;
    const int nPt = update_wave_free_tasks(a.dec, a.r, a.m);
    const int nP = (nPt + RAE_NWAVE - 1) / RAE_NWAVE;
    // logical task order: tiles, cost, very heavy rows, row waves; RAE_ROWS_FIRST dispatches the
    // row part first (physical order: very heavy rows, row waves, tiles, cost)
    int wg = wgp;
    if (RAE_ROWS_FIRST) {
        const int nrow = ngrid - nT - nP;
        wg = wgp < nrow ? nT + nP + wgp : wgp - nrow;
    }
    const int64_t slot = g % a.index_window;
#ifdef RAE_STAMPS
    unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#define RAE_FIRST(kind_)                                                                    \
    do {                                                                                    \
        if (a.stamps && lane == 0) {                                                        \
            a.stamps[(size_t)gw * 4 + 0] = t_start;                                         \
            a.stamps[(size_t)gw * 4 + 1] = (unsigned long long)(kind_);                     \
        }                                                                                   \
    } while (0)
#else
#define RAE_FIRST(kind_) do { } while (0)
#endif
    if (wg < nT) {                                            // dense tiles
        RAE_FIRST(wg < nCt ? 0 : 2);
        if (VS == 2 && a.dpart) {        // dense partials: the ranks' sums (wave 0), no K chain
            if (w == 0) {
                if (wg < nCt) {
                    const int which = wg / (rt * mt), ti = wg - which * rt * mt;
                    tile_from_partials<OPT>(a, which ? a.C2 : a.C1, which ? a.aC2 : a.aC1, a.r, false,
                                            which * a.r * a.m, (ti / mt) * 16, (ti % mt) * 16, wg, lane);
                } else {
                    tile_from_partials<OPT>(a, a.Wb, a.aWb, 1, true, 2 * a.r * a.m, 0,
                                            (wg - nCt) * 16, 0, lane);
                }
            }
            RAE_WAVE_END();
            return;
        }
        if (wg < nCt) {
            const int which = wg / (rt * mt), ti = wg - which * rt * mt;
            wg_tile<OPT>(a, which ? a.C2 : a.C1, which ? a.aC2 : a.aC1, a.r,
                         which ? a.lay.odw2 : a.lay.odw1, false, (ti / mt) * 16, (ti % mt) * 16,
                         wg, w, lane, reinterpret_cast<rae_f4*>(spart));
        } else {
            wg_tile<OPT>(a, a.Wb, a.aWb, 1, 0, true, 0, (wg - nCt) * 16, 0, w, lane,
                         reinterpret_cast<rae_f4*>(spart));
        }
        RAE_WAVE_END();
        return;
    }
    if (wg < nT + nP) {                                       // the cost (one workgroup)
        if (wg == nT) {
            RAE_FIRST(3);
            task_cost(a, w, lane, reinterpret_cast<double*>(lds));
        }
        RAE_WAVE_END();
        return;
    }
    // row tasks from the slot's dispatch table (build_batch_tasks): the task entry and the
    // table header are loaded together -- one round trip from wave start to the row's segment
    const int u = wg - nT - nP;
    const int4* thp = reinterpret_cast<const int4*>(a.thdr) + slot;
    if (u < a.NVC) {                                          // very heavy rows
        int4 seg = reinterpret_cast<const int4*>(a.vtask)[slot * a.NVC + u];
        const int4 th = *thp;
        if (u >= th.y) return;
        const bool isA = seg.x >= 0;
        RAE_FIRST(isA ? 8 : 9);
        if (isA) {
            wg_entity_row<OPT, V4, Q, VS, PP>(a, slot, seg, w, lane, spart, sgb);
        } else {
            seg.x = ~seg.x;
            wg_feature_row<OPT, V4, Q, PP>(a, ex0, slot, seg, w, lane, spart);
        }
        RAE_WAVE_END();
        return;
    }
    // wave tasks: a wave with several (large global batches: the grid's row part is capped
    // near one resident wave per slot) loads its next task's segment while it works on the
    // current one
    const int nw = (ngrid - nT - nP - a.NVC) * RAE_NWAVE;
    const int4* tk = reinterpret_cast<const int4*>(a.task) + slot * a.TC;
    int t = (u - a.NVC) * RAE_NWAVE + w;
    int4 seg = tk[t < a.TC ? t : a.TC - 1];
    const int T = thp->x;
    for (; t < T; t += nw) {
        int4 cur = seg;
        if (t + nw < T) seg = tk[t + nw];
        const bool curA = cur.x >= 0;
        if (!curA) cur.x = ~cur.x;
        RAE_FIRST((curA ? 4 : 5) + (cur.z - cur.y > RAE_HEAVY ? 2 : 0));
        if (curA) task_entity_row<OPT, V4, Q, VS, PP>(a, slot, cur, lane);
        else task_feature_row<OPT, V4, Q, PP>(a, ex0, slot, cur, lane);
        RAE_WAVE_END();
    }
#undef RAE_FIRST
}

// SP and bilinear variants (the bilinear R-row tasks need more registers).
#if RAE_UPD_WPE > 0
#define RAE_UPD_ATTR __attribute__((amdgpu_waves_per_eu(RAE_UPD_WPE, RAE_UPD_WPE)))
#else
#define RAE_UPD_ATTR
#endif
template <int OPT, bool V4, int Q, bool WIRE>
__global__ __launch_bounds__(RAE_BT) RAE_UPD_ATTR void k_update(StepArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[update_lds_floats<V4, Q>()];
    update_body<OPT, V4, Q, WIRE ? 2 : 0, WIRE>(a, blockIdx.x, gridDim.x, lds);
    if (WIRE && a.pipe) p2p_stores_done();   // the row pushes acknowledged before the wave ends
}
template <int OPT, bool V4, int Q, bool PP = false>
__global__ __launch_bounds__(RAE_BT) void k_update_bil(StepArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[update_lds_floats<V4, Q>()];
    update_body<OPT, V4, Q, 1, PP>(a, blockIdx.x, gridDim.x, lds);
    if (PP && a.pipe) p2p_stores_done();
}
// The bilinear decoders' update phase in ONE launch: workgroups [0, gu) run k_update_bil's tasks
// (Wb tiles, cost, A / W rows: latency-bound chains), the rest k_bil_rows' R tiles (16 rows
// (i, j) x all m per wave: the HBM-heavy R sweep) -- the two have no data in common, so the
// row chains run under the R sweep instead of after it.  Dynamic LDS: the R tiles' (DMA'd R and
// accumulator rows); an update workgroup carves its partials from the same allocation.
template <int OPT, bool V4, int Q, bool PP = false>
__global__ __launch_bounds__(RAE_BT) void k_bil_update(StepArgs a, int gu) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wg = __builtin_amdgcn_readfirstlane(blockIdx.x);
    if (wg < gu) {
        update_body<OPT, V4, Q, 1, PP>(a, wg, gu, reinterpret_cast<float*>(smem));
        if (PP && a.pipe) p2p_stores_done();
        return;
    }
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int t = (wg - gu) * RAE_NWAVE + w;
    if (t >= n_rtiles(a.dec, a.r, a.m)) return;
    const int slot = n_ctiles(a.dec, a.r, a.m) + t;
    task_bilinear_rows_lds<OPT>(a, t, slot, threadIdx.x & 63,
                                reinterpret_cast<float*>(smem) + (size_t)w * (OPT == 0 ? 2 : 1) * 16 * a.m);
}
#ifndef RAE_BIL_FUSED_UPD
#define RAE_BIL_FUSED_UPD 1   // bilinear update phase as one launch (k_bil_update)
#endif

// rows split into chunks (StepArgs::hch): each row's chunk sums combined in order + its update
template <int OPT, bool V4, int Q, bool PP = false>
__global__ __launch_bounds__(RAE_BT) void k_heavy_fin(StepArgs a) {
    heavy_fin<OPT, V4, Q, PP>(a, blockIdx.x * RAE_NWAVE + (threadIdx.x >> 6), threadIdx.x & 63);
    if (PP && a.pipe) p2p_stores_done();
}

// Dense W sweep (lambda1/lambda2 != 0): g = sparse-part scratch + l1adj*sgn(W) + 2*l2adj*W,
// reset the scratch, L1/L2 partials of the old W per block (fixed grid -> deterministic).
template <int OPT>
__global__ __launch_bounds__(RAE_BT) void k_dense_w(StepArgs a) {
    __shared__ double red[2 * RAE_NWAVE];
    const int64_t total = a.d * (int64_t)a.m;
    double l1 = 0.0, l2 = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)RAE_BT + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * RAE_BT) {
        const float w = a.W[i];
        const float gg = a.gWs[i] + a.l1adj * sgnf(w) + 2.f * a.l2adj * w;
        a.gWs[i] = 0.f;
        l1 += fabsf(w);
        l2 += (double)w * w;
        float ac = (OPT == 0) ? a.aW[i] : 0.f;
        a.W[i] = opt_update<OPT>(w, &ac, gg, a.lr);
        if (OPT == 0) a.aW[i] = ac;
    }
    l1 = wave_sum_d(l1);
    l2 = wave_sum_d(l2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[2 * w] = l1;
        red[2 * w + 1] = l2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s1 = 0.0, s2 = 0.0;
        for (int i = 0; i < RAE_NWAVE; ++i) {
            s1 += red[2 * i];
            s2 += red[2 * i + 1];
        }
        const int slot = a.nregC + blockIdx.x;
        a.regpart[2 * slot] = s1;
        a.regpart[2 * slot + 1] = s2;
    }
}

// cost = base + lambda1*adjust*L1 + lambda2*adjust*L2   (learning/OieInduction.py:134-135)
__global__ void k_finalize_cost(StepArgs a) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double L1 = 0.0, L2 = 0.0;
    if (a.ext_reg)
        for (int i = 0; i < a.nregC; ++i) {
            L1 += a.regpart[2 * i];
            L2 += a.regpart[2 * i + 1];
        }
    for (int i = 0; i < a.nregW; ++i) {
        L1 += a.regpart[2 * (a.nregC + i)];
        L2 += a.regpart[2 * (a.nregC + i) + 1];
    }
    const int64_t batch = step_batch(a);
    a.costs[batch] = (float)((double)*a.base_cost + (double)a.l1adj * L1 + (double)a.l2adj * L2);
}

// STREAM-style copy (measurement helper): 4 float4 nontemporal loads in flight per lane
// before the stores, one 1024-vector block per workgroup -- the fastest of the forms
// tools/probes/stream_probe.hip measured on MI355X (5.88 TB/s at 2 GiB)
typedef float rae_v4f __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_copy(const rae_v4f* __restrict__ src,
                                                     rae_v4f* __restrict__ dst, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 1024;
    for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
        rae_v4f v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = i + 256 * u;
            if (k < n) v[u] = __builtin_nontemporal_load(src + k);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = i + 256 * u;
            if (k < n) __builtin_nontemporal_store(v[u], dst + k);
        }
    }
}

// bf16 MFMA throughput probe (measurement helper): every wave runs `iters` rounds of 8
// independent v_mfma_f32_16x16x32_bf16 chains (enough in flight to cover the dependent-issue
// latency), operands in registers, one result per wave stored so nothing is dead code
__global__ __launch_bounds__(256) void k_mfma_probe(int64_t iters, float* sink) {
    typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    bf8 x, y;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        x[e] = (__bf16)(1e-3f * (float)((threadIdx.x + e) & 7));
        y[e] = (__bf16)(1e-3f * (float)((threadIdx.x * 3 + e) & 7));
    }
    f4 acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = f4{0.f, 0.f, 0.f, 0.f};
    for (int64_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc[c], 0, 0, 0);
    }
    float t = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) t += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    if ((threadIdx.x & 63) == 0) sink[blockIdx.x * 4 + (threadIdx.x >> 6)] = t;
}

__global__ void k_add_cursor(int64_t* cursor, int64_t count) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *cursor += count;
}
__global__ void k_set_cursor(int64_t* cursor, int64_t v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *cursor = v;
}

// ======================================================================================
// host side / C ABI
// ======================================================================================
static thread_local std::string g_last_error;

static int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess)                                                              \
            return fail(RAE_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_));       \
    } while (0)

struct rae_plan {
    rae_config cfg;
    rae_buffers buf;
    StepArgs args;
    int64_t* d_cursor = nullptr;
    int64_t cursor_moves = 0;  // host count of rae_set_cursor / rae_advance_cursor calls
    int64_t* d_zero = nullptr;
    int* d_err = nullptr;
    int* h_err = nullptr;   // pinned host word of rae_check_on
    unsigned* d_sig = nullptr;  // peer-to-peer signal counters (own allocation: IPC-exported)
    bool peers_set = false;     // rae_set_peer called for every other rank
    int peers_mask = 0;
    char* ws = nullptr;
    size_t smem_fwd = 0;
    size_t smem_idx = 0;    // k_idx_sort<true> (partitions of more than RAE_IDX_FAST keys)
    size_t smem_idxf = 0;   // k_idx_sort<false>
    size_t smem_dec = 0;
    size_t smem_mt = 0;     // k_bil_mt: one 8 x 16 x m block of R in LDS
    size_t smem_mt0 = 0;    // ... its first pass (no transposed image for dP): less LDS per WG
    bool mt_direct = false; // fp32 blocks beyond LDS (m > 320): k_bil_mt reads R from L2
    bool sp_split = false;  // SP forward as enc -> GEMM -> dec -> GEMM -> fin (large shapes)
    size_t smem_spe = 0;    // k_sp_enc
    size_t smem_spd = 0;    // k_sp_dec (one negative side)
    bool mt_bf16 = false;
    int grid_fwd = 0, grid_update = 0, grid_dense = 0;
    bool v4 = false;
    int q = 1;
    int dp2 = 0;            // bf16 dP kernel: 0 none (bil_gemm_dp*), 1 k_bil_dp2<7,7>, 2 <8,8>
    unsigned long long* stamps_fwd = nullptr;
    unsigned long long* stamps_upd = nullptr;
    hipEvent_t t_start = nullptr, t_stop = nullptr;   // armed by rae_time_next for ONE call
};

// Main-step launches go through here.  With a timing pair armed (rae_time_next) the kernels
// are launched by hipExtLaunchKernelGGL: the start event takes the first kernel's dispatch
// begin timestamp, the stop event the last kernel's end timestamp -- the kernels' execution
// span as rocprofv3 --kernel-trace reports it, without the event packets' own overhead.
#define RAE_LAUNCH(p, K, g, b, sh, st, ...)                                                 \
    do {                                                                                  \
        if ((p)->t_stop) {                                                                \
            hipEvent_t e0_ = (p)->t_start;                                                \
            (p)->t_start = nullptr;                                                       \
            hipExtLaunchKernelGGL(K, g, b, sh, st, e0_, (p)->t_stop, 0, __VA_ARGS__);      \
        } else {                                                                          \
            hipLaunchKernelGGL(K, g, b, sh, st, __VA_ARGS__);                             \
        }                                                                                 \
    } while (0)

extern "C" const char* rae_last_error(void) { return g_last_error.c_str(); }
extern "C" int rae_version(void) { return RAE_VERSION; }
#ifndef RAE_BUILD_ID
#define RAE_BUILD_ID "unversioned"
#endif
// a diagnostic build (phase stamps, tools/phase_stamps.py) says so in its id: the Python
// binding loads such a library only when RAE_LIB names it explicitly
#ifdef RAE_DIAG
#define RAE_BUILD_KIND "diag-"
#else
#define RAE_BUILD_KIND ""
#endif
__attribute__((used)) static const char g_build_id[] = "RAE_BUILD_ID:" RAE_BUILD_KIND RAE_BUILD_ID;
extern "C" const char* rae_build_id(void) { return g_build_id + 13; }

// the SP decoder exchanges wire records between ranks (rae_step.hpp): V1 / V2 / G1 are
// recomputed after the all-gather instead of crossing xGMI (1); with dense partials (2) the
// records carry each rank's partial dC1 / dC2 / dWb block instead of every example's dw1 / dw2
static int wire_records(const rae_config& c) {
    if (c.decoder != RAE_DEC_SP || c.world_size <= 1) return 0;
    if (c.dp_dense == RAE_DPDENSE_RECORDS) return 1;
    if (c.dp_dense == RAE_DPDENSE_PARTIALS) return 2;
    // partials when their chunk is at most half of dw1 / dw2 (l >~ 2 m): below that they move
    // about as many bytes and k_dpart (~4 us at C3, l = 100) sits on the critical path
    const int pc = align4((dense_partial_floats(c.embed, c.relations) + c.batch_size - 1) /
                          c.batch_size);
    return pc <= align4(c.embed) ? 2 : 1;
}
extern "C" int64_t rae_exchange_record_floats(const rae_config* cfg) {
    if (!cfg) return -1;
    return make_layout(cfg->decoder, cfg->relations, cfg->embed, cfg->neg_samples,
                       wire_records(*cfg), cfg->batch_size).rec;
}
extern "C" int64_t rae_exchange_floats(const rae_config* cfg) {
    if (!cfg) return -1;
    return rae_exchange_record_floats(cfg) * (int64_t)cfg->batch_size * cfg->world_size;
}

static int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

extern "C" int rae_plan_create(const rae_config* cfg, const rae_buffers* buf, rae_plan** out) {
    if (!cfg || !buf || !out) return fail(RAE_E_INVALID, "null argument");
    const rae_config& c = *cfg;
    if (c.decoder < 0 || c.decoder > 2) return fail(RAE_E_INVALID, "decoder must be 0..2");
    if (c.optimizer < 0 || c.optimizer > 1) return fail(RAE_E_INVALID, "optimizer must be 0..1");
    if (c.relations < 1 || c.relations > 1024)
        return fail(RAE_E_INVALID, "relations must be in [1, 1024]");
    if (c.embed < 1 || c.embed > 1024) return fail(RAE_E_INVALID, "embed must be in [1, 1024]");
    if (c.neg_samples < 1) return fail(RAE_E_INVALID, "neg_samples must be >= 1");
    if (c.sp_forward < RAE_SPFWD_AUTO || c.sp_forward > RAE_SPFWD_SPLIT ||
        c.bil_dp < RAE_BILDP_AUTO || c.bil_dp > RAE_BILDP_MTILE ||
        c.bil_prep < RAE_BILPREP_AUTO || c.bil_prep > RAE_BILPREP_KERNEL ||
        c.dp_update < RAE_DPUPD_REPLICATED || c.dp_update > RAE_DPUPD_PARTITIONED ||
        c.priv_rows < RAE_PRIV_AUTO || c.priv_rows > RAE_PRIV_ON ||
        c.dp_dense < RAE_DPDENSE_AUTO || c.dp_dense > RAE_DPDENSE_PARTIALS ||
        c.heavy_chunk < RAE_HCHUNK_AUTO || c.heavy_chunk > RAE_HCHUNK_ON ||
        c.dp_xchg < RAE_XCHG_COLLECTIVE || c.dp_xchg > RAE_XCHG_P2P_PIPE)
        return fail(RAE_E_INVALID, "unknown kernel form (sp_forward / bil_dp / bil_prep / dp_update / "
                                   "priv_rows / dp_dense / heavy_chunk / dp_xchg)");
    if (c.dp_xchg != RAE_XCHG_COLLECTIVE &&
        (c.dp_update != RAE_DPUPD_PARTITIONED || c.world_size > 31 || c.embed % 4 ||
         c.relations % 4 || c.embed > 512 || c.relations > 512))
        return fail(RAE_E_INVALID, "the peer-to-peer exchange runs the partitioned update "
                                   "(world_size <= 31; embed and relations multiples of 4, <= 512)");
    // the pipelined form marks a row's reading peers in one byte, and its update pushes rows
    // from the row tasks only (not from the private-row tasks)
    if (c.dp_xchg == RAE_XCHG_P2P_PIPE && (c.world_size > 8 || c.priv_rows == RAE_PRIV_ON))
        return fail(RAE_E_INVALID, "the pipelined peer-to-peer exchange needs world_size <= 8 and "
                                   "private rows off");
    if (c.bil_dp == RAE_BILDP_MTILE && !(c.decoder != RAE_DEC_SP && c.mfma_bf16 && c.relations <= 128))
        return fail(RAE_E_INVALID, "bil_dp MTILE needs a bf16 bilinear plan with relations <= 128");
    if (c.dp_update == RAE_DPUPD_PARTITIONED && (c.lambda1 != 0.f || c.lambda2 != 0.f))
        return fail(RAE_E_INVALID, "the partitioned data-parallel update needs lambda1 = lambda2 = 0 "
                                   "(a regulariser makes every W row change every step)");
    if (c.batch_size < 1 || c.world_size < 1 || c.rank < 0 || c.rank >= c.world_size)
        return fail(RAE_E_INVALID, "bad batch_size/world_size/rank");
    if (c.n_examples < (int64_t)c.batch_size * c.world_size)
        return fail(RAE_E_INVALID, "fewer examples than one global batch");
    if (c.n_entities < 1 || c.n_features < 1 || c.n_entities >= (1ll << 31))
        return fail(RAE_E_INVALID, "bad n_entities / n_features");
    if (!buf->W || !buf->Wb || !buf->A || !buf->Ab || !buf->indptr || !buf->indices ||
        !buf->args1 || !buf->args2 || !buf->exchange || !buf->costs)
        return fail(RAE_E_INVALID, "missing required buffer");
    if (c.decoder != RAE_DEC_RESCAL && (!buf->C1 || !buf->C2))
        return fail(RAE_E_INVALID, "C1/C2 required for this decoder");
    if (c.decoder != RAE_DEC_SP && !buf->R3) return fail(RAE_E_INVALID, "R/C tensor required");
    if (c.optimizer == RAE_OPT_ADAGRAD &&
        (!buf->acc_W || !buf->acc_Wb || !buf->acc_A || !buf->acc_Ab ||
         (c.decoder != RAE_DEC_RESCAL && (!buf->acc_C1 || !buf->acc_C2)) ||
         (c.decoder != RAE_DEC_SP && !buf->acc_R3)))
        return fail(RAE_E_INVALID, "AdaGrad accumulators required");

    {
        const RecLayout lay = make_layout(c.decoder, c.relations, c.embed, c.neg_samples,
                                          wire_records(c), c.batch_size);
        if ((int64_t)lay.rec * c.batch_size * c.world_size >= (1ll << 31) ||
            (int64_t)3 * align4(c.embed) * c.batch_size * c.world_size >= (1ll << 31))
            return fail(RAE_E_INVALID, "exchange buffer exceeds 2^31 floats (global batch too large)");
    }
    rae_plan* p = new rae_plan();
    p->cfg = c;
    p->buf = *buf;
    StepArgs& a = p->args;
    memset(&a, 0, sizeof(a));
    const int L = c.batch_size * c.world_size;
    const int NJ = 2 + 2 * c.neg_samples;
    a.dec = c.decoder;
    a.opt = c.optimizer;
    a.N = c.n_examples;
    a.d = c.n_features;
    a.n = c.n_entities;
    a.m = c.relations;
    a.r = c.embed;
    a.s = c.neg_samples;
    a.l = c.batch_size;
    a.L = L;
    a.rank = c.rank;
    a.lr = c.learning_rate;
    a.alpha = c.alpha;
    // adjust = batch / N_train (learning/OieInduction.py:131) with the GLOBAL batch
    const double adjust = (double)L / (double)c.n_examples;
    a.l1adj = (float)(c.lambda1 * adjust);
    a.l2adj = (float)(c.lambda2 * adjust);
    a.invD = (float)(1.0 / (4.0 * L + 2.0 * L * c.neg_samples));
    a.ext_reg = c.ext_reg;
    a.reg_on = (c.lambda1 != 0.f || c.lambda2 != 0.f) ? 1 : 0;
    a.indptr = buf->indptr;
    a.indices = buf->indices;
    a.values = buf->values;
    a.args1 = buf->args1;
    a.args2 = buf->args2;
    a.neg1 = buf->neg1;
    a.neg2 = buf->neg2;
    a.neg_mode = c.neg_mode;
    a.neg_stride = c.neg_stride;
    a.W = buf->W; a.Wb = buf->Wb; a.A = buf->A; a.Ab = buf->Ab;
    a.C1 = buf->C1; a.C2 = buf->C2; a.R3 = buf->R3;
    a.aW = buf->acc_W; a.aWb = buf->acc_Wb; a.aA = buf->acc_A; a.aAb = buf->acc_Ab;
    a.aC1 = buf->acc_C1; a.aC2 = buf->acc_C2; a.aR3 = buf->acc_R3;
    a.ex = buf->exchange;
    a.lay = make_layout(c.decoder, c.relations, c.embed, c.neg_samples, wire_records(c),
                        c.batch_size);
    // the update's record vectors: in the records, or (wire record) the vector buffer
    a.vb = a.ex;
    a.vbs = a.lay.rec;
    a.vG1 = a.lay.oG1; a.vV1 = a.lay.oV1; a.vV2 = a.lay.oV2; a.vG2 = a.lay.oG2;
    if (a.lay.wire) {
        const int r4 = align4(c.embed);
        a.vbs = 3 * r4;
        a.vV1 = 0; a.vV2 = r4; a.vG1 = 2 * r4; a.vG2 = 0;
    }
    // the forward's dw1 / dw2: in the records, or (dense partials) a rank-local buffer
    a.dpart = a.lay.wire == 2 ? 1 : 0;
    a.dwb = a.ex;
    a.dws = a.lay.rec;
    a.dw1o = a.lay.odw1; a.dw2o = a.lay.odw2;
    if (a.dpart) {
        a.dws = 2 * align4(c.embed);
        a.dw1o = 0; a.dw2o = align4(c.embed);
    }
    a.costs = buf->costs;
    p->v4 = (c.relations % 4 == 0) && (c.embed % 4 == 0);
    {
        const int vw = p->v4 ? 4 : 1;
        const int qa = ceil_div(c.embed / vw, 64), qm = ceil_div(c.relations / vw, 64);
        const int q = qa > qm ? qa : qm;
        if (q > 2) {
            delete p;
            return fail(RAE_E_INVALID,
                        "relations/embed are limited to 512 (128 when not multiples of 4)");
        }
        p->q = q <= 1 ? 1 : 2;
    }

    // row-index partitions: ~1024 records per partition on average, LDS holds RAE_KCAP
    a.RA = L * NJ;
    a.RW = c.max_batch_nnz > 0 ? c.max_batch_nnz : 1;
    a.HA = index_partitions(a.RA);
    a.HW = index_partitions(a.RW);
    a.G = c.world_size;
    a.part = c.dp_update == RAE_DPUPD_PARTITIONED ? 1 : 0;
    if (a.HA > RAE_IDX_HMAX || a.HW > RAE_IDX_HMAX) {
        delete p;
        return fail(RAE_E_INVALID, "global batch too large for the row index (more than " +
                                   std::to_string(RAE_IDX_HMAX * RAE_IDX_PART) +
                                   " records of one table)");
    }
    {
        const int64_t nb = c.n_examples / L;
        // partitioned: the peers' row lists take 2 G (LA + LW) ints per slot -> a shorter window
        int64_t win = c.index_window > 0 ? c.index_window : (a.part ? 256 : 2048);
        if (win > nb) win = nb;
        a.index_window = win < 1 ? 1 : win;
    }
    int bbits = 1;
    while ((1 << bbits) < L) ++bbits;
    a.posbits = 31 - bbits;
    if (c.max_row_nnz >= (1 << a.posbits)) {
        delete p;
        return fail(RAE_E_INVALID, "an example has too many features for the record encoding");
    }
    // parameter / dense-row partial slots for the regulariser
    a.nregC = n_ctiles(c.decoder, c.embed, c.relations) + n_rtiles(c.decoder, c.embed, c.relations);
    p->grid_dense = 1024;
    a.nregW = a.reg_on ? p->grid_dense : 0;

    // workspace
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    const size_t o_cursor = take(8), o_zero = take(8), o_err = take(8), o_base = take(8);
    const size_t W_ = (size_t)a.index_window;
    const size_t o_srecA = take(4ull * W_ * a.RA), o_urowA = take(16ull * W_ * a.RA);
    const size_t o_srecW = take(4ull * W_ * a.RW), o_urowW = take(16ull * W_ * a.RW);
    const size_t o_skeyA = take(8ull * W_ * a.RA), o_skeyW = take(8ull * W_ * a.RW);
    const size_t o_gidx = take(4ull * W_ * 4 * RAE_IDX_HMAX);
    const size_t o_pcls = take(16ull * W_ * 2 * RAE_IDX_HMAX);
    a.VCA = a.RA / (RAE_VHEAVY + 1) + 1;       // very heavy rows per batch are fewer than this
    a.VCW = a.RW / (RAE_VHEAVY + 1) + 1;
    // the update's dispatch table: every unique row is at most one task (TC = records), and
    // NVC very heavy rows get a workgroup each (L / RAE_NVC_DIV, at least 32 -- the rest run as
    // wave tasks)
    a.TC = a.RA + a.RW;
    {
        const int Lo = a.part ? (L + a.G - 1) / a.G : L;     // the rows this rank updates
        const int nvc = Lo / RAE_NVC_DIV > RAE_NVC_MIN ? Lo / RAE_NVC_DIV : RAE_NVC_MIN;
        a.NVC = nvc < a.VCA + a.VCW ? nvc : a.VCA + a.VCW;
        // large global batches: very heavy rows with at least 2 RAE_HCH records split into
        // floor(records / RAE_HCH) chunks (every chunk a workgroup task: NVC >= HF + 1 >
        // records / RAE_HCH, the most chunks a batch can have -- rae_index.hpp build_batch_tasks)
        a.hch = (c.heavy_chunk == RAE_HCHUNK_ON ||
                 (c.heavy_chunk == RAE_HCHUNK_AUTO && L >= RAE_HCH_MINL)) ? RAE_HCH : 0;
        if (a.hch) {
            a.HF = (a.RA + a.RW) / a.hch + 1;
            if (a.NVC < a.HF + 1) a.NVC = a.HF + 1;
            a.hps = ((c.embed + 3) & ~3) + 4 > ((c.relations + 3) & ~3) ? ((c.embed + 3) & ~3) + 4
                                                                       : ((c.relations + 3) & ~3);
        }
    }
    const size_t o_thdr = take(16 * W_), o_task = take(16ull * W_ * a.TC);
    const size_t o_vtask = take(16ull * W_ * a.NVC);
    const size_t o_hfin = a.hch ? take(16ull * W_ * a.HF) : 0;
    const size_t o_hpart = a.hch ? take(4ull * a.NVC * a.hps) : 0;
    {
        const int NJd = 2 + 2 * c.neg_samples;
        int cap = c.max_row_nnz > 0 ? c.max_row_nnz : 1;
        if (cap > 256) cap = 256;                    // the fast path's feature capacity
        a.dcap = cap;
        a.dstride = ((2 + NJd + cap) + 31) & ~31;     // whole 128-B lines per example
    }
    // private rows (rows one record of the global batch references, updated per example by the
    // update launch): plans without a regulariser whose record slots fit one wave (NJ <= 64);
    // the example's features from its descriptor (<= dcap, <= 32).  Several ranks: every rank's
    // update takes the private rows it updates (replicated: all; partitioned: its own), so the
    // descriptors cover the whole global batch
    // auto: single-rank and replicated plans below a global batch of RAE_PRIV_MAXL; at larger
    // batches and in the partitioned update (a rank's own private rows: a few per example) the
    // row tasks do them faster (profiles/r04_ab.txt)
    const bool priv_ok = !a.reg_on && NJ <= 64;
    a.priv = (priv_ok && (c.priv_rows == RAE_PRIV_ON ||
                          (c.priv_rows == RAE_PRIV_AUTO && !a.part && L < RAE_PRIV_MAXL))) ? 1 : 0;
    a.dnx = (a.priv && c.world_size > 1) ? L : c.batch_size;
    a.d0 = a.dnx == L ? c.rank * c.batch_size : 0;
    const size_t o_desc = take(4ull * W_ * a.dnx * a.dstride);
    const size_t o_reg = take(16ull * (a.nregC + a.nregW + 1));
    const size_t o_gws = a.reg_on ? take(4ull * c.n_features * c.relations) : 0;
    // partitioned data-parallel update: list capacities are the worst cases of one rank's
    // l examples (every entity id distinct; the largest global batch's features)
    a.LA = a.part ? c.batch_size * NJ : 0;
    a.LW = a.part ? a.RW : 0;
    const size_t o_dpl = a.part ? take(4ull * W_ * dpl_slot_ints(a.G, a.LA, a.LW)) : 0;
    const size_t o_dpc = a.part ? take(4ull * W_ * 2 * a.G * 2) : 0;
    const size_t o_dpm = take(16);
    // peer-to-peer exchange: the peers' mapped buffers and this rank's expected signal counts
    const size_t o_peers = take(sizeof(PeerBufs) * (size_t)c.world_size);
    const size_t o_pexp = take(4ull * 2 * c.world_size);
    // pipelined peer-to-peer form: two parities of row-mark bytes over the owned rows
    a.pipe = (c.dp_xchg == RAE_XCHG_P2P_PIPE && c.world_size > 1) ? 1 : 0;
    a.pmA = a.pipe ? (int)((((c.n_entities + c.world_size - 1) / c.world_size + 3) / 4 + 3) & ~3) : 0;
    a.pmW = a.pipe ? (int)((((c.n_features + c.world_size - 1) / c.world_size + 3) / 4 + 3) & ~3) : 0;
    const size_t o_pm = a.pipe ? take(4ull * 2 * (a.pmA + a.pmW)) : 0;
    const bool bil = c.decoder != RAE_DEC_SP;
    a.bf16 = (bil && c.mfma_bf16) ? 1 : 0;
    // bf16 dP with LDS-staged R slices (k_bil_dp2): the C5 shape compiled exactly, other
    // shapes up to r = 256, K = 128 padded; float4 rows needed (r, K multiples of 4)
    // dP contraction form: in the second M-tile pass (bf16, m <= 128) by default; k_bil_dp2
    // (bf16, LDS-staged R slices: the C5 shape compiled exactly, others up to r = 256, m = 128
    // padded; float4 rows) or the strided k_bil_dp otherwise / on request
    const bool mt_ok = bil && c.mfma_bf16 && c.relations <= 128;
    const bool dp2_ok = a.bf16 && c.embed % 4 == 0 && c.relations % 4 == 0 &&
                        (((c.embed + 31) / 32 == 7 && (c.relations + 15) / 16 == 7) ||
                         (c.embed <= 256 && c.relations <= 128));
    const bool mtdp = mt_ok && (c.bil_dp == RAE_BILDP_AUTO || c.bil_dp == RAE_BILDP_MTILE);
    p->dp2 = 0;
    if (!mtdp && dp2_ok && c.bil_dp != RAE_BILDP_STRIDED)
        p->dp2 = ((c.embed + 31) / 32 == 7 && (c.relations + 15) / 16 == 7) ? 1 : 2;
    a.nib = bil ? (p->dp2 ? (c.embed + RAE_IB2 - 1) / RAE_IB2 : (c.embed + RAE_IB - 1) / RAE_IB) : 0;
    const size_t o_dpp = bil ? take(4ull * a.nib * c.batch_size * c.relations) : 0;
    a.r4 = align4(c.embed);
    const int64_t nbi_mt = (c.embed + RAE_MTI - 1) / RAE_MTI, nbj_mt = (c.embed + RAE_MTJ - 1) / RAE_MTJ;
    const size_t o_mtv = bil ? take(4ull * nbj_mt * c.batch_size * a.r4) : 0;
    const size_t o_mtw = bil ? take(4ull * nbi_mt * c.batch_size * a.r4) : 0;
    a.nmtp = (int)(nbi_mt * nbj_mt);
    const size_t o_mtp = mtdp ? take(4ull * a.nmtp * c.batch_size * c.relations) : 0;
    // split SP forward (rae_sp_split.hpp) for runtime shapes whose decoder matrices stream
    // through every example's workgroup (r*m > RAE_SPLIT_RM; C4: 90 k), or on request
    p->sp_split = !bil && (c.sp_forward == RAE_SPFWD_SPLIT ||
                           (c.sp_forward == RAE_SPFWD_AUTO &&
                            (int64_t)c.embed * c.relations > RAE_SPLIT_RM));
    const size_t o_sps = p->sp_split ? take(4ull * sps_stride(c.embed) * c.batch_size) : 0;
    a.privnf = a.priv ? (a.dcap < 32 ? a.dcap : 32) : 0;
    a.privc = (a.priv && a.part && c.world_size > 1) ? 1 : 0;
    const size_t o_pmask = a.priv ? take(16ull * W_ * L) : 0;
    a.Lp = (L + 31) / 32 * 32;
    a.fuse_prep = (a.bf16 && c.world_size == 1 && c.bil_prep == RAE_BILPREP_AUTO) ? 1 : 0;
    const size_t o_fac = a.bf16 ? take(16ull * c.embed * a.Lp) : 0;
    const size_t o_vb = a.lay.wire ? take(4ull * a.vbs * L) : 0;
    const size_t o_dwb = a.dpart ? take(4ull * a.dws * L) : 0;
    const size_t o_pfr = a.bf16 ? take(16ull * (a.Lp / 32) * ((c.relations + 15) / 16) * 64) : 0;
    hipError_t e = hipMalloc(&p->ws, off);
    if (e != hipSuccess) {
        delete p;
        return fail(RAE_E_HIP, std::string("hipMalloc workspace: ") + hipGetErrorString(e));
    }
    (void)hipMemset(p->ws, 0, off);
    e = hipHostMalloc(reinterpret_cast<void**>(&p->h_err), sizeof(int), hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipFree(p->ws);
        delete p;
        return fail(RAE_E_HIP, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    *p->h_err = 0;
    if (c.dp_xchg != RAE_XCHG_COLLECTIVE) {
        // the peers add to these words over xGMI and this rank polls them: uncached (no L2
        // line of them can go stale; rae_p2p.hpp "Visibility across GPUs")
        e = hipExtMallocWithFlags(reinterpret_cast<void**>(&p->d_sig), 4ull * 2 * c.world_size,
                                  hipDeviceMallocUncached);
        if (e == hipSuccess) e = hipMemset(p->d_sig, 0, 4ull * 2 * c.world_size);
        if (e != hipSuccess) {
            (void)hipFree(p->ws);
            (void)hipHostFree(p->h_err);
            delete p;
            return fail(RAE_E_HIP, std::string("hipMalloc signals: ") + hipGetErrorString(e));
        }
    }
    p->d_cursor = reinterpret_cast<int64_t*>(p->ws + o_cursor);
    p->d_zero = reinterpret_cast<int64_t*>(p->ws + o_zero);
    p->d_err = reinterpret_cast<int*>(p->ws + o_err);
    a.base_cost = reinterpret_cast<float*>(p->ws + o_base);
    a.srecA = reinterpret_cast<int32_t*>(p->ws + o_srecA);
    a.urowA = reinterpret_cast<int32_t*>(p->ws + o_urowA);
    a.srecW = reinterpret_cast<int32_t*>(p->ws + o_srecW);
    a.urowW = reinterpret_cast<int32_t*>(p->ws + o_urowW);
    a.skeyA = reinterpret_cast<unsigned long long*>(p->ws + o_skeyA);
    a.skeyW = reinterpret_cast<unsigned long long*>(p->ws + o_skeyW);
    a.gidx = reinterpret_cast<int32_t*>(p->ws + o_gidx);
    a.pcls = reinterpret_cast<int32_t*>(p->ws + o_pcls);
    a.thdr = reinterpret_cast<int32_t*>(p->ws + o_thdr);
    a.task = reinterpret_cast<int32_t*>(p->ws + o_task);
    a.vtask = reinterpret_cast<int32_t*>(p->ws + o_vtask);
    a.hfin = a.hch ? reinterpret_cast<int32_t*>(p->ws + o_hfin) : nullptr;
    a.hpart = a.hch ? reinterpret_cast<float*>(p->ws + o_hpart) : nullptr;

    a.desc = reinterpret_cast<int32_t*>(p->ws + o_desc);
    a.regpart = reinterpret_cast<double*>(p->ws + o_reg);
    a.gWs = a.reg_on ? reinterpret_cast<float*>(p->ws + o_gws) : nullptr;
    a.dPpart = bil ? reinterpret_cast<float*>(p->ws + o_dpp) : nullptr;
    a.sps = p->sp_split ? reinterpret_cast<float*>(p->ws + o_sps) : nullptr;
    a.spss = sps_stride(c.embed);
    a.mtV = bil ? reinterpret_cast<float*>(p->ws + o_mtv) : nullptr;
    a.mtW = bil ? reinterpret_cast<float*>(p->ws + o_mtw) : nullptr;
    a.mtP = mtdp ? reinterpret_cast<float*>(p->ws + o_mtp) : nullptr;
    a.facT = a.bf16 ? reinterpret_cast<float*>(p->ws + o_fac) : nullptr;
    a.pfrag = a.bf16 ? reinterpret_cast<uint4*>(p->ws + o_pfr) : nullptr;
    a.err = p->d_err;
    a.cursor = p->d_cursor;
    a.dpl = a.part ? reinterpret_cast<int32_t*>(p->ws + o_dpl) : nullptr;
    a.dpc = a.part ? reinterpret_cast<int32_t*>(p->ws + o_dpc) : nullptr;
    a.dpmax = reinterpret_cast<int*>(p->ws + o_dpm);
    a.xchg = c.dp_xchg;
    a.peers = reinterpret_cast<PeerBufs*>(p->ws + o_peers);
    a.p2p_expect = reinterpret_cast<unsigned*>(p->ws + o_pexp);
    a.pm = a.pipe ? reinterpret_cast<uint32_t*>(p->ws + o_pm) : nullptr;
    a.pmask = a.priv ? reinterpret_cast<int32_t*>(p->ws + o_pmask) : nullptr;
    if (a.lay.wire) a.vb = reinterpret_cast<float*>(p->ws + o_vb);
    if (a.dpart) a.dwb = reinterpret_cast<float*>(p->ws + o_dwb);

    const int ex_floats = example_smem_floats(c.decoder, c.relations, c.embed, c.neg_samples);
    const size_t smem_ex = 4ull * ex_floats;
    // k_idx_sort<big>: keys, scan scratch, segment starts (the fast form: RAE_IDX_FAST keys)
    p->smem_idx = 8ull * RAE_KCAP + 4ull * 64 + 4ull * RAE_KCAP;
    p->smem_idxf = 8ull * RAE_IDX_FAST + 4ull * 64 + 4ull * RAE_IDX_FAST;
    p->smem_fwd = smem_ex;
    p->smem_spe = p->sp_split ? 4ull * example_smem_floats(0, c.relations, c.embed, 0) : 0;
    p->smem_spd = p->sp_split ? 4ull * sp_dec_side_smem_floats(c.embed, c.neg_samples) : 0;
    p->smem_dec = bil ? 4ull * bil_dec_smem_floats(c.embed, c.neg_samples) : 0;
    // the M-tile passes: bf16 blocks need m <= 128 (four K steps of 32 per fragment set)
    p->mt_bf16 = bil && a.bf16 && c.relations <= 128;
    p->smem_mt = bil ? bil_mt_lds_bytes(c.relations, p->mt_bf16) : 0;
    // the first pass never stages the transposed image (dP rides on the second): with half the
    // LDS, two of its workgroups fit a CU and all (r/8)(r/16) start at once
    p->smem_mt0 = (bil && p->mt_bf16) ? (size_t)RAE_MTI * RAE_MTJ * (((c.relations + 31) / 32 * 32) + 8) * 2
                                      : p->smem_mt;

    if (p->smem_mt > RAE_MT_LDS_MAX) {        // fp32 block too large to stage (m > 320)
        p->mt_direct = true;
        p->smem_mt = 0;
    }
    if (p->smem_fwd > 160 * 1024 || p->smem_idx > 160 * 1024 || p->smem_dec > 160 * 1024) {
        (void)hipFree(p->ws);
        delete p;
        return fail(RAE_E_INVALID, "configuration needs more than 160 KiB LDS per example "
                                   "workgroup (relations / embed / neg_samples too large)");
    }
    p->grid_fwd = c.batch_size;
    const int64_t gu = update_grid(c.decoder, c.embed, c.relations, a.TC, a.NVC, L, a.priv,
                                   a.privc, a.part ? a.G : 1);
    if (gu >= (1ll << 31)) {
        (void)hipFree(p->ws);
        delete p;
        return fail(RAE_E_INVALID, "update grid too large");
    }
    p->grid_update = (int)gu;
    {
        const void* fns[] = {(const void*)k_forward<true, DimsC3>,
                             (const void*)k_forward<false, DimsC2>,
                             (const void*)k_forward<true, DynDims>,
                             (const void*)k_forward<false, DynDims>,
                             (const void*)k_bil_enc<true>, (const void*)k_bil_enc<false>,
                             (const void*)k_bil_enc_fast<DimsC3>,
                             (const void*)k_sp_dec<true>, (const void*)k_sp_dec<false>};
        for (const void* f : fns)
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)p->smem_fwd);
        if (p->sp_split) {
            (void)hipFuncSetAttribute((const void*)k_sp_enc<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_spe);
            (void)hipFuncSetAttribute((const void*)k_sp_enc<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_spe);
        }
        if (bil) {
            (void)hipFuncSetAttribute((const void*)k_bil_dp2<7, 7>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dp2_lds_bytes<7, 7>());
            (void)hipFuncSetAttribute((const void*)k_bil_dp2<8, 8>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dp2_lds_bytes<8, 8>());
            (void)hipFuncSetAttribute((const void*)k_bil_mt<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_mt);
            (void)hipFuncSetAttribute((const void*)k_bil_mt<true, false, false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_mt);
            (void)hipFuncSetAttribute((const void*)k_bil_mt<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_mt);
            (void)hipFuncSetAttribute((const void*)k_bil_dec<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_dec);
            (void)hipFuncSetAttribute((const void*)k_bil_dec<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_dec);
        }
        (void)hipFuncSetAttribute((const void*)k_idx_sort<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)p->smem_idx);
        (void)hipFuncSetAttribute((const void*)k_build_dplists,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(4 * RAE_DPL_KEYS + 4 * 32));
    }
    a.sig = p->d_sig;
    a.p2p_timeout = RAE_P2P_TIMEOUT_DEFAULT;
    if (a.sig) {                 // this rank's own entry of the peer table
        const PeerBufs own{a.ex, a.W, a.A, a.Ab, a.sig};
        if (hipMemcpy(a.peers + c.rank, &own, sizeof(own), hipMemcpyHostToDevice) != hipSuccess) {
            rae_plan_destroy(p);
            return fail(RAE_E_HIP, "peer table");
        }
    }
    *out = p;
    return RAE_OK;
}

extern "C" int rae_plan_forms(const rae_plan* p, rae_config* out) {
    if (!p || !out) return fail(RAE_E_INVALID, "null argument");
    const bool bil = p->cfg.decoder != RAE_DEC_SP;
    out->sp_forward = bil ? 0 : (p->sp_split ? RAE_SPFWD_SPLIT : RAE_SPFWD_FUSED);
    out->bil_dp = !bil ? 0 : (p->args.mtP ? RAE_BILDP_MTILE
                              : (p->dp2 ? RAE_BILDP_STAGED : RAE_BILDP_STRIDED));
    out->bil_prep = (!bil || !p->args.bf16) ? 0 : (p->args.fuse_prep ? RAE_BILPREP_AUTO
                                                                    : RAE_BILPREP_KERNEL);
    out->dp_update = p->cfg.dp_update;
    out->priv_rows = p->args.priv ? RAE_PRIV_ON : RAE_PRIV_OFF;
    out->dp_dense = p->args.lay.wire == 2 ? RAE_DPDENSE_PARTIALS
                  : (p->args.lay.wire == 1 ? RAE_DPDENSE_RECORDS : 0);
    out->heavy_chunk = p->args.hch ? RAE_HCHUNK_ON : RAE_HCHUNK_OFF;
    out->dp_xchg = p->cfg.dp_xchg;
    return RAE_OK;
}

extern "C" int rae_plan_destroy(rae_plan* p) {
    if (!p) return RAE_OK;
    if (p->ws) (void)hipFree(p->ws);
    if (p->h_err) (void)hipHostFree(p->h_err);
    if (p->d_sig) (void)hipFree(p->d_sig);
    delete p;
    return RAE_OK;
}

extern "C" int rae_set_negatives(rae_plan* p, const int32_t* n1, const int32_t* n2, int32_t mode,
                                 int64_t stride) {
    if (!p || !n1 || !n2) return fail(RAE_E_INVALID, "null argument");
    if (mode != RAE_NEG_PER_CALL && mode != RAE_NEG_PER_EPOCH)
        return fail(RAE_E_INVALID, "bad negatives mode");
    p->args.neg1 = n1;
    p->args.neg2 = n2;
    p->args.neg_mode = mode;
    p->args.neg_stride = stride;
    return RAE_OK;
}

extern "C" int rae_set_cursor(rae_plan* p, int64_t batch, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    hipLaunchKernelGGL(k_set_cursor, dim3(1), dim3(64), 0, (hipStream_t)stream, p->d_cursor, batch);
    ++p->cursor_moves;
    HIPCHK(hipGetLastError());
    return RAE_OK;
}
extern "C" int rae_advance_cursor(rae_plan* p, int64_t count, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    hipLaunchKernelGGL(k_add_cursor, dim3(1), dim3(64), 0, (hipStream_t)stream, p->d_cursor, count);
    ++p->cursor_moves;
    HIPCHK(hipGetLastError());
    return RAE_OK;
}
extern "C" int64_t rae_cursor_moves(const rae_plan* p) { return p ? p->cursor_moves : -1; }

static void launch_fwd_sp(rae_plan* p, const StepArgs& a, hipStream_t st) {
    const dim3 gr(p->grid_fwd), bt(RAE_FBT);
    if (p->sp_split) {
        const dim3 gcp(sp_cp_tasks(a.l, a.r)), gct(sp_ctdw_tasks(a.l, a.m));   // WG per tile
        if (p->v4) RAE_LAUNCH(p, k_sp_enc<true>, gr, bt, p->smem_spe, st, a);
        else RAE_LAUNCH(p, k_sp_enc<false>, gr, bt, p->smem_spe, st, a);
        if (a.m % 4 == 0) RAE_LAUNCH(p, k_sp_cp<true>, gcp, dim3(RAE_BT), 0, st, a);
        else RAE_LAUNCH(p, k_sp_cp<false>, gcp, dim3(RAE_BT), 0, st, a);
        const dim3 gsd(RAE_SPD_NP * p->grid_fwd);          // a workgroup per (example, piece)
        if (p->v4) RAE_LAUNCH(p, k_sp_dec<true>, gsd, bt, p->smem_spd, st, a);
        else RAE_LAUNCH(p, k_sp_dec<false>, gsd, bt, p->smem_spd, st, a);
        if (a.r % 4 == 0) RAE_LAUNCH(p, k_sp_ctdw<true>, gct, dim3(RAE_DW_BT), 0, st, a);
        else RAE_LAUNCH(p, k_sp_ctdw<false>, gct, dim3(RAE_DW_BT), 0, st, a);
        return;
    }
    const bool c3 = a.m == 100 && a.r == 200 && a.s == 20;
    const bool c2 = a.m == 30 && a.r == 100 && a.s == 10;
    if (c3 && p->v4)
        RAE_LAUNCH(p, (k_forward<true, DimsC3>), gr, bt, p->smem_fwd, st, a);
    else if (c2 && !p->v4)
        RAE_LAUNCH(p, (k_forward<false, DimsC2>), gr, bt, p->smem_fwd, st, a);
    else if (p->v4)
        RAE_LAUNCH(p, (k_forward<true, DynDims>), gr, bt, p->smem_fwd, st, a);
    else
        RAE_LAUNCH(p, (k_forward<false, DynDims>), gr, bt, p->smem_fwd, st, a);
}

static void launch_fwd_dp(rae_plan* p, const StepArgs& a, hipStream_t st);
template <bool V4>
static void launch_fwd_bil(rae_plan* p, const StepArgs& a, hipStream_t st) {
    const dim3 ge(p->grid_fwd);
    if (V4 && a.dec == RAE_DEC_RESCAL && a.m == 100 && a.r == 200 && a.s == 20)     // C5 shape
        RAE_LAUNCH(p, (k_bil_enc_fast<DimsC3>), ge, dim3(RAE_FBT), p->smem_fwd, st, a);
    else
        RAE_LAUNCH(p, (k_bil_enc<V4>), ge, dim3(RAE_FBT), p->smem_fwd, st, a);
    const dim3 gmt(((a.r + RAE_MTI - 1) / RAE_MTI) * ((a.r + RAE_MTJ - 1) / RAE_MTJ));
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) RAE_LAUNCH(p, (k_bil_dec<V4>), ge, dim3(RAE_DBT), p->smem_dec, st, a);
        if (p->mt_bf16 && pass == 0)       // no dP: the lighter instantiation, half the LDS
            RAE_LAUNCH(p, (k_bil_mt<true, false, false>), gmt, dim3(RAE_MTT), p->smem_mt0, st, a, pass);
        else if (p->mt_bf16) RAE_LAUNCH(p, (k_bil_mt<true>), gmt, dim3(RAE_MTT), p->smem_mt, st, a, pass);
        else if (p->mt_direct) RAE_LAUNCH(p, (k_bil_mt<false, true>), gmt, dim3(RAE_MTT), 0, st, a, pass);
        else RAE_LAUNCH(p, (k_bil_mt<false>), gmt, dim3(RAE_MTT), p->smem_mt, st, a, pass);
    }
    if (!a.mtP) launch_fwd_dp(p, a, st);              // else dP came with the second pass
    RAE_LAUNCH(p, k_bil_fin, ge, dim3(RAE_FINT), 0, st, a);
}

static void launch_fwd_dp(rae_plan* p, const StepArgs& a, hipStream_t st) {
    const int gd = ceil_div(bil_dp_tasks(a.l, a.m, a.nib), RAE_NWAVE);
    const size_t lds77 = dp2_lds_bytes<7, 7>(), lds88 = dp2_lds_bytes<8, 8>();
    if (p->dp2 == 1)
        RAE_LAUNCH(p, (k_bil_dp2<7, 7>), dim3(a.nib), dim3(dp2_threads<7, 7>()), lds77, st, a);
    else if (p->dp2 == 2)
        RAE_LAUNCH(p, (k_bil_dp2<8, 8>), dim3(a.nib), dim3(dp2_threads<8, 8>()), lds88, st, a);
    else if (a.bf16)
        RAE_LAUNCH(p, k_bil_dp<true>, dim3(gd), dim3(RAE_BT), 0, st, a);
    else
        RAE_LAUNCH(p, k_bil_dp<false>, dim3(gd), dim3(RAE_BT), 0, st, a);
}

// peer-to-peer exchange grids (every rank the same: the peers expect these many signals)
static unsigned p2p_rows_grid(const StepArgs& a) {
    const int64_t g = ((int64_t)a.G * (a.capA + a.capW) + RAE_NWAVE - 1) / RAE_NWAVE;
    return (unsigned)(g < 1 ? 1 : g);
}
static unsigned p2p_recs_grid(const StepArgs& a) {
    const int64_t g = ((int64_t)a.l * a.lay.rec / 4 + RAE_BT - 1) / RAE_BT;
    return (unsigned)(g < 1 ? 1 : g);
}
static bool p2p_on(const rae_plan* p) { return p->args.xchg != RAE_XCHG_COLLECTIVE && p->args.G > 1; }
// k_p2p_pre's grid: marking threads (one per list entry of every list, the own one included)
// + pushing waves (one per entry of the peers' lists)
static int p2p_pre_mark_blocks(const StepArgs& a) {
    const int64_t n = (int64_t)a.G * (a.capA + a.capW);
    return (int)((n + RAE_BT - 1) / RAE_BT);
}

static int launch_forward(rae_plan* p, const int64_t* cursor, int64_t off, hipStream_t st) {
    if (!p->args.neg1 || !p->args.neg2) return fail(RAE_E_STATE, "negatives not set");
    StepArgs a = p->args;
    a.cursor = cursor;
    a.step_offset = off;
    a.stamps = p->stamps_fwd;
    const bool p2p = p2p_on(p);
    if (p2p) {
        if (!p->peers_set) return fail(RAE_E_STATE, "peer buffers not set (rae_set_peer)");
        if (!a.pipe) {        // the owned rows the peers' examples read, into their replicas
            const unsigned gr = p2p_rows_grid(a);   // (>= 1 workgroup: the signal follows anyway)
            RAE_LAUNCH(p, k_p2p_rows, dim3(gr), dim3(RAE_BT), 0, st, a);
            RAE_LAUNCH(p, k_p2p_signal, dim3(1), dim3(64), 0, st, a, 1);
        }                     // pipelined: pushed and signalled by the previous step / prologue
        RAE_LAUNCH(p, k_p2p_wait, dim3(1), dim3(64), 0, st, a, 1, 1u);
    }
    if (a.dec == RAE_DEC_SP) {
        launch_fwd_sp(p, a, st);
        if (a.dpart)          // this rank's dense partials into its records, before the exchange
            RAE_LAUNCH(p, k_dpart, dim3(dpart_tasks(a.r, a.m)), dim3(RAE_BT), 0, st, a);
    }
    else if (p->v4) launch_fwd_bil<true>(p, a, st);
    else launch_fwd_bil<false>(p, a, st);
    if (p2p)                  // this rank's records into every peer's exchange buffer
    {
        // (pipelined: + blocks clearing the next batch's row marks)
        RAE_LAUNCH(p, k_p2p_recs, dim3(p2p_recs_grid(a) + (a.pipe ? 64 : 0)), dim3(RAE_BT), 0, st, a);
        RAE_LAUNCH(p, k_p2p_signal, dim3(1), dim3(64), 0, st, a, 0);
        if (a.pipe) {         // the next batch's rows this step's update leaves unchanged
            const int nmb = p2p_pre_mark_blocks(a);
            RAE_LAUNCH(p, k_p2p_pre, dim3(nmb + p2p_rows_grid(a)), dim3(RAE_BT), 0, st, a, 0, nmb);
        }
    }
    p->t_start = p->t_stop = nullptr;
    HIPCHK(hipGetLastError());
    return RAE_OK;
}

template <int OPT, bool V4, bool BIL>
static void launch_update_b(rae_plan* p, dim3 gu, dim3 bt, hipStream_t st, const StepArgs& a) {
    if constexpr (BIL) {
        // R tensor: k_bil_prep (bf16 operand layout) -> k_bil_rows; then k_update_bil (C / Wb
        // tiles, cost, A / W rows).  Measured at C5 and not kept: a forked stream for the R
        // branch (123 vs 112 us/step: the cross-stream graph edges cost more than the overlap);
        // k_bil_rows with all P fragments in LDS and every load of a tile hoisted into one round
        // trip (29 vs 24 us: two workgroups per CU and the per-workgroup staging cost more).
        if (a.bf16 && !a.fuse_prep) {
            const int gp = 4 * ((a.r + 63) / 64) * (a.Lp / 32) + (a.Lp / 32) * ((a.m + 15) / 16);
            RAE_LAUNCH(p, k_bil_prep, dim3(gp), bt, 0, st, a);
        }
        const int nRt = n_rtiles(a.dec, a.r, a.m);
        const dim3 gr((nRt + RAE_NWAVE - 1) / RAE_NWAVE);
        const size_t lr = bil_rows_lds_bytes(a.m, a.bf16, OPT == 0);
        constexpr size_t lu = 4 * update_lds_floats<V4, 2>();
        if (RAE_BIL_FUSED_UPD && lr >= lu) {
            const dim3 gf(gu.x + gr.x);
            if (a.pipe) {     // (the pipelined peer-to-peer form's row pushes compiled in)
                if (p->q == 1) RAE_LAUNCH(p, (k_bil_update<OPT, V4, 1, true>), gf, bt, lr, st, a, (int)gu.x);
                else RAE_LAUNCH(p, (k_bil_update<OPT, V4, 2, true>), gf, bt, lr, st, a, (int)gu.x);
            } else {
                if (p->q == 1) RAE_LAUNCH(p, (k_bil_update<OPT, V4, 1>), gf, bt, lr, st, a, (int)gu.x);
                else RAE_LAUNCH(p, (k_bil_update<OPT, V4, 2>), gf, bt, lr, st, a, (int)gu.x);
            }
            return;
        }
        if (lr) RAE_LAUNCH(p, (k_bil_rows<OPT, true>), gr, bt, lr, st, a);
        else RAE_LAUNCH(p, (k_bil_rows<OPT, false>), gr, bt, 0, st, a);
        if (a.pipe) {
            if (p->q == 1) RAE_LAUNCH(p, (k_update_bil<OPT, V4, 1, true>), gu, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_update_bil<OPT, V4, 2, true>), gu, bt, 0, st, a);
        } else {
            if (p->q == 1) RAE_LAUNCH(p, (k_update_bil<OPT, V4, 1>), gu, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_update_bil<OPT, V4, 2>), gu, bt, 0, st, a);
        }
    } else {
        // the data-parallel SP update (wire records: vectors in the vector buffer, dense
        // partials) and the single-rank one are separate instantiations
        if (a.lay.wire) {
            if (p->q == 1) RAE_LAUNCH(p, (k_update<OPT, V4, 1, true>), gu, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_update<OPT, V4, 2, true>), gu, bt, 0, st, a);
        } else {
            if (p->q == 1) RAE_LAUNCH(p, (k_update<OPT, V4, 1, false>), gu, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_update<OPT, V4, 2, false>), gu, bt, 0, st, a);
        }
    }
}
template <int OPT, bool V4>
static void launch_update_v(rae_plan* p, dim3 gu, dim3 bt, hipStream_t st, const StepArgs& a) {
    if (a.dec == RAE_DEC_SP) launch_update_b<OPT, V4, false>(p, gu, bt, st, a);
    else launch_update_b<OPT, V4, true>(p, gu, bt, st, a);
}
template <int OPT>
static void launch_update_q(rae_plan* p, dim3 gu, dim3 bt, hipStream_t st, const StepArgs& a) {
    if (p->v4) launch_update_v<OPT, true>(p, gu, bt, st, a);
    else launch_update_v<OPT, false>(p, gu, bt, st, a);
}

// k_heavy_fin for the plan's optimizer / vector width / row slots (PP: pipelined pushes)
template <bool PP>
static void launch_heavy_fin(rae_plan* p, dim3 gh, dim3 bt, hipStream_t st, const StepArgs& a) {
    if (a.opt == RAE_OPT_ADAGRAD) {
        if (p->v4) {
            if (p->q == 1) RAE_LAUNCH(p, (k_heavy_fin<0, true, 1, PP>), gh, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_heavy_fin<0, true, 2, PP>), gh, bt, 0, st, a);
        } else {
            if (p->q == 1) RAE_LAUNCH(p, (k_heavy_fin<0, false, 1, PP>), gh, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_heavy_fin<0, false, 2, PP>), gh, bt, 0, st, a);
        }
    } else {
        if (p->v4) {
            if (p->q == 1) RAE_LAUNCH(p, (k_heavy_fin<1, true, 1, PP>), gh, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_heavy_fin<1, true, 2, PP>), gh, bt, 0, st, a);
        } else {
            if (p->q == 1) RAE_LAUNCH(p, (k_heavy_fin<1, false, 1, PP>), gh, bt, 0, st, a);
            else RAE_LAUNCH(p, (k_heavy_fin<1, false, 2, PP>), gh, bt, 0, st, a);
        }
    }
}

static int launch_update(rae_plan* p, const int64_t* cursor, int64_t off, hipStream_t st) {
    StepArgs a = p->args;
    a.cursor = cursor;
    a.step_offset = off;
    a.stamps = p->stamps_upd;
    const dim3 gu(p->grid_update), bt(RAE_BT);
    if (p2p_on(p))            // every peer's records of this batch are here
        RAE_LAUNCH(p, k_p2p_wait, dim3(1), dim3(64), 0, st, a, 0, 1u);
    if (a.lay.wire)           // the vectors the wire records left out, for the whole batch
    {
        const dim3 gv(ceil_div(vrec_tasks(a.L, a.r), RAE_NWAVE));
        if (a.m % 4 == 0) RAE_LAUNCH(p, k_vrec<true>, gv, bt, 0, st, a);
        else RAE_LAUNCH(p, k_vrec<false>, gv, bt, 0, st, a);
    }
    if (a.opt == RAE_OPT_ADAGRAD) launch_update_q<0>(p, gu, bt, st, a);
    else launch_update_q<1>(p, gu, bt, st, a);
    HIPCHK(hipGetLastError());
    if (a.hch) {              // the rows split into chunks: their chunk sums combined + updated
        const dim3 gh(ceil_div(a.HF, RAE_NWAVE));
        if (a.pipe) launch_heavy_fin<true>(p, gh, bt, st, a);
        else launch_heavy_fin<false>(p, gh, bt, st, a);
        HIPCHK(hipGetLastError());
    }
    if (a.reg_on) {
        if (a.opt == RAE_OPT_ADAGRAD)
            RAE_LAUNCH(p, (k_dense_w<0>), dim3(p->grid_dense), bt, 0, st, a);
        else
            RAE_LAUNCH(p, (k_dense_w<1>), dim3(p->grid_dense), bt, 0, st, a);
        HIPCHK(hipGetLastError());
        RAE_LAUNCH(p, k_finalize_cost, dim3(1), dim3(64), 0, st, a);
        HIPCHK(hipGetLastError());
    }
    if (p2p_on(p) && a.pipe) {   // the next batch's rows are in the peers' replicas
        RAE_LAUNCH(p, k_p2p_signal, dim3(1), dim3(64), 0, st, a, 1);
        HIPCHK(hipGetLastError());
    }
    p->t_start = p->t_stop = nullptr;
    return RAE_OK;
}

static int launch_index(rae_plan* p, int64_t first, int64_t count, hipStream_t st) {
    if (!p->args.neg1 || !p->args.neg2) return fail(RAE_E_STATE, "negatives not set");
    const int64_t nb = p->cfg.n_examples / ((int64_t)p->cfg.batch_size * p->cfg.world_size);
    if (first < 0 || count < 0 || first + count > nb)
        return fail(RAE_E_INVALID, "batch range out of the epoch");
    if (count > p->args.index_window)
        return fail(RAE_E_INVALID, "more batches than the index window holds");
    if (count == 0) return RAE_OK;
    const StepArgs& a = p->args;
    // the slots' partition counts and scatter cursors start at zero (two ranges when the
    // window wraps around the ring)
    {
        const int64_t s0 = first % a.index_window, n0 = std::min(count, a.index_window - s0);
        const size_t per = 4ull * 4 * RAE_IDX_HMAX;
        HIPCHK(hipMemsetAsync(a.gidx + s0 * 4 * RAE_IDX_HMAX, 0, per * n0, st));
        if (count > n0) HIPCHK(hipMemsetAsync(a.gidx, 0, per * (count - n0), st));
    }
    const unsigned nsl = (unsigned)((a.L + RAE_IDX_EPS - 1) / RAE_IDX_EPS);
    const unsigned hmax = (unsigned)(a.HA > a.HW ? a.HA : a.HW);
    hipLaunchKernelGGL(k_idx_count, dim3((unsigned)count, 3, nsl), dim3(RAE_BT), 0, st, a, first);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_idx_scatter, dim3((unsigned)count, 2, nsl), dim3(RAE_BT), 0, st, a, first);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_idx_sort<false>, dim3((unsigned)count, 2, hmax), dim3(RAE_FBT),
                       p->smem_idxf, st, a, first);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_idx_sort<true>, dim3((unsigned)count, 2, hmax), dim3(RAE_FBT),
                       p->smem_idx, st, a, first);
    HIPCHK(hipGetLastError());
    const unsigned ntk = (unsigned)((a.TC + RAE_TASK_PER - 1) / RAE_TASK_PER);
    hipLaunchKernelGGL(k_build_tasks, dim3((unsigned)count, ntk), dim3(RAE_BT), 0, st, a, first);
    HIPCHK(hipGetLastError());
    if (p->args.part) {
        hipLaunchKernelGGL(k_build_dplists, dim3((unsigned)count, p->args.G, 4), dim3(RAE_FBT),
                           4 * RAE_DPL_KEYS + 4 * 32, st, p->args, first);
        HIPCHK(hipGetLastError());
    }
    return RAE_OK;
}

extern "C" int rae_build_index(rae_plan* p, int64_t first, int64_t count, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    return launch_index(p, first, count, (hipStream_t)stream);
}
extern "C" int64_t rae_index_window(rae_plan* p) { return p ? p->args.index_window : -1; }

extern "C" int rae_step_forward(rae_plan* p, int64_t off, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    return launch_forward(p, p->d_cursor, off, (hipStream_t)stream);
}
extern "C" int rae_step_update(rae_plan* p, int64_t off, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    return launch_update(p, p->d_cursor, off, (hipStream_t)stream);
}

// absolute-batch forms: the batch index rides in the launch (no device cursor)
static int check_batch(rae_plan* p, int64_t batch) {
    const int64_t nb = p->cfg.n_examples / ((int64_t)p->cfg.batch_size * p->cfg.world_size);
    if (batch < 0 || batch >= nb) return fail(RAE_E_INVALID, "batch index out of the epoch");
    return RAE_OK;
}
extern "C" int rae_step_forward_at(rae_plan* p, int64_t batch, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (int rc = check_batch(p, batch)) return rc;
    return launch_forward(p, nullptr, batch, (hipStream_t)stream);
}
extern "C" int rae_step_update_at(rae_plan* p, int64_t batch, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (int rc = check_batch(p, batch)) return rc;
    return launch_update(p, nullptr, batch, (hipStream_t)stream);
}

// ---- partitioned data-parallel update (rae_dp.hpp) ----
extern "C" int64_t rae_dp_block_floats(const rae_config* cfg, int32_t cap_entities,
                                       int32_t cap_features) {
    if (!cfg || cap_entities < 0 || cap_features < 0) return -1;
    return dp_block_floats(cfg->embed, cfg->relations, cap_entities, cap_features);
}
extern "C" int rae_set_dp_buffers(rae_plan* p, float* send, float* recv, int32_t cap_entities,
                                  int32_t cap_features) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (!p->args.part) return fail(RAE_E_STATE, "the plan's data-parallel update is not partitioned");
    if ((p->args.xchg == RAE_XCHG_COLLECTIVE && (!send || !recv)) || cap_entities < 0 || cap_features < 0 ||
        cap_entities > p->args.LA || cap_features > p->args.LW)
        return fail(RAE_E_INVALID, "bad row-exchange buffers / capacities");
    StepArgs& a = p->args;
    a.dsend = send;
    a.drecv = recv;
    a.capA = cap_entities;
    a.capW = cap_features;
    a.dblk = dp_block_floats(a.r, a.m, a.capA, a.capW);
    return RAE_OK;
}
extern "C" int rae_dp_list_max(rae_plan* p, int32_t* max_entities, int32_t* max_features) {
    if (!p || !max_entities || !max_features) return fail(RAE_E_INVALID, "null argument");
    int v[2] = {0, 0};
    HIPCHK(hipMemcpy(v, p->args.dpmax, sizeof(v), hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(p->args.dpmax, 0, sizeof(v)));
    *max_entities = v[0];
    *max_features = v[1];
    return RAE_OK;
}
static int launch_dp_move(rae_plan* p, bool pack, const int64_t* cursor, int64_t off, hipStream_t st) {
    const StepArgs& a0 = p->args;
    if (!a0.part) return fail(RAE_E_STATE, "the plan's data-parallel update is not partitioned");
    if (a0.G == 1) return RAE_OK;                   // every row is this rank's
    if (!a0.dsend || !a0.drecv) return fail(RAE_E_STATE, "row-exchange buffers not set (the "
                                                       "peer-to-peer exchange has none: its rows "
                                                       "move inside rae_step_forward)");
    StepArgs a = a0;
    a.cursor = cursor;
    a.step_offset = off;
    const int64_t waves = (int64_t)a.G * (a.capA + a.capW);
    if (waves == 0) return RAE_OK;
    const dim3 gr((unsigned)((waves + RAE_NWAVE - 1) / RAE_NWAVE));
    if (pack) RAE_LAUNCH(p, k_dp_move<true>, gr, dim3(RAE_BT), 0, st, a);
    else RAE_LAUNCH(p, k_dp_move<false>, gr, dim3(RAE_BT), 0, st, a);
    p->t_start = p->t_stop = nullptr;
    HIPCHK(hipGetLastError());
    return RAE_OK;
}
extern "C" int rae_dp_pack(rae_plan* p, int64_t off, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    return launch_dp_move(p, true, p->d_cursor, off, (hipStream_t)stream);
}
extern "C" int rae_dp_unpack(rae_plan* p, int64_t off, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    return launch_dp_move(p, false, p->d_cursor, off, (hipStream_t)stream);
}
extern "C" int rae_dp_pack_at(rae_plan* p, int64_t batch, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (int rc = check_batch(p, batch)) return rc;
    return launch_dp_move(p, true, nullptr, batch, (hipStream_t)stream);
}
extern "C" int rae_dp_unpack_at(rae_plan* p, int64_t batch, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (int rc = check_batch(p, batch)) return rc;
    return launch_dp_move(p, false, nullptr, batch, (hipStream_t)stream);
}

// ---- peer-to-peer exchange (rae_p2p.hpp) ----
extern "C" int rae_ipc_export(const void* ptr, void* handle_out, int64_t* offset_out) {
    if (!ptr || !handle_out || !offset_out) return fail(RAE_E_INVALID, "null argument");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    HIPCHK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr));
    hipIpcMemHandle_t h;
    HIPCHK(hipIpcGetMemHandle(&h, (void*)base));
    static_assert(sizeof(h) == RAE_IPC_HANDLE_BYTES, "IPC handle size");
    memcpy(handle_out, &h, sizeof(h));
    *offset_out = (int64_t)((const char*)ptr - (const char*)base);
    return RAE_OK;
}
extern "C" int rae_ipc_open(const void* handle, void** base_out) {
    if (!handle || !base_out) return fail(RAE_E_INVALID, "null argument");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    HIPCHK(hipIpcOpenMemHandle(base_out, h, hipIpcMemLazyEnablePeerAccess));
    return RAE_OK;
}
extern "C" int rae_ipc_close(void* base) {
    if (!base) return fail(RAE_E_INVALID, "null argument");
    HIPCHK(hipIpcCloseMemHandle(base));
    return RAE_OK;
}
extern "C" void* rae_p2p_signals(rae_plan* p) { return p ? (void*)p->d_sig : nullptr; }
extern "C" int rae_set_peer(rae_plan* p, int32_t peer, float* exchange, float* W, float* A,
                            float* Ab, void* signals) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (p->args.xchg == RAE_XCHG_COLLECTIVE) return fail(RAE_E_STATE, "the plan's exchange is not peer-to-peer");
    if (peer < 0 || peer >= p->args.G || peer == p->args.rank)
        return fail(RAE_E_INVALID, "peer must be another rank");
    if (!exchange || !W || !A || !Ab || !signals) return fail(RAE_E_INVALID, "null peer buffer");
    const PeerBufs pb{exchange, W, A, Ab, (unsigned*)signals};
    HIPCHK(hipMemcpy(p->args.peers + peer, &pb, sizeof(pb), hipMemcpyHostToDevice));
    p->peers_mask |= 1 << peer;
    p->peers_set = p->peers_mask == (((1 << p->args.G) - 1) & ~(1 << p->args.rank));
    return RAE_OK;
}
extern "C" int rae_p2p_prologue(rae_plan* p, int64_t batch, int32_t drain, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (!p2p_on(p) || !p->args.pipe)
        return fail(RAE_E_STATE, "the plan's exchange is not the pipelined peer-to-peer form");
    if (!p->peers_set) return fail(RAE_E_STATE, "peer buffers not set (rae_set_peer)");
    if (int rc = check_batch(p, batch)) return rc;
    const hipStream_t st = (hipStream_t)stream;
    StepArgs a = p->args;
    a.cursor = nullptr;
    a.step_offset = batch;
    if (drain)                // the signal of rows a previous step pushed for another batch
        RAE_LAUNCH(p, k_p2p_wait, dim3(1), dim3(64), 0, st, a, 1, 1u);
    HIPCHK(hipMemsetAsync(a.pm, 0, 4ull * 2 * (a.pmA + a.pmW), st));
    const int nmb = p2p_pre_mark_blocks(a);
    RAE_LAUNCH(p, k_p2p_pre, dim3(nmb + p2p_rows_grid(a)), dim3(RAE_BT), 0, st, a, 1, nmb);
    RAE_LAUNCH(p, k_p2p_signal, dim3(1), dim3(64), 0, st, a, 1);
    HIPCHK(hipGetLastError());
    return RAE_OK;
}
extern "C" int rae_set_p2p_timeout(rae_plan* p, double seconds) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (p->args.xchg == RAE_XCHG_COLLECTIVE) return fail(RAE_E_STATE, "the plan's exchange is not peer-to-peer");
    if (!(seconds > 0.0) || seconds > 3600.0) return fail(RAE_E_INVALID, "timeout must be in (0, 3600] s");
    p->args.p2p_timeout = (unsigned long long)(seconds * 1e8);   // s_memrealtime: 100 MHz
    return RAE_OK;
}

extern "C" int rae_time_next(rae_plan* p, void* start, void* stop) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (!start || !stop) return fail(RAE_E_INVALID, "null event");
    p->t_start = (hipEvent_t)start;
    p->t_stop = (hipEvent_t)stop;
    return RAE_OK;
}
extern "C" int rae_event_create(void** ev) {
    if (!ev) return fail(RAE_E_INVALID, "null argument");
    hipEvent_t e = nullptr;
    HIPCHK(hipEventCreate(&e));
    *ev = (void*)e;
    return RAE_OK;
}
extern "C" int rae_event_destroy(void* ev) {
    if (ev) HIPCHK(hipEventDestroy((hipEvent_t)ev));
    return RAE_OK;
}
extern "C" int rae_event_elapsed_ms(void* start, void* stop, float* ms) {
    if (!start || !stop || !ms) return fail(RAE_E_INVALID, "null argument");
    HIPCHK(hipEventSynchronize((hipEvent_t)stop));
    HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return RAE_OK;
}

extern "C" int rae_train_step(rae_plan* p, int64_t batch, const int32_t* n1, const int32_t* n2,
                              rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    if (p->cfg.world_size != 1)
        return fail(RAE_E_STATE, "rae_train_step is the single-rank func['train'] path");
    const int64_t nb = p->cfg.n_examples / p->cfg.batch_size;
    if (batch < 0 || batch >= nb) return fail(RAE_E_INVALID, "batch index out of range");
    int rc = rae_set_negatives(p, n1, n2, RAE_NEG_PER_CALL, p->cfg.batch_size);
    if (rc) return rc;
    rc = launch_index(p, batch, 1, (hipStream_t)stream);
    if (rc) return rc;
    rc = launch_forward(p, nullptr, batch, (hipStream_t)stream);
    if (rc) return rc;
    return launch_update(p, nullptr, batch, (hipStream_t)stream);
}

#ifdef RAE_STAMPS
// diagnostic build only: point the kernels at a stamp buffer (16 u64 per forward block,
// 4 u64 per update wave); fwd=1 -> forward launches, fwd=0 -> update launches
extern "C" int rae_debug_stamps(rae_plan* p, unsigned long long* buf, int fwd) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    p->stamps_fwd = fwd ? buf : nullptr;
    p->stamps_upd = fwd ? nullptr : buf;
    return RAE_OK;
}
extern "C" int rae_debug_grid(rae_plan* p, int* out) {
    out[0] = p->grid_fwd; out[1] = p->grid_update; out[2] = 0; out[3] = 0;
    return RAE_OK;
}
#endif

// the device error word, bit by bit (rae.h): a peer-to-peer wait timeout is a state error (a
// peer stopped signalling), everything else a capacity overflow
static int err_flags(int e) {
    if (!e) return RAE_OK;
    static const struct { int bit; const char* what; } bits[] = {
        {1, "an entity-row index partition overflowed its LDS sort"},
        {2, "a feature-row index partition overflowed its LDS sort"},
        {4, "a batch exceeded the row index's record capacity"},
        {8, "a data-parallel row list overflowed while being built"},
        {16, "a data-parallel row list is longer than the exchange's row capacity"},
        {64, "a peer-to-peer wait timed out (a peer stopped signalling)"},
    };
    std::string msg;
    for (const auto& b : bits)
        if (e & b.bit) msg += (msg.empty() ? "" : "; ") + std::string(b.what);
    msg += " (device error flags=" + std::to_string(e) + ")";
    return fail(e & 64 ? RAE_E_STATE : RAE_E_OVERFLOW, msg);
}
extern "C" int rae_check(rae_plan* p) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    int e = 0;
    HIPCHK(hipMemcpy(&e, p->d_err, sizeof(int), hipMemcpyDeviceToHost));
    return err_flags(e);
}
// the same read ordered on one stream (pinned host word): the caller waits for that stream's
// queued work only
extern "C" int rae_check_on(rae_plan* p, rae_stream_t stream) {
    if (!p) return fail(RAE_E_INVALID, "null plan");
    HIPCHK(hipMemcpyAsync(p->h_err, p->d_err, sizeof(int), hipMemcpyDeviceToHost,
                          (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return err_flags(*p->h_err);
}

static int launch_neg(const double* cum, int64_t n, const double* u, uint64_t seed,
                      uint64_t offset, int64_t count, int32_t* out, hipStream_t st, bool philox) {
    if (!cum || !out || (!philox && !u)) return fail(RAE_E_INVALID, "null argument");
    if (n < 1 || n >= (1ll << 31)) return fail(RAE_E_INVALID, "CDF size must be in [1, 2^31)");
    if (count <= 0) return RAE_OK;
    int64_t blocks = (count + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (philox)
        hipLaunchKernelGGL(k_neg_sample<true>, dim3((unsigned)blocks), dim3(256), 0, st, cum, n, u,
                           seed, offset, count, out);
    else
        hipLaunchKernelGGL(k_neg_sample<false>, dim3((unsigned)blocks), dim3(256), 0, st, cum, n, u,
                           seed, offset, count, out);
    HIPCHK(hipGetLastError());
    return RAE_OK;
}

extern "C" int rae_neg_sample(const double* cum, int64_t n, const double* u, int64_t count,
                              int32_t* out, rae_stream_t stream) {
    return launch_neg(cum, n, u, 0, 0, count, out, (hipStream_t)stream, false);
}
extern "C" int rae_neg_sample_philox(const double* cum, int64_t n, uint64_t seed, uint64_t offset,
                                     int64_t count, int32_t* out, rae_stream_t stream) {
    return launch_neg(cum, n, nullptr, seed, offset, count, out, (hipStream_t)stream, true);
}

extern "C" int rae_stream_copy(const void* src, void* dst, int64_t bytes, rae_stream_t stream) {
    if (!src || !dst) return fail(RAE_E_INVALID, "null argument");
    if (bytes < 0 || (bytes & 15) || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15))
        return fail(RAE_E_INVALID, "bytes and pointers must be multiples of 16");
    const int64_t n = bytes / 16;
    if (n == 0) return RAE_OK;
    int64_t grid = (n + 1023) / 1024;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream,
                       (const rae_v4f*)src, (rae_v4f*)dst, n);
    HIPCHK(hipGetLastError());
    return RAE_OK;
}

extern "C" int rae_mfma_probe(int64_t iters, int32_t blocks, float* sink, rae_stream_t stream) {
    if (!sink || iters < 1 || blocks < 1) return fail(RAE_E_INVALID, "bad argument");
    hipLaunchKernelGGL(k_mfma_probe, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       iters, sink);
    HIPCHK(hipGetLastError());
    return RAE_OK;
}

extern "C" int rae_label(const int32_t* indptr, const int32_t* indices, const float* values,
                         const float* W, const float* Wb, int32_t m, int64_t row0, int64_t nrows,
                         int64_t* labels, float* probs, rae_stream_t stream) {
    if (!indptr || !indices || !W || !Wb || !labels) return fail(RAE_E_INVALID, "null argument");
    if (m < 1 || m > 512) return fail(RAE_E_INVALID, "relations must be in [1, 512] for labelling");
    const bool v4 = (m % 4) == 0;
    if (!v4 && m > 128)
        return fail(RAE_E_INVALID, "relations must be a multiple of 4 above 128 for labelling");
    if (nrows <= 0) return RAE_OK;
    int64_t blocks = (nrows + RAE_NWAVE - 1) / RAE_NWAVE;
    if (blocks > 65536) blocks = 65536;
    if (v4)
        hipLaunchKernelGGL(k_label<true>, dim3((unsigned)blocks), dim3(RAE_BT), 0, (hipStream_t)stream,
                           indptr, indices, values, W, Wb, m, row0, nrows, labels, probs);
    else
        hipLaunchKernelGGL(k_label<false>, dim3((unsigned)blocks), dim3(RAE_BT), 0, (hipStream_t)stream,
                           indptr, indices, values, W, Wb, m, row0, nrows, labels, probs);
    HIPCHK(hipGetLastError());
    return RAE_OK;
}
