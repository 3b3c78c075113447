// Row-owner partitioned data-parallel update (rae_config.dp_update = RAE_DPUPD_PARTITIONED).
//
// The reference trains on one process (learning/OieInduction.py:186-189); SURVEY.md 8(e) asks
// the build to shard the global batch over G ranks with a deterministic merge of the sparse
// row updates (learning/Optimizers.py:27-33).  In the replicated form every rank runs the
// whole update over the gathered records.  Here a parameter row of A / Ab (entity) or W
// (feature) is OWNED by rank row % G: only its owner updates it (the row index of the global
// batch keeps the owned rows only, rae_index.hpp), so the update's row work -- the part that
// grows with the global batch -- is split G ways.  The dense decoder matrices (C1, C2, Wb,
// R / C) stay replicated: every rank needs all of them in its forward.
//
// A rank's copy of a row it does not own is refreshed only when its own examples read it:
// before the forward of global batch g, every owner k sends rank j the current values of the
// rows j's examples reference in batch g that k owns, and j writes them into its replica
//   k_dp_pack   (rank k): send[j] <- A / Ab / W rows of list(j reads, k owns)     for j != k
//   [caller: all-to-all of the equal-size peer blocks; RCCL over xGMI]
//   k_dp_unpack (rank j): replica <- recv[k] rows of list(j reads, k owns)        for k != j
// The lists depend only on the batch's ids, negatives and CSR rows, so k_build_dplists builds
// them with the row index, a window ahead: per batch slot, direction (0 send: peer p reads, I
// own; 1 recv: I read, peer p owns), peer and table (A, W), the distinct rows in a fixed order
// (by hash pass, then ascending) -- sender and receiver compute the same list from the same
// data, so no row ids travel.  The sum of every owned row's gradient is the replicated form's
// sum (same records, same order), so the trained parameters are bit-identical to it once the
// replicas are gathered (rae/dist.py sync_rows).
#pragma once
#include "rae_common.hpp"
#include "rae_index.hpp"
#include "rae_step.hpp"

namespace rae {

#define RAE_DPL_KEYS 16384      // uint32 keys per LDS sort pass (64 KiB)
#define RAE_DPL_HMAX 1024       // hash passes of one list before an overflow is an error

// list storage of one batch slot: [dir 2][peer G][A list LA | W list LW] ints; counts
// [slot][dir][peer][table] ints
__host__ __device__ inline int64_t dpl_slot_ints(int G, int LA, int LW) {
    return 2ll * G * (LA + LW);
}
__device__ __forceinline__ int32_t* dpl_list(const StepArgs& a, int64_t slot, int dir, int p, int tab) {
    return a.dpl + slot * dpl_slot_ints(a.G, a.LA, a.LW) + ((int64_t)dir * a.G + p) * (a.LA + a.LW) +
           (tab ? a.LA : 0);
}
__device__ __forceinline__ int32_t* dpl_count(const StepArgs& a, int64_t slot, int dir, int p, int tab) {
    return a.dpc + ((slot * 2 + dir) * a.G + p) * 2 + tab;
}

// One list: the distinct rows of table `tab` (0: entities -- e1, e2, neg1, neg2 of every
// example; 1: features) that rank x's l examples of batch g reference and rank y owns.
template <int BT>
__device__ void build_dp_list(const StepArgs& a, int64_t g, int64_t slot, int dir, int p, int tab,
                              char* smem) {
    unsigned* keys = reinterpret_cast<unsigned*>(smem);
    int* sint = reinterpret_cast<int*>(keys + RAE_DPL_KEYS);   // [0] count, [1..] scan scratch
    const int tid = threadIdx.x;
    const int G = a.G;
    const int x = dir == 0 ? p : a.rank, y = dir == 0 ? a.rank : p;
    int32_t* cnt_out = dpl_count(a, slot, dir, p, tab);
    // own rows: nothing travels -- but the pipelined peer-to-peer form marks the rows its own
    // examples read too (rae_p2p.hpp: a batch's marks are the rows its update writes)
    if (p == a.rank && !(a.pipe && dir == 0)) {
        if (tid == 0) *cnt_out = 0;
        return;
    }
    int32_t* out = dpl_list(a, slot, dir, p, tab);
    const int cap = tab ? a.LW : a.LA;
    const int64_t ex0 = g * (int64_t)a.L + (int64_t)x * a.l;
    const int NJ = 2 + 2 * a.s;
    const int P0 = tab ? a.indptr[ex0] : 0;
    const int ncand = tab ? a.indptr[ex0 + a.l] - P0 : a.l * NJ;
    // candidate idx: a feature id of the rank's CSR rows, or entity slot j of example b
    // (j-major: coalesced columns)
    auto cand = [&](int idx) -> int {
        if (tab) return a.indices[P0 + idx];
        const int j = idx / a.l, b = idx - j * a.l;
        const int64_t ex = ex0 + b;
        const int64_t col = a.neg_mode ? ex : (int64_t)x * a.l + b;
        if (j == 0) return a.args1[ex];
        if (j == 1) return a.args2[ex];
        if (j < 2 + a.s) return a.neg1[(int64_t)(j - 2) * a.neg_stride + col];
        return a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
    };
    // the rows rank y owns are y + G q, q < nq: when a bit per q fits the LDS, the list is a
    // bitmap -- one atomicOr per candidate, then the set bits in ascending q by a block scan of
    // the words' popcounts: ascending rows, the sort path's order, without the sort (which was
    // 9.4 of the 19.7 us per batch of the partitioned index at G = 8, l = 1024)
    const int64_t nq = ((tab ? a.d : a.n) - y + G - 1) / G;
    if (nq <= 32ll * RAE_DPL_KEYS) {
        const int nw = (int)((nq + 31) >> 5);
        for (int i = tid; i < nw; i += BT) keys[i] = 0u;
        __syncthreads();
        for (int idx = tid; idx < ncand; idx += BT) {
            const int row = cand(idx);
            if (row % G == y) {
                const int q = row / G;
                atomicOr(&keys[q >> 5], 1u << (q & 31));
            }
        }
        __syncthreads();
        const int per = (nw + BT - 1) / BT, w0 = min(tid * per, nw), w1 = min(w0 + per, nw);
        int c = 0;
        for (int k = w0; k < w1; ++k) c += __popc(keys[k]);
        int tot;
        int pos = block_int_scan<BT>(c, sint, &tot);
        for (int k = w0; k < w1; ++k) {
            unsigned wv = keys[k];
            while (wv) {
                const int b = __ffs(wv) - 1;
                wv &= wv - 1;
                if (pos < cap) out[pos] = y + G * (k * 32 + b);
                ++pos;
            }
        }
        if (tid == 0) {
            *cnt_out = tot;
            atomicMax(a.dpmax + tab, tot);
            if (tot > cap) atomicOr(a.err, 8);
        }
        return;
    }
    // larger vocabularies: hash passes (row / G) % H, each sorting its owned candidates in
    // LDS.  H is sized from the owned candidates counted first (duplicates included: a pass
    // holds every occurrence), twice over for the hash's imbalance; a pass that still
    // overflows (a Zipf-heavy row's occurrences in one bucket) restarts the list with H doubled
    //  -- an overflow is an error only beyond RAE_DPL_HMAX passes
    int own = 0;
    for (int idx = tid; idx < ncand; idx += BT) own += cand(idx) % G == y;
    int nown;
    (void)block_int_scan<BT>(own, sint + 1, &nown);
    int H = max(1, (2 * nown + RAE_DPL_KEYS - 1) / RAE_DPL_KEYS);
    int total = 0;
    for (;;) {
        bool over = false;
        total = 0;
        for (int h = 0; h < H; ++h) {
            if (tid == 0) sint[0] = 0;
            __syncthreads();
            for (int idx = tid; idx < ncand; idx += BT) {
                const int row = cand(idx);
                if (row % G == y && (H <= 1 || (row / G) % H == h)) {
                    const int sl = atomicAdd(&sint[0], 1);
                    if (sl < RAE_DPL_KEYS) keys[sl] = (unsigned)row;
                }
            }
            __syncthreads();
            const int cnt = sint[0];
            __syncthreads();                      // every thread has read cnt before a reset
            if (cnt > RAE_DPL_KEYS) {
                over = true;
                break;
            }
            int n2 = 1;
            while (n2 < cnt) n2 <<= 1;
            for (int i = cnt + tid; i < n2; i += BT) keys[i] = 0xffffffffu;
            __syncthreads();
            for (int k = 2; k <= n2; k <<= 1) {                      // bitonic sort, ascending
                for (int j = k >> 1; j > 0; j >>= 1) {
                    for (int i = tid; i < n2; i += BT) {
                        const int ixj = i ^ j;
                        if (ixj > i) {
                            const unsigned u = keys[i], v = keys[ixj];
                            if ((u > v) == ((i & k) == 0)) {
                                keys[i] = v;
                                keys[ixj] = u;
                            }
                        }
                    }
                    __syncthreads();
                }
            }
            // distinct rows in order
            for (int i0 = 0; i0 < cnt; i0 += BT) {
                const int i = i0 + tid;
                const bool head = i < cnt && (i == 0 || keys[i - 1] != keys[i]);
                int tot;
                const int pos = total + block_flag_scan<BT>(head, sint + 1, &tot);
                if (head && pos < cap) out[pos] = (int32_t)keys[i];
                total += tot;
            }
            __syncthreads();
        }
        if (!over) break;
        H *= 2;
        if (H > RAE_DPL_HMAX) {
            if (tid == 0) atomicOr(a.err, 8);
            return;
        }
    }
    if (tid == 0) {
        *cnt_out = total;
        atomicMax(a.dpmax + tab, total);
        if (total > cap) atomicOr(a.err, 8);
    }
}

// peer block layout (floats): A rows (capA x r4) | Ab (align4(capA)) | W rows (capW x m4)
__host__ __device__ inline int64_t dp_block_floats(int r, int m, int capA, int capW) {
    return (int64_t)capA * align4(r) + align4(capA) + (int64_t)capW * align4(m);
}

// One wave per row slot of every peer block: pack (dir 0: my rows -> send[peer]) or unpack
// (dir 1: recv[peer] -> my replica).  Rows are float4-moved when r / m are multiples of 4.
template <bool PACK>
__device__ void dp_move(const StepArgs& a, int64_t t, int lane) {
    const int per = a.capA + a.capW;
    const int p = (int)(t / per), i0 = (int)(t - (int64_t)p * per);
    if (p >= a.G || p == a.rank) return;
    const int64_t slot = step_batch(a) % a.index_window;
    const int tab = i0 >= a.capA ? 1 : 0;
    const int i = tab ? i0 - a.capA : i0;
    const int cap = tab ? a.capW : a.capA;
    // the list length and the entry load together (one round trip; the list's storage holds
    // LA / LW >= cap entries, so entry i < cap is always in bounds -- used only when i < n)
    const int n = *dpl_count(a, slot, PACK ? 0 : 1, p, tab);
    const int row = dpl_list(a, slot, PACK ? 0 : 1, p, tab)[i < cap ? i : 0];
    if (i == 0 && lane == 0 && n > cap) atomicOr(a.err, 16);   // the host sizes cap >= every n
    if (i >= n || i >= cap) return;
    const int w = tab ? a.m : a.r, w4 = align4(w);
    float* blk = (PACK ? a.dsend : a.drecv) + (int64_t)p * a.dblk;
    float* buf = tab ? blk + (int64_t)a.capA * align4(a.r) + align4(a.capA) + (int64_t)i * w4
                     : blk + (int64_t)i * w4;
    float* prow = (tab ? a.W : a.A) + (int64_t)row * w;
    if ((w & 3) == 0) {
        float4* d = reinterpret_cast<float4*>(PACK ? buf : prow);
        const float4* s = reinterpret_cast<const float4*>(PACK ? prow : buf);
        for (int c = lane; c < w / 4; c += RAE_WAVE) d[c] = s[c];
    } else {
        float* d = PACK ? buf : prow;
        const float* s = PACK ? prow : buf;
        for (int c = lane; c < w; c += RAE_WAVE) d[c] = s[c];
    }
    if (!tab && lane == 0) {
        float* ab = blk + (int64_t)a.capA * align4(a.r) + i;
        if (PACK) *ab = a.Ab[row];
        else a.Ab[row] = *ab;
    }
}

}  // namespace rae
