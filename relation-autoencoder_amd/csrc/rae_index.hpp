// Per-step row index of the global batch, built by dedicated "index workgroups" that run
// inside the forward kernel beside the per-example workgroups.
//
// The reference's T.grad produces DENSE gradients dW (d,m) / dA (n,r) / dAb (n) by
// inc-subtensor scatter-adds (learning/Optimizers.py:27; the A[...] and Ab[...] reads of
// SelectionalPreferences.py:34-48, Bilinear.py:30-46, BilinearPlusSP.py:39-54, and the
// sparse.dot of RelationClassifier.py:35), then AdaGrad sweeps every row.  Only rows
// referenced by the batch have non-zero gradient (and a zero-gradient AdaGrad step leaves
// a row bit-unchanged), so the update only has to visit the referenced rows once each.
// This index lists, for every distinct referenced row, its contributing records in a
// FIXED order (row, record id) -- the per-row gradient sums are then deterministic and
// identical on every data-parallel rank.
//
// Records are hash-partitioned by row % H; partition h is built by one workgroup:
//   gather its records -> 64-bit keys (row << 32 | rec) in LDS -> bitonic sort ->
//   head flags + block scan -> unique rows with segment starts.
#pragma once
#include "rae_common.hpp"
#include "rae_step.hpp"

namespace rae {

// Block-wide exclusive scan of a 0/1 flag (RAE_BT threads). Returns this thread's
// exclusive prefix; *total receives the block total.  `ws` is >= RAE_NWAVE+1 ints.
__device__ __forceinline__ int block_flag_scan(int flag, int* ws, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long bal = __ballot(flag);
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int pre = __popcll(bal & lt);
    __syncthreads();
    if (lane == 0) ws[w] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < RAE_NWAVE; ++i) {
        const int c = ws[i];
        off += (i < w) ? c : 0;
        tot += c;
    }
    *total = tot;
    return off + pre;
}

// isA: entity-row index (A / Ab), records (b, j), j < 2+2s:
//   j = 0 -> e1, 1 -> e2, 2+t -> neg1[t], 2+s+t -> neg2[t]        (rec = b*NJ + j)
// !isA: feature-row index (W), records = CSR entries of the batch:
//   rec = b << posbits | position-in-row
__device__ void build_index_partition(const StepArgs& a, int64_t g, bool isA, int h,
                                      char* smem) {
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);
    int* sint = reinterpret_cast<int*>(keys + RAE_KCAP);   // [0] count, [1..] scan scratch
    const int tid = threadIdx.x;
    const int H = isA ? a.HA : a.HW;
    const int R = isA ? a.RA : a.RW;
    int32_t* hdr = (isA ? a.hdrA : a.hdrW) + 2 * h;
    int32_t* srec = (isA ? a.srecA : a.srecW) + (int64_t)h * R;
    int32_t* urow = (isA ? a.urowA : a.urowW) + (int64_t)h * R;
    int32_t* ustart = (isA ? a.ustartA : a.ustartW) + (int64_t)h * R;

    if (tid == 0) sint[0] = 0;
    __syncthreads();
    const int64_t ex0 = g * (int64_t)a.L;
    if (isA) {
        const int NJ = 2 + 2 * a.s;
        const int nrec = a.L * NJ;
        for (int rec = tid; rec < nrec; rec += RAE_BT) {
            const int b = rec / NJ;
            const int j = rec - b * NJ;
            const int64_t ex = ex0 + b;
            const int64_t col = a.neg_mode ? ex : (int64_t)b;
            int row;
            if (j == 0) row = a.args1[ex];
            else if (j == 1) row = a.args2[ex];
            else if (j < 2 + a.s) row = a.neg1[(int64_t)(j - 2) * a.neg_stride + col];
            else row = a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
            if (row % H == h) {
                const int slot = atomicAdd(&sint[0], 1);
                if (slot < RAE_KCAP)
                    keys[slot] = ((unsigned long long)(unsigned)row << 32) | (unsigned)rec;
            }
        }
    } else {
        for (int b = tid; b < a.L; b += RAE_BT) {
            const int64_t ex = ex0 + b;
            const int p0 = a.indptr[ex], p1 = a.indptr[ex + 1];
            for (int p = p0; p < p1; ++p) {
                const int row = a.indices[p];
                if (row % H == h) {
                    const int slot = atomicAdd(&sint[0], 1);
                    const unsigned rec = ((unsigned)b << a.posbits) | (unsigned)(p - p0);
                    if (slot < RAE_KCAP)
                        keys[slot] = ((unsigned long long)(unsigned)row << 32) | rec;
                }
            }
        }
    }
    __syncthreads();
    const int cnt = sint[0];
    if (cnt > RAE_KCAP || cnt > R) {
        if (tid == 0) {
            atomicOr(a.err, isA ? 1 : 2);
            hdr[0] = 0;
            hdr[1] = 0;
        }
        return;
    }
    int n2 = 1;
    while (n2 < cnt) n2 <<= 1;
    for (int i = cnt + tid; i < n2; i += RAE_BT) keys[i] = ~0ull;
    __syncthreads();
    // bitonic sort, ascending
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < n2; i += RAE_BT) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long x = keys[i], y = keys[ixj];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) {
                        keys[i] = y;
                        keys[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    // segmentation
    int base = 0;
    for (int i0 = 0; i0 < cnt; i0 += RAE_BT) {
        const int i = i0 + tid;
        int head = 0;
        unsigned row = 0;
        if (i < cnt) {
            const unsigned long long k = keys[i];
            row = (unsigned)(k >> 32);
            head = (i == 0) || ((unsigned)(keys[i - 1] >> 32) != row);
            srec[i] = (int32_t)(unsigned)(k & 0xffffffffull);
        }
        int tot;
        const int u = base + block_flag_scan(head, sint + 1, &tot);
        if (head) {
            urow[u] = (int32_t)row;
            ustart[u] = i;
        }
        base += tot;
    }
    if (tid == 0) {
        hdr[0] = cnt;
        hdr[1] = base;
    }
}

// Locate task t among the unique rows of H partitions: returns partition, sets *u.
__device__ __forceinline__ int locate_row(const int32_t* hdr, int H, int t, int* u) {
    int h = 0;
    for (; h < H; ++h) {
        const int U = hdr[2 * h + 1];
        if (t < U) break;
        t -= U;
    }
    *u = t;
    return h;
}

__device__ __forceinline__ int total_rows(const int32_t* hdr, int H) {
    int tot = 0;
    for (int h = 0; h < H; ++h) tot += hdr[2 * h + 1];
    return tot;
}

}  // namespace rae
