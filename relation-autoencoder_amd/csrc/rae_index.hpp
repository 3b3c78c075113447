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
// Records are hash-partitioned by row % H (~RAE_PART records per partition); partition h
// is built by one workgroup: load its records' rows with coalesced, independent loads ->
// 64-bit keys (row << 32 | rec) -> bitonic sort (in registers + wave shuffles for strides
// < 64, through LDS for larger strides) -> head flags + block scan -> unique rows.
#pragma once
#include "rae_common.hpp"
#include "rae_step.hpp"

namespace rae {

// Block-wide exclusive scan of a 0/1 flag (BT threads).  Returns this thread's exclusive
// prefix; *total receives the block total.  `ws` is >= BT/64 ints.
template <int BT>
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
    for (int i = 0; i < BT / 64; ++i) {
        const int c = ws[i];
        off += (i < w) ? c : 0;
        tot += c;
    }
    *total = tot;
    return off + pre;
}

// bitonic compare-exchange step for the element held by thread `i`
__device__ __forceinline__ unsigned long long bitonic_pick(unsigned long long mine,
                                                           unsigned long long other, int i,
                                                           int j, int k) {
    const bool up = (i & k) == 0;
    const bool lower = (i & j) == 0;
    const unsigned long long lo = mine < other ? mine : other;
    const unsigned long long hi = mine < other ? other : mine;
    return (lower == up) ? lo : hi;
}

template <int BT>
__device__ void sort_keys(unsigned long long* keys, int n2) {
    const int tid = threadIdx.x;
    if (n2 <= BT) {
        // one key per thread: strides < 64 through wave shuffles, larger through LDS
        unsigned long long key = keys[tid];
        for (int k = 2; k <= n2; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                unsigned long long other;
                if (j >= 64) {
                    __syncthreads();
                    keys[tid] = key;
                    __syncthreads();
                    other = keys[tid ^ j];
                } else {
                    other = shfl_xor_u64(key, j);
                }
                key = bitonic_pick(key, other, tid, j, k);
            }
        }
        __syncthreads();
        keys[tid] = key;
        __syncthreads();
        return;
    }
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < n2; i += BT) {
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
}

// isA: entity-row index (A / Ab), records (b, j), j < 2+2s:
//   j = 0 -> e1, 1 -> e2, 2+t -> neg1[t], 2+s+t -> neg2[t]        (rec = b*NJ + j)
// !isA: feature-row index (W), records = CSR entries of the batch:
//   rec = b << posbits | position-in-row
template <int BT>
__device__ void build_index_partition(const StepArgs& a, int64_t g, bool isA, int h,
                                      char* smem) {
    constexpr int E = 16;                      // records per thread per pass
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);
    int* sint = reinterpret_cast<int*>(keys + RAE_KCAP);   // [0] count, [1..] scan scratch
    int* sptr = sint + 32;                                   // batch indptr (W index)
    const int tid = threadIdx.x;
    const int H = isA ? a.HA : a.HW;
    const int R = isA ? a.RA : a.RW;
    int32_t* hdr = (isA ? a.hdrA : a.hdrW) + 2 * h;
    int32_t* srec = (isA ? a.srecA : a.srecW) + (int64_t)h * R;
    int32_t* urow = (isA ? a.urowA : a.urowW) + (int64_t)h * R;
    int32_t* ustart = (isA ? a.ustartA : a.ustartW) + (int64_t)h * R;

    if (tid == 0) sint[0] = 0;
    const int64_t ex0 = g * (int64_t)a.L;
    if (!isA)
        for (int b = tid; b <= a.L; b += BT) sptr[b] = a.indptr[ex0 + b];
    __syncthreads();
    if (isA) {
        const int NJ = 2 + 2 * a.s;
        const int nrec = a.L * NJ;
        // enumerate j-major (consecutive threads -> consecutive columns: coalesced)
        for (int base = 0; base < nrec; base += BT * E) {
            int rows[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int idx = base + tid + BT * e;
                rows[e] = -1;
                if (idx < nrec) {
                    const int j = idx / a.L, b = idx - j * a.L;
                    const int64_t ex = ex0 + b;
                    const int64_t col = a.neg_mode ? ex : (int64_t)b;
                    if (j == 0) rows[e] = a.args1[ex];
                    else if (j == 1) rows[e] = a.args2[ex];
                    else if (j < 2 + a.s) rows[e] = a.neg1[(int64_t)(j - 2) * a.neg_stride + col];
                    else rows[e] = a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
                }
            }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int idx = base + tid + BT * e;
                if (rows[e] >= 0 && rows[e] % H == h) {
                    const int j = idx / a.L, b = idx - j * a.L;
                    const unsigned rec = (unsigned)(b * NJ + j);
                    const int slot = atomicAdd(&sint[0], 1);
                    if (slot < RAE_KCAP)
                        keys[slot] = ((unsigned long long)(unsigned)rows[e] << 32) | rec;
                }
            }
        }
    } else {
        const int P0 = sptr[0], nnz = sptr[a.L] - P0;
        for (int base = 0; base < nnz; base += BT * E) {
            int rows[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int idx = base + tid + BT * e;
                rows[e] = (idx < nnz) ? a.indices[P0 + idx] : -1;
            }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int idx = base + tid + BT * e;
                if (rows[e] >= 0 && rows[e] % H == h) {
                    // example of nnz position P0+idx: binary search in the batch indptr
                    int lo = 0, hi = a.L - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (sptr[mid] - P0 <= idx) lo = mid; else hi = mid - 1;
                    }
                    const unsigned rec =
                        ((unsigned)lo << a.posbits) | (unsigned)(idx - (sptr[lo] - P0));
                    const int slot = atomicAdd(&sint[0], 1);
                    if (slot < RAE_KCAP)
                        keys[slot] = ((unsigned long long)(unsigned)rows[e] << 32) | rec;
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
    const int npad = n2 > BT ? n2 : BT;
    for (int i = cnt + tid; i < npad; i += BT) keys[i] = ~0ull;
    __syncthreads();
    sort_keys<BT>(keys, n2);
    // segmentation
    int base = 0;
    for (int i0 = 0; i0 < cnt; i0 += BT) {
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
        const int u = base + block_flag_scan<BT>(head, sint + 1, &tot);
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
