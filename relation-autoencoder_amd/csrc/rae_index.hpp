// Row index of a global batch: for every distinct parameter row the batch references, the
// list of its contributing records in a FIXED order.
//
// The reference's T.grad produces DENSE gradients dW (d,m) / dA (n,r) / dAb (n) by
// inc-subtensor scatter-adds (learning/Optimizers.py:27; the A[...] and Ab[...] reads of
// SelectionalPreferences.py:34-48, Bilinear.py:30-46, BilinearPlusSP.py:39-54, and the
// sparse.dot of RelationClassifier.py:35), then AdaGrad sweeps every row.  Only rows
// referenced by the batch have non-zero gradient (and a zero-gradient AdaGrad step leaves
// a row bit-unchanged), so the update only has to visit the referenced rows once each.
// With records in (row, record id) order the per-row gradient sums are deterministic and
// identical on every data-parallel rank.
//
// The index depends only on the batch's entity ids, negatives and CSR rows -- not on the
// parameters -- so it is built ahead of the steps, for a window of batches per launch
// (k_idx_count -> k_idx_scatter -> k_idx_sort -> k_build_tasks), off the step's critical path.
// Layout per batch slot (slot = batch % window), per table (A: entity rows, W: feature rows):
//   srec[slot][i]        = record id, i in sorted (row, record) order, partition after partition
//   seg[slot][x]         = (row, first sorted position, end position, first record id) of a
//                          distinct row, at its partition's offset in class order: heavy (more
//                          than RAE_HEAVY records: the Zipf-frequent entities / features), light,
//                          very heavy (more than RAE_VHEAVY: split over a workgroup's four waves
//                          by the update); a one-record row needs no srec read (its record rides
//                          in the segment)
//   pcls[slot][p]        = (heavy, light, very heavy rows, offset) of partition p
// Records: A-index rec = b*NJ + j (j = 0 e1, 1 e2, 2+t neg1[t], 2+s+t neg2[t]);
//          W-index rec = b << posbits | position of the feature in row b.
// Rows are hash-partitioned (row % H, ~RAE_IDX_PART records per partition) so one LDS sort
// holds a partition; every partition is sorted by its own workgroup (k_idx_sort).
#pragma once
#include "rae_common.hpp"
#include "rae_step.hpp"

namespace rae {

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

// exclusive block-wide prefix sum of one int per thread (fixed order), and the block total
template <int BT>
__device__ __forceinline__ int block_int_scan(int v, int* ws, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    __syncthreads();
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < BT / 64; ++i) {
        const int c = ws[i];
        off += (i < w) ? c : 0;
        tot += c;
    }
    *total = tot;
    return off + incl - v;
}

// Bitonic sort of n2 (a power of two) 64-bit keys in LDS: one compare-exchange pair (i, i + j)
// per thread and step (pair p -> i with bit j clear), a workgroup barrier per step.  (Running
// the steps whose pairs stay inside one wave's block without the barrier measured no faster.)
template <int BT>
__device__ void lds_bitonic_sort(unsigned long long* keys, int n2) {
    const int tid = threadIdx.x;
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = tid; p < (n2 >> 1); p += BT) {
                const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), ixj = i + j;
                const unsigned long long x = keys[i], y = keys[ixj];
                const bool up = (i & k) == 0;
                if ((x > y) == up) {
                    keys[i] = y;
                    keys[ixj] = x;
                }
            }
            __syncthreads();
        }
    }
}

// records per partition (hash of the row): the bitonic sort's length is the next power of two
// of a partition's records, so ~RAE_IDX_PART keys per partition keep the padding small
#ifndef RAE_IDX_PART
#define RAE_IDX_PART 1024      // measured at C3: 4096 -> 0.98, 2048 -> 0.83, 1024 -> 0.79 us per batch
#endif
#define RAE_IDX_HMAX 1024      // partitions per batch and table (k_build_tasks' LDS prefix tables)
#define RAE_IDX_EPS 32         // examples per slice of the binning launches
__host__ __device__ inline int index_partitions(int nrec) {
    return nrec <= RAE_IDX_PART ? 1 : (nrec + RAE_IDX_PART - 1) / RAE_IDX_PART;
}

// ---- the row index, built in four launches per window of batches ---------------------------
//   k_idx_count    (batch, table, slice of RAE_IDX_EPS examples): the slice's kept records per
//                  hash partition, added into the slot's partition counts (gidx[.][0])
//   k_idx_scatter  (batch, table, slice): the partitions' offsets (exclusive prefix of the
//                  counts), a block per (slice, partition) reserved from the scatter cursors
//                  (gidx[.][1]), the slice's (row, record) keys written there -- binned by
//                  partition, in no particular order inside a partition
//   k_idx_sort     (batch, table, partition): the partition's keys sorted in LDS -> the sorted
//                  record ids (srec, at the partition's offset) and its segments -- one per
//                  distinct row: (row, first position, end position, first record id) --
//                  class-ordered at the same offset: heavy (> RAE_HEAVY records), light, very
//                  heavy (> RAE_VHEAVY); private rows (one record, StepArgs::priv) set their
//                  example's mask bit instead; the class counts per partition (pcls)
//   k_build_tasks  (batch): the update's dispatch table from the partitions' class lists
// Every launch's work is spread over (batch x partition) workgroups -- the whole GPU at a
// data-parallel global batch, where one workgroup per batch and table had sorted every
// partition in turn (28.9 / 65.4 us per batch at G = 8, l = 1024).  Keys are unique
// (row, record) pairs, so the sorted order -- and everything built from it -- is independent of
// the scatter's arbitrary order.
struct IdxTab {
    int nrec, H;                 // records of the table in the batch, hash partitions
    int Rcap;
    int32_t* srec;
    int4* seg;
    unsigned long long* skey;
};
__device__ __forceinline__ IdxTab idx_tab(const StepArgs& a, int64_t g, int64_t slot, int tab) {
    IdxTab t;
    const int64_t ex0 = g * (int64_t)a.L;
    t.nrec = tab ? a.indptr[ex0 + a.L] - a.indptr[ex0] : a.L * (2 + 2 * a.s);
    t.H = index_partitions(a.part ? (t.nrec + a.G - 1) / a.G : t.nrec);
    t.Rcap = tab ? a.RW : a.RA;
    t.srec = (tab ? a.srecW : a.srecA) + slot * (int64_t)t.Rcap;
    t.seg = reinterpret_cast<int4*>(tab ? a.urowW : a.urowA) + slot * (int64_t)t.Rcap;
    t.skey = (tab ? a.skeyW : a.skeyA) + slot * (int64_t)t.Rcap;
    return t;
}
// the slot's partition counts (which 0) / scatter cursors (which 1) of a table
__device__ __forceinline__ int32_t* idx_gc(const StepArgs& a, int64_t slot, int tab, int which) {
    return a.gidx + ((slot * 2 + tab) * 2 + which) * RAE_IDX_HMAX;
}
__device__ __forceinline__ int4* idx_cls(const StepArgs& a, int64_t slot, int tab) {
    return reinterpret_cast<int4*>(a.pcls) + (slot * 2 + tab) * RAE_IDX_HMAX;
}
// partitioned data-parallel update: this rank keeps only the rows it owns (row % G == rank) and
// hashes on row / G (row % H would leave whole partitions empty when gcd(G, H) > 1)
__device__ __forceinline__ bool idx_keep(const StepArgs& a, int row) { return !a.part || row % a.G == a.rank; }
__device__ __forceinline__ int idx_part(const StepArgs& a, int row, int H) {
    return (a.part ? row / a.G : row) % H;
}

// The records of the examples [b0, b1) of global batch g: f(row, record id).
// A-index record = b * NJ + j (j = 0 e1, 1 e2, 2+t neg1[t], 2+s+t neg2[t]), enumerated j-major
// (coalesced columns); W-index record = b << posbits | position of the feature in row b.
template <int BT, class F>
__device__ __forceinline__ void idx_slice_records(const StepArgs& a, int64_t g, int tab, int b0,
                                                  int b1, int* sptr, F&& f) {
    const int tid = threadIdx.x, nb = b1 - b0;
    const int64_t ex0 = g * (int64_t)a.L;
    if (tab == 0) {
        const int NJ = 2 + 2 * a.s;
        for (int idx = tid; idx < NJ * nb; idx += BT) {
            const int j = idx / nb, b = b0 + (idx - j * nb);
            const int64_t ex = ex0 + b;
            const int64_t col = a.neg_mode ? ex : (int64_t)b;
            int row;
            if (j == 0) row = a.args1[ex];
            else if (j == 1) row = a.args2[ex];
            else if (j < 2 + a.s) row = a.neg1[(int64_t)(j - 2) * a.neg_stride + col];
            else row = a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
            f(row, (unsigned)(b * NJ + j));
        }
    } else {
        // the slice's CSR row starts in LDS (sptr: nb + 1 ints), a position's example by
        // binary search there
        const int P0 = sptr[0], n = sptr[nb] - P0;
        for (int idx = tid; idx < n; idx += BT) {
            int lo = 0, hi = nb - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (sptr[mid] - P0 <= idx) lo = mid; else hi = mid - 1;
            }
            const int pos = P0 + idx;
            f(a.indices[pos], ((unsigned)(b0 + lo) << a.posbits) | (unsigned)(pos - sptr[lo]));
        }
    }
}

// k_idx_count: also zeroes the slice's private-row mask words of this table
template <int BT>
__device__ void index_count(const StepArgs& a, int64_t g, int64_t slot, int tab, int z, int* sh) {
    const int tid = threadIdx.x;
    const int b0 = z * RAE_IDX_EPS;
    if (b0 >= a.L) return;
    const int b1 = min(b0 + RAE_IDX_EPS, a.L);
    const IdxTab t = idx_tab(a, g, slot, tab);
    int* hist = sh;
    int* sptr = sh + RAE_IDX_HMAX;
    if (t.H > RAE_IDX_HMAX || t.nrec > t.Rcap) {
        if (tid == 0) atomicOr(a.err, tab ? 2 : 1);
        return;
    }
    for (int h = tid; h < t.H; h += BT) hist[h] = 0;
    if (tab) {
        const int64_t ex0 = g * (int64_t)a.L;
        for (int b = tid; b <= b1 - b0; b += BT) sptr[b] = a.indptr[ex0 + b0 + b];
    }
    if (a.priv) {
        int2* pm = reinterpret_cast<int2*>(a.pmask + slot * (int64_t)a.L * 4) + tab;
        for (int b = b0 + tid; b < b1; b += BT) pm[2 * b] = make_int2(0, 0);
    }
    __syncthreads();
    idx_slice_records<BT>(a, g, tab, b0, b1, sptr, [&](int row, unsigned) {
        if (idx_keep(a, row)) atomicAdd(&hist[idx_part(a, row, t.H)], 1);
    });
    __syncthreads();
    int32_t* gc = idx_gc(a, slot, tab, 0);
    for (int h = tid; h < t.H; h += BT)
        if (hist[h]) atomicAdd(&gc[h], hist[h]);
}

// exclusive prefix sum over n <= RAE_IDX_HMAX ints of LDS `v` in place (BT threads)
template <int BT>
__device__ __forceinline__ void lds_exclusive_scan(int* v, int n, int* ws) {
    constexpr int PER = (RAE_IDX_HMAX + BT - 1) / BT;
    const int tid = threadIdx.x, h0 = tid * PER;
    int x[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        x[k] = h0 + k < n ? v[h0 + k] : 0;
        sum += x[k];
    }
    int tot;
    int ex = block_int_scan<BT>(sum, ws, &tot);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (h0 + k < n) v[h0 + k] = ex;
        ex += x[k];
    }
    __syncthreads();
}

template <int BT>
__device__ void index_scatter(const StepArgs& a, int64_t g, int64_t slot, int tab, int z, int* sh) {
    const int tid = threadIdx.x;
    const int b0 = z * RAE_IDX_EPS;
    if (b0 >= a.L) return;
    const int b1 = min(b0 + RAE_IDX_EPS, a.L);
    const IdxTab t = idx_tab(a, g, slot, tab);
    if (t.H > RAE_IDX_HMAX || t.nrec > t.Rcap) return;         // k_idx_count flagged it
    int* pre = sh;                                   // partition offsets
    int* cur = sh + RAE_IDX_HMAX;                    // this slice's block cursors
    int* sptr = sh + 2 * RAE_IDX_HMAX;
    int* ws = sptr + RAE_IDX_EPS + 1;
    const int32_t* gc = idx_gc(a, slot, tab, 0);
    for (int h = tid; h < t.H; h += BT) {
        pre[h] = gc[h];
        cur[h] = 0;
    }
    if (tab) {
        const int64_t ex0 = g * (int64_t)a.L;
        for (int b = tid; b <= b1 - b0; b += BT) sptr[b] = a.indptr[ex0 + b0 + b];
    }
    __syncthreads();
    lds_exclusive_scan<BT>(pre, t.H, ws);
    idx_slice_records<BT>(a, g, tab, b0, b1, sptr, [&](int row, unsigned) {
        if (idx_keep(a, row)) atomicAdd(&cur[idx_part(a, row, t.H)], 1);
    });
    __syncthreads();
    int32_t* gcur = idx_gc(a, slot, tab, 1);
    for (int h = tid; h < t.H; h += BT)
        if (cur[h]) cur[h] = pre[h] + atomicAdd(&gcur[h], cur[h]);
    __syncthreads();
    idx_slice_records<BT>(a, g, tab, b0, b1, sptr, [&](int row, unsigned rec) {
        if (idx_keep(a, row)) {
            const int pos = atomicAdd(&cur[idx_part(a, row, t.H)], 1);
            t.skey[pos] = ((unsigned long long)(unsigned)row << 32) | rec;
        }
    });
}

// exclusive block-wide prefix sums of NF flags per thread at once: one ballot per flag and wave,
// one barrier pair for all of them (ws >= NF * BT / 64 ints)
template <int BT, int NF>
__device__ __forceinline__ void block_flags_scan(const bool (&f)[NF], int* ws, int (&pre)[NF],
                                                 int (&tot)[NF]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int in[NF];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NF; ++q) {
        const unsigned long long bal = __ballot(f[q]);
        in[q] = __popcll(bal & lt);
        if (lane == 0) ws[q * (BT / 64) + w] = __popcll(bal);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NF; ++q) {
        int off = 0, t = 0;
#pragma unroll
        for (int i = 0; i < BT / 64; ++i) {
            const int c = ws[q * (BT / 64) + i];
            off += (i < w) ? c : 0;
            t += c;
        }
        pre[q] = off + in[q];
        tot[q] = t;
    }
}

// Bitonic sort of the partition's keys held in registers, RAE_IDX_KPT per thread (position
// p = KPT tid + e), over the first n2 (a power of two <= KPT BT) positions: compare-exchange
// partners inside a thread are register pairs, inside a wave DPP / permlane lane swaps, across
// waves an LDS round (keys, KPT BT entries) -- 6 of the 66 steps at 2048 keys carry a barrier,
// where the all-LDS sort had a barrier and four LDS accesses per step.
#define RAE_IDX_KPT 4
#define RAE_IDX_FAST (RAE_IDX_KPT * RAE_FBT)    // partitions of up to 2048 keys: k_idx_sort
// one compare-exchange step (k = 2^LK, j = 2^LJ) on the register keys
template <int BT, int LK, int LJ>
__device__ __forceinline__ void reg_bitonic_step(unsigned long long (&kv)[RAE_IDX_KPT],
                                                 unsigned long long* keys) {
    constexpr int KPT = RAE_IDX_KPT, k = 1 << LK, j = 1 << LJ;
    const int tid = threadIdx.x;
    unsigned long long pv[KPT];
    if constexpr (j >= KPT * RAE_WAVE) {              // partner in another wave: LDS
#pragma unroll
        for (int e = 0; e < KPT; ++e) keys[KPT * tid + e] = kv[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < KPT; ++e) pv[e] = keys[(KPT * tid + e) ^ j];
        __syncthreads();
    } else if constexpr (j >= KPT) {                  // partner lane: lane ^ (j / KPT)
#pragma unroll
        for (int e = 0; e < KPT; ++e) pv[e] = xor_lane_u64(kv[e], j / KPT);
    } else {                                          // partner register
#pragma unroll
        for (int e = 0; e < KPT; ++e) pv[e] = kv[e ^ j];
    }
#pragma unroll
    for (int e = 0; e < KPT; ++e) {
        const int p = KPT * tid + e;
        const bool take_min = ((p & k) == 0) == ((p & j) == 0);
        const unsigned long long lo = kv[e] < pv[e] ? kv[e] : pv[e];
        const unsigned long long hi = kv[e] < pv[e] ? pv[e] : kv[e];
        kv[e] = take_min ? lo : hi;
    }
}
template <int BT, int LK, int LJ>
__device__ __forceinline__ void reg_bitonic_level(unsigned long long (&kv)[RAE_IDX_KPT],
                                                  unsigned long long* keys) {
    reg_bitonic_step<BT, LK, LJ>(kv, keys);
    if constexpr (LJ > 0) reg_bitonic_level<BT, LK, LJ - 1>(kv, keys);
}
template <int BT, int LK, int LOGN>
__device__ __forceinline__ void reg_bitonic_levels(unsigned long long (&kv)[RAE_IDX_KPT], int n2,
                                                   unsigned long long* keys) {
    if ((1 << LK) > n2) return;                      // uniform: the first n2 positions are sorted
    reg_bitonic_level<BT, LK, LK - 1>(kv, keys);
    if constexpr (LK < LOGN) reg_bitonic_levels<BT, LK + 1, LOGN>(kv, n2, keys);
}
template <int BT>
__device__ __forceinline__ void reg_bitonic_sort(unsigned long long (&kv)[RAE_IDX_KPT], int n2,
                                                 unsigned long long* keys) {
    constexpr int LOGN = 11;                          // 2^11 = KPT * BT (BT = 512)
    static_assert(RAE_IDX_KPT * BT == (1 << LOGN), "fast sort size");
    reg_bitonic_levels<BT, 1, LOGN>(kv, n2, keys);
}

// k_idx_sort (big = false: partitions of up to RAE_IDX_FAST keys, register sort, small LDS ->
// several workgroups per CU) and k_idx_sort_big (the rare larger partitions, up to RAE_KCAP
// keys, LDS sort): partition h of a table
template <int BT, bool BIG>
__device__ void index_sort(const StepArgs& a, int64_t g, int64_t slot, int tab, int h, char* smem) {
    const int tid = threadIdx.x;
    const IdxTab t = idx_tab(a, g, slot, tab);
    if (h >= t.H || t.H > RAE_IDX_HMAX || t.nrec > t.Rcap) return;
    const int32_t* gc = idx_gc(a, slot, tab, 0);
    const int cnt = gc[h];
    if (BIG != (cnt > RAE_IDX_FAST)) return;            // the other launch's partition
    constexpr int KC = BIG ? RAE_KCAP : RAE_IDX_FAST;
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);
    int* sint = reinterpret_cast<int*>(keys + KC);      // [0..63] scan scratch
    int* sstart = sint + 64;                             // segment starts (<= KC)
    // the partition's offset: the counts of partitions 0..h-1
    int part = 0;
    for (int k = tid; k < h; k += BT) part += gc[k];
    int base;
    block_int_scan<BT>(part, sint, &base);
    int4* cls = idx_cls(a, slot, tab);
    if (cnt > RAE_KCAP) {
        if (tid == 0) {
            atomicOr(a.err, tab ? 2 : 1);
            cls[h] = make_int4(0, 0, 0, base);
        }
        return;
    }
    int n2 = 1;
    while (n2 < cnt) n2 <<= 1;
    if constexpr (BIG) {
        for (int i = tid; i < cnt; i += BT) keys[i] = t.skey[base + i];
        for (int i = cnt + tid; i < n2; i += BT) keys[i] = ~0ull;
        __syncthreads();
        lds_bitonic_sort<BT>(keys, n2);
    } else {
        unsigned long long kv[RAE_IDX_KPT];
#pragma unroll
        for (int e = 0; e < RAE_IDX_KPT; ++e) {
            const int p = RAE_IDX_KPT * tid + e;
            kv[e] = p < cnt ? t.skey[base + p] : ~0ull;
        }
        reg_bitonic_sort<BT>(kv, n2, keys);
#pragma unroll
        for (int e = 0; e < RAE_IDX_KPT; ++e) keys[RAE_IDX_KPT * tid + e] = kv[e];
        __syncthreads();
    }
    // segment heads in sorted order -> sstart[segment]
    int nu = 0;
    for (int i0 = 0; i0 < cnt; i0 += BT) {
        const int i = i0 + tid;
        bool head[1] = {false};
        if (i < cnt) {
            const unsigned long long k = keys[i];
            head[0] = (i == 0) || ((unsigned)(keys[i - 1] >> 32) != (unsigned)(k >> 32));
            t.srec[base + i] = (int32_t)(unsigned)(k & 0xffffffffull);
        }
        int pre[1], tot[1];
        block_flags_scan<BT, 1>(head, sint, pre, tot);
        if (head[0]) sstart[nu + pre[0]] = i;
        nu += tot[0];
    }
    __syncthreads();
    const int64_t ex0 = g * (int64_t)a.L;
    const int NJ = 2 + 2 * a.s;
    // segment v's class: 0 heavy, 1 light, 2 very heavy, 3 private (mask bit set, no task)
    auto seg_class = [&](int v, int& st, int& en, bool mark) {
        st = sstart[v];
        en = (v + 1 < nu) ? sstart[v + 1] : cnt;
        // private row (StepArgs::priv): one record, of an example whose features the
        // descriptor holds (at most privnf) -- the update's per-example workgroups take it
        // (SP: e2's rows, with no A gradient, stay in the table)
        if (a.priv && en - st == 1) {
            const unsigned rec = (unsigned)(keys[st] & 0xffffffffull);
            bool psg;
            if (tab == 0) {
                const int b = (int)(rec / (unsigned)NJ), j = (int)rec - b * NJ;
                psg = (j != 1 || a.dec != 0) && a.indptr[ex0 + b + 1] - a.indptr[ex0 + b] <= a.privnf;
                if (psg && mark) atomicOr(a.pmask + (slot * a.L + b) * 4 + (j >> 5), 1 << (j & 31));
            } else {
                const int b = (int)(rec >> a.posbits);
                const int pos = (int)(rec & ((1u << a.posbits) - 1u));
                psg = a.indptr[ex0 + b + 1] - a.indptr[ex0 + b] <= a.privnf;
                if (psg && mark) atomicOr(a.pmask + (slot * a.L + b) * 4 + 2, 1 << pos);
            }
#ifdef RAE_DIAG_NOSINGLE      // timing knockout (wrong results): rows with one record are skipped
            psg = true;
#endif
            if (psg) return 3;
        }
#ifdef RAE_DIAG_NOSINGLE
        if (en - st == 1) return 3;
#endif
        return (en - st) > RAE_VHEAVY ? 2 : ((en - st) > RAE_HEAVY ? 0 : 1);
    };
    // pass 1: class counts; pass 2: every segment at its class position (order kept per class)
    int n[3] = {0, 0, 0};
    for (int v0 = 0; v0 < nu; v0 += BT) {
        const int v = v0 + tid;
        int st, en, c = -1;
        if (v < nu) c = seg_class(v, st, en, false);
        const bool f[3] = {c == 0, c == 1, c == 2};
        int pre[3], tot[3];
        block_flags_scan<BT, 3>(f, sint, pre, tot);
#pragma unroll
        for (int k = 0; k < 3; ++k) n[k] += tot[k];
    }
    int o[3] = {0, n[0], n[0] + n[1]};
    for (int v0 = 0; v0 < nu; v0 += BT) {
        const int v = v0 + tid;
        int st = 0, en = 0, c = -1;
        if (v < nu) c = seg_class(v, st, en, true);
        const bool f[3] = {c == 0, c == 1, c == 2};
        int pre[3], tot[3];
        block_flags_scan<BT, 3>(f, sint, pre, tot);
        if (c >= 0 && c < 3) {
            const unsigned long long k = keys[st];
            const int pos = c == 0 ? o[0] + pre[0] : (c == 1 ? o[1] + pre[1] : o[2] + pre[2]);
            t.seg[base + pos] = make_int4((int)(unsigned)(k >> 32), base + st, base + en,
                                                    (int)(unsigned)(k & 0xffffffffull));
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) o[k] += tot[k];
    }
    if (tid == 0) cls[h] = make_int4(n[0], n[1], n[2], base);
}

// The update's dispatch table of a slot, built once every partition of the batch is sorted:
// the update's row waves then find their task with ONE load issued at wave start in parallel
// with the table header.
//   vtask[slot][v]  very heavy rows (A first, then W), v < NVC: one workgroup each
//   task[slot][t]   wave tasks in dispatch order: heavy A, heavy W, light A, light W, then the
//                   very heavy rows beyond NVC (none at all in plans whose NVC covers them)
//   thdr[slot]      (wave tasks, workgroup tasks, chunked rows, 0)
// W rows are stored as ~row (negative), A rows as row.  Workgroup z of the batch copies table
// entries [z RAE_TASK_PER, (z + 1) RAE_TASK_PER); workgroup 0 also lays out the very heavy rows.
// LDS: for each table and class (heavy, light, very heavy) the exclusive prefix of the
// partitions' class counts (RAE_IDX_HMAX + 1 ints each); an entry's partition is found by
// binary search there.
#define RAE_TASK_PER 2048
template <int BT>
__device__ void build_batch_tasks(const StepArgs& a, int64_t g, int64_t slot, int z, int* sh) {
    __shared__ int sws[BT / 64];
    int Ht[2];
    const int4* clsT[2] = {idx_cls(a, slot, 0), idx_cls(a, slot, 1)};
    int tot[2][3];
    for (int tab = 0; tab < 2; ++tab) {
        Ht[tab] = idx_tab(a, g, slot, tab).H;
        if (Ht[tab] > RAE_IDX_HMAX) Ht[tab] = 0;           // flagged by k_idx_count
        for (int c = 0; c < 3; ++c) {
            int* pf = sh + (tab * 3 + c) * (RAE_IDX_HMAX + 1);
            int x = 0;
            for (int h = threadIdx.x; h < Ht[tab]; h += BT) {
                const int4 q = clsT[tab][h];
                pf[h] = c == 0 ? q.x : (c == 1 ? q.y : q.z);
                x += pf[h];
            }
            int t_;
            block_int_scan<BT>(x, sws, &t_);
            tot[tab][c] = t_;
            lds_exclusive_scan<BT>(pf, Ht[tab], sws);
        }
    }
    // entry x of class c of table tab -> its segment
    auto seg_of = [&](int tab, int c, int x) {
        const int* pf = sh + (tab * 3 + c) * (RAE_IDX_HMAX + 1);
        int lo = 0, hi = Ht[tab] - 1;                      // last partition with pf[h] <= x
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pf[mid] <= x) lo = mid; else hi = mid - 1;
        }
        const int4 q = clsT[tab][lo];
        const int off = c == 0 ? 0 : (c == 1 ? q.x : q.x + q.y);
        int4 sg = reinterpret_cast<const int4*>(tab ? a.urowW : a.urowA)[slot * (int64_t)(tab ? a.RW : a.RA) +
                                                                          q.w + off + (x - pf[lo])];
        if (tab) sg.x = ~sg.x;
        return sg;
    };
    const int VA = tot[0][2], VW = tot[1][2];
    const int HA = tot[0][0], HW = tot[1][0], LA = tot[0][1], LW = tot[1][1];
    const int TH = HA + HW + LA + LW;
    int4* vt = reinterpret_cast<int4*>(a.vtask) + slot * a.NVC;
    int4* tk = reinterpret_cast<int4*>(a.task) + slot * a.TC;
    for (int t = z * RAE_TASK_PER + threadIdx.x; t < min(TH, (z + 1) * RAE_TASK_PER); t += BT) {
        int x = t;
        int4 sg;
        if (x < HA) sg = seg_of(0, 0, x);
        else if ((x -= HA) < HW) sg = seg_of(1, 0, x);
        else if ((x -= HW) < LA) sg = seg_of(0, 1, x);
        else sg = seg_of(1, 1, x - LA);
        tk[t] = sg;
    }
    if (z != 0) return;
    auto vrow = [&](int v) { return v < VA ? seg_of(0, 2, v) : seg_of(1, 2, v - VA); };
    // very heavy rows: rows with at least 2 hch records become floor(records / hch) chunk tasks
    // (the first vtask entries; chunk k = records [st + k hch, st + (k+1) hch), the last one
    // to the row's end: hch .. 2 hch - 1 records) plus a combine entry; the others keep one
    // workgroup task each, overflowing to wave tasks beyond NVC.  With floor counting a batch
    // has at most records / hch < HF < NVC chunks and fewer than HF chunked rows (rae.hip sizes
    // NVC >= HF + 1), so every chunk and combine entry has its slot (ceil counting
    // could exceed NVC and leave k_heavy_fin reading partials no chunk task wrote).
    auto nchunks = [&](int cnt) { return (a.hch > 0 && cnt >= 2 * a.hch) ? cnt / a.hch : 0; };
    int NC = 0, NF = 0, NU = 0;
    if (a.hch > 0) {
        int4* hf = reinterpret_cast<int4*>(a.hfin) + slot * a.HF;
        for (int v0 = 0; v0 < VA + VW; v0 += BT) {
            const int v = v0 + threadIdx.x;
            int4 sg = make_int4(0, 0, 0, 0);
            int nch = 0;
            if (v < VA + VW) {
                sg = vrow(v);
                nch = nchunks(sg.z - sg.y);
            }
            int tc, tf;
            const int cb = NC + block_int_scan<BT>(nch, sws, &tc);
            const int fb = NF + block_int_scan<BT>(nch > 0 ? 1 : 0, sws, &tf);
            for (int k = 0; k < nch; ++k) {
                const int c = cb + k;
                const int e = (k + 1 == nch) ? sg.z : sg.y + (k + 1) * a.hch;
                vt[c] = make_int4(sg.x, sg.y + k * a.hch, e, -1 - c);
            }
            if (nch > 0) hf[fb] = make_int4(sg.x, cb, nch, 0);
            NC += tc;
            NF += tf;
        }
    }
    for (int v0 = 0; v0 < VA + VW; v0 += BT) {        // the unchunked very heavy rows
        const int v = v0 + threadIdx.x;
        int4 sg = make_int4(0, 0, 0, 0);
        bool un = false;
        if (v < VA + VW) {
            sg = vrow(v);
            un = nchunks(sg.z - sg.y) == 0;
        }
        int tu;
        const int i = NC + NU + block_int_scan<BT>(un ? 1 : 0, sws, &tu);
        if (un) {
            if (i < a.NVC) vt[i] = sg;
            else tk[TH + i - a.NVC] = sg;
        }
        NU += tu;
    }
    const int NV = min(NC + NU, a.NVC), XV = NC + NU - NV;
    if (threadIdx.x == 0) reinterpret_cast<int4*>(a.thdr)[slot] = make_int4(TH + XV, NV, NF, 0);
}

// Per-example descriptors of the rank's l examples of batch g (slot): everything the forward
// needs before its W-row gather in ONE coalesced read -- the feature count and CSR start,
// the NJ entity ids (e1, e2, neg1[t], neg2[t]) and the first dcap feature ids -- instead of
// the dependent indptr -> indices -> W-row chain (parameter independent, so built ahead).
// With the update's private-row tasks on several ranks (dnx == L) every example of the global
// batch gets one (each rank's update applies all examples' private rows, or its owned ones).
// (descriptor examples [z RAE_IDX_EPS, (z + 1) RAE_IDX_EPS) of the slot: one slice)
template <int BT>
__device__ void build_batch_desc(const StepArgs& a, int64_t g, int64_t slot, int z) {
    const int NJ = 2 + 2 * a.s, DS = a.dstride;
    int32_t* out = a.desc + slot * (int64_t)a.dnx * DS;
    const int first = a.dnx == a.L ? 0 : a.rank * a.l;
    const int e0 = z * RAE_IDX_EPS, e1 = min(e0 + RAE_IDX_EPS, a.dnx);
    for (int idx = e0 * DS + threadIdx.x; idx < e1 * DS; idx += BT) {
        const int bl = idx / DS, t = idx - bl * DS;
        const int bg = first + bl;
        const int64_t ex = g * (int64_t)a.L + bg;
        const int64_t col = a.neg_mode ? ex : (int64_t)bg;
        const int p0 = a.indptr[ex];
        int v = 0;
        if (t == 0) v = a.indptr[ex + 1] - p0;
        else if (t == 1) v = p0;
        else if (t < 2 + NJ) {
            const int j = t - 2;
            v = (j == 0) ? a.args1[ex] : (j == 1) ? a.args2[ex]
              : (j < 2 + a.s) ? a.neg1[(int64_t)(j - 2) * a.neg_stride + col]
                              : a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
        } else {
            const int f = t - 2 - NJ;
            if (f < a.dcap && f < a.indptr[ex + 1] - p0) v = a.indices[p0 + f];
        }
        out[idx] = v;
    }
}

}  // namespace rae
