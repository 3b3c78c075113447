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
// (k_build_index, one workgroup per (batch, A|W)), off the step's critical path.
// Layout per batch slot (slot = batch % window):
//   hdr[slot]            = (records, heavy + light rows, heavy rows, very heavy rows)
//   srec[slot][i]        = record id, i in sorted order
//   seg[slot][x]         = (row, first sorted position, end position, first record id) of a
//                          unique row with at most RAE_VHEAVY records; rows with more than
//                          RAE_HEAVY ("heavy": the Zipf-frequent entities / features) fill
//                          x = 0, 1, ... and the light rows fill x = Rcap-1, Rcap-2, ... so the
//                          update can hand the heavy rows -- its longest one-wave tasks -- to
//                          the first-dispatched waves, and a one-record row needs no srec read
//                          (its record rides in the segment)
//   vseg[slot][x]        = the same for rows with more than RAE_VHEAVY records ("very heavy":
//                          tens to hundreds of records at a large global batch), which the
//                          update splits over the four waves of a workgroup
// Records: A-index rec = b*NJ + j (j = 0 e1, 1 e2, 2+t neg1[t], 2+s+t neg2[t]);
//          W-index rec = b << posbits | position of the feature in row b.
// Rows are hash-partitioned (row % H) when a batch has more records than one LDS sort
// holds; partitions are processed one after another by the same workgroup.
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
__host__ __device__ inline int index_partitions(int nrec) {
    return nrec <= RAE_IDX_PART ? 1 : (nrec + RAE_IDX_PART - 1) / RAE_IDX_PART;
}

template <int BT>
__device__ void build_batch_index(const StepArgs& a, int64_t g, int64_t slot, bool isA,
                                  char* smem) {
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);
    int* sint = reinterpret_cast<int*>(keys + RAE_KCAP);   // [0] count, [1..24] scan scratch
    int* sptr = sint + 32;                                   // batch indptr (W index)
    int* sstart = sptr + a.L + 1;                            // segment starts of a partition
    const int tid = threadIdx.x;
    const int64_t ex0 = g * (int64_t)a.L;
    const int NJ = 2 + 2 * a.s;
    const int Rcap = isA ? a.RA : a.RW;
    int32_t* hdr = (isA ? a.hdrA : a.hdrW) + 4 * slot;
    int32_t* srec = (isA ? a.srecA : a.srecW) + slot * (int64_t)Rcap;
    int4* seg = reinterpret_cast<int4*>(isA ? a.urowA : a.urowW) + slot * (int64_t)Rcap;
    const int Vcap = isA ? a.VCA : a.VCW;
    int4* vseg = reinterpret_cast<int4*>(isA ? a.vrowA : a.vrowW) + slot * (int64_t)Vcap;
    if (!isA)
        for (int b = tid; b <= a.L; b += BT) sptr[b] = a.indptr[ex0 + b];
    if (a.priv) {                // private-row masks of this batch: A words 0, 1 / W words 2, 3
        int2* pm = reinterpret_cast<int2*>(a.pmask + slot * (int64_t)a.L * 4) + (isA ? 0 : 1);
        for (int b = tid; b < a.L; b += BT) pm[2 * b] = make_int2(0, 0);
    }
    __syncthreads();
    const int P0 = isA ? 0 : sptr[0];
    const int nrec = isA ? a.L * NJ : sptr[a.L] - P0;
    if (nrec > Rcap) {
        if (tid == 0) {
            atomicOr(a.err, 4);
            hdr[0] = hdr[1] = hdr[2] = hdr[3] = 0;
        }
        return;
    }
    // partitioned data-parallel update: this rank keeps only the rows it owns (row % G == rank),
    // ~nrec / G records, so it sizes its partitions from that share and hashes on row / G (row %
    // H would leave whole partitions empty when gcd(G, H) > 1)
    const int H = index_partitions(a.part ? (nrec + a.G - 1) / a.G : nrec);
    // record at position idx of the batch: its parameter row (and, want_rec, its record id)
    auto rec_at = [&](int idx, int& row, unsigned& rec, bool want_rec) {
        if (isA) {
            const int j = idx / a.L, b = idx - j * a.L;          // j-major: coalesced columns
            const int64_t ex = ex0 + b;
            const int64_t col = a.neg_mode ? ex : (int64_t)b;
            if (j == 0) row = a.args1[ex];
            else if (j == 1) row = a.args2[ex];
            else if (j < 2 + a.s) row = a.neg1[(int64_t)(j - 2) * a.neg_stride + col];
            else row = a.neg2[(int64_t)(j - 2 - a.s) * a.neg_stride + col];
            rec = (unsigned)(b * NJ + j);
        } else {
            row = a.indices[P0 + idx];
            rec = 0;
            if (want_rec) {
                int lo = 0, hi = a.L - 1;                               // example of position idx
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (sptr[mid] - P0 <= idx) lo = mid; else hi = mid - 1;
                }
                rec = ((unsigned)lo << a.posbits) | (unsigned)(idx - (sptr[lo] - P0));
            }
        }
    };
    // partitioned data-parallel update: this rank's update visits only the rows it owns (rae_dp.hpp)
    auto keep = [&](int row) { return !a.part || row % a.G == a.rank; };
    auto part_of = [&](int row) { return (a.part ? row / a.G : row) % H; };
    // More than one partition: the records are binned by partition in ONE pass (an LDS
    // histogram, its prefix sums, a scatter of (row, record) into the slot's srow / srec at the
    // partition's final position -- partition h's sorted records end up in the same range), so
    // the work is two scans of the batch instead of one scan per partition (H ~ records / 1024:
    // 33 scans of 34 k records per batch at L = 800).
    int* hcnt = sstart + RAE_KCAP;                           // H partition sizes
    int* hcur = hcnt + H;                                    // H scatter cursors
    int32_t* srow = (isA ? a.srowA : a.srowW) + slot * (int64_t)Rcap;
    if (H > 1) {
        for (int h = tid; h < H; h += BT) hcnt[h] = 0;
        __syncthreads();
        for (int idx = tid; idx < nrec; idx += BT) {
            int row;
            unsigned rec;
            rec_at(idx, row, rec, false);
            if (keep(row)) atomicAdd(&hcnt[part_of(row)], 1);
        }
        __syncthreads();
        if (tid < RAE_WAVE) {                                // exclusive prefix sum, wave 0
            const int per = (H + RAE_WAVE - 1) / RAE_WAVE, h0 = tid * per;
            int sum = 0;
            for (int h = h0; h < H && h < h0 + per; ++h) sum += hcnt[h];
            int incl = sum;
            for (int o = 1; o < RAE_WAVE; o <<= 1) {
                const int t = __shfl_up(incl, o, RAE_WAVE);
                if (tid >= o) incl += t;
            }
            int ex = incl - sum;
            for (int h = h0; h < H && h < h0 + per; ++h) {
                hcur[h] = ex;
                ex += hcnt[h];
            }
        }
        __syncthreads();
        for (int idx = tid; idx < nrec; idx += BT) {
            int row;
            unsigned rec;
            rec_at(idx, row, rec, true);
            if (keep(row)) {
                const int pos = atomicAdd(&hcur[part_of(row)], 1);
                srow[pos] = row;
                srec[pos] = (int32_t)rec;
            }
        }
        __syncthreads();
    }
    int base_i = 0, nh = 0, nl = 0, nv = 0;
    for (int h = 0; h < H; ++h) {
        if (H > 1) {
            // partition h: its binned records (base == base_i: bins in partition order)
            const int cnt_h = hcnt[h];
            if (tid == 0) sint[0] = cnt_h;
            for (int i = tid; i < cnt_h && i < RAE_KCAP; i += BT)
                keys[i] = ((unsigned long long)(unsigned)srow[base_i + i] << 32) |
                          (unsigned)srec[base_i + i];
        } else {
            if (tid == 0) sint[0] = 0;
            __syncthreads();
            for (int idx = tid; idx < nrec; idx += BT) {
                int row;
                unsigned rec;
                rec_at(idx, row, rec, true);
                if (keep(row)) {
                    const int sl = atomicAdd(&sint[0], 1);
                    if (sl < RAE_KCAP) keys[sl] = ((unsigned long long)(unsigned)row << 32) | rec;
                }
            }
        }
        __syncthreads();
        const int cnt = sint[0];
        if (cnt > RAE_KCAP) {
            if (tid == 0) {
                atomicOr(a.err, isA ? 1 : 2);
                hdr[0] = hdr[1] = hdr[2] = hdr[3] = 0;
            }
            return;
        }
        int n2 = 1;
        while (n2 < cnt) n2 <<= 1;
        for (int i = cnt + tid; i < n2; i += BT) keys[i] = ~0ull;
        __syncthreads();
        lds_bitonic_sort<BT>(keys, n2);
        // segment heads in sorted order -> sstart[local segment]
        int nu = 0;
        for (int i0 = 0; i0 < cnt; i0 += BT) {
            const int i = i0 + tid;
            int head = 0;
            if (i < cnt) {
                const unsigned long long k = keys[i];
                const unsigned row = (unsigned)(k >> 32);
                head = (i == 0) || ((unsigned)(keys[i - 1] >> 32) != row);
                srec[base_i + i] = (int32_t)(unsigned)(k & 0xffffffffull);
            }
            int tot;
            const int u = nu + block_flag_scan<BT>(head, sint + 1, &tot);
            if (head) sstart[u] = i;
            nu += tot;
        }
        __syncthreads();
        // segments -> very heavy rows to vseg, heavy rows at the front of seg, light rows at
        // its back (order kept in each class)
        for (int v0 = 0; v0 < nu; v0 += BT) {
            const int v = v0 + tid;
            const bool valid = v < nu;
            int st = 0, en = 0;
            if (valid) {
                st = sstart[v];
                en = (v + 1 < nu) ? sstart[v + 1] : cnt;
            }
            // private row (StepArgs::priv): one record, of an example whose features the
            // descriptor holds (at most privnf) -- the update's per-example workgroups take it
            // (SP: e2's rows, with no A gradient, stay in the table)
            bool psg = false;
            if (a.priv && valid && en - st == 1) {
                const unsigned rec = (unsigned)(keys[st] & 0xffffffffull);
                if (isA) {
                    const int b = (int)(rec / (unsigned)NJ), j = (int)rec - b * NJ;
                    psg = (j != 1 || a.dec != 0) && a.indptr[ex0 + b + 1] - a.indptr[ex0 + b] <= a.privnf;
                    if (psg) atomicOr(a.pmask + (slot * a.L + b) * 4 + (j >> 5), 1 << (j & 31));
                } else {
                    const int b = (int)(rec >> a.posbits);
                    const int pos = (int)(rec & ((1u << a.posbits) - 1u));
                    psg = sptr[b + 1] - sptr[b] <= a.privnf;
                    if (psg) atomicOr(a.pmask + (slot * a.L + b) * 4 + 2, 1 << pos);
                }
            }
#ifdef RAE_DIAG_NOSINGLE      // timing knockout (wrong results): rows with one record are skipped
            psg = psg || (valid && en - st == 1);
#endif
            const bool vheavy = valid && (en - st) > RAE_VHEAVY;
            const bool heavy = valid && !vheavy && (en - st) > RAE_HEAVY;
            int htot, ltot, vtot;
            const int hp = block_flag_scan<BT>(heavy, sint + 1, &htot);
            const int lp = block_flag_scan<BT>(valid && !psg && (en - st) <= RAE_HEAVY, sint + 12, &ltot);
            const int vp = block_flag_scan<BT>(vheavy, sint + 21, &vtot);
            if (valid) {
                const unsigned long long k = keys[st];
                const int4 sg = make_int4((int)(unsigned)(k >> 32), base_i + st, base_i + en,
                                          (int)(unsigned)(k & 0xffffffffull));
                if (vheavy) vseg[nv + vp] = sg;
                else if (!psg) seg[heavy ? nh + hp : Rcap - 1 - (nl + lp)] = sg;
            }
            nh += htot;
            nl += ltot;
            nv += vtot;
        }
        base_i += cnt;
        __syncthreads();
    }
    if (tid == 0) {
        hdr[0] = base_i;
        hdr[1] = nh + nl;
        hdr[2] = nh;
        hdr[3] = nv;
    }
}

// The update's dispatch table of a slot, built once the A and W indexes of the batch exist
// (a second launch): the update's row waves then find their task with ONE load issued at wave
// start in parallel with the table header, instead of header -> (class counts) -> segment.
//   vtask[slot][v]  very heavy rows (A first, then W), v < NVC: one workgroup each
//   task[slot][t]   wave tasks in dispatch order: very heavy rows beyond NVC, heavy A, heavy W,
//                   light A, light W (the order the update used to derive from the header)
//   thdr[slot]      (wave tasks, workgroup tasks, 0, 0)
// W rows are stored as ~row (negative), A rows as row.
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

template <int BT>
__device__ void build_batch_tasks(const StepArgs& a, int64_t slot) {
    __shared__ int sws[BT / 64];
    const int4 hA = reinterpret_cast<const int4*>(a.hdrA)[slot];
    const int4 hW = reinterpret_cast<const int4*>(a.hdrW)[slot];
    const int HA = hA.z, HW = hW.z, LA = hA.y - hA.z, VA = hA.w, VW = hW.w;
    int4* vt = reinterpret_cast<int4*>(a.vtask) + slot * a.NVC;
    int4* tk = reinterpret_cast<int4*>(a.task) + slot * a.TC;
    const int4* urA = reinterpret_cast<const int4*>(a.urowA) + slot * a.RA;
    const int4* urW = reinterpret_cast<const int4*>(a.urowW) + slot * a.RW;
    auto vrow = [&](int v) {
        int4 sg = v < VA ? reinterpret_cast<const int4*>(a.vrowA)[slot * a.VCA + v]
                         : reinterpret_cast<const int4*>(a.vrowW)[slot * a.VCW + v - VA];
        if (v >= VA) sg.x = ~sg.x;
        return sg;
    };
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
            else tk[i - a.NVC] = sg;
        }
        NU += tu;
    }
    const int NV = min(NC + NU, a.NVC), XV = NC + NU - NV;
    const int T = XV + hA.y + hW.y;
    for (int t = threadIdx.x; t < T - XV; t += BT) {
        int x = t;
        int4 sg;
        if (x < HA) sg = urA[x];
        else if ((x -= HA) < HW) { sg = urW[x]; sg.x = ~sg.x; }
        else if ((x -= HW) < LA) sg = urA[a.RA - 1 - x];
        else { sg = urW[a.RW - 1 - (x - LA)]; sg.x = ~sg.x; }
        tk[XV + t] = sg;
    }
    if (threadIdx.x == 0) reinterpret_cast<int4*>(a.thdr)[slot] = make_int4(T, NV, NF, 0);
}

// Per-example descriptors of the rank's l examples of batch g (slot): everything the forward
// needs before its W-row gather in ONE coalesced read -- the feature count and CSR start,
// the NJ entity ids (e1, e2, neg1[t], neg2[t]) and the first dcap feature ids -- instead of
// the dependent indptr -> indices -> W-row chain (parameter independent, so built ahead).
// With the update's private-row tasks on several ranks (dnx == L) every example of the global
// batch gets one (each rank's update applies all examples' private rows, or its owned ones).
template <int BT>
__device__ void build_batch_desc(const StepArgs& a, int64_t g, int64_t slot) {
    const int NJ = 2 + 2 * a.s, DS = a.dstride;
    int32_t* out = a.desc + slot * (int64_t)a.dnx * DS;
    const int first = a.dnx == a.L ? 0 : a.rank * a.l;
    for (int idx = threadIdx.x; idx < a.dnx * DS; idx += BT) {
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
