// Kernel argument block and exchange-record layout shared by the step kernels.
#pragma once
#include <stdint.h>

namespace rae {

// Per-example record in the exchange buffer (floats).
//   P (m) | dS (m) | V1 (r) | V2 (r) | dw1 (r) | dw2 (r) | G1 (r) |
//   [bilinear: G2 (r) | X (r) | Y (r) | A1 (r) | A2 (r) | z = S - max S (m) | aux (4)] |
//   coef (2*NJ) | loss (1) | pad
// coef[j] = (c_j, gamma_j) for record j (0: e1, 1: e2, 2+t: neg1[t], 2+s+t: neg2[t]):
// record j's A-row gradient is c_j * vec_j and its Ab gradient gamma_j, with
// vec_0 = G1, vec_1 = G2 (bilinear; SP: c_1 = 0), vec_{neg1} = V1, vec_{neg2} = V2 -- one
// vector per record, so the update reads exactly one r-vector per referencing record.
// SP       : V1 = wC1 = C1.P, V2 = wC2, G1 = dl*wC1 + dr*wC2 (e1's whole A gradient),
//            dw1/dw2 = dCost/dwC1, dCost/dwC2.
// bilinear : V1 = M a2 (+ wC1), V2 = M^T a1 (+ wC2) with M = sum_k P_k R[:,:,k];
//            G1/G2 = the full A-row gradients of e1/e2; X, Y, A1, A2 the rank-2 factors of
//            dCost/dM = X A2^T + A1 Y^T (A1/A2 = copies of A[e1], A[e2] taken before the
//            update kernel changes A); dw1/dw2 as SP for the hybrid.  Forward scratch:
//            G1/G2 hold M a2 / M^T a1 until k_bil_fin, aux = (dOne, c_a1, c_a2) from
//            k_bil_dec.
//
// Wire record (SP decoder, world_size > 1): what crosses xGMI in the all-gather.  V1, V2 and G1
// are dropped -- every rank recomputes them for the whole global batch after the exchange
// (k_vrec: V = P.C^T on fp32 MFMA, G1 = dl V1 + dr V2 from aux = (dl, dr)), which the update
// reads from the vector buffer (StepArgs::vb) -- 692 instead of 1,288 floats per example at C3:
//   P (m) | dS (m) | dw1 (r) | dw2 (r) | aux (4: dl, dr) | coef (2*NJ) | loss (1) | pad
// With dense partials (wire 2, rae.h RAE_DPDENSE_PARTIALS) the rank reduces the decoder-matrix
// gradients of its OWN l examples (k_dpart: dC1, dC2, dWb over K = l) and the records carry that
// partial block -- pc floats each, rank k's element e in record k l + e / pc -- instead of dw1 /
// dw2; the update sums the G partials in rank order (no K = L chain):
//   P (m) | dS (m) | aux (4) | coef (2*NJ) | loss (1) | pad | partial chunk (pc)
struct RecLayout {
    int oP, odS, oV1, oV2, odw1, odw2, oG1, ocoef, oloss, rec;
    int oG2, oX, oY, oA1, oA2, oZ, oAux;   // bilinear decoders (and oAux of the SP wire record)
    int wire;                              // 1: SP wire record (no V1 / V2 / G1: -1); 2: + partials
    int oPart, pc;                         // wire 2: the partial chunk (-1 / 0 otherwise)
};

__host__ __device__ inline int align4(int x) { return (x + 3) & ~3; }

// wire: the SP decoder's data-parallel exchange record (ignored for the bilinear decoders)
// floats of one rank's dense partial block: dC1 (r, m) | dC2 (r, m) | dWb (m)
__host__ __device__ inline int dense_partial_floats(int r, int m) { return 2 * r * m + m; }

__host__ __device__ inline RecLayout make_layout(int dec, int m, int r, int s, int wire = 0,
                                                 int l = 1) {
    RecLayout L{};
    const int NJ = 2 + 2 * s;
    const int m4 = align4(m), r4 = align4(r);
    L.oP = 0;
    L.odS = m4;
    L.oPart = -1;
    if (dec == 0 && wire) {
        L.wire = wire;
        L.oV1 = L.oV2 = L.oG1 = -1;
        int o = 2 * m4;
        if (wire == 1) {
            L.odw1 = o;
            L.odw2 = o + r4;
            o += 2 * r4;
        } else {
            L.odw1 = L.odw2 = -1;
        }
        L.oAux = o;
        L.ocoef = L.oAux + 4;
        L.oloss = L.ocoef + align4(2 * NJ);
        o = align4(L.oloss + 1);
        if (wire == 2) {
            L.pc = align4((dense_partial_floats(r, m) + l - 1) / l);
            L.oPart = o;
            o += L.pc;
        }
        L.rec = o;
        return L;
    }
    L.oV1 = 2 * m4;
    L.oV2 = L.oV1 + r4;
    L.odw1 = L.oV2 + r4;
    L.odw2 = L.odw1 + r4;
    L.oG1 = L.odw2 + r4;
    int o = L.oG1 + r4;
    if (dec != 0) {
        L.oG2 = o; o += r4;
        L.oX = o; o += r4;
        L.oY = o; o += r4;
        L.oA1 = o; o += r4;
        L.oA2 = o; o += r4;
        L.oZ = o; o += m4;
        L.oAux = o; o += 4;
    }
    L.ocoef = o;
    o += align4(2 * NJ);
    L.oloss = o;
    L.rec = align4(o + 1);
    return L;
}

// one data-parallel peer's buffers as this rank maps them (rae_set_peer; the peer-to-peer
// exchange, rae_p2p.hpp); peer == rank: this rank's own
struct PeerBufs {
    float* ex;
    float* W;
    float* A;
    float* Ab;
    unsigned* sig;        // [2 kinds][G writers] signal counters
};

struct StepArgs {
    // configuration
    int dec, opt;
    int64_t N, d, n;
    int m, r, s, l, L, rank;
    float lr, alpha, l1adj, l2adj, invD;
    int ext_reg, reg_on;
    // data
    const int32_t* indptr;
    const int32_t* indices;
    const float* values;
    const int32_t* args1;
    const int32_t* args2;
    const int32_t* neg1;
    const int32_t* neg2;
    int neg_mode;
    int64_t neg_stride;
    // parameters / accumulators
    float *W, *Wb, *A, *Ab, *C1, *C2, *R3;
    float *aW, *aWb, *aA, *aAb, *aC1, *aC2, *aR3;
    // exchange records
    float* ex;
    RecLayout lay;
    // the per-example gradient vectors the update reads for A rows: vec(e1) = G1, vec(e2) = G2
    // (bilinear), vec(neg1) = V1, vec(neg2) = V2 -- example b's at vb + b * vbs + v* (floats).
    // The records themselves (vb = ex, vbs = rec), or for the SP wire record the vector buffer
    // k_vrec fills after the exchange (V1 | V2 | G1, 3 r4 floats per example of the batch)
    const float* vb;
    int vbs, vG1, vV1, vV2, vG2;
    // where the forward leaves dCost/dwC1, dCost/dwC2 of example b (the dense C1 / C2 gradient
    // operands): the record (dwb = ex), or -- dense partials -- a rank-local buffer that k_dpart
    // reduces before the exchange
    float* dwb;
    int dws, dw1o, dw2o;
    int dpart;           // dense partials (RecLayout wire 2)
    // row index of the global batches (rae_index.hpp), one slot per batch % index_window
    int HA, HW, RA, RW, posbits;
    int64_t index_window;
    int32_t *srecA, *urowA;             // sorted record ids; urow*: the partitions' segments
    int32_t *srecW, *urowW;             // (row, first position, end, first record), class-ordered
    unsigned long long *skeyA, *skeyW;  // build scratch: (row, record) keys binned by partition
    int32_t* gidx;                      // build scratch: per slot and table, partition counts +
                                        // scatter cursors (RAE_IDX_HMAX each; zeroed per build)
    int32_t* pcls;                      // per slot, table, partition: (heavy, light, very heavy,
                                        // offset) -- k_build_tasks' input
    int VCA, VCW;                       // bounds on the very heavy rows of a batch
    // the update's dispatch table per slot (rae_index.hpp build_batch_tasks): every row task in
    // dispatch order (W rows as ~row), the first NVC very heavy rows as workgroup tasks, and a
    // header (tasks, workgroup tasks) -- one load away from the wave that runs the task
    int32_t *thdr, *task, *vtask;
    int TC, NVC;
    // very heavy rows with more than hch records (StepArgs::hch > 0: large global batches) are
    // split into chunks of hch records: one workgroup task per chunk (a vtask entry whose .w is
    // -(1 + chunk)) writes its partial gradient to hpart[chunk]; k_heavy_fin sums each row's
    // chunks in order and applies the update -- the hfin list per slot: (row | ~row for W, first
    // chunk, chunks, 0), thdr .z entries
    int hch, HF, hps;    // records per chunk (0: off); combine-list capacity; floats per partial
    float* hpart;
    int32_t* hfin;
    // per-example descriptors of this rank's l examples per slot (rae_index.hpp):
    // [nf, p0, entity ids (NJ), feature ids (<= dcap)], dstride ints each
    int32_t* desc;
    int dstride, dcap;
    int dnx, d0;         // examples per descriptor slot (l; L when the update's private-row
                         // tasks read every example's descriptor) and this rank's first one
    // batch addressing, outputs, scratch
    const int64_t* cursor;
    int64_t step_offset;
    float* costs;
    float* gWs;          // dense W gradient scratch (reg_on only)
    float* dPpart;       // bilinear: dCost/dP partial sums over i-blocks (nib, l, m)
    float* sps;          // split SP forward (rae_sp_split.hpp): per example of the rank, the
    int spss;            //   decoder halves' N1 | N2 | A[e1] rows and their scalars (stride spss)
    float* mtV;          // bilinear: k_bil_mt partials over j-blocks (nblk, l, r4): M a2 / M y
    float* mtW;          //           ... over i-blocks: M^T a1 / M^T x
    float* mtP;          //           dP partials of the second pass, per block (nmtp, l, m)
    int nmtp;            //           blocks of a k_bil_mt pass
    int r4;              // align4(r): row stride of the partials
    int nib;             // bilinear: number of i-blocks of the dP contraction
    int bf16;            // bilinear: bf16 MFMA operands (fp32 accumulation) for the R GEMMs
    // bf16 R-gradient operands laid out by k_bil_prep after the exchange: the rank-2 factors
    // X, A1, A2, Y of the global batch transposed to (4, r, Lp) bf16 (RAE_FAC_BF16; example-minor, Lp = L
    // rounded up to 32, zero padded) and P as ready B fragments (L/32, K/16, 64 lanes) x 8 bf16
    float* facT;
    uint4* pfrag;
    int Lp;
    int fuse_prep;       // single rank: the forward kernels write facT / pfrag themselves (no
                         // k_bil_prep launch); padding (b >= L, k >= m) stays zero from creation
    double* regpart;     // [nreg][2] L1/L2 partials of regularised rows
    int nregC;           // number of decoder-row partial slots
    int nregW;           // number of dense-W block partial slots
    float* base_cost;    // cost before the regulariser (reg_on only)
    int* err;            // device error word
    // row-owner partitioned data-parallel update (rae_dp.hpp): G ranks, rows owned row % G
    int G, part;         // world size; 1 when dp_update is partitioned
    int32_t* dpl;        // per slot: the peers' row lists (dpl_slot_ints each)
    int32_t* dpc;        // per slot: their lengths [dir][peer][table]
    int LA, LW;          // list capacities (entity rows, feature rows)
    float* dsend;        // caller's all-to-all buffers: G peer blocks of dblk floats
    float* drecv;
    int capA, capW;      // rows per peer block (set with the buffers; <= LA / LW)
    int64_t dblk;
    int* dpmax;          // longest list built since the last rae_dp_list_max [entity, feature]
    // peer-to-peer exchange (rae.h RAE_XCHG_P2P, rae_p2p.hpp): the peers' mapped buffers, this
    // rank's signal counters (written by the peers) and its expected counts (private)
    int xchg;
    PeerBufs* peers;
    unsigned* sig;       // uncached allocation (rae.hip: hipDeviceMallocUncached)
    unsigned* p2p_expect;
    unsigned long long p2p_timeout;   // s_memrealtime ticks (100 MHz) a wait may spin
    // pipelined form (RAE_XCHG_P2P_PIPE, rae_p2p.hpp): per batch parity, one byte per owned row
    // (entity rows then feature rows, pmA / pmW words of 4) -- bit p: peer p's examples of that
    // batch read the row (bit rank: this rank's own); a byte != 0: the batch updates the row
    int pipe;
    uint32_t* pm;
    int pmA, pmW;
    // private rows: rows a single record of the global batch references (rae.h RAE_PRIV_AUTO;
    // single-rank SP plans), updated per example by the update launch's leading workgroups;
    // pmask per slot and example = (entity-slot bits j < 32, j >= 32, feature-position bits,
    // 0); the row index leaves these rows out of the update's dispatch table
    int priv, privnf;    // enabled; longest feature row whose rows may be private
    int privc;           // one workgroup per example (partitioned plans: ~1/G of the rows)
    int32_t* pmask;
    unsigned long long* stamps;   // diagnostic build only (RAE_STAMPS): phase timestamps
};

// The global batch a step kernel works on: a device cursor + offset (graphs replayed over an
// epoch window), or -- cursor == nullptr -- the absolute batch baked into the launch (graphs
// captured per chunk of the epoch; no dependent cursor load at kernel start).
__device__ __forceinline__ int64_t step_batch(const StepArgs& a) {
    return a.cursor ? *a.cursor + a.step_offset : a.step_offset;
}

#if defined(RAE_DIAG_NOSINGLE) && !defined(RAE_DIAG)
#error "RAE_DIAG_NOSINGLE is a timing knockout with wrong results: a diagnostic build (-DRAE_DIAG)"
#endif
#if defined(RAE_STAMPS) && !defined(RAE_DIAG)
#error "RAE_STAMPS instruments the kernels for tools/phase_stamps.py: a diagnostic build (-DRAE_DIAG)"
#endif
#ifdef RAE_STAMPS
#define RAE_STAMP(a, slot)                                                                  \
    do {                                                                                    \
        if ((a).stamps && threadIdx.x == 0)                                                 \
            (a).stamps[(size_t)blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define RAE_STAMP(a, slot) do { } while (0)
#endif

}  // namespace rae
