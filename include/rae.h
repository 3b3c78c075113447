/*
 * rae.h -- C ABI of the MI355X-native relation-autoencoder training path.
 *
 * This is the drop-in boundary for the reference's compiled Theano function
 *
 *   self.func['train'] = theano.function(inputs=[batch_index, neg1, neg2], outputs=cost,
 *                                        updates=..., givens={xFeats, ents_1, ents_2})
 *        (learning/OieInduction.py:146-149, called at :189)
 *   self.func['label_<split>'] = theano.function(inputs=[batch_index],
 *                                        outputs=(labels, probs), ...)
 *        (learning/OieInduction.py:151-155, called at :245,259,337)
 *
 * and for the model/optimizer objects that function is built from
 * (OieModelFunctions learning/OieModel.py:16-101, AdaGrad/SGD learning/Optimizers.py:6-52).
 *
 * Conventions
 *  - plain C types only; every pointer named *_dev is a device pointer (HBM, gfx950);
 *  - the caller owns all parameter / accumulator / data / exchange memory (they are
 *    Theano shared variables in the reference: learning/OieInduction.py:439-449,
 *    learning/Optimizers.py:12-15); the plan holds borrowed pointers plus a private
 *    workspace allocated once in rae_plan_create;
 *  - every call returns 0 on success and a negative RAE_E* code on error;
 *    rae_last_error() returns a thread-local message for the last failure;
 *  - hot calls (rae_step_*, rae_train_step, rae_label) never allocate or synchronise, so
 *    they can be captured into a HIP graph; they are stream-ordered on `stream`;
 *  - a plan is single-caller (like a Theano function); different plans may run on
 *    different streams concurrently.
 */
#ifndef RAE_H
#define RAE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* rae_stream_t;   /* == hipStream_t */

#define RAE_OK 0
#define RAE_E_INVALID (-1)     /* bad argument / unsupported configuration           */
#define RAE_E_HIP (-2)         /* HIP runtime error                                  */
#define RAE_E_OVERFLOW (-3)    /* a per-step row-index partition overflowed its LDS  */
#define RAE_E_STATE (-4)       /* call sequence error; a peer-to-peer wait timed out */
/* device error word bits (rae_check; rae_last_error names each set bit): 1 / 2 an A / W
 * row-index partition overflowed its LDS sort, 4 a batch exceeded the index's record capacity,
 * 8 a data-parallel row list overflowed while being built, 16 a row list is longer than the
 * exchange's row capacity (RAE_E_OVERFLOW for these); 64 a peer-to-peer wait timed out -- a
 * peer stopped signalling (RAE_E_STATE)                                                      */

/* decoder type: learning/models/decoders/Decoder.py:84-93 ('sp', 'rescal', 'rescal+sp') */
#define RAE_DEC_SP 0
#define RAE_DEC_RESCAL 1
#define RAE_DEC_HYBRID 2

/* optimizer: learning/OieInduction.py:261-269 ('adagrad', 'sgd') */
#define RAE_OPT_ADAGRAD 0
#define RAE_OPT_SGD 1

/* negative-sample column addressing */
#define RAE_NEG_PER_CALL 0     /* neg arrays are (s, l_global): column = example-in-batch */
#define RAE_NEG_PER_EPOCH 1    /* neg arrays are (s, N): column = global example index     */

typedef struct rae_config {
    int32_t decoder;          /* RAE_DEC_*                                                */
    int32_t optimizer;        /* RAE_OPT_*                                                */
    int64_t n_examples;       /* N: rows of the train split (learning/OieData.py:78)     */
    int64_t n_features;       /* d: feature dimensionality (OieData.py:96-98)             */
    int64_t n_entities;       /* n: entity vocabulary (OieData.py:92-94)                  */
    int32_t relations;        /* m = K (--relations, OieInduction.py:469)                 */
    int32_t embed;            /* r (--embed-size, :468)                                   */
    int32_t neg_samples;      /* s (--neg-samples, :470)                                  */
    int32_t batch_size;       /* l: examples per rank per step (--batch-size, :467)       */
    int32_t world_size;       /* data-parallel ranks G (1 = single GPU)                   */
    int32_t rank;             /* this rank                                                */
    float learning_rate;      /* --learning-rate (:466)                                   */
    float alpha;              /* entropy scale (--alpha, :479; OieModel.py:81)            */
    float lambda1;            /* --l1 (:471)                                              */
    float lambda2;            /* --l2 (:472)                                              */
    int32_t ext_reg;          /* --ext-reg (:477; OieModel.py:60-62)                      */
    int32_t max_batch_nnz;    /* max nnz over global batches (sizes the W row index)      */
    int32_t max_row_nnz;      /* max nnz of one example row                               */
    int32_t neg_mode;         /* RAE_NEG_*                                                */
    int64_t neg_stride;       /* row stride (elements) of the neg arrays                  */
    int64_t index_window;     /* batches whose row index is held at once (0 = default)   */
    int32_t mfma_bf16;        /* RESCAL / hybrid: bf16 MFMA operands for the R/C GEMMs    *
                               * (fp32 accumulate; BASELINE config 5); 0 = exact fp32     */
    /* kernel forms (0 = the plan's own choice for the shape; the others exist so tests can
     * pin one form against another -- every form computes the same step):                 */
    int32_t sp_forward;       /* SP forward: RAE_SPFWD_*                                    */
    int32_t bil_dp;           /* bilinear dCost/dP contraction: RAE_BILDP_*                 */
    int32_t bil_prep;         /* bf16 R-gradient operands: RAE_BILPREP_*                    */
    int32_t dp_update;        /* data-parallel update: RAE_DPUPD_*                          */
    int32_t priv_rows;        /* rows one record of the batch references: RAE_PRIV_*        */
    int32_t dp_dense;         /* data-parallel SP: dense decoder-matrix gradients RAE_DPDENSE_* */
    int32_t heavy_chunk;      /* very heavy rows split into record chunks: RAE_HCHUNK_*      */
    int32_t dp_xchg;          /* data-parallel exchange: RAE_XCHG_*                          */
} rae_config;

#define RAE_SPFWD_AUTO 0      /* fused per-example kernel unless r*m > 32768                  */
#define RAE_SPFWD_FUSED 1     /* k_forward: one workgroup per example                         */
#define RAE_SPFWD_SPLIT 2     /* k_sp_enc -> P.C^T GEMM -> k_sp_dec -> dw.C GEMM (+ dS epilogue)  */
#define RAE_BILDP_AUTO 0      /* inside the second M-tile pass when bf16 and m <= 128          */
#define RAE_BILDP_STRIDED 1   /* k_bil_dp (one wave per 16x16 tile of dP)                      */
#define RAE_BILDP_STAGED 2    /* k_bil_dp2 (bf16, LDS-staged R slices; r <= 256, m <= 128)      */
#define RAE_BILDP_MTILE 3     /* inside the second k_bil_mt pass (bf16, m <= 128)               */
#define RAE_BILPREP_AUTO 0    /* single rank: the forward writes the operands (no launch)      */
#define RAE_BILPREP_KERNEL 1  /* k_bil_prep after the exchange                                 */
#define RAE_DPUPD_REPLICATED 0 /* every rank updates every referenced row (bit-identical     *
                                * replicas after every step)                                  */
#define RAE_DPUPD_PARTITIONED 1 /* rank k updates the rows it owns (row % G == k) and pushes *
                                 * the next step's rows to the ranks that read them            */
#define RAE_PRIV_AUTO 0       /* rows exactly one record of the global batch references are left  *
                               * out of the update's row tasks and updated by per-example        *
                               * workgroups of the same update launch (task_private_rows; the    *
                               * one-record row task's arithmetic, bit-identical parameters) in  *
                               * single-rank and replicated plans with a global batch below 4096 *
                               * examples, without a regulariser (lambda1 = lambda2 = 0) and     *
                               * with 2 + 2s <= 64 record slots, any decoder                     */
#define RAE_PRIV_OFF 1        /* every row updated by the update's row tasks                      */
#define RAE_PRIV_ON 2         /* private rows whenever admissible (no regulariser, <= 64 slots),   *
                               * any global batch; the partitioned update takes the private rows *
                               * it owns, one wave per example                                    */
#define RAE_DPDENSE_AUTO 0    /* partials when they are at most half of dw1 / dw2 in the records *
                               * (per-rank partial chunk <= r floats: l >~ 2 relations)          */
#define RAE_DPDENSE_RECORDS 1 /* dw1 / dw2 of every example in the exchange records; the update *
                               * reduces dC1 / dC2 / dWb over the global batch (K = L)           */
#define RAE_DPDENSE_PARTIALS 2 /* each rank reduces its own l examples' dC1 / dC2 / dWb before   *
                                * the exchange (k_dpart); the records carry the partial block,  *
                                * the update sums the ranks' blocks in rank order               */
#define RAE_HCHUNK_AUTO 0     /* global batches of >= 2048 examples: rows with at least 256      *
                               * records of the batch summed as floor(records / 128) chunks in   *
                               * parallel (128 records each, the last one to the row's end; one  *
                               * partial per chunk, k_heavy_fin adds them in chunk order and     *
                               * applies the optimiser); smaller batches: off                    */
#define RAE_HCHUNK_OFF 1      /* every very heavy row summed by one workgroup                      */
#define RAE_HCHUNK_ON 2       /* chunks at any global batch                                        */
#define RAE_XCHG_COLLECTIVE 0 /* the caller moves records / rows between the step launches (an    *
                               * all-gather; rae_dp_pack -> all-to-all -> rae_dp_unpack)         */
#define RAE_XCHG_P2P 1        /* partitioned update only: the kernels store records and rows     *
                               * straight into the peers' buffers (rae_set_peer) and wait on     *
                               * their signal counters -- no caller collective in the step       */
#define RAE_XCHG_P2P_PIPE 2   /* RAE_XCHG_P2P with the next batch's rows pushed during this step: *
                               * the rows the update leaves unchanged right after the forward,   *
                               * every updated row by the update task that writes it -- so the   *
                               * row bytes travel under the update; world_size <= 8, private     *
                               * rows off; rae_p2p_prologue before the first step of a run       */

/* Caller-owned device buffers.  Shapes are the reference's (fp32 everywhere):
 *   W (d,m)  Wb (m)  A (n,r)  Ab (n)  C1,C2 (r,m)  R (r,r,m) [rescal] / C (r,r,m) [hybrid]
 *   (RelationClassifier.py:24-25, OieModel.py:105, SelectionalPreferences.py:13-19,
 *    Bilinear.py:14-17, BilinearPlusSP.py:14-23), acc_* the AdaGrad accumulators of the
 *   same shapes (Optimizers.py:12-15; unused for SGD, may be NULL).
 * data: the train split CSR (OieData.py:83-90) + entity ids.  values may be NULL
 *   (binary features: every stored value is 1.0, OieData.py:88).
 * exchange: per-example records of the global batch, rae_exchange_floats() floats; rank k
 *   writes rows [k*l, (k+1)*l); between rae_step_forward and rae_step_update the caller
 *   all-gathers it across ranks (no-op for world_size == 1).
 * costs: one float per batch index (the value func['train'] returns).
 */
typedef struct rae_buffers {
    float* W; float* Wb; float* A; float* Ab;
    float* C1; float* C2; float* R3;             /* R3 = R (rescal) or C (hybrid) */
    float* acc_W; float* acc_Wb; float* acc_A; float* acc_Ab;
    float* acc_C1; float* acc_C2; float* acc_R3;
    const int32_t* indptr; const int32_t* indices; const float* values;
    const int32_t* args1; const int32_t* args2;
    const int32_t* neg1; const int32_t* neg2;   /* may be NULL until rae_set_negatives */
    float* exchange;
    float* costs;
} rae_buffers;

typedef struct rae_plan rae_plan;

/* --- lifetime ---------------------------------------------------------------------- */
int rae_plan_create(const rae_config* cfg, const rae_buffers* buf, rae_plan** out);
int rae_plan_destroy(rae_plan* plan);
const char* rae_last_error(void);
int rae_version(void);
/* hash of the sources and flags the library was built from (rae/_lib.py source_build_id);
 * the Python binding refuses a library whose id differs from the sources beside it       */
const char* rae_build_id(void);

/* floats per example record and per global batch in the exchange buffer */
int64_t rae_exchange_record_floats(const rae_config* cfg);
int64_t rae_exchange_floats(const rae_config* cfg);

/* The kernel forms the plan resolved for its shape (RAE_SPFWD_FUSED / _SPLIT, RAE_BILDP_*,
 * RAE_BILPREP_*, RAE_DPUPD_*, RAE_PRIV_*; 0 where a form does not apply to the decoder), written into
 * the matching fields of *out (the other fields are left as they are).                  */
int rae_plan_forms(const rae_plan* plan, rae_config* out);

/* --- negatives --------------------------------------------------------------------- */
/* Point the plan at negative-sample arrays (learning/NegativeExampleGenerator.py:14-32
 * output, int32).  mode RAE_NEG_PER_EPOCH: (s, N) arrays for the whole epoch
 * (OieInduction.py:183-184); RAE_NEG_PER_CALL: (s, l_global) arrays of one batch
 * (OieInduction.py:187-189). */
int rae_set_negatives(rae_plan* plan, const int32_t* neg1_dev, const int32_t* neg2_dev,
                      int32_t mode, int64_t stride);

/* --- the row index ----------------------------------------------------------------- */
/* Build the per-batch row index (for every parameter row a batch references, its
 * contributing records in a fixed order) for global batches [first, first+count), from the
 * current negatives; count <= rae_index_window().  Batch b uses slot b % window, so build
 * a window before stepping through it.  Independent of the parameters. */
int rae_build_index(rae_plan* plan, int64_t first_batch, int64_t count, rae_stream_t stream);
int64_t rae_index_window(rae_plan* plan);

/* --- the training step (func['train']) --------------------------------------------- */
/* Batch addressed as  batch = *cursor + step_offset  (cursor: device int64 owned by the
 * plan) so a captured sequence of steps can be replayed for successive batches.        */
int rae_set_cursor(rae_plan* plan, int64_t batch, rae_stream_t stream);
int rae_advance_cursor(rae_plan* plan, int64_t count, rae_stream_t stream);
/* Number of rae_set_cursor / rae_advance_cursor calls made on this plan so far (host count;
 * a captured graph's replays make no calls).  A driver that caches where the cursor points
 * compares it with the count it saw last, so a move made by anyone else is never missed.  */
int64_t rae_cursor_moves(const rae_plan* plan);
/* K1: per-example encoder + decoder forward/backward of this rank's l examples.  Writes the
 * exchange records.  The batch's row index must have been built (rae_build_index).      */
int rae_step_forward(rae_plan* plan, int64_t step_offset, rae_stream_t stream);
/* K2 (+K3 when lambda1/lambda2 != 0): deterministic per-row gradient reduction over the
 * global batch and the optimizer update of every parameter; writes costs[batch].        */
int rae_step_update(rae_plan* plan, int64_t step_offset, rae_stream_t stream);
/* The same two phases for an absolute global batch index (no device cursor: the index is a
 * launch argument; rae_train_step runs this way).  Measured on MI355X: no faster than the
 * cursor form inside graphs (the cursor load overlaps the kernels' other start-up loads),
 * and per-chunk graphs cost more to replay than one graph replayed over an epoch window.
 * `batch` in [0, n_examples / (batch_size * world_size)).                                */
int rae_step_forward_at(rae_plan* plan, int64_t batch, rae_stream_t stream);
int rae_step_update_at(rae_plan* plan, int64_t batch, rae_stream_t stream);
/* One whole func['train'](batch_index, neg1, neg2) call on a single rank:
 * rae_set_negatives(PER_CALL) + index + forward + update for `batch_index`.            */
int rae_train_step(rae_plan* plan, int64_t batch_index, const int32_t* neg1_dev,
                   const int32_t* neg2_dev, rae_stream_t stream);
/* --- partitioned data-parallel update (dp_update = RAE_DPUPD_PARTITIONED) ------------- *
 * Row r of A / Ab / W is owned by rank r % world_size; rae_step_update updates the owned rows
 * only (the dense C1 / C2 / Wb / R / C stay replicated).  Before each step's forward every
 * rank refreshes the non-owned rows its examples read:
 *     rae_dp_pack -> [caller: all-to-all of world_size equal blocks, send -> recv] -> rae_dp_unpack
 * (the same cursor / absolute batch addressing as rae_step_forward / _at).  The peers' row lists
 * are built with the row index (rae_build_index).  Parameters equal the replicated form's
 * bitwise once the owners' rows are gathered (the caller's sync; rae/dist.py sync_rows).
 * Requires lambda1 = lambda2 = 0.                                                          */
/* floats of one peer block for the given row capacities (entity rows, feature rows)      */
int64_t rae_dp_block_floats(const rae_config* cfg, int32_t cap_entities, int32_t cap_features);
/* caller-owned send / recv buffers of world_size blocks each, and their row capacities;
 * every list the plan builds must fit (rae_dp_list_max; a longer one sets error flag 16)   */
int rae_set_dp_buffers(rae_plan* plan, float* send_dev, float* recv_dev, int32_t cap_entities,
                       int32_t cap_features);
/* longest list built since the previous call (synchronises; resets the maxima)           */
int rae_dp_list_max(rae_plan* plan, int32_t* max_entities, int32_t* max_features);
int rae_dp_pack(rae_plan* plan, int64_t step_offset, rae_stream_t stream);
int rae_dp_unpack(rae_plan* plan, int64_t step_offset, rae_stream_t stream);
int rae_dp_pack_at(rae_plan* plan, int64_t batch, rae_stream_t stream);
int rae_dp_unpack_at(rae_plan* plan, int64_t batch, rae_stream_t stream);

/* --- peer-to-peer exchange (dp_xchg = RAE_XCHG_P2P) ---------------------------------- *
 * Every rank maps its peers' exchange buffer, W, A, Ab and signal words (IPC handles, traded
 * once through the caller's process group) and hands them to its plan; rae_step_forward then
 * pushes the owned rows each peer's examples read into that peer's replica, waits for the
 * peers' rows, runs the forward and pushes its records into every peer's exchange buffer;
 * rae_step_update waits for the peers' records.  Graph-capturable (kernels only).  The row
 * capacities come from rae_set_dp_buffers(plan, NULL, NULL, caps) as in the collective form.
 * Replaces (learning/OieInduction.py:186-189 runs one process): the all-gather / all-to-all. */
#define RAE_IPC_HANDLE_BYTES 64
/* handle of the allocation holding dev_ptr, and dev_ptr's offset in it                     */
int rae_ipc_export(const void* dev_ptr, void* handle_out, int64_t* offset_out);
/* map another process's allocation (its base address; add the exported offset)            */
int rae_ipc_open(const void* handle, void** base_out);
int rae_ipc_close(void* base);
/* the plan's signal counters (device, uncached; export them to the peers)                  */
void* rae_p2p_signals(rae_plan* plan);
/* peer `peer`'s buffers as this process maps them                                          */
int rae_set_peer(rae_plan* plan, int32_t peer, float* exchange_dev, float* W_dev, float* A_dev,
                 float* Ab_dev, void* signals_dev);
/* how long one wait kernel may spin for a peer's signal before it sets error bit 64 and
 * gives up (default 5 s; a driver that does host work between steps -- per-batch evaluation
 * -- raises it or puts a host barrier in front of the next step)                          */
int rae_set_p2p_timeout(rae_plan* plan, double seconds);
/* RAE_XCHG_P2P_PIPE: each step pushes (and signals) the rows of the NEXT batch, so the first
 * step of a run needs its own batch's rows pushed first: marks and pushes the rows of
 * `batch` and signals them (every rank calls it with the same batch).  drain != 0: the step
 * before this run pushed rows for another batch -- consume that signal first.  The row index
 * (rae_build_index) of a step's batch + 1 must be built before the step runs.            */
int rae_p2p_prologue(rae_plan* plan, int64_t batch, int32_t drain, rae_stream_t stream);

/* Kernel timing (bench / profiling; no reference counterpart).  Arms the NEXT
 * rae_step_forward or rae_step_update call on this plan: its kernels are launched with
 * hipExtLaunchKernelGGL so `start_event` takes the first kernel's dispatch-begin timestamp
 * and `stop_event` the last kernel's end timestamp -- the execution span rocprofv3
 * --kernel-trace reports, without event-packet overhead.  Not for graph capture.
 * Events are hipEvent_t handles (rae_event_create makes them).                         */
int rae_time_next(rae_plan* plan, void* start_event, void* stop_event);
int rae_event_create(void** event_out);
int rae_event_destroy(void* event);
/* waits for stop_event, then *ms = hipEventElapsedTime(start_event, stop_event) */
int rae_event_elapsed_ms(void* start_event, void* stop_event, float* ms);
/* Device error word (overflow flags); host reads it with rae_check() (a blocking read: waits
 * for all the device's queued work) or rae_check_on() (ordered on `stream` only: waits for
 * the work queued on that stream, e.g. a row-index build on a side stream).              */
int rae_check(rae_plan* plan);
int rae_check_on(rae_plan* plan, rae_stream_t stream);

/* --- negative sampling (learning/NegativeExampleGenerator.py:14-32) ----------------- */
/* out[i] = first j with cum[j] >= x_i  (numpy searchsorted side='left' over the float64 CDF
 * negSamplingCum, learning/OieData.py:57-59), i < count, int32.
 * rae_neg_sample:        x_i = uniforms[i], the caller's draws of U(0, cum[n-1]) -- with the
 *                        model's RandomState stream this is the reference sampler bit for bit.
 * rae_neg_sample_philox: x_i = cum[n-1] * U_i, U_i from Philox4x32-10 at counter offset + i
 *                        under key seed (device-only perf mode, not the reference's stream). */
int rae_neg_sample(const double* cum_dev, int64_t n, const double* uniforms_dev, int64_t count,
                   int32_t* out_dev, rae_stream_t stream);
int rae_neg_sample_philox(const double* cum_dev, int64_t n, uint64_t seed, uint64_t offset,
                          int64_t count, int32_t* out_dev, rae_stream_t stream);

/* --- labelling (func['label_<split>'], RelationClassifier.py:39-48) ----------------- */
/* rows [row0, row0+nrows) of any CSR split with the current W/Wb: labels = argmax(S)
 * (int64, first max) and probs = softmax(S) (fp32, may be NULL).                        */
int rae_label(const int32_t* indptr, const int32_t* indices, const float* values,
              const float* W, const float* Wb, int32_t relations, int64_t row0,
              int64_t nrows, int64_t* labels_out, float* probs_out, rae_stream_t stream);

/* --- measurement helper (bench.py; no reference counterpart) ------------------------- */
/* STREAM-style device copy of `bytes` (multiple of 16, 16-byte aligned pointers) with float4
 * loads and stores: the measured HBM ceiling bench.py reports next to the 8 TB/s spec.   */
int rae_stream_copy(const void* src_dev, void* dst_dev, int64_t bytes, rae_stream_t stream);
/* bf16 MFMA throughput probe: `blocks` workgroups of 4 waves, each wave `iters` rounds of 8
 * independent v_mfma_f32_16x16x32_bf16 (16384 flops each); writes one float per wave to
 * sink_dev (blocks * 4 floats).  bench.py times it: the measured dense bf16 MFMA ceiling.  */
int rae_mfma_probe(int64_t iters, int32_t blocks, float* sink_dev, rae_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RAE_H */
