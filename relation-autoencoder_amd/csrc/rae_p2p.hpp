// Peer-to-peer data-parallel exchange (rae_config.dp_xchg = RAE_XCHG_P2P; partitioned update).
//
// The reference trains on one process (learning/OieInduction.py:186-189); the data-parallel
// step shards its global batch over G ranks.  With the collective exchange the
// partitioned step is   pack -> all-to-all -> unpack -> forward -> all-gather -> update, and
// each collective is a host-launched RCCL call with its own latency on the step's dependence
// chain.  Here every rank maps its peers' buffers (IPC handles exchanged once at set-up: their
// exchange buffer, W, A, Ab and signal words) and the kernels store straight into them:
//   k_p2p_rows   (start of step b, after the update of b-1): the owner stores every row it owns
//                that peer p's examples of batch b read into p's OWN replica (the row lists of
//                rae_dp.hpp, direction 0) -- no send buffer, no all-to-all, no unpack
//   k_p2p_wait   (rows): until every owner's row stores of batch b are visible
//   forward(b)   this rank's records into its own exchange buffer, as before
//   k_p2p_recs   its l records into every peer's exchange buffer, at the same rows
//   k_p2p_wait   (records): until every peer's records of batch b are here
//   update(b)    the owned rows, as before
// Signalling: after a push kernel a one-wave signal kernel adds one to the peer's signal word
// (kind, this rank) with a system-scope atomic -- a counter that grows by one every step (fences per workgroup inside the pushes cost an L2 write-back each:
// 55-81 us per step in the loopback model).  The waiting kernel (one wave: lane p watches peer
// p) spins on relaxed system-scope loads until each counter reaches its expected value (kept in
// this rank's private words, advanced by the wait kernel itself, so graph replays stay in
// step), with a bounded spin: after StepArgs::p2p_timeout (rae_set_p2p_timeout; 5 s by default)
// it sets error bit 64 and returns (the host sees it at rae_check) rather than hold the GPU.
// Visibility across GPUs ("peer-to-peer visibility"), each side made explicit:
//  * producer: every push store is a system-scope write-through (`global_store ... sc0 sc1`,
//    store_sys below) and each pushing wave waits for its stores to complete (vmcnt(0)) before
//    it ends -- no pushed byte can sit dirty in one of this GPU's eight L2s (a peer's memory is
//    mapped non-coherent here, and the signal kernel's single-wave fence writes back one XCD's
//    L2 only), so the bytes are in the peer's memory before the kernel boundary, and the
//    signal add follows that boundary;
//  * signal words: allocated uncached (hipDeviceMallocUncached), so neither the polls nor the
//    peers' atomic adds go through an L2 line that could be stale;
//  * consumer: the pushed rows / records land in this rank's own coarse-grained memory; the
//    peers' stores reach it through its data fabric like another XCD's write-backs do, and the
//    kernels that read them start after the wait kernel's acquire and their own dispatch
//    acquire (L1 invalidated) -- the same hand-off the MI355X guide measures cross-XCD with an
//    L1 invalidate alone (MI355X_MICROARCH.md:161-174).  Untested across physical GPUs.
// Hazards (all ranks run the same step sequence): a peer's replica rows and exchange rows are
// overwritten only after that peer has consumed them -- owner k's row stores of batch b follow
// k's update of b - 1, which needed peer p's records of b - 1, which p pushed after its forward
// of b - 1 (the rows' last reader); k's record stores of batch b follow k's forward of b, which
// needed p's rows of b, which p pushed after its update of b - 1 (the records' last reader).
// Each row is stored by its owner only, with the value the collective form would have unpacked,
// so the parameters are bit-identical to the collective partitioned (and replicated) update.
#pragma once
#include "rae_common.hpp"
#include "rae_dp.hpp"
#include "rae_step.hpp"

namespace rae {

#define RAE_P2P_TIMEOUT_DEFAULT 500000000ull   // s_memrealtime ticks (100 MHz): 5 s

// system-scope write-through stores into a peer's memory (sc0 sc1: not held in this GPU's L2);
// the caller's wave waits for them with p2p_stores_done() before it ends.  Buffer-store
// builtins (cache-policy operand 17 = sc0 sc1) rather than inline asm: the compiler's hazard
// and wait-count passes see these stores (an inline-asm store they cannot see lets them reuse
// or wait wrongly around it -- measured: asm sc1 row stores in the update gave non-finite
// costs, the same stores as builtins did not; profiles/r06_ab.txt).
// base: a wave-uniform base pointer (made scalar here); c: the lane's element index.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(const float* base) {
    const uint64_t u = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    float* b = reinterpret_cast<float*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, -1, 0x00020000);
}
__device__ __forceinline__ void store_sys(const float* base, int c, float4 v) {
    const rae_v4u u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(u, sys_rsrc(base), c * 16, 0, 17);
}
__device__ __forceinline__ void store_sys(const float* base, int c, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), sys_rsrc(base), c * 4, 0, 17);
}
__device__ __forceinline__ void p2p_stores_done() { asm volatile("s_waitcnt vmcnt(0)" : : : "memory"); }

// k_p2p_signal (one wave, after a push kernel): every store of the pushes is a system-scope
// write-through that its wave waited for (store_sys + vmcnt(0): the push kernels, and the
// update kernels' row pushes of the pipelined form) -- complete at system scope before the
// kernel boundary this launch follows -- so the add needs no release fence: a relaxed
// system-scope add into every peer's (uncached) word (kind, rank).  (A release here would
// write back this XCD's whole L2 -- the update's dirty parameter rows -- on every signal.)
__device__ void p2p_signal(const StepArgs& a, int kind) {
    if (threadIdx.x < a.G && threadIdx.x != a.rank) {
        unsigned* s = a.peers[threadIdx.x].sig + kind * a.G + a.rank;
        __hip_atomic_fetch_add(s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// k_p2p_recs: this rank's l records (float4 slices) into every peer's buffer.  Pipelined form:
// the blocks past the records clear the row marks of batch b + 1's parity (they held batch
// b - 1's, whose last readers -- the pre-push of step b - 1, the update of b - 2 -- are done),
// which k_p2p_pre of this step then fills
__device__ void p2p_push_records(const StepArgs& a) {
    const int64_t n4 = (int64_t)a.l * a.lay.rec / 4;                 // rec is a multiple of 4
    const int64_t nrb = (n4 + blockDim.x - 1) / blockDim.x;
    if (a.pipe && (int64_t)blockIdx.x >= nrb) {
        const int64_t b = step_batch(a);
        // (stored like the pushes, so every store of this kernel is one kind)
        const float* pm = reinterpret_cast<const float*>(a.pm + (int64_t)((b + 1) & 1) * (a.pmA + a.pmW));
        const int64_t nw4 = (a.pmA + a.pmW) / 4;                      // pmA, pmW multiples of 4
        for (int64_t i = (blockIdx.x - nrb) * blockDim.x + threadIdx.x; i < nw4;
             i += (gridDim.x - nrb) * blockDim.x)
            store_sys(pm, (int)i, make_float4(0.f, 0.f, 0.f, 0.f));
        p2p_stores_done();
        return;
    }
    const int64_t o4 = (int64_t)a.rank * a.l * a.lay.rec / 4;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const float4 v = reinterpret_cast<const float4*>(a.ex)[o4 + i];
    for (int p = 0; p < a.G; ++p)
        if (p != a.rank) store_sys(a.peers[p].ex, (int)(o4 + i), v);
    p2p_stores_done();
}

// one owned row of table tab into peer p's replica (one wave; Ab with the entity rows)
__device__ __forceinline__ void push_row_to(const StepArgs& a, int p, int tab, int row, int lane) {
    const int w = tab ? a.m : a.r;                   // r, m multiples of 4, <= 512
    const float4* s = reinterpret_cast<const float4*>((tab ? a.W : a.A) + (int64_t)row * w);
    const float* d = (tab ? a.peers[p].W : a.peers[p].A) + (int64_t)row * w;    // row: wave-uniform
    const int w4 = w / 4;
    float4 v0, v1;
    if (lane < w4) v0 = s[lane];
    if (lane + 64 < w4) v1 = s[lane + 64];
    const float ab = (!tab && lane == 0) ? a.Ab[row] : 0.f;
    if (lane < w4) store_sys(d, lane, v0);
    if (lane + 64 < w4) store_sys(d, lane + 64, v1);
    if (!tab && lane == 0) store_sys(a.peers[p].Ab, row, ab);
}

// k_p2p_rows: one wave per (peer, list entry) of batch step_batch(a)'s direction-0 lists (rows
// this rank owns that the peer's examples read): the row into that peer's replica
__device__ void p2p_push_rows(const StepArgs& a) {
    const int lane = threadIdx.x & 63;
    const int per = a.capA + a.capW;
    const int64_t t = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int p = (int)(t / per), i0 = (int)(t - (int64_t)p * per);
    if (p >= a.G || p == a.rank) return;
    const int64_t slot = step_batch(a) % a.index_window;
    const int tab = i0 >= a.capA ? 1 : 0;
    const int i = tab ? i0 - a.capA : i0;
    const int cap = tab ? a.capW : a.capA;
    // the list length and the entry load together (one round trip; the list's storage holds
    // LA / LW >= cap entries, so entry i < cap is in bounds -- used only when i < n)
    const int n = *dpl_count(a, slot, 0, p, tab);
    const int row = dpl_list(a, slot, 0, p, tab)[i < cap ? i : 0];
    if (i == 0 && lane == 0 && n > cap) atomicOr(a.err, 16);
    if (i >= n || i >= cap) return;
    push_row_to(a, p, tab, row, lane);
    p2p_stores_done();
}

// ---- pipelined form (RAE_XCHG_P2P_PIPE) ------------------------------------------------------
// The rows peer p's examples read in batch b + 1 (direction-0 list) leave during step b:
//   k_p2p_pre(b), right after the forward and the record push: marks batch b + 1's lists into
//     the row-mark bytes of its parity (bit p per list p, the own list included), and pushes the
//     listed rows that batch b does NOT update (mark byte of b's parity == 0: no list of b holds
//     the row, so no row task of update(b) writes it) -- final values, pushed while the peers'
//     records are still on their way;
//   update(b): every row task, as it writes an owned row, stores it into each peer whose bit is
//     set in batch b + 1's mark byte (pipe_push_row) -- the updated rows travel under the update;
//   k_p2p_signal (kind 1) after the update: batch b + 1's rows are all in place.
// A run's first batch has no previous step: rae_p2p_prologue marks and pushes its whole lists.
// Hazards: a pre-pushed row is one update(b) leaves alone, so its value equals what a peer
// that reads it in batch b already holds (an identical overwrite while that peer's forward(b)
// may read it); an update push reaches a peer after its forward(b) (this rank's update waited
// for the peer's records of b) and before its forward(b + 1) (which waits for kind 1).
__device__ __forceinline__ uint8_t* pipe_marks(const StepArgs& a, int64_t batch, int tab) {
    return reinterpret_cast<uint8_t*>(a.pm + (batch & 1) * (int64_t)(a.pmA + a.pmW) + (tab ? a.pmA : 0));
}
__device__ __forceinline__ int64_t epoch_batches(const StepArgs& a) { return a.N / a.L; }

// k_p2p_pre: blocks [0, nmb): one thread per list entry marks batch tb's lists; the rest: one
// wave per (peer, list entry) pushes -- prologue: every listed row of tb = step_batch; else tb =
// step_batch + 1 and only the rows step_batch does not update
__device__ void p2p_pre(const StepArgs& a, int prologue, int nmb) {
    const int64_t b = step_batch(a);
    const int64_t tb = prologue ? b : b + 1;
    if (tb >= epoch_batches(a)) return;               // the epoch's last step: nothing follows
    const int64_t slot = tb % a.index_window;
    const int per = a.capA + a.capW;
    if ((int)blockIdx.x < nmb) {
        const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        const int p = (int)(t / per), i0 = (int)(t - (int64_t)p * per);
        if (p >= a.G) return;
        const int tab = i0 >= a.capA ? 1 : 0;
        const int i = tab ? i0 - a.capA : i0;
        const int cap = tab ? a.capW : a.capA;
        const int n = *dpl_count(a, slot, 0, p, tab);
        if (i == 0 && n > cap) atomicOr(a.err, 16);
        if (i >= n || i >= cap) return;
        const int q = dpl_list(a, slot, 0, p, tab)[i] / a.G;
        uint32_t* w = reinterpret_cast<uint32_t*>(pipe_marks(a, tb, tab)) + (q >> 2);
        atomicOr(w, (1u << p) << (8 * (q & 3)));
        return;
    }
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)(blockIdx.x - nmb) * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int p = (int)(t / per), i0 = (int)(t - (int64_t)p * per);
    if (p >= a.G || p == a.rank) return;
    const int tab = i0 >= a.capA ? 1 : 0;
    const int i = tab ? i0 - a.capA : i0;
    const int cap = tab ? a.capW : a.capA;
    const int n = *dpl_count(a, slot, 0, p, tab);
    const int row = dpl_list(a, slot, 0, p, tab)[i < cap ? i : 0];
    if (i == 0 && lane == 0 && n > cap) atomicOr(a.err, 16);
    if (i >= n || i >= cap) return;
    if (!prologue && pipe_marks(a, b, tab)[row / a.G] != 0) return;   // update(b) pushes it
    push_row_to(a, p, tab, row, lane);
    p2p_stores_done();
}

// update(b), pipelined form: the peers (bits) that read owned row `row` of table tab in batch
// b + 1 -- loaded by the row task when it issues its parameter loads, so the byte's round trip
// is not on the task's chain; 0 when not pipelined or b is the epoch's last batch
// PP: the update instantiation may run a pipelined plan (data parallel); the single-rank
// instantiations compile the pushes out (a runtime-off branch still cost the C4 update 1.3 us)
template <bool PP>
__device__ __forceinline__ unsigned pipe_mark(const StepArgs& a, int tab, int row) {
    if constexpr (!PP) return 0u;
    if (!a.pipe) return 0u;
    const int64_t tb = step_batch(a) + 1;
    if (tb >= epoch_batches(a)) return 0u;
    // the row is wave-uniform: one word load the compiler can keep scalar (no VGPR held
    // across the task)
    const int q = __builtin_amdgcn_readfirstlane(row / a.G);
    const uint32_t wd = reinterpret_cast<const uint32_t*>(pipe_marks(a, tb, tab))[q >> 2];
    return __builtin_amdgcn_readfirstlane((wd >> (8 * (q & 3))) & 0xffu & ~(1u << a.rank));
}
// ... and once the row is written (its new values in the lanes' vectors v[0..Q)): into the
// replica of every peer in mk
template <class VT, int Q>
__device__ __forceinline__ void pipe_push_row(const StepArgs& a, int tab, int row, unsigned mk,
                                              const VT (&v)[Q], int nv, int lane) {
#if defined(RAE_DIAG) && defined(RAE_PIPE_NOPUSH)   // diagnostic A/B only: no update pushes
    return;
#endif
    if (!mk) return;
    const int w = tab ? a.m : a.r;
    for (int p = 0; p < a.G; ++p) {
        if (!((mk >> p) & 1u)) continue;
        const float* d = (tab ? a.peers[p].W : a.peers[p].A) + (int64_t)row * w;   // row: wave-uniform
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int c = lane + RAE_WAVE * q;
#if defined(RAE_DIAG) && defined(RAE_PIPE_PLAIN)   // diagnostic A/B only: plain stores
            if (c < nv) const_cast<VT*>(reinterpret_cast<const VT*>(d))[c] = v[q];
#else
            if (c < nv) store_sys(d, c, v[q]);
#endif
        }
    }
}
// ... an entity row's Ab (one lane)
__device__ __forceinline__ void pipe_push_ab(const StepArgs& a, int row, unsigned mk, float v) {
    for (int p = 0; p < a.G; ++p)
        if ((mk >> p) & 1u) store_sys(a.peers[p].Ab, row, v);
}

// k_p2p_wait: lane p waits for peer p's `per` signals of this step (kind 0 records, 1 rows):
// relaxed system-scope polls (no cache invalidation per poll), one acquire fence at the end
__device__ void p2p_wait(const StepArgs& a, int kind, unsigned per) {
    const int p = threadIdx.x;
    if (p >= a.G || p == a.rank) return;
    unsigned* ex = a.p2p_expect + kind * a.G + p;
    const unsigned target = *ex + per;
    const unsigned* s = a.sig + kind * a.G + p;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    // a wait that already timed out this run: do not wait again (fail fast; rae_check raises)
    const bool dead = (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 64) != 0;
    while (!dead && (int)(__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.p2p_timeout) {
            atomicOr(a.err, 64);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);         // system scope: the peer's stores
    *ex = target;
}

}  // namespace rae
