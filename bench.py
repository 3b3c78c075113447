"""Benchmark: train examples/sec (fwd+bwd+update) of the relation-VAE training step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--batch-size 100]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

A "step" is one func['train'] call on one global batch (l examples per rank): encoder +
decoder forward/backward + AdaGrad update of every parameter.  Inputs (dataset, per-epoch
negatives) are resident in HBM before the timed region; negative sampling (host RNG, as in
the reference) is timed separately.  K steps are timed between barrier+synchronize pairs,
max over ranks.  The parameter-independent row index is built as the epoch loop builds it
(engine index_overlap): for K >= OVERLAP_MIN_STEPS the next window's index on a side stream
beside the steps -- the timed region holds the K steps AND the index build of the next K
batches, running concurrently; shorter runs (the driver's 20 steps) time the steps alone and
add the index at its serial per-batch cost measured over a whole window; value =
K * global_batch / seconds -- end-to-end training throughput.  Rank 0 prints one JSON line.

Also reported: the roofline of the step's dominant kernel (the one with the longest average
launch; algorithmic bytes per launch by SURVEY.md 8(d)'s accounting / its average duration
from HIP events on the launch stream), both kernels' lines, and the CPU baseline -- the
reference's dense Theano schedule restated in torch (oracle/cpu_ref.py), float64 and float32,
timed on the host's CPU share on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))

METRIC = "train examples/sec (fwd+bwd) K=100 d=200 neg=20 at 1/2/4/8 MI355X"
OVERLAP_MIN_STEPS = 128     # timed runs this long build the next batches' index beside the steps
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F32_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: dense fp32 MFMA (v_mfma_f32_16x16x4_f32)
MFMA_BF16_PEAK_TFS = 2500.0
TIMING = ("HIP events stamped by the kernels' own dispatch packets (hipExtLaunchKernelGGL via "
          "rae_time_next) on the launch stream, eager launches of the steps after the timed region")  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)

# BASELINE.json configs: N triples, feature dim, K, embed, neg, decoder
CONFIGS = {
    "c2": dict(N=100_000, d=2 ** 17, m=30, r=100, s=10, dec="sp", ntrue=30,
               name="C2 synthetic 100k triples K=30 embed=100 neg=10 sp"),
    "c3": dict(N=1_000_000, d=2 ** 17, m=100, r=200, s=20, dec="sp", ntrue=100,
               name="C3 synthetic 1M triples K=100 embed=200 neg=20 sp (headline)"),
    # dp_update: the data-parallel update form --dp-update auto picks at N > 1 (tools/probes/
    # dp_update_model.py, DESIGN.md 4: at G = 8, l = 100 C4 projects 32.6 % partitioned vs
    # 27.5 % replicated over RCCL, C3 24.0 % vs 25.4 %)
    "c4": dict(N=10_000_000, d=2 ** 20, m=300, r=300, s=50, dec="sp", ntrue=300,
               dp_update="partitioned", name="C4 synthetic 10M triples K=300 embed=300 neg=50 sp"),
    "c5": dict(N=1_000_000, d=2 ** 17, m=100, r=200, s=20, dec="rescal", ntrue=100, bf16=True,
               name="C5 synthetic 1M triples K=100 embed=200 neg=20 rescal, bf16 MFMA"),
}


def step_bytes(host, ex0, L, l, rank, m, r, s, dec):
    """Algorithmic HBM bytes of one step per kernel, two accountings, U_W / U_A counted
    exactly from the batch's feature ids and entity ids (nA = A rows read per example: SP
    1 + 2s -- A[e2] is unused, SelectionalPreferences.py:34-35 -- bilinear 2 + 2s;
    P_dec = 2rm SP, r^2 m RESCAL, r^2 m + 2rm hybrid):

    SURVEY.md 8(d) ("s8d", the roofline's numerator):
      k_forward (this rank's l examples): per example encoder 4(f+1) + 8 f m (CSR ids, W-row
        gather + its gradient scatter), decoder 8(1+s) + 8 r nA + 16(1+s) (ids, A-row gather +
        scatter, Ab gather + scatter); per launch the dense parameters' forward read 4(m + P_dec)
      k_update (global batch): sparse AdaGrad 20 (m U_W + r U_A + U_A) (read p, g, acc; write
        p, acc) + the dense parameters' gradient write + AdaGrad 24 (m + P_dec)
    minimal ("min": every byte this design must move, once; no gradient buffer exists):
      k_forward: 4(f+1) + 4 f m + 16(1+s) + 4 r nA per example, 4(m + P_dec) per launch
      k_update: 16 (m U_W + r U_A + U_A) + 16 (m + P_dec)
    Returns {"s8d": (fwd, upd), "min": (fwd, upd)}."""
    indptr = host["indptr"]
    rows = slice(ex0 + rank * l, ex0 + rank * l + l)
    f = np.diff(indptr[rows.start:rows.stop + 1]).astype(np.int64)
    nA = (1 + 2 * s) if dec == "sp" else (2 + 2 * s)
    pdec = {"sp": 2 * r * m, "rescal": r * r * m, "rescal+sp": r * r * m + 2 * r * m}[dec]
    gfe = slice(ex0, ex0 + L)
    feats = host["indices"][indptr[gfe.start]:indptr[gfe.stop]]
    ents = np.concatenate([host["args1"][gfe], host["args2"][gfe],
                           host["neg1"][:, gfe].ravel(), host["neg2"][:, gfe].ravel()])
    UW, UA = np.unique(feats).size, np.unique(ents).size
    rows_el = m * UW + r * UA + UA
    fwd_8d = int((4 * (f + 1) + 8 * f * m + 8 * (1 + s) + 8 * r * nA + 16 * (1 + s)).sum()) \
        + 4 * (m + pdec)
    upd_8d = 20 * rows_el + 24 * (m + pdec)
    fwd_min = int((4 * (f + 1) + 4 * f * m + 16 * (1 + s) + 4 * r * nA).sum()) + 4 * (m + pdec)
    upd_min = 16 * rows_el + 16 * (m + pdec)
    return {"s8d": (fwd_8d, upd_8d), "min": (fwd_min, upd_min)}


def step_flops(L, l, m, r, dec):
    """MFMA flops of one step for the bilinear decoders: M = P.R (2 l r^2 m), the dP
    contraction (2 l r^2 m) and the R/C gradient (2 L r^2 m)."""
    if dec == "sp":
        return 0
    return 2 * r * r * m * (2 * l + L)


def pmc_traffic(config, batch_size=100):
    """L2-to-fabric (HBM + Infinity Cache) bytes per launch from the newest committed
    rocprofv3 PMC passes (profiles/rNN_<config>_pmc_traffic.json) taken at this per-rank batch
    size (the passes' bench arguments name it; none means the default 100), if any:
    2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE counts half of a wide
    coalesced read on gfx950; the same pass's rae_stream_copy, of known bytes, confirms the
    factor), averaged over the launches of each kernel."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc_traffic.json")) +
                   glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_l*_pmc_traffic.json")))
    found = None
    for path in paths:
        with open(path) as fh:
            out = json.load(fh)
        src = out.get("source", "")
        bs = int(src.split("--batch-size", 1)[1].split()[0]) if "--batch-size" in src else 100
        if bs == batch_size and (found is None or os.path.basename(path)[:3] >= found[0]):
            found = (os.path.basename(path)[:3], path, out)
    if found is None:
        return None
    _, path, out = found
    out["file"] = os.path.relpath(path, ROOT)
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:                                    # pragma: no cover
        pass
    return "unknown"


def _cpu_dense_steps(data, cfg, l, dtype, threads, budget_s, warm=5, max_steps=200, seed=2):
    """The reference's dense Theano schedule (oracle/cpu_ref.py: forward, dense T.grad,
    dense AdaGrad over every parameter) on `threads` host threads: `warm` untimed steps,
    then up to `max_steps` timed steps within `budget_s`.  Returns (examples/s, steps, s)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref
    torch.set_num_threads(threads)
    sp_ = data.split["train"]
    rng = np.random.RandomState(seed)
    p = cpu_ref.init_params(rng, cfg["dec"], data.get_dimensionality(), cfg["m"],
                            data.get_arg_voc_size(), cfg["r"], dtype)
    step = cpu_ref.DenseScheduleStep(cfg["dec"], p, lr=0.1, alpha=1.0)
    cum = data.negSamplingCum
    nb = sp_.args1.shape[0] // l
    # per-epoch negatives of the batches used (host RandomState, outside the timing as in
    # the GPU leg); inputs staged as torch tensors before the timed steps
    nsteps = warm + max_steps
    u1 = rng.uniform(0, cum[-1], (cfg["s"], nsteps * l))
    u2 = rng.uniform(0, cum[-1], (cfg["s"], nsteps * l))
    n1 = torch.as_tensor(cum.searchsorted(u1).astype(np.int64))
    n2 = torch.as_tensor(cum.searchsorted(u2).astype(np.int64))
    a1 = torch.as_tensor(sp_.args1.astype(np.int64))
    a2 = torch.as_tensor(sp_.args2.astype(np.int64))

    def one(i):
        b = i % nb
        rows = slice(b * l, (b + 1) * l)
        X = cpu_ref.batch_csr(sp_.xFeats, rows, dtype)
        cols = slice(i * l, (i + 1) * l)
        return step(X, a1[rows], a2[rows], n1[:, cols], n2[:, cols])
    for i in range(warm):
        one(i)
    steps, t0 = 0, time.perf_counter()
    while steps < max_steps and (time.perf_counter() - t0 < budget_s or steps < 2):
        one(warm + steps)
        steps += 1
    el = time.perf_counter() - t0
    del p, step
    return steps * l / el, steps, el


def _cgroup_cpu_quota():
    """CPUs the container's cgroup may use (cpu.max quota / period), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_baseline(data, cfg, l, budget_s, max_steps=200):
    """CPU baseline: the reference's dense schedule on this host's CPU share, float64
    (Theano's default floatX) and float32, BASELINE.md sec. 2: 5 warm-up + 200 timed steps
    (each variant stops earlier only past `budget_s`).  Threads: the OMP_NUM_THREADS share a
    GPU box gives this process (its cgroup quota; the whole host's CPUs would oversubscribe
    it), else every CPU of the affinity mask.  The faster precision is reported."""
    import torch
    aff = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    th = omp if 0 < omp < aff else aff
    prev = torch.get_num_threads()
    runs = {}
    for prec, dt in (("fp64", torch.float64), ("fp32", torch.float32)):
        v, n, el = _cpu_dense_steps(data, cfg, l, dt, th, budget_s, max_steps=max_steps)
        runs[prec] = {"value": v, "steps": n, "seconds": el, "threads": th}
    torch.set_num_threads(prev)
    best = max(runs, key=lambda k: runs[k]["value"])
    return dict(value=runs[best]["value"], unit="examples/s", cores=th, kind="port",
                sample=(f"oracle/cpu_ref.py dense Theano schedule (forward, dense T.grad, dense "
                        f"AdaGrad over all params), same workload l={l}, torch CPU on {th} "
                        f"threads, 5 warm-up + {max_steps} timed steps per precision (budget "
                        f"{budget_s:.0f} s each); the faster precision reported"),
                precision=best, fp64_value=runs["fp64"]["value"], runs=runs,
                affinity_cpus=aff, omp_num_threads=omp or None,
                cgroup_cpu_quota=_cgroup_cpu_quota(), cpu_model=_cpu_model(),
                ms_per_step=1e3 * l / runs[best]["value"])


def warm_up(eng, W, K, prebuilt, graphed):
    """Capture every graph the warm-up and the timed steps replay (no capture inside the timed
    region), then run the W warm-up steps.  A step with a collective the runtime cannot capture
    (data-parallel exchange) falls back to eager launches; returns whether graphs are used.
    (tests/test_dist.py::test_rccl_one_rank_captured_exchange exercises the fallback.)"""
    import torch
    try:
        if graphed:
            eng.capture_for(0, W)
            eng.capture_for(W, K, last_advance=False)
        eng.run(0, W, index=not prebuilt)
    except RuntimeError as e:              # e.g. a collective the runtime cannot capture
        if eng.exchange is None or not graphed:
            raise
        print(f"warning: graph capture of the data-parallel step failed ({e}); timing eager "
              f"launches instead", file=sys.stderr)
        graphed = False
        eng.graph_chunk = 1
        eng._graphs.clear()
        eng.cursor_moved()
        torch.cuda.synchronize()
        eng.run(0, W, index=not prebuilt)
    return graphed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--no-index-overlap", action="store_true",
                    help="build each window's row index on the step stream (serial, counted at "
                         "its per-batch cost) instead of beside the previous window's steps")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--batch-size", type=int, default=100)
    ap.add_argument("--graph-chunk", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=75.0,
                    help="budget per CPU-baseline precision (200 timed steps normally fit)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=200)
    ap.add_argument("--no-label-pass", action="store_true")
    ap.add_argument("--kernel-form", action="append", default=[], metavar="KEY=VALUE",
                    help="pin a kernel form (include/rae.h; e.g. sp_forward=split); recorded in "
                         "config.kernel_forms")
    ap.add_argument("--dp-update", default="auto", choices=["auto", "replicated", "partitioned"],
                    help="data-parallel update (N > 1): every rank updates every row, or each "
                         "rank the rows it owns (rows pulled from their owners each step); auto: "
                         "the config's projected better form (C4 partitioned, else replicated)")
    ap.add_argument("--dp-xchg", default="collective", choices=["collective", "p2p", "p2p_pipe"],
                    help="partitioned update, N > 1: RCCL collectives between the step launches, or "
                         "the kernels' own stores into the peers' IPC-mapped buffers (include/rae.h "
                         "RAE_XCHG_P2P)")
    ap.add_argument("--p2p-cross-device", action="store_true",
                    help="--dp-xchg p2p with ranks on different GPUs (verified on ranks sharing "
                         "one GPU only; refused without this flag)")
    args = ap.parse_args()
    if args.dp_xchg != "collective":
        args.dp_update = "partitioned"
        args.kernel_form.append(f"dp_xchg={args.dp_xchg}")

    import torch
    from rae import dist as rdist
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer

    ws, rk, lrank = rdist.init()
    if args.dp_update == "auto":         # one rank: the plan has no data-parallel update
        args.dp_update = CONFIGS[args.config].get("dp_update", "replicated") if ws > 1 else "replicated"
    if ws != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
    # one GPU per local rank; ranks beyond the node's GPUs share them (a rehearsal of the
    # multi-rank path on a one-GPU box, RAE_DIST_BACKEND=gloo)
    dev = torch.device("cuda", lrank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    cfg = CONFIGS[args.config]
    l = args.batch_size
    L = l * ws
    t0 = time.perf_counter()
    data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
    t_data = time.perf_counter() - t0
    exchange = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, cfg["r"], cfg["m"],
                             cfg["s"], 0.0, 0.0, "adagrad", "bench", cfg["dec"], False, True, False,
                             1.0, device=dev, world_size=ws, rank=rk, exchange=exchange,
                             graph_chunk=args.graph_chunk, mfma_bf16=cfg.get("bf16", False),
                             dp_update=args.dp_update,
                             kernel_forms=dict(kv.split("=", 1) for kv in args.kernel_form),
                             index_overlap=not args.no_index_overlap,
                             p2p_cross_device=args.p2p_cross_device)
    ind.compile_function()
    eng = ind.engine
    # per-epoch negatives: the reference's RandomState stream, CDF search on the device
    # (parity mode, rae_neg_sample) -- timed separately, outside the metric
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    torch.cuda.synchronize()
    t_neg = time.perf_counter() - t0
    neg1, neg2 = eng.neg1.cpu().numpy(), eng.neg2.cpu().numpy()
    rdist.warm_up(exchange, eng.exchange_buf)
    nb = eng.nb
    K, W = args.steps, args.warmup
    if K + W > nb:
        raise SystemExit(f"steps+warmup={K + W} exceed the {nb} global batches of one epoch")

    # The per-batch row index (rae_build_index) depends only on the batch's ids, negatives and
    # CSR rows -- not on the parameters -- so the epoch loop builds it a window of batches
    # ahead.  Here it is built for the warm-up + timed batches before the timed region, and
    # its per-batch cost over a whole window (how the epoch loop pays it) is added to the
    # timed seconds for the headline value.
    # (the pipelined peer-to-peer form's last step reads the row lists of the batch after it)
    look = min(eng._look, nb - W - K)
    prebuilt = W + K + look <= eng.index_window
    if prebuilt:
        eng.build_index(0, W + K + look)
        eng.check()                        # a partition overflow is reported before any step
    if eng._dp:                            # the rows all-to-all's communicator, before capture
        if not prebuilt:
            eng.build_index(0, min(eng.index_window, W + K))
        if not eng._p2p:
            exchange.rows(eng._dp_send, eng._dp_recv)
        torch.cuda.synchronize()
    graphed = warm_up(eng, W, K, prebuilt, args.graph_chunk > 1)
    timed_graphs = eng.graph_sizes(W, K) if graphed else []
    torch.cuda.synchronize()
    rdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # the index of the K batches after the timed ones, built beside them as the epoch loop
    # builds a window's successor (engine.run prefetch) -- for runs of at least
    # OVERLAP_MIN_STEPS steps; a shorter run is timed without it and the build is counted at its
    # serial per-batch cost over a whole window (measured below): beside only 20 steps the side
    # build's interference costs the steps more (0.6-0.8 us each, profiles/r05_ab.txt) than the
    # whole serial build (0.39 us per batch)
    npref = 0
    if prebuilt and eng.index_overlap and 2 * K <= eng.index_window and K >= OVERLAP_MIN_STEPS:
        npref = max(0, min(K, nb - W - K))
    # no run follows the timed one on this cursor: its last graph skips the cursor advance
    eng.run(W, K, index=not prebuilt, last_advance=False,
            prefetch=None if not prebuilt else npref > 0, sync_peers=False)
    t_host = time.perf_counter() - t0          # host time to queue the timed region's work
    torch.cuda.synchronize()
    rdist.barrier()
    torch.cuda.synchronize()
    elapsed = rdist.max_over_ranks(time.perf_counter() - t0)
    eng.check()
    costs = eng.costs[W:W + K].cpu().numpy()
    assert np.all(np.isfinite(costs)), "non-finite cost"
    # row-index build cost per batch, over one whole window (as the epoch loop builds it)
    st0 = torch.cuda.current_stream()
    nwin = min(eng.index_window, nb)
    ie = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ie[0].record(st0)
    eng.build_index(0, nwin)
    ie[1].record(st0)
    torch.cuda.synchronize()
    index_us = ie[0].elapsed_time(ie[1]) * 1e3 / nwin
    index_us = rdist.max_over_ranks(index_us)

    # ---- per-kernel durations: eager launches of the same step sequence continuing the
    # epoch, each phase launched through rae_time_next (hipExtLaunchKernelGGL), so the HIP
    # events carry the kernels' own dispatch begin/end timestamps -- the span rocprofv3
    # --kernel-trace reports -- on the stream the kernels run on
    lib, plan = eng.lib, eng.plan
    st = torch.cuda.current_stream()
    sp_ = C.c_void_p(st.cuda_stream)
    b0 = W + K
    n_it = min(args.kernel_iters, nb - b0, eng.index_window)
    eng.build_index(b0, n_it)
    eng.set_cursor(b0)

    def _ev():
        h = C.c_void_p()
        assert lib.rae_event_create(C.byref(h)) == 0, lib.rae_last_error()
        return h
    fev = [(_ev(), _ev()) for _ in range(n_it)]
    uev = [(_ev(), _ev()) for _ in range(n_it)]
    xev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(n_it)]
    pev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(n_it)]
    for i in range(n_it):
        if eng._dp and not eng._p2p:       # partitioned update: rows pulled from their owners
            pev[i][0].record(st)
            assert lib.rae_dp_pack(plan, i, sp_) == 0, lib.rae_last_error()
            exchange.rows(eng._dp_send, eng._dp_recv)
            assert lib.rae_dp_unpack(plan, i, sp_) == 0, lib.rae_last_error()
            pev[i][1].record(st)
        assert lib.rae_time_next(plan, fev[i][0], fev[i][1]) == 0
        assert lib.rae_step_forward(plan, i, sp_) == 0, lib.rae_last_error()
        if exchange is not None and not eng._p2p:   # the records all-gather (data parallel)
            xev[i][0].record(st)
            exchange(eng.exchange_buf)
            xev[i][1].record(st)
        assert lib.rae_time_next(plan, uev[i][0], uev[i][1]) == 0
        assert lib.rae_step_update(plan, i, sp_) == 0, lib.rae_last_error()
    torch.cuda.synchronize()

    def _ms(pair):
        v = C.c_float()
        assert lib.rae_event_elapsed_ms(pair[0], pair[1], C.byref(v)) == 0, lib.rae_last_error()
        return v.value
    fwd_ms = np.array([_ms(e) for e in fev])
    upd_ms = np.array([_ms(e) for e in uev])
    xch_ms = np.array([a.elapsed_time(b) for a, b in xev]) \
        if exchange is not None and not eng._p2p else None
    for e in fev + uev:
        lib.rae_event_destroy(e[0])
        lib.rae_event_destroy(e[1])
    fwd_us = float(np.mean(fwd_ms) * 1e3)
    upd_us = float(np.mean(upd_ms) * 1e3)
    dec = cfg["dec"]
    xs = data.split["train"]
    host = dict(indptr=np.asarray(xs.xFeats.indptr, dtype=np.int64), indices=xs.xFeats.indices,
                args1=xs.args1, args2=xs.args2, neg1=neg1, neg2=neg2)
    per = [step_bytes(host, (b0 + i) * L, L, l, rk, cfg["m"], cfg["r"], cfg["s"], dec)
           for i in range(n_it)]
    by = np.array([p_["s8d"] for p_ in per], dtype=np.float64).mean(axis=0)
    bmin = np.array([p_["min"] for p_ in per], dtype=np.float64).mean(axis=0)
    traffic = pmc_traffic(args.config, args.batch_size)
    build_id = lib.rae_build_id().decode()
    kern = {}
    for i, (name, us) in enumerate((("k_forward", fwd_us), ("k_update", upd_us))):
        kern[name] = {"avg_launch_us": us,
                      "bytes_per_launch": by[i], "achieved_GBs": by[i] / (us * 1e-6) / 1e9,
                      "frac": by[i] / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                      "bytes_min_per_launch": bmin[i],
                      "achieved_min_GBs": bmin[i] / (us * 1e-6) / 1e9,
                      "frac_min": bmin[i] / (us * 1e-6) / 1e9 / HBM_PEAK_GBS}
        t = (traffic or {}).get(name)
        if t is not None:
            kern[name]["traffic"] = t
    if dec != "sp":
        kern["k_forward"]["kernels"] = "k_bil_enc + k_bil_mt + k_bil_dec + k_bil_mt [+ k_bil_dp*] + k_bil_fin"
        kern["k_update"]["kernels"] = "[k_bil_prep +] k_bil_rows + k_update_bil"
    elif eng.kernel_forms_in_use()["sp_forward"] == "split":
        kern["k_forward"]["kernels"] = "k_sp_enc + k_sp_cp + k_sp_dec + k_sp_ctdw (with the softmax backward)"
    # the roofline line names the dominant kernel: the longer average launch of the step
    dom = "k_forward" if fwd_us >= upd_us else "k_update"
    if dec == "sp":
        k = kern[dom]
        roof = {"kernel": dom, "bound": "hbm", "achieved": k["achieved_GBs"], "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": k["frac"], "traffic": k.get("traffic"),
                "bytes_per_launch": k["bytes_per_launch"], "avg_launch_us": k["avg_launch_us"],
                "bytes": "SURVEY.md 8(d) algorithmic bytes (bench.py step_bytes 's8d'); "
                         "frac_min counts each byte this design moves once",
                "frac_min": k["frac_min"], "timing": TIMING,
                "traffic_source": None}
    else:
        fl = step_flops(L, l, cfg["m"], cfg["r"], dec)
        pk = MFMA_BF16_PEAK_TFS if cfg.get("bf16") else MFMA_F32_PEAK_TFS
        ach = fl / ((fwd_us + upd_us) * 1e-6) / 1e12
        roof = {"kernel": "step (forward phase + update phase)", "dominant_phase": dom,
                "bound": "mfma", "achieved": ach,
                "peak": pk, "unit": "TFLOP/s", "frac": ach / pk,
                "traffic": kern[dom].get("traffic"), "traffic_of": dom + " phase, per step",
                "flops_per_step": fl, "avg_step_kernel_us": fwd_us + upd_us,
                "timing": TIMING}
    if traffic:
        # HBM (+ Infinity-Cache) bytes of the dominant kernel per launch from the committed PMC
        # passes, and whether they profiled the library this run uses
        roof["traffic_source"] = (traffic.get("file", "") + ": " + traffic.get("source", ""))
        roof["traffic_build_id"] = traffic.get("build_id")
        roof["traffic_current"] = traffic.get("build_id") == build_id

    # ---- labelling pass over the whole train split (func['label_train'] at full-split scale,
    # the encoder kernel K1 in inference mode): fixed weights, probs + labels
    label = None
    if not args.no_label_pass:
        split = eng.split
        Nl = split.N
        lab = torch.empty(Nl, dtype=torch.int64, device=dev)
        pr = torch.empty((Nl, cfg["m"]), dtype=torch.float32, device=dev)
        Wt, Wbt = ind.modelFunc.params[0], ind.modelFunc.params[1]

        def _label():
            lib.rae_label(C.c_void_p(split.indptr.data_ptr()), C.c_void_p(split.indices.data_ptr()),
                          None, C.c_void_p(Wt.data_ptr()), C.c_void_p(Wbt.data_ptr()), cfg["m"], 0, Nl,
                          C.c_void_p(lab.data_ptr()), C.c_void_p(pr.data_ptr()), sp_)
        _label()
        torch.cuda.synchronize()
        le = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(5)]
        for a_, b_ in le:
            a_.record(st)
            _label()
            b_.record(st)
        torch.cuda.synchronize()
        lus = float(np.mean([a_.elapsed_time(b_) for a_, b_ in le]) * 1e3)
        nnz = int(split.indptr_np[Nl])
        lbytes = 4 * (Nl + 1) + 4 * nnz + 4 * nnz * cfg["m"] + 4 * Nl * cfg["m"] + 8 * Nl + 4 * cfg["m"]
        lach = lbytes / (lus * 1e-6) / 1e9
        # compulsory HBM bytes: every input read once (indptr, feature ids, W once -- its rows
        # are gathered again and again, from L2 / MALL), every output written once
        cbytes = 4 * (Nl + 1) + 4 * nnz + 4 * cfg["d"] * cfg["m"] + 4 * Nl * cfg["m"] + 8 * Nl + \
            4 * cfg["m"]
        label = {"kernel": "k_label (rae_label over the whole train split)", "rows": Nl,
                 "avg_launch_us": lus, "bytes_per_launch": lbytes, "achieved": lach,
                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": lach / HBM_PEAK_GBS,
                 "rows_per_s": Nl / (lus * 1e-6),
                 "bytes": "per row 4 (indptr) + 4f (ids) + 4fm (W rows) + 4m (probs) + 8 (label); "
                          "no W-row reuse credited (SURVEY 8d) -- W (4dm bytes) is L2/MALL "
                          "resident, so most of these bytes never reach HBM",
                 "compulsory_bytes": cbytes,
                 "compulsory_frac": cbytes / (lus * 1e-6) / 1e9 / HBM_PEAK_GBS,
                 "compulsory": "each input read once from HBM (indptr, ids, W), probs + labels "
                               "written once: the bytes that must cross HBM; 'frac' is the "
                               "no-reuse gather rate (W rows mostly from MALL)"}
        lt = ((traffic or {}).get("per_kernel") or {}).get("rae::k_label")
        if lt:
            label["traffic"] = lt["traffic_bytes"]
            label["traffic_GBs"] = lt["traffic_bytes"] / (lus * 1e-6) / 1e9
            label["traffic_frac"] = label["traffic_GBs"] / HBM_PEAK_GBS
            label["traffic_source"] = (f"{traffic.get('file')}: 2*FETCH_SIZE + WRITE_SIZE per "
                                       f"launch (L2 misses: HBM and Infinity-Cache bytes)")
        del lab, pr

    # ---- measured copy bandwidth of this HBM: our own STREAM-style float4 copy kernel
    # (rae_stream_copy), 2 GiB each way -- the practical ceiling next to the 8 TB/s spec the
    # roofline fractions quote (MI355X_MICROARCH.md: 6.29 TB/s for a float4 copy)
    hbm_copy = None
    if not args.no_label_pass:
        nbytes = 1 << 31
        src = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        dst = torch.empty_like(src)

        def _copy():
            assert lib.rae_stream_copy(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                       nbytes, sp_) == 0, lib.rae_last_error()
        _copy()
        torch.cuda.synchronize()
        ce = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(7)]
        for a_, b_ in ce:
            a_.record(st)
            _copy()
            b_.record(st)
        torch.cuda.synchronize()
        cus = float(np.median([a_.elapsed_time(b_) for a_, b_ in ce]) * 1e3)
        assert bool(torch.equal(src[-4:], dst[-4:]))
        hbm_copy = {"GBs": 2 * nbytes / (cus * 1e-6) / 1e9, "bytes": 2 * nbytes, "us": cus,
                    "how": "rae_stream_copy: float4 loads/stores, 2 GiB read + 2 GiB written, "
                           "median of 7"}
        if label is not None:
            label["frac_of_measured_copy"] = label["achieved"] / hbm_copy["GBs"]
            if "traffic_GBs" in label:
                label["traffic_frac_of_measured_copy"] = label["traffic_GBs"] / hbm_copy["GBs"]
        roof["frac_of_measured_copy"] = (roof["achieved"] / hbm_copy["GBs"]
                                         if roof.get("unit") == "GB/s" else None)
        del src, dst

    # ---- measured dense bf16 MFMA ceiling (rae_mfma_probe): the denominator next to the
    # 2.5 PF datasheet label for the bilinear decoders' MFMA roofline
    mfma_peak = None
    if not args.no_label_pass:
        blocks, iters = 256 * 8, 4096
        sink = torch.empty(blocks * 4, dtype=torch.float32, device=dev)

        def _mfma():
            assert lib.rae_mfma_probe(iters, blocks, C.c_void_p(sink.data_ptr()), sp_) == 0, \
                lib.rae_last_error()
        _mfma()
        torch.cuda.synchronize()
        me = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(5)]
        for a_, b_ in me:
            a_.record(st)
            _mfma()
            b_.record(st)
        torch.cuda.synchronize()
        mus = float(np.median([a_.elapsed_time(b_) for a_, b_ in me]) * 1e3)
        fl = blocks * 4.0 * iters * 8 * 16384
        mfma_peak = {"TFLOPs": fl / (mus * 1e-6) / 1e12, "flops": fl, "us": mus,
                     "how": "rae_mfma_probe: 2048 WGs x 4 waves, 8 independent "
                            "v_mfma_f32_16x16x32_bf16 chains per wave, median of 5"}
        if roof.get("unit") == "TFLOP/s" and cfg.get("bf16"):
            roof["frac_of_measured_peak"] = roof["achieved"] / mfma_peak["TFLOPs"]

    # headline: end-to-end training throughput with the row index counted in -- built inside
    # the timed region beside the steps (npref batches), the rest at its serial cost
    e2e = elapsed + ((K - npref) * index_us * 1e-6 if prebuilt else 0.0)
    ms_per_step = 1e3 * e2e / K
    out = {
        "metric": METRIC,
        "value": K * L / e2e,
        "unit": "examples/s",
        "n_gpus": ws,
        "steps": K,
        "warmup": W,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 MFMA operands, fp32 accumulate" if cfg.get("bf16") else "fp32",
        "data": "synthetic (SURVEY 8d generator, seed 1234; random-init params, seed 2)",
        "config": {"workload": cfg["name"], "global_batch": L, "batch_per_gpu": l,
                   "n_examples": cfg["N"], "n_features": cfg["d"], "relations": cfg["m"],
                   "embed": cfg["r"], "neg_samples": cfg["s"], "decoder": cfg["dec"],
                   "optimizer": "adagrad", "parallelism": f"dp{ws}",
                   "n_entities": data.get_arg_voc_size(),
                   "graph_chunk": args.graph_chunk if graphed else 1,
                   "timed_graph_steps": timed_graphs,
                   "graph_batches": "absolute" if (graphed and eng.graph_absolute) else "cursor",
                   "kernel_forms": eng.kernel_forms_in_use()},
        "roofline": roof,
        "kernels": kern,
        "kernel_us": {"forward": fwd_us, "update": upd_us,
                      "forward_p50": float(np.median(fwd_ms) * 1e3),
                      "update_p50": float(np.median(upd_ms) * 1e3)},
        "label_pass": label,
        "hbm_copy": hbm_copy,
        "mfma_bf16_peak": mfma_peak,
        "negative_sampling_s": t_neg,
        "negative_sampling": "host RandomState uniforms (reference stream) + device CDF search",
        "timed_region_host_queue_us": t_host * 1e6,
        "index_build_us_per_batch": index_us,
        "index_build": ("k_build_index + k_build_tasks (parameter-independent per-batch row "
                        "index): the next batches' index built on a side stream beside the "
                        "timed steps (index_batches_built_in_timed_region); batches it could "
                        "not build there are counted at index_build_us_per_batch (serial, "
                        "over a whole window)"),
        "index_batches_built_in_timed_region": npref if prebuilt else K,
        "index_overlap": eng.index_overlap,
        "index_mode": ("beside the timed steps (side stream)" if npref > 0 else
                       "serial, counted at index_build_us_per_batch per step") if prebuilt else
                      "on the step stream before each window (inside the timed region)",
        "build_id": build_id,
        "dataset_build_s": t_data,
    }
    if xch_ms is not None:
        out["kernel_us"]["exchange"] = float(np.mean(xch_ms) * 1e3)
    if eng._dp and not eng._p2p:
        out["kernel_us"]["row_pull"] = float(np.mean([a.elapsed_time(b) for a, b in pev]) * 1e3)
        out["config"]["dp_row_caps"] = list(eng._dp_caps)
    if rk == 0 and ws == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(data, cfg, l, args.cpu_seconds)
        out["cpu_baseline"]["host_cpus"] = os.cpu_count()
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    if rk == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
