"""Single-GPU cost model of the data-parallel step at world size G (no peers: the collectives
are no-ops, the other ranks' records stay zero -- a timing probe only).

    python tools/probes/dp_update_model.py [--G 8] [--l 100] [--config c3]
                                           [--link-gbs 76.8] [--links 7] [--eff 0.7] [--lat-us 10]

Times, per step, with the kernels' own dispatch timestamps (rae_time_next):
  single       the G = 1 plan at the same l (the weak-scaling denominator): forward, update, and
               the row index's per-batch cost over a window (bench.py counts it in the step);
  replicated   rank 0 of a G-rank plan: forward (l examples), update over the global batch
               L = G*l (with the SP wire record: k_vrec + k_update), row index of the global batch;
  partitioned  the same with the row-owner partitioned update: + the row pull's pack / unpack.
  p2p_pipe     the same with the next batch's rows pushed during the step (RAE_XCHG_P2P_PIPE):
               the rows' link time is credited as hidden under the update (project_p2p_pipe);
  p2p          the partitioned update over the peer-to-peer exchange (include/rae.h RAE_XCHG_P2P):
               the row and record pushes and the signal waits are kernels of the step; here the
               "peers" are local dummy buffers and the signal words loop back to this rank's own
               counters (a push's signals are the waits' expected counts), so the pushes' stores
               and the waits' polling are timed, the link is not.
Whole steps as the epoch loop runs them (graph replays of n steps, HIP events): alone
("graph_step") and with the next n batches' row index built beside them on the side stream
("graph_step_with_index": engine index_overlap).
Bytes: the records all-gather and the rows all-to-all inbound per rank per step.  The
projection takes graph_step_with_index (kernels, launch gaps and the overlapped index, the
no-op collectives' slots empty) and adds each collective at
lat_us + inbound bytes / (links * link_gbs * eff)  (no overlap with the kernels); it reports
the weak-scaling efficiency t_single / t_G, t_single the same measure of the G = 1 plan.
DESIGN.md sec. 4 holds the table of one run."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))
sys.path.insert(0, ROOT)


class NoPeers:
    def __init__(self, G):
        self.world_size, self.rank = G, 0

    def __call__(self, buf):
        pass

    def rows(self, send, recv):
        pass

    def max_int(self, v):
        return int(v)

    def sync_rows(self, ts):
        pass

    def barrier(self):
        pass


def loopback_p2p_setup(eng):
    """Peers of a G-rank plan with no peer processes: every peer's exchange buffer / replica
    is a local dummy buffer set of its own (distinct addresses, as distinct GPUs would have:
    pushes of one row to several peers are not stores to one address), and peer p's signal
    words start (p - rank) words before this rank's, so the push's add on "peer p's word
    (kind, rank)" lands on this rank's word (kind, p) -- the count the wait for peer p
    expects."""
    import torch
    named = eng._named
    eng._loop = []
    sig = int(eng.lib.rae_p2p_signals(eng.plan))
    for p in range(eng.world_size):
        if p != eng.rank:
            bufs = [torch.zeros_like(eng.exchange_buf), torch.empty_like(named["W"]),
                    torch.empty_like(named["A"]), torch.empty_like(named["Ab"])]
            eng._loop.append(bufs)
            ex, W, A, Ab = (C.c_void_p(t.data_ptr()) for t in bufs)
            rc = eng.lib.rae_set_peer(eng.plan, p, ex, W, A, Ab, C.c_void_p(sig + 4 * (p - eng.rank)))
            assert rc == 0, eng.lib.rae_last_error()


def measure(args, cfg, data, gold, G, mode):
    import torch
    from rae import engine as E
    from rae.inducer import ReconstructInducer
    dev = torch.device("cuda", 0)
    forms = dict(kv.split("=", 1) for kv in args.kernel_form) if G > 1 else {}
    p2p = mode in ("p2p", "p2p_pipe")
    pipe = mode == "p2p_pipe"
    if p2p:
        forms["dp_xchg"] = mode
        mode = "partitioned"
        E.TrainEngine._p2p_setup = loopback_p2p_setup
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, args.l, cfg["r"],
                             cfg["m"], cfg["s"], 0.0, 0.0, "adagrad", "dpm", cfg["dec"], False,
                             True, False, 1.0, device=dev, world_size=G, rank=0,
                             exchange=NoPeers(G) if G > 1 else None, graph_chunk=args.graph_n,
                             mfma_bf16=cfg.get("bf16", False), dp_update=mode,
                             kernel_forms=forms or None)
    ind.compile_function()
    eng = ind.engine
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    # the row index: per-batch cost over a whole window (as the epoch loop builds it)
    nw = min(eng.nb, eng.index_window)
    st0 = torch.cuda.current_stream()
    ie = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    eng.build_index(0, nw)
    torch.cuda.synchronize()
    ie[0].record(st0)
    eng.build_index(0, nw)
    ie[1].record(st0)
    torch.cuda.synchronize()
    index_us = ie[0].elapsed_time(ie[1]) * 1e3 / nw
    n = min(args.iters, eng.nb - eng._look, eng.index_window - eng._look)
    eng.build_index(0, n + eng._look)
    eng.set_cursor(0)
    lib, plan = eng.lib, eng.plan
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if pipe:                               # the first step's rows (no previous step pushed them)
        assert lib.rae_p2p_prologue(plan, 0, 0, st) == 0, lib.rae_last_error()

    def ev():
        h = C.c_void_p()
        assert lib.rae_event_create(C.byref(h)) == 0
        return h
    part = mode == "partitioned" and G > 1 and not p2p
    t = {"forward": [], "update": []}
    if part:
        t.update(pack=[], unpack=[])
    evs = []
    for i in range(n):
        e = {k: (ev(), ev()) for k in t}
        if part:
            assert lib.rae_time_next(plan, *e["pack"]) == 0
            assert lib.rae_dp_pack(plan, i, st) == 0, lib.rae_last_error()
            assert lib.rae_time_next(plan, *e["unpack"]) == 0
            assert lib.rae_dp_unpack(plan, i, st) == 0, lib.rae_last_error()
        assert lib.rae_time_next(plan, *e["forward"]) == 0
        assert lib.rae_step_forward(plan, i, st) == 0
        assert lib.rae_time_next(plan, *e["update"]) == 0
        assert lib.rae_step_update(plan, i, st) == 0
        evs.append(e)
    if pipe:                               # the last step signalled batch n's rows (engine state)
        eng._p2p_next, eng._p2p_valid = n, True
    torch.cuda.synchronize()
    for e in evs:
        for k in t:
            v = C.c_float()
            if lib.rae_event_elapsed_ms(e[k][0], e[k][1], C.byref(v)) == 0:
                t[k].append(v.value * 1e3)
    out = {k: float(np.median(v[3:])) for k, v in t.items() if v}
    out["index_per_batch"] = index_us
    out["record_floats"] = eng.rec_floats
    if G > 1:
        out["records_allgather_in_bytes"] = (G - 1) * args.l * eng.rec_floats * 4
    if part or p2p:
        ca, cw = eng._dp_caps
        blk = int(lib.rae_dp_block_floats(C.byref(eng.cfg), ca, cw)) * 4
        out["rows_alltoall_in_bytes"] = (G - 1) * blk
        out["row_caps"] = [ca, cw]
    if p2p and not pipe:
        out["xchg"] = "p2p (forward = row push + wait + forward + record push; update = wait + "\
                      "update)"
    if pipe:
        out["xchg"] = "p2p_pipe (forward = wait + forward + record push + next batch's unchanged "\
                      "rows' push; update = wait + update with the updated rows' pushes)"
    out["kernel_forms"] = eng.kernel_forms_in_use()
    out.update(graph_steps(eng, args))
    ind._drop_engine()
    return out


def graph_steps(eng, args):
    """us per step of n graph-replayed steps, alone and with the next n batches' index built
    beside them (prefetch_index on the side stream), medians over reps."""
    import torch
    n = min(args.graph_n, eng.index_window // 2 - eng._look, eng.nb // 2 - eng._look)
    eng.cursor_moved()
    eng.build_index(0, n + eng._look)
    eng.capture_for(0, n)
    eng.run(0, n, index=False)
    main = torch.cuda.current_stream()
    alone, ovl = [], []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        eng.run(0, n, index=False)
        b.record(main)
        torch.cuda.synchronize()
        alone.append(a.elapsed_time(b) * 1e3 / n)
        eng._ready = None                   # force the rebuild of [n, 2n) each rep
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        eng.prefetch_index(n + eng._look, n)
        eng.run(0, n, index=False)
        main.wait_event(eng._ready[3])
        b.record(main)
        torch.cuda.synchronize()
        ovl.append(a.elapsed_time(b) * 1e3 / n)
    return {"graph_steps_n": n, "graph_step": float(np.median(alone)),
            "graph_step_with_index": float(np.median(ovl))}


def project_p2p_pipe(r, t1, args):
    """The pipelined peer-to-peer step: the measured graph step (its pushes' local stores and
    the waits' polling included) + the records' link time not hidden by their push kernel + the
    rows' link time not hidden under the update (the next batch's rows leave from the pre-push
    right after the forward and from the update's row tasks; the peers wait for them only at
    their next forward) + one signal latency per exchange."""
    bw = args.links * args.link_gbs * args.eff * 1e3          # bytes per us
    tg = r["graph_step_with_index"]
    rec_t = r["records_allgather_in_bytes"] / bw
    row_t = r["rows_alltoall_in_bytes"] / bw
    hide = r["update"]                                         # wait + update (events)
    extra = max(0.0, rec_t - args.push_us) + max(0.0, row_t - hide) + 2 * args.p2p_lat_us
    return {"step_us": tg + extra, "kernels_us": tg, "link_and_signal_us": extra,
            "records_in_us": rec_t, "rows_in_us": row_t, "rows_hidden_under_us": hide,
            "efficiency": t1 / (tg + extra), "efficiency_if_link_free": t1 / tg,
            "model": "graph step + max(0, records bytes / rate - push_us) + max(0, rows bytes / "
                     "rate - update us) + 2 signal latencies"}


def project_p2p(r, t1, args):
    """The peer-to-peer step: the measured graph step (its pushes' local stores and the waits'
    polling included) + whatever of each push's inbound bytes the link cannot move while the
    push kernel runs + one signal latency per exchange (a system-scope release seen by the
    peer's poll over xGMI)."""
    bw = args.links * args.link_gbs * args.eff * 1e3          # bytes per us
    tg = r["graph_step_with_index"]
    rec_t = r["records_allgather_in_bytes"] / bw
    row_t = r["rows_alltoall_in_bytes"] / bw
    extra = max(0.0, rec_t - args.push_us) + max(0.0, row_t - args.push_us) + 2 * args.p2p_lat_us
    return {"step_us": tg + extra, "kernels_us": tg, "link_and_signal_us": extra,
            "records_in_us": rec_t, "rows_in_us": row_t, "efficiency": t1 / (tg + extra),
            "efficiency_if_link_free": t1 / tg,
            "model": "graph step (pushes + waits local) + max(0, inbound bytes / rate - "
                     "push_us) per push + 2 signal latencies"}


def project(res, args):
    bw = args.links * args.link_gbs * args.eff * 1e3          # bytes per us
    coll = lambda b: args.lat_us + b / bw                      # noqa: E731
    s = res["single"]
    t1 = s["graph_step_with_index"]
    proj = {"single_step_us": t1,
            "assumptions": {"link_gbs_per_direction": args.link_gbs, "links": args.links,
                            "efficiency": args.eff, "collective_latency_us": args.lat_us,
                            "inbound_GBs": bw / 1e3,
                            "model": "step = graph-replayed step with the index built beside "
                                     "it (measured) + A2A (partitioned) + AG, every collective "
                                     "lat + bytes / inbound rate, not overlapped"}}
    if res.get("p2p_pipe"):
        proj["p2p_pipe"] = project_p2p_pipe(res["p2p_pipe"], t1, args)
        proj["assumptions"]["p2p_signal_latency_us"] = args.p2p_lat_us
    if res.get("p2p"):
        proj["p2p"] = project_p2p(res["p2p"], t1, args)
        proj["assumptions"]["p2p_signal_latency_us"] = args.p2p_lat_us
        proj["assumptions"]["push_overlap_us"] = args.push_us
    for mode in ("replicated", "partitioned"):
        r = res.get(mode)
        if not r:
            continue
        tg = r["graph_step_with_index"]
        comm = 0.0
        if "records_allgather_in_bytes" in r:
            comm += coll(r["records_allgather_in_bytes"])
        if "rows_alltoall_in_bytes" in r:
            comm += coll(r["rows_alltoall_in_bytes"])
        proj[mode] = {"step_us": tg + comm, "kernels_us": tg, "collectives_us": comm,
                      "efficiency": t1 / (tg + comm),
                      "efficiency_if_collectives_free": t1 / tg}
    return proj


def main():
    import bench
    from rae.data import synthetic_dataset
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--l", type=int, default=100)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--graph-n", type=int, default=64, help="steps per timed graph replay")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="replicated,partitioned,p2p,p2p_pipe")
    ap.add_argument("--kernel-form", action="append", default=[], metavar="KEY=VALUE",
                    help="kernel form of the G-rank plans (e.g. priv_rows=off)")
    ap.add_argument("--link-gbs", type=float, default=76.8,
                    help="xGMI GB/s per link and direction (MI355X: 153.6 GB/s bidirectional)")
    ap.add_argument("--links", type=int, default=7)
    ap.add_argument("--eff", type=float, default=0.7, help="achievable fraction of the links")
    ap.add_argument("--lat-us", type=float, default=10.0, help="per-collective latency")
    ap.add_argument("--p2p-lat-us", type=float, default=3.0,
                    help="peer-to-peer signal latency (release -> the peer's poll sees it)")
    ap.add_argument("--push-us", type=float, default=0.0,
                    help="link time hidden under each push kernel (its own measured duration "
                         "is in the graph step)")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
    res = {"G": args.G, "l": args.l, "config": args.config}
    res["single"] = measure(args, cfg, data, gold, 1, "replicated")
    for mode in args.modes.split(","):
        res[mode] = measure(args, cfg, data, gold, args.G, mode)
    res["projection"] = project(res, args)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
