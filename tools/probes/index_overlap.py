"""Does the row-index build hide behind the step graphs when it runs on a second stream?

    python tools/probes/index_overlap.py [--config c3] [--l 100] [--G 1] [--dp-update replicated]
                                         [--n 128] [--reps 5]

The index is parameter independent, so the next window's build could run beside the current
window's steps.  Times (HIP events, medians over reps):
  steps     n graph-replayed steps alone (batches [0, n), their index built beforehand)
  index     the build of n other batches ([n, 2n): other ring slots) alone
  serial    index then steps on one stream
  overlap   steps on the main stream and the build on a low-priority side stream at once
With --G > 1 the plan is rank 0 of a G-rank plan with no-op collectives (dp_update_model.py)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    import bench
    from dp_update_model import NoPeers
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--l", type=int, default=100)
    ap.add_argument("--G", type=int, default=1)
    ap.add_argument("--dp-update", default="replicated")
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--graph-chunk", type=int, default=0, help="steps per graph (0: n)")
    ap.add_argument("--slices", type=int, default=1, help="prefetch slices (one per graph)")
    ap.add_argument("--priority", default="low", choices=["low", "normal"])
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
    G = args.G
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, args.l, cfg["r"],
                             cfg["m"], cfg["s"], 0.0, 0.0, "adagrad", "ovl", cfg["dec"], False,
                             True, False, 1.0, device=dev, world_size=G, rank=0,
                             exchange=NoPeers(G) if G > 1 else None,
                             graph_chunk=args.graph_chunk or args.n,
                             mfma_bf16=cfg.get("bf16", False), dp_update=args.dp_update)
    ind.compile_function()
    eng = ind.engine
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    n = args.n
    assert 2 * n <= eng.index_window and 2 * n <= eng.nb, (eng.index_window, eng.nb)
    main_s = torch.cuda.current_stream(dev)
    lo, hi = torch.cuda.Stream.priority_range()
    side = torch.cuda.Stream(dev, priority=lo if args.priority == "low" else 0)
    eng.build_index(0, 2 * n)
    eng.capture_for(0, n)
    eng.run(0, n, index=False)                          # warm

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def build_on(stream):
        import ctypes as C
        from rae import _lib
        _lib.check(eng.lib.rae_build_index(eng.plan, n, n, C.c_void_p(stream.cuda_stream)),
                   "rae_build_index")

    import time
    res = {k: [] for k in ("steps", "index", "serial", "overlap", "overlap_sliced",
                           "host_queue_sliced_us", "engine_sliced", "engine_sliced_host_us",
                           "engine_sliced_own_stream", "engine_sliced_own_stream_host_us")}
    own = torch.cuda.Stream(dev)
    gc = args.graph_chunk or n

    def build_slice(stream, b, c):
        import ctypes as C
        from rae import _lib
        _lib.check(eng.lib.rae_build_index(eng.plan, b, c, C.c_void_p(stream.cuda_stream)),
                   "rae_build_index")
    for _ in range(args.reps):
        torch.cuda.synchronize()
        a, b = ev(), ev()
        a.record(main_s)
        eng.run(0, n, index=False)
        b.record(main_s)
        torch.cuda.synchronize()
        res["steps"].append(a.elapsed_time(b) * 1e3 / n)

        a, b = ev(), ev()
        a.record(side)
        build_on(side)
        b.record(side)
        torch.cuda.synchronize()
        res["index"].append(a.elapsed_time(b) * 1e3 / n)

        a, b = ev(), ev()
        a.record(main_s)
        build_on(main_s)
        eng.run(0, n, index=False)
        b.record(main_s)
        torch.cuda.synchronize()
        res["serial"].append(a.elapsed_time(b) * 1e3 / n)

        a, b, c = ev(), ev(), ev()
        a.record(main_s)
        side.wait_event(a)
        build_on(side)
        c.record(side)
        eng.run(0, n, index=False)
        main_s.wait_event(c)
        b.record(main_s)
        torch.cuda.synchronize()
        res["overlap"].append(a.elapsed_time(b) * 1e3 / n)

        # sliced: one prefetch slice in front of each graph replay, as engine.run does
        torch.cuda.synchronize()
        a, b = ev(), ev()
        a.record(main_s)
        t0 = time.perf_counter()
        eng.set_cursor(0)
        k = max(1, args.slices)
        q = -(-n // k)
        cs = []
        for g0 in range(0, n, gc):
            i = g0 // gc
            if i < k and i * q < n:
                side.wait_stream(main_s)
                build_slice(side, n + i * q, min(q, n - i * q))
                c = ev()
                c.record(side)
                cs.append(c)
            eng._graph(min(gc, n - g0)).replay()
        res["host_queue_sliced_us"].append((time.perf_counter() - t0) * 1e6)
        for c in cs:
            main_s.wait_event(c)
        b.record(main_s)
        torch.cuda.synchronize()
        eng.cursor_moved()
        res["overlap_sliced"].append(a.elapsed_time(b) * 1e3 / n)

        # the engine's own path: run(prefetch=True) on the default stream, then on a stream
        for key, strm in (("engine_sliced", main_s), ("engine_sliced_own_stream", own)):
            torch.cuda.synchronize()
            with torch.cuda.stream(strm):
                eng._ready = (0, n, eng._neg_version, None)
                a, b = ev(), ev()
                a.record(strm)
                t0 = time.perf_counter()
                eng.run(0, n, index=False, prefetch=True)
                res[key + "_host_us"].append((time.perf_counter() - t0) * 1e6)
                strm.wait_stream(eng._idx_stream)
                b.record(strm)
            torch.cuda.synchronize()
            res[key].append(a.elapsed_time(b) * 1e3 / n)
    out = {k: float(np.median(v)) for k, v in res.items()}
    out.update(config=args.config, l=args.l, G=G, dp_update=args.dp_update, n=n,
               unit="us per step", kernel_forms=eng.kernel_forms_in_use())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
