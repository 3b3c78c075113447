"""Host-side time of the calls bench.py's timed region makes (engine.prefetch_index, graph
replays, the torch stream/event calls inside): bench.main() with those methods wrapped.

    python tools/probes/bench_host_trace.py [bench.py arguments]

Prints one line per wrapped call made inside engine.run (name, host microseconds) to stderr
after bench's JSON line."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from rae import engine as E
    log = []
    state = {"on": False}

    def wrap(obj, name, label):
        fn = getattr(obj, name)

        def w(*a, **k):
            t0 = time.perf_counter()
            r = fn(*a, **k)
            if state["on"]:
                log.append((label, (time.perf_counter() - t0) * 1e6))
            return r
        setattr(obj, name, w)

    run = E.TrainEngine.run

    def run_w(self, *a, **k):
        state["on"] = True
        log.append(("---- run", 0.0))
        t0 = time.perf_counter()
        try:
            return run(self, *a, **k)
        finally:
            log.append(("run total", (time.perf_counter() - t0) * 1e6))
            state["on"] = False
    E.TrainEngine.run = run_w
    wrap(E.TrainEngine, "prefetch_index", "prefetch_index")
    wrap(torch.cuda.Stream, "wait_stream", "  Stream.wait_stream")
    wrap(torch.cuda.Stream, "record_event", "  Stream.record_event")
    wrap(torch.cuda.Event, "record", "  Event.record")
    wrap(torch.cuda.CUDAGraph, "replay", "graph replay")
    import bench
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
    starts = [i for i, (k, _) in enumerate(log) if k == "---- run"]
    timed = max(range(len(starts)), key=lambda j: (log[starts[j + 1] - 1][1] if j + 1 < len(starts)
                                                   else log[-1][1]))
    end = starts[timed + 1] if timed + 1 < len(starts) else len(log)
    for k, v in log[starts[timed]:end]:
        print(f"{k:28s} {v:9.1f}", file=sys.stderr)


if __name__ == "__main__":
    main()
