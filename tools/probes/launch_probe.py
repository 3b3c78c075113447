"""Probe: the fixed cost of a short timed run (bench.py's driver command times 20 C3 steps) --
host time of each graph replay and wall time from the host clock, for one 20-step graph against
a short head graph followed by the rest (the GPU starts on the head while the host submits the
rest).  Prints one line per split: median wall us over reps, us per step, host us per replay.

    python tools/probes/launch_probe.py [--config c3] [--steps 20] [--reps 15]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    args = ap.parse_args()
    import torch
    import bench
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 100, cfg["r"], cfg["m"],
                             cfg["s"], 0.0, 0.0, "adagrad", "probe", cfg["dec"], False, True, False,
                             1.0, device=dev, graph_chunk=64)
    ind.compile_function()
    eng = ind.engine
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    K = args.steps
    eng.build_index(0, min(eng.index_window, 8 * K))
    eng.run(0, K, index=False)                     # warm-up (captures the K-step graph)
    torch.cuda.synchronize()
    splits = [[K], [1, K - 1], [2, K - 2], [4, K - 4], [1, 3, K - 4], [2, 6, K - 8]]
    for sp in splits:
        for n in sp:
            eng._graph(n, advance=True)
    torch.cuda.synchronize()
    for sp in splits:
        walls, hosts = [], []
        for rep in range(args.reps):
            eng.set_cursor(K)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hs = []
            for n in sp:
                h0 = time.perf_counter()
                eng._graph(n, advance=True).replay()
                hs.append((time.perf_counter() - h0) * 1e6)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            hosts.append(hs)
        w = float(np.median(walls))
        h = np.median(np.array(hosts), axis=0)
        print(f"split {sp}: wall {w:.1f} us ({w / K:.2f} us/step), host per replay "
              f"{[round(float(x), 1) for x in h]}", flush=True)


if __name__ == "__main__":
    main()
