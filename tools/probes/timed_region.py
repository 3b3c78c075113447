"""Fixed cost of bench.py's timed region: wall time (synchronize -> run -> synchronize) and the
GPU span (events on the stream) of K consecutive C3 steps, for several K, launched as one
captured graph (cursor or absolute batches) or eagerly.  intercept = wall(K) - K * slope.
Diagnostic only.   python tools/probes/timed_region.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from rae.data import synthetic_dataset  # noqa: E402
from rae.inducer import ReconstructInducer  # noqa: E402

dev = torch.device("cuda", 0)
cfg = bench.CONFIGS["c3"]
data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
out = {}
for mode in ("graph", "graph_abs", "eager"):
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 100, cfg["r"], cfg["m"],
                             cfg["s"], 0.0, 0.0, "adagrad", "probe", "sp", False, True, False, 1.0,
                             device=dev, graph_chunk=1 if mode == "eager" else 128)
    ind.compile_function()
    eng = ind.engine
    eng.graph_absolute = mode == "graph_abs"
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    Ks = (1, 5, 10, 20, 40, 80)
    first = 0
    plan = []
    for K in Ks:
        for rep in range(4):
            plan.append((first, K))
            first += K + 1
    eng.build_index(0, first)
    for b, K in plan:
        eng.capture_for(b, K, last_advance=False)
    res = {K: {"wall": [], "gpu": []} for K in Ks}
    for b, K in plan:
        eng.run(b - 1 if b else 0, 1, index=False)            # warm / position the cursor
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        eng.run(b, K, index=False, last_advance=False)
        e1.record()
        torch.cuda.synchronize()
        res[K]["wall"].append((time.perf_counter() - t0) * 1e6)
        res[K]["gpu"].append(e0.elapsed_time(e1) * 1e3)
    wall = np.array([np.median(res[K]["wall"]) for K in Ks])
    gpu = np.array([np.median(res[K]["gpu"]) for K in Ks])
    sw, iw = np.polyfit(Ks, wall, 1)
    sg, ig = np.polyfit(Ks, gpu, 1)
    out[mode] = {"K": list(Ks), "wall_us": wall.round(1).tolist(), "gpu_us": gpu.round(1).tolist(),
                 "wall_slope_us": round(sw, 2), "wall_intercept_us": round(iw, 1),
                 "gpu_slope_us": round(sg, 2), "gpu_intercept_us": round(ig, 1)}
    print(mode, json.dumps(out[mode]), flush=True)
    ind._drop_engine()
print(json.dumps(out))
