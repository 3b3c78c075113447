"""Host-side cost of launching a captured step graph: torch's CUDAGraph.replay() against
hipGraphLaunch on the raw exec through ctypes, and engine.run() as bench.py calls it.
Diagnostic only.   python tools/probes/replay_overhead.py"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))
import torch  # noqa: E402
from rae.data import synthetic_dataset  # noqa: E402
from rae.inducer import ReconstructInducer  # noqa: E402

dev = torch.device("cuda", 0)
data, gold = synthetic_dataset(20000, 4000, 20, seed=1)
ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 100, 200, 100, 20, 0.0, 0.0,
                         "adagrad", "probe", "sp", False, True, False, 1.0, device=dev, graph_chunk=64)
ind.compile_function()
eng = ind.engine
n1, n2 = ind.draw_epoch_negatives()
eng.set_epoch_negatives(n1, n2)
eng.build_index(0, 100)
eng.capture_for(0, 20, last_advance=False)
g = eng._graph(20, advance=False)
hip = C.CDLL("libamdhip64.so")
hip.hipGraphLaunch.argtypes = [C.c_void_p, C.c_void_p]
ex = C.c_void_p(g.raw_cuda_graph_exec())
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
eng.run(0, 20, index=False, last_advance=False)
torch.cuda.synchronize()
for name, fn in (("CUDAGraph.replay", g.replay), ("hipGraphLaunch", lambda: hip.hipGraphLaunch(ex, st)),
                 ("engine.run", lambda: eng.run(0, 20, index=False, last_advance=False))):
    ts = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    print(f"{name:18s} host us: median {np.median(ts) * 1e6:.1f}  min {np.min(ts) * 1e6:.1f}", flush=True)
eng.close()
