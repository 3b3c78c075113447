"""Debug probe: private rows (priv_rows auto) vs the update launch (off), step by step -- the
first batch whose parameters differ and where.   python tools/probes/priv_diff.py [opt]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "relation-autoencoder_amd"))
from rae.data import synthetic_dataset  # noqa: E402
from rae.inducer import ReconstructInducer  # noqa: E402

opt = sys.argv[1] if len(sys.argv) > 1 else "sgd"
dev = torch.device("cuda", 0)
engs = []
for form in ("auto", "off"):
    data, gold = synthetic_dataset(400, 3000, 10, seed=21)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 100, 200, 100, 20,
                             0.0, 0.0, opt, "priv", "sp", False, True, False, 1.0, device=dev,
                             graph_chunk=1, kernel_forms={"priv_rows": form})
    ind.compile_function()
    n1, n2 = ind.draw_epoch_negatives()
    ind.engine.set_epoch_negatives(n1, n2)
    engs.append(ind)
for b in range(4):
    snap = []
    for ind in engs:
        ind.engine.run(b, 1, graph=False)
        torch.cuda.synchronize()
        snap.append({k: v.detach().cpu().numpy().copy() for k, v in ind.modelFunc.named_params().items()})
    for k in snap[0]:
        d = snap[0][k] != snap[1][k]
        if d.any():
            idx = np.argwhere(d)
            print(f"batch {b}: {k} differs at {len(idx)} entries, first {idx[:5].tolist()}, "
                  f"values {snap[0][k][tuple(idx[0])]!r} vs {snap[1][k][tuple(idx[0])]!r}")
    print(f"batch {b} done")
