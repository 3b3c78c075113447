import sys, os, numpy as np
sys.path.insert(0, "relation-autoencoder_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import test_gpu_train as T
import torch
from rae.data import synthetic_dataset
from rae.inducer import ReconstructInducer
dev = torch.device("cuda", 0)
for shape in [(60, 96, 5, 40), (100, 200, 20, 100)]:
    for dec in ["rescal", "rescal+sp"]:
        m, r, s, l = shape
        data, gold = synthetic_dataset(200, 2000, 10, seed=99)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0, 0.0,
                                 "adagrad", "bf16", dec, False, True, False, 1.0, device=dev,
                                 graph_chunk=2, mfma_bf16=True)
        ind.learn(verbose=False)
        tr, costs = T._oracle_trajectory(dec, data, 2, m, r, s, l, 1, lr=0.1, alpha=1.0)
        got = T._params(ind)
        rels = {k: float(np.linalg.norm(got[k] - v) / max(np.linalg.norm(v), 1e-12)) for k, v in tr.params.items()}
        cr = float(np.max(np.abs(np.array(ind.epoch_costs) - costs) / np.abs(costs)))
        print(os.environ.get("RAE_DP2", "1"), shape, dec, "cost", f"{cr:.2e}", {k: f"{v:.2e}" for k, v in rels.items()}, flush=True)
