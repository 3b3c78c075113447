"""Rank body of the data-parallel tests (launched by tests/test_dist.py through
``python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1``).

    python _dist_worker.py MODE OUT_DIR [decoder]

MODE
  exchange   rae.dist.make_exchange over gloo: every rank ends with all ranks' rows.
  oracle     the partition of SURVEY 8(e) on the float64 oracle: rank k takes rows
             [b*L + k*l, b*L + (k+1)*l) of global batch b and the same columns of the
             per-epoch negatives, normalises its loss by the GLOBAL denominator 4L + 2Ls,
             gradients are summed over ranks (gloo all-reduce), every rank applies the
             identical AdaGrad step.  Each rank saves its params.
  gpu        the real HIP path with world_size 2: both ranks share cuda:0, the exchange
             records go through gloo (host-staged), eager steps.  Each rank saves its
             params and per-batch costs.
  gpu_c3     the same at BASELINE config 3's full size with global batch L = 800 (2 x 400).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "relation-autoencoder_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# shapes shared with test_dist.py
DP_SHAPE = dict(N=240, d=400, ntrue=4, m=8, r=12, s=3, l=15, epochs=2, seed=11)


def _dataset():
    from rae.data import synthetic_dataset
    return synthetic_dataset(DP_SHAPE["N"], DP_SHAPE["d"], DP_SHAPE["ntrue"], seed=DP_SHAPE["seed"])


def run_exchange(out):
    from rae import dist as rdist
    ws, rk = dist.get_world_size(), dist.get_rank()
    ex = rdist.make_exchange(ws, rk)
    n = 5
    buf = torch.full((ws * n,), -1.0)
    buf[rk * n:(rk + 1) * n] = torch.arange(n, dtype=torch.float32) + 100 * (rk + 1)
    ex(buf)
    np.save(os.path.join(out, f"exchange_{rk}.npy"), buf.numpy())


def run_oracle(out, decoder, lambda1=0.0):
    import rae_oracle as O
    ws, rk = dist.get_world_size(), dist.get_rank()
    data, _ = _dataset()
    sp_ = data.split["train"]
    m, r, s, l = DP_SHAPE["m"], DP_SHAPE["r"], DP_SHAPE["s"], DP_SHAPE["l"]
    L = ws * l
    N = sp_.xFeats.shape[0]
    rng = np.random.RandomState(2)
    p = O.init_params(rng, decoder, data.get_dimensionality(), m, data.get_arg_voc_size(), r)
    acc = {k: np.zeros_like(v) for k, v in p.items()}
    D = 4 * L + 2 * L * s
    adjust = L / N
    costs = []
    for ep in range(DP_SHAPE["epochs"]):
        n1 = O.negative_samples(rng, data.negSamplingCum, N, s)
        n2 = O.negative_samples(rng, data.negSamplingCum, N, s)
        for b in range(N // L):
            rows = slice(b * L + rk * l, b * L + (rk + 1) * l)
            res = O.train_step_grads(decoder, p, sp_.xFeats[rows], sp_.args1[rows],
                                     sp_.args2[rows], n1[:, rows], n2[:, rows], alpha=1.0,
                                     lambda1=lambda1 if rk == 0 else 0.0, adjust=adjust,
                                     denom=D)
            names = list(res.grads)
            flat = torch.from_numpy(np.concatenate([res.grads[k].ravel() for k in names] +
                                                   [np.array([res.cost])]))
            dist.all_reduce(flat)
            flat = flat.numpy()
            o = 0
            grads = {}
            for k in names:
                grads[k] = flat[o:o + res.grads[k].size].reshape(res.grads[k].shape)
                o += res.grads[k].size
            costs.append(flat[o])
            O.adagrad_apply(p, acc, grads, 0.1)
    np.savez(os.path.join(out, f"oracle_{decoder}_{rk}.npz"), costs=np.array(costs), **p)


def run_gpu(out, decoder):
    from rae import dist as rdist
    from rae.inducer import ReconstructInducer
    ws, rk = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)                 # both ranks share the one GPU of the box
    torch.cuda.set_device(dev)
    data, gold = _dataset()
    m, r, s, l = DP_SHAPE["m"], DP_SHAPE["r"], DP_SHAPE["s"], DP_SHAPE["l"]
    ex = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), DP_SHAPE["epochs"], 0.1, l, r,
                             m, s, 0.0, 0.0, "adagrad", "dp", decoder, False, True, False, 1.0,
                             device=dev, world_size=ws, rank=rk, exchange=ex, graph_chunk=1)
    ind.learn(verbose=False)
    params = {k: v.detach().cpu().double().numpy() for k, v in ind.modelFunc.named_params().items()}
    np.savez(os.path.join(out, f"gpu_{decoder}_{rk}.npz"),
             costs=np.concatenate(ind.epoch_costs), **params)


def run_gpu_c3(out, steps=3):
    """BASELINE config 3 at full size (1M triples) with the global batch of 8 ranks at l=100,
    L = 800, split over 2 ranks of l = 400: the first `steps` batches of an epoch, negatives
    from the reference's RandomState stream (device CDF search)."""
    from rae import dist as rdist
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    ws, rk = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data, gold = synthetic_dataset(1_000_000, 2 ** 17, 100, seed=1234)
    ex = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 800 // ws, 200, 100,
                             20, 0.0, 0.0, "adagrad", "dp800", "sp", False, True, False, 1.0,
                             device=dev, world_size=ws, rank=rk, exchange=ex, graph_chunk=1)
    ind.compile_function()
    eng = ind.engine
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    eng.run(0, steps)
    torch.cuda.synchronize()
    eng.check()
    np.save(os.path.join(out, f"c3_costs_{rk}.npy"), eng.costs[:steps].cpu().numpy())
    for k, v in ind.modelFunc.named_params().items():
        np.save(os.path.join(out, f"c3_{k}_{rk}.npy"), v.detach().cpu().numpy())


def main():
    mode, out = sys.argv[1], sys.argv[2]
    dec = sys.argv[3] if len(sys.argv) > 3 else "sp"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo")
    try:
        if mode == "exchange":
            run_exchange(out)
        elif mode == "oracle":
            run_oracle(out, dec, lambda1=float(sys.argv[4]) if len(sys.argv) > 4 else 0.0)
        elif mode == "gpu":
            run_gpu(out, dec)
        elif mode == "gpu_c3":
            run_gpu_c3(out)
        else:
            raise SystemExit(f"unknown mode {mode}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
