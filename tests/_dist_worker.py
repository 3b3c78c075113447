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
  gpu_c3     the same at BASELINE config 3's full size with global batch L = 800 (2 x 400);
             argument 3: the data-parallel update ("replicated" | "partitioned").
  oracle_part  the row-owner partitioned update's protocol on the float64 oracle.
  rows       rae.dist.Exchange.rows / sync_rows / max_int over gloo.
  gpu_c4dp   BASELINE config 4's model shape (split SP forward + wire records + k_vrec) on a
             reduced synthetic set; argument 3: the data-parallel update.
  gpu_ckpt   partitioned update, gather() on every rank, then a rank-0-only checkpoint.
  nccl1      one rank over RCCL: the captured exchange == no exchange, bitwise (run_nccl1).
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


# the DP_SHAPE set relabelled into vocabularies whose owned rows per rank exceed the row
# lists' LDS bitmap (32 * RAE_DPL_KEYS = 524288 rows at G = 2): entity e -> e * BIG_E, feature
# f -> f * BIG_F, so k_build_dplists takes its hash-pass path for both tables
BIG_E, BIG_F = 25013, 5243


def _dataset_big():
    import scipy.sparse as sp
    from rae.data import DatasetManager, DatasetSplit
    data, gold = _dataset()
    n, d = data.get_arg_voc_size(), data.get_dimensionality()
    splits = {}
    for k, v in data.split.items():
        x = v.xFeats.tocoo()
        xb = sp.csr_matrix((x.data, (x.row, x.col * BIG_F)), shape=(x.shape[0], d * BIG_F))
        splits[k] = DatasetSplit(v.args1 * BIG_E, v.args2 * BIG_E, xb)
    freqs = np.zeros(n * BIG_E, dtype=np.int64)
    freqs[np.arange(n) * BIG_E] = data.entity_freqs
    return DatasetManager(splits, freqs, d * BIG_F), gold


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


def _reads(sp_, n1, n2, rows):
    """Entity rows (e1, e2, negatives) and feature rows the examples `rows` read."""
    ents = np.unique(np.concatenate([sp_.args1[rows], sp_.args2[rows], n1[:, rows].ravel(),
                                     n2[:, rows].ravel()]))
    return ents, np.unique(sp_.xFeats[rows].indices)


def run_oracle_part(out, decoder):
    """The row-owner partitioned update (include/rae.h RAE_DPUPD_PARTITIONED) on the float64
    oracle: every rank keeps a replica, only row x's owner (x % G) applies x's A / Ab / W
    update, and before each forward every owner sends each peer the rows that peer's examples
    read.  Non-owned rows nobody pulled go stale -- if the pull lists missed a row, a forward
    would read a stale value and the run would leave the global-batch trajectory.  At the end
    the owners' rows are gathered (Exchange.sync_rows)."""
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
    own = {"A": np.arange(p["A"].shape[0]) % ws == rk, "W": np.arange(p["W"].shape[0]) % ws == rk}
    own["Ab"] = own["A"]
    D = 4 * L + 2 * L * s
    costs = []
    for ep in range(DP_SHAPE["epochs"]):
        n1 = O.negative_samples(rng, data.negSamplingCum, N, s)
        n2 = O.negative_samples(rng, data.negSamplingCum, N, s)
        for b in range(N // L):
            # pull: owner -> reader, exactly the rows each peer reads and this rank owns
            send = {}
            for j in range(ws):
                if j != rk:
                    e, f = _reads(sp_, n1, n2, slice(b * L + j * l, b * L + (j + 1) * l))
                    e, f = e[e % ws == rk], f[f % ws == rk]
                    send[j] = (e, p["A"][e].copy(), p["Ab"][e].copy(), f, p["W"][f].copy())
            box = [None] * ws
            dist.all_gather_object(box, send)
            for k in range(ws):
                if k != rk:
                    e, a_, ab_, f, w_ = box[k][rk]
                    p["A"][e], p["Ab"][e], p["W"][f] = a_, ab_, w_
            rows = slice(b * L + rk * l, b * L + (rk + 1) * l)
            res = O.train_step_grads(decoder, p, sp_.xFeats[rows], sp_.args1[rows],
                                     sp_.args2[rows], n1[:, rows], n2[:, rows], alpha=1.0,
                                     denom=D)
            names = list(res.grads)
            flat = torch.from_numpy(np.concatenate([res.grads[k].ravel() for k in names] +
                                                   [np.array([res.cost])]))
            dist.all_reduce(flat)                # == the records' contributions, summed
            flat = flat.numpy()
            o = 0
            for k in names:
                g = flat[o:o + res.grads[k].size].reshape(res.grads[k].shape)
                o += res.grads[k].size
                msk = own.get(k)                 # rows: the owner only; dense: every rank
                if msk is None:
                    O.adagrad_apply({k: p[k]}, {k: acc[k]}, {k: g}, 0.1)
                else:
                    sub_p, sub_a = {k: p[k][msk]}, {k: acc[k][msk]}
                    O.adagrad_apply(sub_p, sub_a, {k: g[msk]}, 0.1)
                    p[k][msk], acc[k][msk] = sub_p[k], sub_a[k]
            costs.append(flat[o])
    # gather every row from its owner (the replicas now identical)
    box = [None] * ws
    dist.all_gather_object(box, {k: p[k][own[k]] for k in ("A", "Ab", "W")})
    for k in ("A", "Ab", "W"):
        for j in range(ws):
            p[k][np.arange(p[k].shape[0]) % ws == j] = box[j][k]
    np.savez(os.path.join(out, f"oraclepart_{decoder}_{rk}.npz"), costs=np.array(costs), **p)


def run_sync_rows(out):
    """Exchange.rows (all-to-all of equal blocks) and Exchange.sync_rows over gloo."""
    from rae import dist as rdist
    ws, rk = dist.get_world_size(), dist.get_rank()
    ex = rdist.make_exchange(ws, rk)
    send = torch.arange(ws * 3, dtype=torch.float32) + 1000 * rk     # block j -> rank j
    recv = torch.full_like(send, -1.0)
    ex.rows(send, recv)
    t2 = torch.full((11, 3), -1.0)
    t2[rk::ws] = torch.arange(11, dtype=torch.float32)[rk::ws, None] * 10 + rk
    t1 = torch.full((7,), -1.0)
    t1[rk::ws] = torch.arange(7, dtype=torch.float32)[rk::ws] + 0.5
    ex.sync_rows([t2, t1])
    assert ex.max_int(rk * 3 + 1) == (ws - 1) * 3 + 1
    np.savez(os.path.join(out, f"rows_{rk}.npz"), recv=recv.numpy(), t2=t2.numpy(), t1=t1.numpy())


def run_gpu(out, decoder, dp_update="replicated", dense="auto", priv="auto", index_window=0,
            xchg="collective", graph_chunk=1, vocab="small"):
    from rae import dist as rdist
    from rae.inducer import ReconstructInducer
    ws, rk = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)                 # both ranks share the one GPU of the box
    torch.cuda.set_device(dev)
    data, gold = _dataset_big() if vocab == "big" else _dataset()
    m, r, s, l = DP_SHAPE["m"], DP_SHAPE["r"], DP_SHAPE["s"], DP_SHAPE["l"]
    ex = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), DP_SHAPE["epochs"], 0.1, l, r,
                             m, s, 0.0, 0.0, "adagrad", "dp", decoder, False, True, False, 1.0,
                             device=dev, world_size=ws, rank=rk, exchange=ex,
                             graph_chunk=graph_chunk, dp_update=dp_update,
                             kernel_forms=dict({"dp_dense": dense} if decoder == "sp" else {},
                                               priv_rows=priv, dp_xchg=xchg),
                             index_window=index_window)
    ind.learn(verbose=False)
    if xchg != "collective":
        assert ind.engine.kernel_forms_in_use()["dp_xchg"] == xchg
    if decoder == "sp" and dense != "auto":
        assert ind.engine.kernel_forms_in_use()["dp_dense"] == dense
    if priv != "auto":
        assert ind.engine.kernel_forms_in_use()["priv_rows"] == priv
    ind.engine.sync_replicas()
    params = {k: v.detach().cpu().double().numpy() for k, v in ind.modelFunc.named_params().items()}
    tag = dp_update if xchg == "collective" else f"{dp_update}_{xchg}"
    if vocab != "small":
        tag += "_" + vocab
    np.savez(os.path.join(out, f"gpu_{tag}_{decoder}_{rk}.npz"),
             costs=np.concatenate(ind.epoch_costs), **params)


def run_gpu_delay(out, xchg, delay):
    """a rank that spends host time between single-batch runs (per-batch evaluation,
    checkpoints) must not make a peer's bounded GPU wait time out.  The peer-to-peer forms with a
    0.3 s wait bound; rank 1 sleeps `delay` seconds before every batch; run() meets the peers at a
    host barrier first, so the early rank waits there, not in a wait kernel.  Saves the costs and
    parameters after `steps` batches (bitwise equal with and without the delay)."""
    import time
    from rae import dist as rdist
    from rae.inducer import ReconstructInducer
    ws, rk = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data, gold = _dataset()
    m, r, s, l = DP_SHAPE["m"], DP_SHAPE["r"], DP_SHAPE["s"], DP_SHAPE["l"]
    ex = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "delay", "sp", False, True, False, 1.0, device=dev,
                             world_size=ws, rank=rk, exchange=ex, graph_chunk=1,
                             dp_update="partitioned", kernel_forms={"dp_xchg": xchg},
                             p2p_timeout=0.3)
    ind.compile_function()
    eng = ind.engine
    assert eng.kernel_forms_in_use()["dp_xchg"] == xchg
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    steps = 4
    for b in range(steps):
        if rk == 1 and delay > 0:
            torch.cuda.synchronize()
            time.sleep(delay)
        eng.run(b, 1)
    torch.cuda.synchronize()
    eng.check()                          # a timed-out wait sets error bit 64: raises here
    eng.sync_replicas()
    params = {k: v.detach().cpu().numpy() for k, v in ind.modelFunc.named_params().items()}
    np.savez(os.path.join(out, f"delay_{xchg}_{delay}_{rk}.npz"),
             costs=eng.costs[:steps].cpu().numpy(), **params)


def run_gpu_c3(out, steps=3, dp_update="replicated", heavy_chunk="auto"):
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
                             device=dev, world_size=ws, rank=rk, exchange=ex, graph_chunk=1,
                             dp_update=dp_update, kernel_forms={"heavy_chunk": heavy_chunk})
    ind.compile_function()
    if heavy_chunk != "auto":
        assert ind.engine.kernel_forms_in_use()["heavy_chunk"] == heavy_chunk
    eng = ind.engine
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    eng.run(0, steps)
    torch.cuda.synchronize()
    eng.check()
    eng.sync_replicas()
    np.save(os.path.join(out, f"c3_costs_{rk}.npy"), eng.costs[:steps].cpu().numpy())
    for k, v in ind.modelFunc.named_params().items():
        np.save(os.path.join(out, f"c3_{k}_{rk}.npy"), v.detach().cpu().numpy())


C4DP_SHAPE = dict(N=20_000, d=2 ** 15, ntrue=300, m=300, r=300, s=50, l=100, steps=3, seed=1234)


def c4dp_dataset():
    from rae.data import synthetic_dataset
    c = C4DP_SHAPE
    return synthetic_dataset(c["N"], c["d"], c["ntrue"], seed=c["seed"])


def run_gpu_c4dp(out, dp_update="replicated"):
    xchg = "collective"
    if dp_update in ("p2p", "p2p_pipe"):   # the partitioned update over a peer-to-peer exchange
        dp_update, xchg = "partitioned", dp_update
    """BASELINE config 4's model shape (K = 300, embed 300, neg 50, l = 100 per rank) on a
    reduced synthetic set: the data-parallel kernels the 8-GPU config runs together -- the split
    SP forward (r m > 32768), the wire records with every example's dw1 / dw2 (dp_dense records
    at l = 100), k_vrec rebuilding V1 / V2 / G1 after the exchange, 102 record slots (private rows
    off) -- for the first `steps` global batches of an epoch."""
    from rae import dist as rdist
    from rae.inducer import ReconstructInducer
    ws, rk = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = C4DP_SHAPE
    data, gold = c4dp_dataset()
    ex = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, c["l"], c["r"], c["m"],
                             c["s"], 0.0, 0.0, "adagrad", "c4dp", "sp", False, True, False, 1.0,
                             device=dev, world_size=ws, rank=rk, exchange=ex, graph_chunk=1,
                             dp_update=dp_update, kernel_forms={"dp_xchg": xchg})
    ind.compile_function()
    eng = ind.engine
    forms = eng.kernel_forms_in_use()
    want = {"sp_forward": "split", "dp_update": dp_update, "priv_rows": "off", "dp_dense": "records",
            "dp_xchg": xchg}
    assert {k: forms[k] for k in want} == want, forms
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    snap = {}
    for b in range(c["steps"]):          # one step at a time: the parameters after every step
        eng.run(b, 1)
        torch.cuda.synchronize()
        eng.check()
        eng.sync_replicas()
        for k, v in ind.modelFunc.named_params().items():
            snap[f"{k}@{b}"] = v.detach().cpu().numpy()
    np.savez(os.path.join(out, f"c4dp_{dp_update if xchg == 'collective' else xchg}_{rk}.npz"),
             costs=eng.costs[:c["steps"]].cpu().numpy(), **snap)


def run_gpu_ckpt(out, decoder):
    """Partitioned update, then a rank-0-only checkpoint: every rank calls gather() (the
    collective), then rank 0 alone saves -- which must not start a collective -- and every
    rank's replica equals the others'."""
    from rae import dist as rdist
    from rae.inducer import ReconstructInducer
    ws, rk = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data, gold = _dataset()
    m, r, s, l = DP_SHAPE["m"], DP_SHAPE["r"], DP_SHAPE["s"], DP_SHAPE["l"]
    ex = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), DP_SHAPE["epochs"], 0.1, l, r,
                             m, s, 0.0, 0.0, "adagrad", "dp", decoder, False, True, False, 1.0,
                             device=dev, world_size=ws, rank=rk, exchange=ex, graph_chunk=1,
                             dp_update="partitioned")
    ind.learn(verbose=False)
    assert ind.engine.stale()
    ind.gather()                                   # every rank
    assert not ind.engine.stale()
    if rk == 0:                                    # rank 0 alone: no collective may start here
        ind.save_checkpoint(os.path.join(out, "ckpt_part.npz"))
        lab, _ = ind.engine.label(ind.engine.split, 0, 64, probs=False)
        np.save(os.path.join(out, "ckpt_labels.npy"), lab.cpu().numpy())
    dist.barrier()
    params = {k: v.detach().cpu().numpy() for k, v in ind.modelFunc.named_params().items()}
    np.savez(os.path.join(out, f"ckpt_replica_{rk}.npz"), **params)


def run_nccl1(out):
    """One rank over RCCL (the "nccl" backend; one GPU forms a 1-rank communicator): the
    data-parallel exchange as bench.py runs it at N > 1 -- an in-place all_gather_into_tensor
    of the records between the forward and the update, captured into the step graphs -- must
    leave parameters and costs bitwise equal to the same run with no exchange; the same with a
    forced capture failure (bench.warm_up's eager fallback); and an all_to_all_single (the
    partitioned update's row pull) captured into a graph and replayed delivers its blocks."""
    import bench
    from rae import dist as rdist
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    dev = torch.device("cuda", 0)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1

    class NoCapture(rdist.Exchange):
        """An exchange the runtime 'cannot capture' (raises inside a graph capture)."""
        def __call__(self, buf):
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("collective not capturable (test)")
            super().__call__(buf)

    res = {}
    W_, K_ = 6, 20
    for name, exch in (("plain", None), ("rccl", rdist.Exchange(1, 0)),
                       ("fallback", NoCapture(1, 0))):
        data, gold = synthetic_dataset(6000, 3000, 16, seed=7)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 100, 200, 100, 20,
                                 0.0, 0.0, "adagrad", "nccl1", "sp", False, True, False, 1.0,
                                 device=dev, exchange=exch, graph_chunk=8)
        ind.compile_function()
        eng = ind.engine
        eng.sample_epoch_negatives(ind.negativeSampler, "device")
        rdist.warm_up(exch, eng.exchange_buf)
        eng.build_index(0, W_ + K_)
        graphed = bench.warm_up(eng, W_, K_, True, True)
        eng.run(W_, K_, index=False, last_advance=False)
        torch.cuda.synchronize()
        eng.check()
        res[name] = ({k: v.detach().cpu().numpy() for k, v in ind.modelFunc.named_params().items()},
                     eng.costs[:W_ + K_].cpu().numpy(), graphed)
        ind._drop_engine()
    assert res["plain"][2] and res["rccl"][2] and not res["fallback"][2], \
        [v[2] for v in res.values()]
    for name in ("rccl", "fallback"):
        assert np.array_equal(res[name][1], res["plain"][1]), name
        for k, v in res["plain"][0].items():
            assert np.array_equal(res[name][0][k], v), (name, k)
    # the rows all-to-all, captured and replayed
    ex = rdist.Exchange(1, 0)
    send = torch.arange(4096, dtype=torch.float32, device=dev)
    recv = torch.zeros_like(send)
    ex.rows(send, recv)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.graph(g, stream=st):
        send.add_(1.0)
        ex.rows(send, recv)
    torch.cuda.current_stream(dev).wait_stream(st)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(recv, torch.arange(4096, dtype=torch.float32, device=dev) + 3.0)
    with open(os.path.join(out, "nccl1.ok"), "w") as fh:
        fh.write(f"rccl {torch.cuda.nccl.version()}\n")


def main():
    mode, out = sys.argv[1], sys.argv[2]
    dec = sys.argv[3] if len(sys.argv) > 3 else "sp"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if mode == "nccl1":                  # one rank over RCCL on the box's one GPU
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    try:
        if mode == "exchange":
            run_exchange(out)
        elif mode == "oracle":
            run_oracle(out, dec, lambda1=float(sys.argv[4]) if len(sys.argv) > 4 else 0.0)
        elif mode == "oracle_part":
            run_oracle_part(out, dec)
        elif mode == "rows":
            run_sync_rows(out)
        elif mode == "gpu":
            run_gpu(out, dec, sys.argv[4] if len(sys.argv) > 4 else "replicated",
                    sys.argv[5] if len(sys.argv) > 5 else "auto",
                    sys.argv[6] if len(sys.argv) > 6 else "auto",
                    int(sys.argv[7]) if len(sys.argv) > 7 else 0,
                    sys.argv[8] if len(sys.argv) > 8 else "collective",
                    int(sys.argv[9]) if len(sys.argv) > 9 else 1,
                    sys.argv[10] if len(sys.argv) > 10 else "small")
        elif mode == "gpu_c3":
            run_gpu_c3(out, dp_update=dec if dec != "sp" else "replicated",
                       heavy_chunk=sys.argv[4] if len(sys.argv) > 4 else "auto")
        elif mode == "gpu_c4dp":
            run_gpu_c4dp(out, dp_update=dec if dec != "sp" else "replicated")
        elif mode == "gpu_ckpt":
            run_gpu_ckpt(out, dec)
        elif mode == "gpu_delay":
            run_gpu_delay(out, dec, float(sys.argv[4]))
        elif mode == "nccl1":
            run_nccl1(out)
        else:
            raise SystemExit(f"unknown mode {mode}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
