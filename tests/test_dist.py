"""Data-parallel path with world_size 2, 4 and 8, one process per rank, launched the
way bench.py is launched for N > 1 (torch.distributed.run, 127.0.0.1).

CPU (gloo): the exchange all-gather, and the row/negative-column partition + global loss
normaliser on the float64 oracle == the single-process oracle at the global batch.
GPU: the HIP path itself with two / four / eight ranks on one GPU (gloo, host-staged exchange) == the
oracle at the global batch, and all replicas bit-identical.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import rae_oracle as O
from _dist_worker import C4DP_SHAPE, DP_SHAPE, _dataset, c4dp_dataset

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "_dist_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(args, timeout=300, nproc=2):
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), WORKER,
           *args]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]


def _single_process_oracle(decoder, lambda1=0.0, ws=2):
    data, _ = _dataset()
    sp_ = data.split["train"]
    L = ws * DP_SHAPE["l"]
    tr = O.OracleTrainer(decoder, sp_.xFeats, sp_.args1, sp_.args2, data.negSamplingCum,
                         np.random.RandomState(2), DP_SHAPE["m"], DP_SHAPE["r"], DP_SHAPE["s"], L,
                         lr=0.1, alpha=1.0, lambda1=lambda1)
    costs = np.concatenate([tr.epoch()[0] for _ in range(DP_SHAPE["epochs"])])
    return tr, costs


def test_exchange_all_gather_gloo(tmp_path):
    _launch(["exchange", str(tmp_path)])
    want = np.concatenate([np.arange(5, dtype=np.float32) + 100 * (k + 1) for k in range(2)])
    for k in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"exchange_{k}.npy"), want)


@pytest.mark.parametrize("decoder,lambda1,ws", [("sp", 0.0, 2), ("rescal", 0.0, 2),
                                                ("rescal+sp", 0.0, 2), ("sp", 0.01, 2),
                                                ("sp", 0.0, 4), ("rescal+sp", 0.01, 4),
                                                ("sp", 0.0, 8)])
def test_partition_equals_global_batch(tmp_path, decoder, lambda1, ws):
    _launch(["oracle", str(tmp_path), decoder, str(lambda1)], nproc=ws)
    tr, costs = _single_process_oracle(decoder, lambda1, ws)
    rs = [np.load(tmp_path / f"oracle_{decoder}_{k}.npz") for k in range(ws)]
    np.testing.assert_allclose(rs[0]["costs"], costs, rtol=1e-10, atol=1e-12)
    for k, v in tr.params.items():
        for rk in rs[1:]:
            np.testing.assert_array_equal(rs[0][k], rk[k])    # replicas identical
        np.testing.assert_allclose(rs[0][k], v, rtol=1e-9, atol=1e-11, err_msg=k)


@pytest.mark.parametrize("ws", [2, 4])
def test_row_exchange_and_sync_gloo(tmp_path, ws):
    """Exchange.rows delivers block k of rank j's send buffer to block j of rank k's receive
    buffer; Exchange.sync_rows gives every rank row x from rank x % G."""
    _launch(["rows", str(tmp_path)], nproc=ws)
    t2 = np.arange(11, dtype=np.float32)[:, None] * 10 + (np.arange(11) % ws)[:, None]
    t2 = np.repeat(t2, 3, axis=1)
    t1 = np.arange(7, dtype=np.float32) + 0.5
    for k in range(ws):
        z = np.load(tmp_path / f"rows_{k}.npz")
        want = np.concatenate([np.arange(3 * k, 3 * k + 3, dtype=np.float32) + 1000 * j
                               for j in range(ws)])
        np.testing.assert_array_equal(z["recv"], want)
        np.testing.assert_array_equal(z["t2"], t2)
        np.testing.assert_array_equal(z["t1"], t1)


@pytest.mark.parametrize("decoder,ws", [("sp", 2), ("rescal", 2), ("rescal+sp", 2), ("sp", 4),
                                        ("rescal+sp", 4), ("sp", 8)])
def test_partitioned_update_equals_global_batch(tmp_path, decoder, ws):
    """The row-owner partitioned update's protocol (owners update their rows, readers pull
    exactly the rows their examples read before each forward) on the float64 oracle == the
    single-process oracle at the global batch; replicas identical after the final gather."""
    _launch(["oracle_part", str(tmp_path), decoder], nproc=ws)
    tr, costs = _single_process_oracle(decoder, ws=ws)
    rs = [np.load(tmp_path / f"oraclepart_{decoder}_{k}.npz") for k in range(ws)]
    np.testing.assert_allclose(rs[0]["costs"], costs, rtol=1e-10, atol=1e-12)
    for k, v in tr.params.items():
        for rk in rs[1:]:
            np.testing.assert_array_equal(rs[0][k], rk[k])
        np.testing.assert_allclose(rs[0][k], v, rtol=1e-9, atol=1e-11, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("decoder,ws,dense", [("sp", 2, "auto"), ("rescal", 2, "auto"),
                                              ("rescal+sp", 2, "auto"), ("sp", 4, "auto"),
                                              ("sp", 8, "auto"), ("rescal+sp", 8, "auto"),
                                              ("sp", 2, "partials"), ("sp", 4, "partials"),
                                              ("sp", 8, "partials")])
def test_gpu_ranks_match_global_batch(built_lib, cuda_dev, tmp_path, decoder, ws, dense):
    """The HIP path on `ws` ranks sharing the GPU (replicated update) == the oracle at the
    global batch, replicas bit-identical; SP both ways of moving the dense decoder-matrix
    gradients (rae.h RAE_DPDENSE_*: each rank's partials, or -- auto at this shape -- every
    example's dw1 / dw2 in the records)."""
    _launch(["gpu", str(tmp_path), decoder, "replicated", dense], nproc=ws)
    tr, costs = _single_process_oracle(decoder, ws=ws)
    gs = [np.load(tmp_path / f"gpu_replicated_{decoder}_{k}.npz") for k in range(ws)]
    np.testing.assert_allclose(gs[0]["costs"], costs, rtol=2e-5, atol=2e-5)
    for k, v in tr.params.items():
        for gk in gs[1:]:
            np.testing.assert_array_equal(gs[0][k], gk[k])    # bit-identical replicas
        err = np.abs(gs[0][k] - v)
        assert np.all(err <= 2e-4 + 2e-3 * np.abs(v)), f"{k}: max err {err.max():.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("decoder,ws,dense,priv,iw", [("sp", 2, "auto", "auto", 0),
                                                      ("rescal+sp", 2, "auto", "auto", 0),
                                                      ("sp", 4, "auto", "auto", 0),
                                                      ("rescal", 4, "auto", "auto", 0),
                                                      ("sp", 8, "auto", "auto", 0),
                                                      ("sp", 4, "partials", "auto", 0),
                                                      ("sp", 8, "partials", "auto", 0),
                                                      ("sp", 4, "auto", "on", 0),
                                                      ("rescal", 2, "auto", "on", 0),
                                                      ("sp", 2, "auto", "auto", 4)])
def test_gpu_partitioned_update(built_lib, cuda_dev, tmp_path, decoder, ws, dense, priv, iw):
    """The HIP path with the row-owner partitioned update (k_build_dplists, k_dp_move, the
    owned-rows row index) on `ws` ranks sharing the GPU: == the oracle at the global batch,
    and bit-identical to the replicated update's parameters and costs (priv "on": the
    partitioned update's own private rows per example, compact form, against the replicated
    update's; iw = 4: a ring of four batches, so every epoch runs many windows with the next
    window's index and row lists built beside the steps and the row-list capacities agreed per
    window)."""
    _launch(["gpu", str(tmp_path), decoder, "partitioned", dense, priv, str(iw)], nproc=ws)
    _launch(["gpu", str(tmp_path), decoder, "replicated", dense, priv, str(iw)], nproc=ws)
    tr, costs = _single_process_oracle(decoder, ws=ws)
    gp = [np.load(tmp_path / f"gpu_partitioned_{decoder}_{k}.npz") for k in range(ws)]
    gr = np.load(tmp_path / f"gpu_replicated_{decoder}_0.npz")
    np.testing.assert_array_equal(gp[0]["costs"], gr["costs"])
    np.testing.assert_allclose(gp[0]["costs"], costs, rtol=2e-5, atol=2e-5)
    for k, v in tr.params.items():
        for g in gp[1:]:
            np.testing.assert_array_equal(gp[0][k], g[k])
        np.testing.assert_array_equal(gp[0][k], gr[k])
        err = np.abs(gp[0][k] - v)
        assert np.all(err <= 2e-4 + 2e-3 * np.abs(v)), f"{k}: max err {err.max():.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("xchg", ["collective", "p2p", "p2p_pipe"])
def test_gpu_partitioned_large_vocabulary(built_lib, cuda_dev, tmp_path, xchg):
    """vocabularies whose owned rows exceed the row lists' LDS bitmap take
    k_build_dplists' hash passes (sized from the owned candidates, restarted with more passes
    when one overflows); the partitioned update on two ranks (both exchanges) is bitwise equal
    to the replicated one on the same relabelled data -- a missing or stale row in a list would
    change the trajectory."""
    from _dist_worker import BIG_E, BIG_F
    data, _ = _dataset()
    n, d = data.get_arg_voc_size() * BIG_E, data.get_dimensionality() * BIG_F
    assert min(n, d) // 2 > 32 * 16384          # rae_dp.hpp: nq > 32 * RAE_DPL_KEYS, G = 2
    _launch(["gpu", str(tmp_path), "sp", "partitioned", "auto", "auto", "0", xchg, "1", "big"])
    _launch(["gpu", str(tmp_path), "sp", "replicated", "auto", "auto", "0", "collective", "1",
             "big"])
    tag = "partitioned" if xchg == "collective" else f"partitioned_{xchg}"
    gp = [np.load(tmp_path / f"gpu_{tag}_big_sp_{k}.npz") for k in range(2)]
    gr = np.load(tmp_path / "gpu_replicated_big_sp_0.npz")
    for k in gr.files:
        np.testing.assert_array_equal(gp[0][k], gp[1][k], err_msg=k)
        np.testing.assert_array_equal(gp[0][k], gr[k], err_msg=k)


@pytest.mark.gpu
def test_partitioned_gather_then_rank0_checkpoint(built_lib, cuda_dev, tmp_path):
    """under the partitioned update a checkpoint from rank 0 alone must not start a
    collective.  Every rank calls ReconstructInducer.gather(); rank 0 then saves and labels by
    itself; the checkpoint equals every rank's replica and the replicated run's parameters."""
    _launch(["gpu_ckpt", str(tmp_path), "sp"], nproc=2, timeout=240)
    _launch(["gpu", str(tmp_path), "sp", "replicated"], nproc=2)
    ck = np.load(tmp_path / "ckpt_part.npz")
    gr = np.load(tmp_path / "gpu_replicated_sp_0.npz")
    for rk in range(2):
        rep = np.load(tmp_path / f"ckpt_replica_{rk}.npz")
        for k in rep.files:
            np.testing.assert_array_equal(ck["param/" + k], rep[k])
            np.testing.assert_array_equal(ck["param/" + k].astype(np.float64), gr[k])
    assert np.load(tmp_path / "ckpt_labels.npy").shape == (64,)


@pytest.mark.gpu
def test_rccl_one_rank_captured_exchange(built_lib, cuda_dev, tmp_path):
    """the RCCL ("nccl") branch of rae/dist.py on hardware -- one torchrun
    rank (a 1-GPU box forms a 1-rank communicator): the in-place all-gather captured inside the
    step graphs leaves the trained parameters and costs bitwise equal to the run without an
    exchange; bench.warm_up's eager fallback (capture refused) too; a captured all_to_all_single
    replays correctly."""
    _launch(["nccl1", str(tmp_path)], nproc=1, timeout=300)
    assert (tmp_path / "nccl1.ok").exists()


_C4DP = {}


def _c4dp_reference(cuda_dev, ws):
    """(float64 oracle costs + params, single-rank HIP run) at the global batch ws * l of the
    C4-shape data-parallel test, cached per ws.  The single-rank plan runs the same split SP
    forward with full records (V1 / V2 / G1 written by the forward itself)."""
    if ws in _C4DP:
        return _C4DP[ws]
    import torch
    from rae.inducer import ReconstructInducer
    c = C4DP_SHAPE
    L = ws * c["l"]
    data, gold = c4dp_dataset()
    sp_ = data.split["train"]
    tr = O.OracleTrainer("sp", sp_.xFeats, sp_.args1, sp_.args2, data.negSamplingCum,
                         np.random.RandomState(2), c["m"], c["r"], c["s"], L, lr=0.1, alpha=1.0)
    N = sp_.xFeats.shape[0]
    n1 = O.negative_samples(tr.rng, data.negSamplingCum, N, c["s"])
    n2 = O.negative_samples(tr.rng, data.negSamplingCum, N, c["s"])
    costs = np.array([tr.train_batch(b, n1[:, b * L:(b + 1) * L], n2[:, b * L:(b + 1) * L])
                      for b in range(c["steps"])])
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, L, c["r"], c["m"],
                             c["s"], 0.0, 0.0, "adagrad", "c4dp1", "sp", False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=1)
    ind.compile_function()
    eng = ind.engine
    assert eng.kernel_forms_in_use()["sp_forward"] == "split"
    assert eng.kernel_forms_in_use()["priv_rows"] == "off"
    eng.sample_epoch_negatives(ind.negativeSampler, "device")
    snap = {}
    for b in range(c["steps"]):
        eng.run(b, 1)
        torch.cuda.synchronize()
        eng.check()
        for k, v in ind.modelFunc.named_params().items():
            snap[f"{k}@{b}"] = v.detach().cpu().numpy()
    single = (snap, eng.costs[:c["steps"]].cpu().numpy())
    ind._drop_engine()
    _C4DP[ws] = (costs, tr.params, single)
    return _C4DP[ws]


@pytest.mark.gpu
@pytest.mark.parametrize("ws", [2, 4, 8])
def test_gpu_c4_shape_data_parallel(built_lib, cuda_dev, tmp_path, ws):
    """BASELINE config 4's data-parallel kernel combination --
    K = 300, embed 300, neg 50, l = 100 per rank, up to the 8 ranks of the config (global batch
    800, L = 800 update with 102 record slots): the split SP forward, the wire records (dw1 / dw2 per
    example), k_vrec and 102 record slots with private rows off -- on `ws` ranks sharing the GPU
    (gloo), both update forms, the partitioned one also over the peer-to-peer exchange (the
    worker asserts the resolved forms).  Checked:
      * replicas bit-identical, partitioned == replicated bitwise;
      * == the float64 oracle at the global batch (fp32 tolerance);
      * == a single-rank plan at the global batch, whose split forward writes V1 / V2 / G1 into
        the records itself, BITWISE: k_vrec rebuilds exactly the split forward's vectors
        (k_vrec) and the update sums them in the same order."""
    _launch(["gpu_c4dp", str(tmp_path), "replicated"], nproc=ws, timeout=600)
    _launch(["gpu_c4dp", str(tmp_path), "partitioned"], nproc=ws, timeout=600)
    _launch(["gpu_c4dp", str(tmp_path), "p2p"], nproc=ws, timeout=600)
    _launch(["gpu_c4dp", str(tmp_path), "p2p_pipe"], nproc=ws, timeout=600)
    want_c, want_p, (single_p, single_c) = _c4dp_reference(cuda_dev, ws)
    gr = [np.load(tmp_path / f"c4dp_replicated_{k}.npz") for k in range(ws)]
    gp = [np.load(tmp_path / f"c4dp_partitioned_{k}.npz") for k in range(ws)] + \
        [np.load(tmp_path / f"c4dp_p2p_{k}.npz") for k in range(ws)] + \
        [np.load(tmp_path / f"c4dp_p2p_pipe_{k}.npz") for k in range(ws)]
    last = C4DP_SHAPE["steps"] - 1
    for g in gr[1:] + gp:
        np.testing.assert_array_equal(g["costs"], gr[0]["costs"])
        for k in gr[0].files:
            np.testing.assert_array_equal(g[k], gr[0][k], err_msg=k)
    np.testing.assert_allclose(gr[0]["costs"], want_c, rtol=2e-5, atol=2e-5)
    for k, v in want_p.items():
        err = np.abs(gr[0][f"{k}@{last}"].astype(np.float64) - v)
        assert np.all(err <= 2e-4 + 2e-3 * np.abs(v)), f"{k}: max err {err.max():.3e}"
    np.testing.assert_array_equal(gr[0]["costs"], single_c)
    diff = {k: int(np.sum(gr[0][k] != single_p[k])) for k in sorted(single_p)}
    assert not any(diff.values()), f"data-parallel vs single-rank elements differing: {diff}"


@pytest.mark.gpu
@pytest.mark.parametrize("xchg", ["p2p", "p2p_pipe"])
def test_gpu_p2p_delayed_rank(built_lib, cuda_dev, tmp_path, xchg):
    """one rank sleeps 1 s of host time before every single-batch run while the
    peer-to-peer waits are bounded at 0.3 s (rae_set_p2p_timeout).  run() meets the peers at a
    host barrier before any wait kernel starts, so no wait times out (error bit 64 would raise in
    eng.check()), and the costs and parameters equal the undelayed run's bitwise."""
    _launch(["gpu_delay", str(tmp_path), xchg, "1.0"], nproc=2, timeout=300)
    _launch(["gpu_delay", str(tmp_path), xchg, "0"], nproc=2, timeout=300)
    for k in range(2):
        a = np.load(tmp_path / f"delay_{xchg}_1.0_{k}.npz")
        b = np.load(tmp_path / f"delay_{xchg}_0.0_{k}.npz")
        for key in a.files:
            np.testing.assert_array_equal(a[key], b[key], err_msg=key)


@pytest.mark.gpu
@pytest.mark.parametrize("decoder,ws,graph_chunk,iw,xchg", [
    ("sp", 2, 1, 0, "p2p"), ("sp", 4, 4, 0, "p2p"), ("rescal", 2, 1, 0, "p2p"),
    ("rescal+sp", 4, 1, 0, "p2p"), ("sp", 8, 4, 0, "p2p"), ("sp", 2, 2, 4, "p2p"),
    ("sp", 2, 1, 0, "p2p_pipe"), ("sp", 4, 4, 0, "p2p_pipe"), ("rescal", 2, 1, 0, "p2p_pipe"),
    ("rescal+sp", 4, 1, 0, "p2p_pipe"), ("sp", 8, 4, 0, "p2p_pipe"), ("sp", 2, 2, 4, "p2p_pipe"),
    ("sp", 2, 4, 6, "p2p_pipe")])
def test_gpu_p2p_exchange(built_lib, cuda_dev, tmp_path, decoder, ws, graph_chunk, iw, xchg):
    """the partitioned update over the peer-to-peer exchange (include/rae.h
    RAE_XCHG_P2P, csrc/rae_p2p.hpp) -- owners store the rows each peer's next batch reads into
    the peer's IPC-mapped replica, every forward stores its records into every peer's exchange
    buffer, and the kernels wait on the peers' system-scope signal counters -- on `ws` ranks
    sharing the GPU, eager (graph_chunk 1) and graph-replayed (no collective inside a step, so
    the steps capture under gloo too), iw = 4: a ring of four batches (many windows, the row-list
    capacities agreed per window).  == the collective replicated update bitwise (costs and
    parameters), replicas bit-identical after the final gather, == the float64 oracle.
    p2p_pipe (RAE_XCHG_P2P_PIPE): the next batch's rows leave during the step -- those the
    update leaves unchanged right after the forward, the updated ones from the row tasks --
    with the lookahead of one batch past every window (ring of 4 / 6: windows of one and two
    batches, the next window's index built beside the steps) and a prologue per epoch."""
    _launch(["gpu", str(tmp_path), decoder, "partitioned", "auto", "auto", str(iw), xchg,
             str(graph_chunk)], nproc=ws, timeout=420)
    _launch(["gpu", str(tmp_path), decoder, "replicated", "auto", "auto", str(iw)], nproc=ws)
    tr, costs = _single_process_oracle(decoder, ws=ws)
    gp = [np.load(tmp_path / f"gpu_partitioned_{xchg}_{decoder}_{k}.npz") for k in range(ws)]
    gr = np.load(tmp_path / f"gpu_replicated_{decoder}_0.npz")
    np.testing.assert_array_equal(gp[0]["costs"], gr["costs"])
    np.testing.assert_allclose(gp[0]["costs"], costs, rtol=2e-5, atol=2e-5)
    for k, v in tr.params.items():
        for g in gp[1:]:
            np.testing.assert_array_equal(gp[0][k], g[k])
        np.testing.assert_array_equal(gp[0][k], gr[k])
        err = np.abs(gp[0][k] - v)
        assert np.all(err <= 2e-4 + 2e-3 * np.abs(v)), f"{k}: max err {err.max():.3e}"
