"""HIP training path vs the oracle / the reference's golden vectors (needs an MI355X).

Tolerances (fp32 device arithmetic vs the float64 reference, Theano's default floatX):
  per-batch cost        |dc| <= 2e-5 * max(1, |c|)
  parameters            |dp| <= 2e-4 + 2e-3*|p|   after whole training runs
  labels                identical wherever the reference's top-2 score margin > 1e-5
"""
import glob
import os

import numpy as np
import pytest
import scipy.sparse as sp

import rae_oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

COST_RTOL = 2e-5


def _case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    X = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(int(z["N"]), int(z["d"])))
    return z, X


def _inducer(z, X, dev, **kw):
    from rae.data import DatasetManager, DatasetSplit
    from rae.inducer import ReconstructInducer
    data = DatasetManager({"train": DatasetSplit(z["args1"], z["args2"], X)}, z["freqs"],
                          int(z["d"]))
    assert np.array_equal(data.negSamplingCum, z["cum"])
    rng = np.random.RandomState(int(z["seed"]))
    ind = ReconstructInducer(data, {"train": {}}, rng, int(z["epochs"]), float(z["lr"]),
                             int(z["l"]), int(z["r"]), int(z["m"]), int(z["s"]), float(z["l1"]),
                             float(z["l2"]), str(z["optimizer"]), "golden", str(z["decoder"]),
                             False, bool(int(z["ext_reg"])), False, float(z["alpha"]),
                             device=dev, **kw)
    return ind


def _params(ind):
    return {k: v.detach().cpu().double().numpy() for k, v in ind.modelFunc.named_params().items()}


def _assert_params_close(got, want, what):
    for k in want:
        err = np.abs(got[k] - want[k])
        tol = 2e-4 + 2e-3 * np.abs(want[k])
        assert np.all(err <= tol), f"{what} {k}: max err {err.max():.3e}"


SP_CASES = ["sp_basic", "sp_reg", "sp_sgd_noext"]
BIL_CASES = ["rescal_basic", "rescal_reg", "hybrid_basic", "hybrid_testpy"]
ALL_CASES = SP_CASES + BIL_CASES


@pytest.mark.parametrize("name", ALL_CASES)
@pytest.mark.parametrize("graph", [True, False])
def test_epoch_path_matches_reference_golden(built_lib, cuda_dev, name, graph):
    z, X = _case(name)
    ind = _inducer(z, X, cuda_dev, graph_chunk=2 if graph else 1)
    for k, v in _params(ind).items():                     # init on the shared RNG
        assert np.array_equal(v, z["init_" + k].astype(np.float32).astype(np.float64)), k
    errs = ind.learn(verbose=False)
    np.testing.assert_allclose(errs, z["errs"], rtol=COST_RTOL * 3, atol=0)
    _assert_params_close(_params(ind), {k: z["final_" + k] for k in _params(ind)}, name)
    lab = ind.func["label_train"].all_labels(ind.batch_reps["train"])
    _assert_labels(lab, z, X)


def _assert_labels(lab, z, X):
    nrow = lab.shape[0]
    S = np.asarray(X[:nrow] @ z["final_W"]) + z["final_Wb"]
    srt = np.sort(S, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-5
    assert np.array_equal(lab[clear], z["labels"][:nrow][clear])


@pytest.mark.parametrize("name", ALL_CASES)
def test_func_train_per_call_matches_reference_golden(built_lib, cuda_dev, name):
    """The reference's own call pattern: err += func['train'](b, neg1[:, cols], neg2[:, cols])."""
    z, X = _case(name)
    ind = _inducer(z, X, cuda_dev)
    ind.compile_function()
    l, nb = int(z["l"]), int(z["N"]) // int(z["l"])
    for ep in range(int(z["epochs"])):
        n1, n2 = z[f"neg1_e{ep}"], z[f"neg2_e{ep}"]
        for b in range(nb):
            c = ind.func["train"](b, n1[:, b * l:(b + 1) * l], n2[:, b * l:(b + 1) * l])
            want = z["costs"][ep, b]
            assert abs(c - want) <= COST_RTOL * max(1.0, abs(want)), (ep, b, c, want)
    _assert_params_close(_params(ind), {k: z["final_" + k] for k in _params(ind)}, name)
    labels, probs = ind.func["label_train"](0)
    np.testing.assert_allclose(probs, z["probs"][:l], rtol=0, atol=2e-5)


def _oracle_trajectory(decoder, data, seed, m, r, s, l, epochs, **hp):
    tr = O.OracleTrainer(decoder, data.split["train"].xFeats, data.split["train"].args1,
                         data.split["train"].args2, data.negSamplingCum,
                         np.random.RandomState(seed), m, r, s, l, **hp)
    costs = [tr.epoch()[0] for _ in range(epochs)]
    return tr, np.array(costs)


@pytest.mark.parametrize("shape", [
    dict(N=400, d=300, m=8, r=16, s=4, l=50, ntrue=4),
    dict(N=300, d=2000, m=100, r=200, s=20, l=100, ntrue=10),   # headline K/r/s/l
    dict(N=240, d=500, m=30, r=100, s=10, l=60, ntrue=6),       # config 2 K/r/s
    dict(N=210, d=700, m=7, r=13, s=3, l=70, ntrue=5),          # non-multiple-of-4 (scalar path)
    # the fused general path's other branches: s > 32 and r / 4 > 64 (the barrier-based
    # coefficient / weighted-row blocks), m > 128 (S formed by all threads)
    dict(N=300, d=400, m=8, r=16, s=36, l=40, ntrue=4),
    dict(N=300, d=400, m=8, r=300, s=4, l=40, ntrue=4),
    dict(N=300, d=800, m=200, r=16, s=4, l=40, ntrue=6),
    dict(N=400, d=300, m=8, r=16, s=4, l=50, ntrue=4, dec="rescal"),
    dict(N=210, d=700, m=7, r=13, s=3, l=70, ntrue=5, dec="rescal"),
    dict(N=200, d=2000, m=100, r=200, s=20, l=100, ntrue=10, dec="rescal", epochs=1),  # C5 shape
    dict(N=400, d=300, m=8, r=16, s=4, l=50, ntrue=4, dec="rescal+sp"),
    dict(N=210, d=700, m=7, r=13, s=3, l=70, ntrue=5, dec="rescal+sp"),
    dict(N=200, d=1000, m=30, r=60, s=10, l=100, ntrue=6, dec="rescal+sp"),
])
def test_synthetic_vs_oracle(built_lib, cuda_dev, shape):
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    data, gold = synthetic_dataset(shape["N"], shape["d"], shape["ntrue"], seed=99)
    m, r, s, l = shape["m"], shape["r"], shape["s"], shape["l"]
    dec = shape.get("dec", "sp")
    ep = shape.get("epochs", 2)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), ep, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "syn", dec, False, True, False, 1.0, device=cuda_dev,
                             graph_chunk=2)
    errs = ind.learn(verbose=False)
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, ep, lr=0.1, alpha=1.0)
    got = np.array(ind.epoch_costs)
    np.testing.assert_allclose(got, costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "synthetic")


@pytest.mark.parametrize("shape", [
    dict(N=400, d=300, m=8, r=16, s=4, l=50, ntrue=4, force=True),
    dict(N=210, d=700, m=7, r=13, s=3, l=70, ntrue=5, force=True),      # scalar path
    dict(N=300, d=2000, m=100, r=200, s=20, l=100, ntrue=10, force=True),
    dict(N=200, d=3000, m=300, r=300, s=50, l=100, ntrue=10, epochs=1),  # C4 K/r/s: split by default
    # r > 16 ceil(m / 16): k_sp_ctdw's tiles store dw / G1 over several column strides; l not a
    # multiple of 16, odd s
    dict(N=300, d=500, m=8, r=44, s=5, l=37, ntrue=4, force=True),
], ids=["small", "odd", "c3shape", "c4shape", "wide"])
def test_split_sp_forward_vs_oracle(built_lib, cuda_dev, shape):
    """The split SP forward (rae_sp_split.hpp: encoder, P.C^T GEMM, decoder per negative side,
    dw.C GEMM with the softmax backward in its epilogue) against the float64 oracle, with the
    same tolerances as the fused example kernel."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    forms = {"sp_forward": "split"} if shape.get("force") else {}
    data, gold = synthetic_dataset(shape["N"], shape["d"], shape["ntrue"], seed=99)
    m, r, s, l = shape["m"], shape["r"], shape["s"], shape["l"]
    ep = shape.get("epochs", 2)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), ep, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "split", "sp", False, True, False, 1.0, device=cuda_dev,
                             graph_chunk=2, kernel_forms=forms)
    ind.learn(verbose=False)
    tr, costs = _oracle_trajectory("sp", data, 2, m, r, s, l, ep, lr=0.1, alpha=1.0)
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "split")


@pytest.mark.parametrize("dec", ["sp", "rescal"])
def test_index_overlap_matches_serial(built_lib, cuda_dev, dec):
    """engine.run builds the next window's row index on a lowest-priority side stream while the
    current window's steps run (index_overlap; windows of half the ring).  A ring of 8 batches
    over two epochs (many windows, every side build behind the step stream's queue), serial
    windows of 8, and one window per epoch train bit-identically; so does a run cut into
    per-batch runs (frequentEval mode 2's pattern: every window already built by the last
    run's prefetch)."""
    import torch
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    out = []
    for iw, ov in ((8, True), (8, False), (0, True)):
        data, gold = synthetic_dataset(1500, 3000, 10, seed=31)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 2, 0.1, 50, 24, 12, 5,
                                 0.0, 0.0, "adagrad", "ovl", dec, False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=2, index_window=iw,
                                 index_overlap=ov)
        ind.learn(verbose=False)
        eng = ind.engine
        assert eng.index_overlap == ov
        if iw:
            assert eng.index_window == 8
            assert len(eng.windows(0, eng.nb)) >= (6 if ov else 3)
        out.append((_params(ind), np.array(ind.epoch_costs)))
    # per-batch runs (eager, as frequentEval mode 2 runs them) on a fresh model
    data, gold = synthetic_dataset(1500, 3000, 10, seed=31)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 50, 24, 12, 5,
                             0.0, 0.0, "adagrad", "ovl1", dec, False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=2, index_window=8)
    ind.compile_function()
    eng = ind.engine
    n1, n2 = ind.draw_epoch_negatives()
    eng.set_epoch_negatives(n1, n2)
    for b in range(eng.nb):
        eng.run(b, 1, graph=False)
    torch.cuda.synchronize()
    eng.check()
    ref = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 50, 24, 12, 5,
                             0.0, 0.0, "adagrad", "ovl2", dec, False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=2, index_overlap=False)
    ref.compile_function()
    n1r, n2r = ref.draw_epoch_negatives()
    assert np.array_equal(n1, n1r)
    ref.engine.set_epoch_negatives(n1r, n2r)
    ref.engine.run(0, ref.engine.nb)
    torch.cuda.synchronize()
    for k, v in _params(ref).items():
        assert np.array_equal(_params(ind)[k], v), f"per-batch runs: {k}"
    for k in out[0][0]:
        for o in out[1:]:
            assert np.array_equal(out[0][0][k], o[0][k]), k
    for o in out[1:]:
        assert np.array_equal(out[0][1], o[1])


def test_bitwise_deterministic(built_lib, cuda_dev):
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    out = []
    for _ in range(2):
        data, gold = synthetic_dataset(500, 900, 5, seed=7)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 2, 0.1, 50, 24, 12, 5,
                                 0.0, 0.0, "adagrad", "det", "sp", False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=4)
        ind.learn(verbose=False)
        out.append(_params(ind))
    for k in out[0]:
        assert np.array_equal(out[0][k], out[1][k]), k


def test_label_pass_matches_oracle(built_lib, cuda_dev):
    import torch
    from rae.engine import DeviceSplit
    from rae.data import synthetic_dataset
    data, _ = synthetic_dataset(3000, 4000, 8, seed=5)
    g = np.random.RandomState(0)
    m = 100
    W = g.standard_normal((4000, m)).astype(np.float32)
    Wb = g.standard_normal(m).astype(np.float32)
    split = DeviceSplit(data.split["train"], cuda_dev)
    lab = torch.empty(3000, dtype=torch.int64, device=cuda_dev)
    pr = torch.empty((3000, m), dtype=torch.float32, device=cuda_dev)
    import ctypes as C
    from rae import _lib
    lib = _lib.load()
    Wt, Wbt = torch.as_tensor(W, device=cuda_dev), torch.as_tensor(Wb, device=cuda_dev)
    _lib.check(lib.rae_label(C.c_void_p(split.indptr.data_ptr()), C.c_void_p(split.indices.data_ptr()),
                             None, C.c_void_p(Wt.data_ptr()), C.c_void_p(Wbt.data_ptr()), m, 0, 3000,
                             C.c_void_p(lab.data_ptr()), C.c_void_p(pr.data_ptr()), None))
    torch.cuda.synchronize()
    want_lab, want_p = O.label(data.split["train"].xFeats, W.astype(np.float64), Wb.astype(np.float64))
    S = np.asarray(data.split["train"].xFeats @ W.astype(np.float64)) + Wb
    srt = np.sort(S, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-4
    assert np.array_equal(lab.cpu().numpy()[clear], want_lab[clear])
    np.testing.assert_allclose(pr.cpu().numpy(), want_p, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name", ALL_CASES)
def test_single_step_each_parameter(built_lib, cuda_dev, name):
    """One func['train'] call: every parameter vs the reference's params after step 1."""
    z, X = _case(name)
    ind = _inducer(z, X, cuda_dev)
    ind.compile_function()
    l = int(z["l"])
    c = ind.func["train"](0, z["neg1_e0"][:, :l], z["neg2_e0"][:, :l])
    assert abs(c - float(z["costs"][0, 0])) <= COST_RTOL * max(1.0, abs(float(z["costs"][0, 0])))
    got = _params(ind)
    bad = []
    for k in got:
        err = np.abs(got[k] - z["step1_" + k])
        tol = 1e-5 + 1e-4 * np.abs(z["step1_" + k])
        if not np.all(err <= tol):
            idx = np.unravel_index(np.argmax(err - tol), err.shape)
            bad.append(f"{k}: max err {err.max():.3e} at {idx} got {got[k][idx]:.6g} "
                       f"want {z['step1_' + k][idx]:.6g} init {z['init_' + k][idx]:.6g}")
    assert not bad, "; ".join(bad)


@pytest.mark.parametrize("decoder", ["sp", "rescal+sp"])
def test_cli_end_to_end(built_lib, cuda_dev, decoder):
    """python -m rae (the OieInduction.py command line) trains on the GPU end to end."""
    import subprocess
    import sys
    from conftest import PKG
    env = dict(os.environ)
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    p = subprocess.run([sys.executable, "-m", "rae", "synthetic:1000:2000:5", "--model-name", "t",
                        "--decoder", decoder, "--epochs", "2", "--batch-size", "100",
                        "--relations", "10", "--embed-size", "16", "--neg-samples", "4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    errs = [float(line.split(":")[1]) for line in p.stdout.splitlines()
            if line.startswith("Training error")]
    assert len(errs) == 2 and all(np.isfinite(errs))


def test_checkpoint_resume_is_bit_identical(built_lib, cuda_dev, tmp_path):
    """2 epochs straight == 1 epoch, checkpoint, a fresh inducer loads it, 1 more epoch."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    data, gold = synthetic_dataset(600, 900, 5, seed=8)

    def make(epochs):
        return ReconstructInducer(data, gold, np.random.RandomState(2), epochs, 0.1, 50, 16, 8, 4,
                                  0.0, 0.0, "adagrad", "ck", "sp", False, True, False, 1.0,
                                  device=cuda_dev, graph_chunk=4)
    a = make(2)
    a.learn(verbose=False)
    b = make(1)
    b.learn(verbose=False)
    b.save_checkpoint(tmp_path / "ck.npz")
    c = make(2)
    c.load_checkpoint(tmp_path / "ck.npz")
    c.learn(verbose=False)
    pa, pc = _params(a), _params(c)
    for k in pa:
        assert np.array_equal(pa[k], pc[k]), k
    assert a.train_errors == c.train_errors


@pytest.mark.parametrize("shape", [(100, 200, 20, 100), (60, 96, 5, 40), (20, 50, 3, 30),
                                   (30, 64, 10, 64)], ids=["c5", "padded", "ragged", "mid"])
@pytest.mark.parametrize("dec", ["rescal", "rescal+sp"])
def test_bf16_mfma_path_tracks_oracle(built_lib, cuda_dev, dec, shape):
    """BASELINE config 5's bf16-operand MFMA path (fp32 accumulation) over a whole epoch at
    four shapes, against the float64 oracle with the derived tolerance of
    test_gpu_fullscale.check_bf16: as close to float64 as bf16 operand rounding itself
    allows (the oracle with the same rounding emulated), and far closer to that emulation
    than to float64."""
    from test_gpu_fullscale import bf16_trajectories, check_bf16
    m, r, s, l = shape
    out, _ = bf16_trajectories(cuda_dev, dec, N=200 if l >= 64 else 5 * l, d=2000, m=m, r=r, s=s,
                               l=l, ntrue=10, steps=(200 if l >= 64 else 5 * l) // l,
                               seed_data=99)
    check_bf16(out, None, f"{dec} {shape}")


@pytest.mark.parametrize("dec", ["rescal", "rescal+sp"])
def test_bf16_bilinear_bitwise_deterministic(built_lib, cuda_dev, dec):
    """Two runs of the C5 path (bf16 MFMA, M-tile passes with dP, R-update kernel) give
    bit-identical parameters and costs: every partial is combined in a fixed order.  (A
    dynamically indexed MFMA accumulator once made the dP partials vary run to run.)"""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    m, r, s, l = 100, 200, 20, 100
    out = []
    for _ in range(2):
        data, gold = synthetic_dataset(2 * l, 2000, 10, seed=99)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0,
                                 0.0, "adagrad", "det", dec, False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=2, mfma_bf16=True)
        ind.learn(verbose=False)
        out.append((_params(ind), np.array(ind.epoch_costs)))
    assert np.array_equal(out[0][1], out[1][1])
    for k in out[0][0]:
        assert np.array_equal(out[0][0][k], out[1][0][k]), k


def test_cursor_and_absolute_batch_launches_agree(built_lib, cuda_dev):
    # the two ways include/rae.h addresses a step's batch: a device cursor + offset
    # (rae_step_forward / rae_step_update) and the absolute index in the launch
    # (rae_step_*_at; the func['train'] path rae_train_step uses it) -- bit-identical training
    import ctypes as C
    import torch
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    out = []
    for mode in ("cursor", "absolute"):
        data, gold = synthetic_dataset(600, 900, 5, seed=11)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 40, 24, 12, 5,
                                 0.0, 0.0, "adagrad", "abs", "sp", False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=3)
        ind.compile_function()
        eng = ind.engine
        n1, n2 = ind.draw_epoch_negatives()
        eng.set_epoch_negatives(n1, n2)
        nb = eng.nb
        lib, st = eng.lib, C.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert lib.rae_build_index(eng.plan, 0, nb, st) == 0
        if mode == "absolute":
            for b in range(nb):
                assert lib.rae_step_forward_at(eng.plan, b, st) == 0
                assert lib.rae_step_update_at(eng.plan, b, st) == 0
        else:
            assert lib.rae_set_cursor(eng.plan, 0, st) == 0
            for i in range(nb):
                assert lib.rae_step_forward(eng.plan, i, st) == 0
                assert lib.rae_step_update(eng.plan, i, st) == 0
        torch.cuda.synchronize()
        eng.check()
        out.append((_params(ind), eng.costs[:nb].cpu().numpy().copy()))
    for k in out[0][0]:
        assert np.array_equal(out[0][0][k], out[1][0][k]), k
    assert np.array_equal(out[0][1], out[1][1])


def test_consecutive_runs_skip_cursor_reset(built_lib, cuda_dev):
    """engine.run() skips its rae_set_cursor launch when the device cursor already points at the
    requested batch (bench.py's warm-up -> timed region): split runs, an explicit cursor move in
    between and one whole run all train bit-identically."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    out = []
    for mode in ("whole", "split", "moved", "noadv"):
        data, gold = synthetic_dataset(1200, 900, 5, seed=13)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 40, 24, 12, 5,
                                 0.0, 0.0, "adagrad", "cur", "sp", False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=4)
        ind.compile_function()
        eng = ind.engine
        n1, n2 = ind.draw_epoch_negatives()
        eng.set_epoch_negatives(n1, n2)
        nb = eng.nb
        if mode == "whole":
            eng.run(0, nb)
        else:
            eng.run(0, 5, last_advance=(mode != "noadv"))   # noadv: the next run resets it
            if mode == "moved":                     # someone else drove the cursor meanwhile
                import ctypes as C
                import torch
                st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
                # a direct ABI move, no cursor_moved(): the plan's move count tells the engine
                assert eng.lib.rae_set_cursor(eng.plan, 17, st) == 0
            eng.run(5, nb - 5)
        import torch
        torch.cuda.synchronize()
        eng.check()
        out.append((_params(ind), eng.costs[:nb].cpu().numpy().copy()))
    for o in out[1:]:
        for k in out[0][0]:
            assert np.array_equal(out[0][0][k], o[0][k]), k
        assert np.array_equal(out[0][1], o[1])


@pytest.mark.parametrize("shape", [(100, 200, 20, 100), (60, 96, 5, 40)], ids=["c5", "padded"])
@pytest.mark.parametrize("dec", ["rescal", "rescal+sp"])
def test_bf16_dp_kernels_agree(built_lib, cuda_dev, dec, shape):
    """The LDS-staged bf16 dP kernel (k_bil_dp2, compiled for the C5 shape and padded for
    others) against the strided bf16 kernel it replaces (bil_dp="strided"): the same bf16 operands,
    only the fp32 summation order differs, so whole runs agree to 5e-4 relative Frobenius
    distance -- far inside the derived bf16-vs-float64 tolerance above.  Two batches only: over longer runs the drift between the
    two orders depends on the trajectory (it grew from 1e-4 to 8e-4 over a five-batch epoch as
    unrelated kernels changed their own rounding)."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    m, r, s, l = shape
    out = []
    for form in ("staged", "strided"):        # dP from k_bil_dp2 / k_bil_dp, not k_bil_mt
        # two batches: longer runs amplify the summation-order difference chaotically
        data, gold = synthetic_dataset(2 * l, 2000, 10, seed=99)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0,
                                 0.0, "adagrad", "dp2", dec, False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=2, mfma_bf16=True,
                                 kernel_forms={"bil_dp": form})
        ind.learn(verbose=False)
        out.append((_params(ind), np.array(ind.epoch_costs)))
    # the per-batch costs drift with the parameters (up to 2.6e-5 relative seen)
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=1e-4, atol=2e-6)
    for k in out[0][0]:
        a, b = out[0][0][k], out[1][0][k]
        rel = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)
        assert rel < 5e-4, f"{k}: relative distance {rel:.3e}"


@pytest.mark.parametrize("shape", [(100, 200, 20, 100), (60, 96, 5, 40), (20, 50, 3, 30)],
                         ids=["c5", "padded", "ragged"])
@pytest.mark.parametrize("dec", ["rescal", "rescal+sp"])
def test_bf16_dp_in_mtile_pass_agrees(built_lib, cuda_dev, dec, shape):
    """dP computed inside the second k_bil_mt pass (per 8x16 block of R, partials summed by
    k_bil_fin) against k_bil_dp2 / k_bil_dp (bil_dp="staged"): the same bf16 operands, another fp32
    summation order -> two batches agree to 5e-4 relative (as test_bf16_dp_kernels_agree)."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    m, r, s, l = shape
    out = []
    for form in ("mtile", "staged"):
        data, gold = synthetic_dataset(2 * l, 2000, 10, seed=99)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0,
                                 0.0, "adagrad", "mtdp", dec, False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=2, mfma_bf16=True,
                                 kernel_forms={"bil_dp": form})
        ind.learn(verbose=False)
        out.append((_params(ind), np.array(ind.epoch_costs)))
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=1e-4, atol=2e-6)
    for k in out[0][0]:
        a, b = out[0][0][k], out[1][0][k]
        rel = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)
        assert rel < 5e-4, f"{k}: relative distance {rel:.3e}"


@pytest.mark.parametrize("dec,m,hp", [
    ("sp", 10, dict(l2=0.1, alpha=0.1)),          # README.md:44 (C1: K=10, embed 10, neg 5, l=100)
    ("rescal+sp", 5, dict(l2=0.1, alpha=0.1)),    # test.py:33 (2 epochs, rescal+sp, 5 relations)
])
def test_c1_data_sample_vs_oracle(built_lib, cuda_dev, dec, m, hp):
    """BASELINE config 1: data-sample.txt ingested by rae.preprocess (fixture c1_sample.npz,
    oracle/gen_c1_fixture.py) trained on the GPU, against the float64 oracle on the same
    seed; relation assignments identical where the margin is clear; B^3 on the gold labels."""
    from rae.data import load_npz
    from rae.evaluation import construct_split_evaluator
    from rae.inducer import ReconstructInducer
    data, gold = load_npz(os.path.join(GOLDEN, "c1_sample.npz"))
    r, s, l, ep = 10, 5, 100, 2
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), ep, 0.1, l, r, m, s, 0.0,
                             hp["l2"], "adagrad", "c1", dec, False, True, False, hp["alpha"],
                             device=cuda_dev, graph_chunk=4)
    ind.learn(verbose=False)
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, ep, lr=0.1, alpha=hp["alpha"],
                                   lambda2=hp["l2"])
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "c1")
    lab = ind.func["label_train"].all_labels(ind.batch_reps["train"])
    want, _ = tr.labels()
    X = data.split["train"].xFeats
    S = np.asarray(X @ tr.params["W"]) + tr.params["Wb"]
    srt = np.sort(S, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-5
    assert clear.mean() > 0.9
    assert np.array_equal(lab[clear], want[clear])
    f = []
    for labels in (lab, want):
        ev = construct_split_evaluator(gold["train"], "train")
        ev.feed_induced_clusters({i: set(np.flatnonzero(labels == i).tolist()) for i in range(m)})
        f.append(ev.compute_metrics())
    if np.array_equal(lab, want):
        assert f[0] == f[1]


def _edge_dataset(seed=11, mid_rows=False):
    """Ragged inputs the reference accepts: examples with no features (every feature of the
    example thresholded away, OiePreprocessor.py:200-208 -> an empty CSR row), examples longer
    than the fast path's descriptor (general path), e1 == e2, negatives equal to the positive
    entities (Zipf-heavy CDF), and N not a multiple of l (tail dropped, OieInduction.py:98)."""
    from rae.data import DatasetManager
    g = np.random.RandomState(seed)
    N, d, n = 530, 900, 25
    lens = g.randint(1, 20, size=N)
    lens[::17] = 0                                   # empty rows
    lens[5::97] = 300                                # longer than the descriptor capacity
    if mid_rows:                                     # around the fast paths' W-row registers (30)
        lens[3::11] = g.randint(25, 64, size=len(lens[3::11]))
    rows = np.repeat(np.arange(N), lens)
    cols = np.concatenate([g.choice(d, size=k, replace=False) for k in lens])
    X = sp.csr_matrix((np.ones(len(rows), np.float32), (rows, cols)), shape=(N, d))
    a1 = (g.zipf(1.6, N) % n).astype(np.int32)
    a2 = (g.zipf(1.6, N) % n).astype(np.int32)
    a2[::7] = a1[::7]                                # e1 == e2
    a1[:n] = np.arange(n)
    return DatasetManager.from_arrays(X, a1, a2, n_entities=n)


@pytest.mark.parametrize("dec", ["sp", "rescal+sp"])
def test_ragged_inputs_vs_oracle(built_lib, cuda_dev, dec):
    from rae.inducer import ReconstructInducer
    data = _edge_dataset()
    X = data.split["train"].xFeats
    assert np.diff(X.indptr).min() == 0 and np.diff(X.indptr).max() == 300
    m, r, s, l, ep = 12, 16, 4, 100, 2
    ind = ReconstructInducer(data, {"train": {}}, np.random.RandomState(2), ep, 0.1, l, r, m, s,
                             0.0, 0.0, "adagrad", "edge", dec, False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=2)
    ind.learn(verbose=False)
    assert ind.batch_reps["train"] == 5                         # 530 // 100, tail dropped
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, ep, lr=0.1, alpha=1.0)
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "ragged")
    lab = ind.func["label_train"].all_labels(ind.batch_reps["train"])
    want, _ = tr.labels()
    # the labelling kernel is the argmax of the trained (device) parameters; against the
    # float64 trajectory the labels agree except at near-ties within the parameter tolerance
    got = _params(ind)
    S = np.asarray(X[:len(want)] @ got["W"]) + got["Wb"]
    srt = np.sort(S, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-4
    assert np.array_equal(lab[clear], np.argmax(S, axis=1)[clear])
    assert np.mean(lab == want) > 0.97
    # empty rows score Wb alone: one shared label
    empty = np.flatnonzero(np.diff(X.indptr)[:len(want)] == 0)
    assert len(set(lab[empty].tolist())) == 1


@pytest.mark.parametrize("dec", ["sp", "rescal"])
def test_fast_paths_ragged_vs_oracle(built_lib, cuda_dev, dec):
    """The compile-time-shape kernels (C3's SP forward, C5's RESCAL encoder: K=100, r=200, s=20)
    on ragged rows: empty rows, rows around the 30 features their W-row registers hold and rows
    longer than the descriptor -- the longer rows take the runtime-shape path inside the same
    launch."""
    from rae.inducer import ReconstructInducer
    data = _edge_dataset(mid_rows=True)
    nf = np.diff(data.split["train"].xFeats.indptr)
    assert nf.min() == 0 and ((nf > 30) & (nf < 64)).any() and nf.max() == 300
    m, r, s, l, ep = 100, 200, 20, 100, 1
    ind = ReconstructInducer(data, {"train": {}}, np.random.RandomState(2), ep, 0.1, l, r, m, s,
                             0.0, 0.0, "adagrad", "edge", dec, False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=2)
    ind.learn(verbose=False)
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, ep, lr=0.1, alpha=1.0)
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "ragged-fast")


@pytest.mark.parametrize("opt,values,dec,bf16", [("adagrad", False, "sp", False),
                                                 ("sgd", False, "sp", False),
                                                 ("adagrad", True, "sp", False),
                                                 ("adagrad", False, "rescal", False),
                                                 ("adagrad", False, "rescal", True),
                                                 ("adagrad", False, "rescal+sp", False),
                                                 ("sgd", False, "rescal+sp", True)])
def test_private_rows_match_update_launch(built_lib, cuda_dev, opt, values, dec, bf16):
    """Rows one record of the batch references, updated by per-example workgroups of the update
    launch (rae.h RAE_PRIV_AUTO: every single-rank plan without a regulariser), train
    bit-identically to the update launch's row tasks doing every row (priv_rows=off): same
    parameters, accumulators and costs -- for SP and for the bilinear decoders, whose e2 row has
    its own gradient vector (task_private_rows' XY branch: G2), fp32 and bf16 MFMA operands."""
    s = 20
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    out = []
    for form in ("on", "off"):
        data, gold = synthetic_dataset(400, 3000, 10, seed=21)
        if values:                                   # non-binary features: x_f != 1
            x = data.split["train"].xFeats
            x.data = np.random.RandomState(5).uniform(0.5, 2.0, size=x.data.shape).astype(np.float32)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 2, 0.1, 100, 200, 100, s,
                                 0.0, 0.0, opt, "priv", dec, False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=2, kernel_forms={"priv_rows": form},
                                 mfma_bf16=bf16)
        ind.compile_function()
        assert ind.engine.kernel_forms_in_use()["priv_rows"] == form
        ind.learn(verbose=False)
        acc = {}
        if ind.optimizer.accumulator is not None:
            acc = {f"acc_{k}": v.detach().cpu().numpy().copy()
                   for k, v in zip(ind.modelFunc.param_names, ind.optimizer.accumulator)}
        out.append(({**_params(ind), **acc}, np.array(ind.epoch_costs)))
    for k in out[0][0]:
        assert np.array_equal(out[0][0][k], out[1][0][k]), k
    assert np.array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("m", [12, 100, 300, 7])      # 16 / 32 / 64 lanes per row; scalar path
def test_label_pass_every_row_length(built_lib, cuda_dev, m):
    """rae_label on rows of every length 0..130 (each length ten times): the lane-group
    gather's partial last rounds (nnz = 17, 33, ... once dropped a feature) and the
    64-feature chunking, against the float64 oracle's probabilities and labels."""
    import ctypes as C
    import torch
    from rae import _lib
    from rae.engine import DeviceSplit
    from rae.data import DatasetSplit
    g = np.random.RandomState(m)
    d = 4000
    lens = np.repeat(np.arange(131), 10)
    rows = np.repeat(np.arange(len(lens)), lens)
    cols = np.concatenate([g.choice(d, size=k, replace=False) for k in lens])
    X = sp.csr_matrix((np.ones(len(rows), np.float32), (rows, cols)), shape=(len(lens), d))
    n = X.shape[0]
    split = DeviceSplit(DatasetSplit(np.zeros(n, np.int32), np.zeros(n, np.int32), X), cuda_dev)
    W = g.standard_normal((d, m)).astype(np.float32)
    Wb = g.standard_normal(m).astype(np.float32)
    lab = torch.empty(n, dtype=torch.int64, device=cuda_dev)
    pr = torch.empty((n, m), dtype=torch.float32, device=cuda_dev)
    lib = _lib.load()
    Wt, Wbt = torch.as_tensor(W, device=cuda_dev), torch.as_tensor(Wb, device=cuda_dev)
    _lib.check(lib.rae_label(C.c_void_p(split.indptr.data_ptr()), C.c_void_p(split.indices.data_ptr()),
                             None, C.c_void_p(Wt.data_ptr()), C.c_void_p(Wbt.data_ptr()), m, 0, n,
                             C.c_void_p(lab.data_ptr()), C.c_void_p(pr.data_ptr()), None))
    torch.cuda.synchronize()
    want_lab, want_p = O.label(X, W.astype(np.float64), Wb.astype(np.float64))
    np.testing.assert_allclose(pr.cpu().numpy(), want_p, rtol=1e-4, atol=1e-6)
    S = np.asarray(X @ W.astype(np.float64)) + Wb
    srt = np.sort(S, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-4
    assert np.array_equal(lab.cpu().numpy()[clear], want_lab[clear])


@pytest.mark.parametrize("dec", ["sp", "rescal", "rescal+sp"])
@pytest.mark.parametrize("shape", [(1, 4, 1, 1), (3, 1, 1, 3), (2, 5, 2, 7), (17, 3, 1, 5)],
                         ids=["m1_l1", "r1", "odd", "m17"])
def test_degenerate_shapes_vs_oracle(built_lib, cuda_dev, dec, shape):
    """Smallest shapes the reference's constructor accepts: one relation, one-dimensional
    embeddings, a single negative, a batch of one example (K = 1 MFMA chains, scalar
    paths, partial tiles everywhere)."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    m, r, s, l = shape
    data, gold = synthetic_dataset(60, 300, 3, seed=21)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "tiny", dec, False, True, False, 1.0, device=cuda_dev,
                             graph_chunk=2)
    ind.learn(verbose=False)
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, 1, lr=0.1, alpha=1.0)
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "tiny")


@pytest.mark.parametrize("dec", ["rescal", "rescal+sp"])
def test_bilinear_many_relations_vs_oracle(built_lib, cuda_dev, dec):
    """K = 400 relations on a bilinear decoder (fp32): an 8 x 16 x K block of R no longer fits
    in LDS (512 K bytes > 160 KiB above K = 320), so the M-tile passes read R from L2
    (k_bil_mt<false, true>); float4 rows (K multiple of 4) and the R-row update's non-LDS path."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    m, r, s, l = 400, 24, 3, 40
    data, gold = synthetic_dataset(120, 600, 6, seed=31)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "bigk", dec, False, True, False, 1.0, device=cuda_dev,
                             graph_chunk=2)
    ind.learn(verbose=False)
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, 1, lr=0.1, alpha=1.0)
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "bigk")


@pytest.mark.parametrize("dec", ["sp", "rescal+sp"])
def test_hot_rows_vs_oracle(built_lib, cuda_dev, dec):
    """Collisions at their worst: five entities, every e1 the same entity, one feature in every
    example -- a single A row and a single W row receive hundreds of contributions per step
    (the update's multi-chunk record loops and wide rounds)."""
    from rae.data import DatasetManager
    from rae.inducer import ReconstructInducer
    g = np.random.RandomState(3)
    N, d, n = 400, 50, 5
    lens = g.randint(1, 6, size=N)
    rows = np.repeat(np.arange(N), lens + 1)
    cols = np.concatenate([np.concatenate([[0], 1 + g.choice(d - 1, size=k, replace=False)])
                           for k in lens])
    X = sp.csr_matrix((np.ones(len(rows), np.float32), (rows, cols)), shape=(N, d))
    a1 = np.zeros(N, np.int32)
    a2 = g.randint(0, n, N).astype(np.int32)
    a2[:n] = np.arange(n)
    data = DatasetManager.from_arrays(X, a1, a2, n_entities=n)
    m, r, s, l, ep = 8, 16, 4, 100, 2
    ind = ReconstructInducer(data, {"train": {}}, np.random.RandomState(2), ep, 0.1, l, r, m, s,
                             0.0, 0.0, "adagrad", "hot", dec, False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=2)
    ind.learn(verbose=False)
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, ep, lr=0.1, alpha=1.0)
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "hot")


@pytest.mark.parametrize("dec", ["sp", "rescal+sp"])
def test_very_heavy_rows_beyond_workgroup_slots(built_lib, cuda_dev, dec):
    """More very heavy rows (> 16 records per step) than the update has workgroup slots for
    (NVC = max(32, L/2) = 32 at L = 64): the dispatch table hands the excess to single waves
    (rae_index.hpp build_batch_tasks).  60 entities and 40 features under a 64-example batch
    give ~23 records per entity and ~22 per feature: ~90 very heavy rows per step."""
    from rae.data import DatasetManager
    from rae.inducer import ReconstructInducer
    g = np.random.RandomState(5)
    N, d, n = 640, 40, 60
    lens = g.randint(10, 18, size=N)
    rows = np.repeat(np.arange(N), lens)
    cols = np.concatenate([g.choice(d, size=k, replace=False) for k in lens])
    X = sp.csr_matrix((np.ones(len(rows), np.float32), (rows, cols)), shape=(N, d))
    a1 = g.randint(0, n, N).astype(np.int32)
    a2 = g.randint(0, n, N).astype(np.int32)
    a1[:n] = np.arange(n)
    data = DatasetManager.from_arrays(X, a1, a2, n_entities=n)
    m, r, s, l, ep = 8, 16, 10, 64, 2
    # the W rows alone already exceed the 32 workgroup slots in every batch
    vh_w = [int((np.bincount(cols[rows_b], minlength=d) > 16).sum())
            for rows_b in (np.isin(rows, np.arange(b * l, (b + 1) * l)) for b in range(N // l))]
    assert min(vh_w) > 32, vh_w
    ind = ReconstructInducer(data, {"train": {}}, np.random.RandomState(2), ep, 0.1, l, r, m, s,
                             0.0, 0.0, "adagrad", "vheavy", dec, False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=4)
    ind.learn(verbose=False)
    tr, costs = _oracle_trajectory(dec, data, 2, m, r, s, l, ep, lr=0.1, alpha=1.0)
    np.testing.assert_allclose(np.array(ind.epoch_costs), costs, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr.params, "vheavy")


def test_initialize_then_train_restarts_like_reference(built_lib, cuda_dev):
    """test.py:33-46's sequence: train(), initialize(), train().  The second train() runs all
    its epochs again from epoch 0 with a fresh zero-accumulator optimizer
    (OieInduction.py:103-108,137,175) on parameters re-drawn from the same shared RNG."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    m, r, s, l, ep = 8, 16, 4, 50, 2
    data, gold = synthetic_dataset(400, 300, 4, seed=9)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), ep, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "restart", "sp", False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=2)
    ind.train()
    first = np.array(ind.epoch_costs)
    ind.initialize()
    assert ind.cur_epoch == 0 and ind.optimizer is None
    ind.train()
    assert ind.cur_epoch == ep
    second = np.array(ind.epoch_costs)
    assert second.shape == first.shape
    # the oracle: one RandomState drives init, epoch negatives, re-init, epoch negatives
    xs = data.split["train"]
    rng = np.random.RandomState(2)
    tr = O.OracleTrainer("sp", xs.xFeats, xs.args1, xs.args2, data.negSamplingCum, rng, m, r, s,
                         l, lr=0.1, alpha=1.0)
    want1 = np.array([tr.epoch()[0] for _ in range(ep)])
    tr2 = O.OracleTrainer("sp", xs.xFeats, xs.args1, xs.args2, data.negSamplingCum, rng, m, r, s,
                          l, lr=0.1, alpha=1.0)          # re-draw + zero accumulators
    want2 = np.array([tr2.epoch()[0] for _ in range(ep)])
    np.testing.assert_allclose(first, want1, rtol=COST_RTOL, atol=COST_RTOL)
    np.testing.assert_allclose(second, want2, rtol=COST_RTOL, atol=COST_RTOL)
    _assert_params_close(_params(ind), tr2.params, "restart")


def test_frequent_eval_mode2_evaluates_valid_and_test_every_batch(built_lib, cuda_dev, capsys):
    """frequentEval with train/valid/test splits (mode 2): after every batch the valid and
    test clusters are labelled and B^3-evaluated (OieInduction.py:194-198), and again at the
    end of every epoch (:214-217)."""
    from rae.data import DatasetManager, DatasetSplit, synthetic_dataset
    from rae.inducer import ReconstructInducer
    full, gold = synthetic_dataset(300, 200, 3, seed=4)
    xs = full.split["train"]
    cut = [slice(0, 200), slice(200, 250), slice(250, 300)]
    splits = {k: DatasetSplit(xs.args1[c], xs.args2[c], xs.xFeats[c])
              for k, c in zip(("train", "valid", "test"), cut)}
    g = {k: {i - c.start: v for i, v in gold["train"].items() if c.start <= i < c.stop}
         for k, c in zip(("train", "valid", "test"), cut)}
    for k in ("valid", "test"):
        g[k].setdefault(0, ["REL0"])            # at least one gold label per split
    data = DatasetManager(splits, full.entity_freqs, full.n_features)
    ind = ReconstructInducer(data, g, np.random.RandomState(2), 2, 0.1, 25, 8, 4, 3, 0.0, 0.0,
                             "adagrad", "mode2", "sp", False, True, True, 1.0, device=cuda_dev)
    ind.learn()
    out = capsys.readouterr().out
    nb = 200 // 25
    assert out.count("valid f1:") == 2 * (nb + 1)
    assert out.count("test f1:") == 2 * (nb + 1)


def test_label_argmax_nan_and_inf_follow_numpy(built_lib, cuda_dev):
    """A diverged row still gets a label in [0, m): argmax treats NaN as the maximum (first
    NaN wins) and an all -inf row gives 0, as numpy's / Theano's argmax do."""
    import torch
    from rae.engine import DeviceSplit
    from rae.data import DatasetSplit
    from rae import _lib
    import ctypes as C
    g = np.random.RandomState(1)
    N, d, m = 64, 30, 12
    rows = np.repeat(np.arange(N), 3)
    X = sp.csr_matrix((np.ones(3 * N, np.float32), (rows, g.randint(0, d, 3 * N))), shape=(N, d))
    X.sum_duplicates()
    X.data[:] = 1.0
    W = g.uniform(-1, 1, (d, m)).astype(np.float32)
    Wb = np.zeros(m, np.float32)
    W[5, 7] = np.nan
    W[5, 3] = np.nan
    W[9, :] = -np.inf
    ds = DeviceSplit(DatasetSplit(np.zeros(N), np.zeros(N), X), cuda_dev)
    Wt = torch.as_tensor(W, device=cuda_dev)
    Wbt = torch.as_tensor(Wb, device=cuda_dev)
    lab = torch.empty(N, dtype=torch.int64, device=cuda_dev)
    lib = _lib.load()
    _lib.check(lib.rae_label(C.c_void_p(ds.indptr.data_ptr()), C.c_void_p(ds.indices.data_ptr()),
                             None, C.c_void_p(Wt.data_ptr()), C.c_void_p(Wbt.data_ptr()), m, 0, N,
                             C.c_void_p(lab.data_ptr()), None, None), "rae_label")
    torch.cuda.synchronize()
    Xd = X.toarray().astype(np.float64)
    S = np.zeros((N, m))
    for i in range(N):                       # S = X.W + Wb with inf/nan propagation per row
        S[i] = sum(Xd[i, f] * W[f].astype(np.float64) for f in np.nonzero(Xd[i])[0]) + Wb
    want = np.argmax(S, axis=1)
    got = lab.cpu().numpy()
    assert np.all((got >= 0) & (got < m))
    special = ~np.all(np.isfinite(S), axis=1)
    assert special.sum() > 0
    assert np.array_equal(got[special], want[special])


def _record_offsets(dec, m, r, s):
    """The exchange record's field offsets (rae_step.hpp make_layout: P, dS, V1, V2, dw1, dw2,
    G1, [G2, X, Y, A1, A2, Z, aux,] coefficients, loss; m and r padded to multiples of 4)."""
    a4 = lambda x: (x + 3) & ~3
    m4, r4 = a4(m), a4(r)
    o = {"P": 0, "V1": 2 * m4, "V2": 2 * m4 + r4}
    end = 2 * m4 + 5 * r4
    if dec != "sp":
        end += 5 * r4 + m4 + 4
    o["loss"] = end + a4(2 * (2 + 2 * s))
    return o


@pytest.mark.parametrize("dec", ["sp", "rescal"])
def test_forward_launch_alone_vs_oracle(built_lib, cuda_dev, dec):
    """One forward launch by itself (rae_step_forward, no update) at the C3 / C5 shapes
    (m=100, r=200, s=20, l=100: the compile-time-shape fast encoders): the exchange records of
    batch 0 hold the relation probabilities P (RelationClassifier.py:35-36), SP's wC1 / wC2
    (SelectionalPreferences.py:31-32) and per-example loss terms that sum to -cost * D
    (OieModel.py:90) -- the forward half of SURVEY 8(b)'s entry points checked in isolation
    against the float64 oracle's forward."""
    import ctypes as C
    import torch
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    m, r, s, l = 100, 200, 20, 100
    data, gold = synthetic_dataset(300, 2000, 10, seed=7)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s,
                             0.0, 0.0, "adagrad", "fwd", dec, False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=1)
    ind.compile_function()
    eng = ind.engine
    n1, n2 = ind.draw_epoch_negatives()
    eng.set_epoch_negatives(n1, n2)
    p0 = _params(ind)
    lib, st = eng.lib, C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.rae_build_index(eng.plan, 0, 1, st) == 0
    assert lib.rae_set_cursor(eng.plan, 0, st) == 0
    assert lib.rae_step_forward(eng.plan, 0, st) == 0
    torch.cuda.synchronize()
    eng.check()
    assert eng.rec_floats > 0
    rec = eng.exchange_buf.detach().cpu().double().numpy()[:l * eng.rec_floats].reshape(l, eng.rec_floats)
    tr = data.split["train"]
    rows = slice(0, l)
    res = O.train_step_grads(dec, p0, tr.xFeats[rows], tr.args1[rows], tr.args2[rows],
                             n1[:, rows], n2[:, rows], alpha=1.0)
    o = _record_offsets(dec, m, r, s)
    np.testing.assert_allclose(rec[:, o["P"]:o["P"] + m], res.P, rtol=1e-4, atol=1e-6)
    if dec == "sp":
        np.testing.assert_allclose(rec[:, o["V1"]:o["V1"] + r], res.P @ p0["C1"].T, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(rec[:, o["V2"]:o["V2"] + r], res.P @ p0["C2"].T, rtol=1e-4, atol=1e-5)
    D = 4 * l + 2 * l * s
    np.testing.assert_allclose(rec[:, o["loss"]].sum(), -res.cost * D, rtol=2e-5)
    # nothing was updated: the parameters are the ones the forward read
    for k, v in _params(ind).items():
        assert np.array_equal(v, p0[k]), k
