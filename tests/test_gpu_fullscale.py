"""Parity at BASELINE.json's full headline size (config 3: 1M synthetic triples, d = 2^17,
K = 100, embed 200, neg 20, l = 100, SP decoder, AdaGrad) and at the config-4 shape.

The HIP epoch path (graph-captured steps, device row index, sparse row updates) runs the
first batches of an epoch; the float64 oracle runs the same batches with the reference's
DENSE schedule (dense dW / dA, AdaGrad over every row, learning/Optimizers.py:27-33) from the
same RandomState(2) initialisation and the same negatives.  At this size the row-index
partitions, the heavy-row task ordering and the Zipf-frequent rows (tens of records per
step) are all exercised, which the small golden cases cannot reach.

Tolerances as in test_gpu_train.py: costs 2e-5 relative, parameters 2e-4 + 2e-3|p|; plus a
size-independent property: every row the batches did not reference is bit-unchanged.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import rae_oracle as O

pytestmark = pytest.mark.gpu

COST_RTOL = 2e-5


LABEL_ROWS = 100_000      # rows of the trained split the relation assignments are checked on
LABEL_MARGIN = 1e-5       # labels compared where the oracle's top-2 score margin exceeds this


def _gpu_labels(eng, nrows=LABEL_ROWS):
    """func['label_train'] on the device (rae_label, RelationClassifier.py:39-48) over the first
    `nrows` rows of the trained split, with the parameters the steps left."""
    lab, _ = eng.label(eng.split, 0, min(nrows, eng.split.N), probs=False)
    return lab.cpu().numpy()


def _scores(xs, W, Wb, n):
    return np.asarray(xs.xFeats[:n].astype(np.float64) @ W) + Wb[None, :]


def check_labels(got, xs, W, Wb, margin=LABEL_MARGIN, what="", W_gpu=None, Wb_gpu=None,
                 min_decisive=0.9):
    """Relation assignments (argmax S, S = X.W + Wb; RelationClassifier.py:39-48,
    OieInduction.py:321-340) of the GPU equal the oracle's wherever the oracle's top-2 margin
    exceeds `margin` -- and, given the GPU's trained W_gpu / Wb_gpu, also exceeds twice the row's
    largest score difference between the two models (bf16 runs: the trajectories differ by the
    operand rounding, so a label may only flip where the models' scores disagree by more than
    the margin).  At least `min_decisive` of the rows must be checked.  Returns the share."""
    n = got.shape[0]
    S = _scores(xs, W, Wb, n)
    top2 = np.partition(S, -2, axis=1)[:, -2:]
    gap = top2[:, 1] - top2[:, 0]
    need = np.full(n, margin)
    if W_gpu is not None:
        Sg = _scores(xs, W_gpu, Wb_gpu, n)
        need = np.maximum(need, 2.0 * np.abs(Sg - S).max(axis=1))
        # the kernel's argmax is the argmax of its own model's scores (fp32 sums: 1e-5 margin)
        tg = np.partition(Sg, -2, axis=1)[:, -2:]
        own = (tg[:, 1] - tg[:, 0]) > LABEL_MARGIN
        assert np.all(got[own] == Sg[own].argmax(axis=1)), what
    decisive = gap > need
    want = S.argmax(axis=1)
    bad = np.flatnonzero(decisive & (got != want))
    agree = float((got == want).mean())
    print(what, f"labels: {n} rows, {decisive.mean():.4f} decisive, agreement {agree:.5f}")
    assert decisive.mean() >= min_decisive, (what, decisive.mean())
    assert bad.size == 0, (what, bad[:10], got[bad[:10]], want[bad[:10]])
    return float(decisive.mean())


def _run(cuda_dev, N, d, m, r, s, l, ntrue, steps, seed_data=1234, labels=False,
         kernel_forms=None):
    import torch
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    data, gold = synthetic_dataset(N, d, ntrue, seed=seed_data)
    xs = data.split["train"]
    tr = O.OracleTrainer("sp", xs.xFeats, xs.args1, xs.args2, data.negSamplingCum,
                         np.random.RandomState(2), m, r, s, l, lr=0.1, alpha=1.0)
    init = {k: v.copy() for k, v in tr.params.items()}
    neg1 = O.negative_samples(tr.rng, tr.cum, tr.N, s)
    neg2 = O.negative_samples(tr.rng, tr.cum, tr.N, s)
    want = [tr.train_batch(b, neg1[:, O.batch_rows(b, l)], neg2[:, O.batch_rows(b, l)])
            for b in range(steps)]

    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "fullscale", "sp", False, True, False, 1.0,
                             device=cuda_dev, graph_chunk=2, kernel_forms=kernel_forms)
    ind.compile_function()
    eng = ind.engine
    for k, v in (kernel_forms or {}).items():
        assert eng.kernel_forms_in_use()[k] == v
    eng.set_epoch_negatives(neg1, neg2)
    eng.run(0, steps)
    torch.cuda.synchronize()
    eng.check()
    got = eng.costs[:steps].cpu().numpy().astype(np.float64)
    params = {k: v.detach().cpu().double().numpy()
              for k, v in ind.modelFunc.named_params().items()}
    if labels:
        check_labels(_gpu_labels(eng), xs, tr.params["W"], tr.params["Wb"],
                     what=f"N={N} m={m} r={r} s={s} l={l}", W_gpu=params["W"],
                     Wb_gpu=params["Wb"])
    return np.array(want), got, tr.params, params, init


def test_c2_full_size(built_lib, cuda_dev):
    # BASELINE config 2 at its real size: 100k synthetic triples, d = 2^17, K = 30, embed 100,
    # neg 10, l = 100 (the compile-time C2 specialisation of the forward, scalar lanes: K is
    # not a multiple of 4)
    want_c, got_c, want_p, got_p, init = _run(cuda_dev, N=100_000, d=2 ** 17, m=30, r=100,
                                              s=10, l=100, ntrue=30, steps=6, labels=True)
    _check(want_c, got_c, want_p, got_p, init, min_untouched=0.5)


# --------------------------------------------------------------------------------------------
# bf16 MFMA operands (BASELINE config 5): the tolerance is derived per trajectory
# --------------------------------------------------------------------------------------------
def bf16_trajectories(cuda_dev, dec, N, d, m, r, s, l, ntrue, steps, seed_data=1234,
                      graph_chunk=2, labels=False):
    """The GPU bf16 path, the exact float64 oracle and the float64 oracle with the bf16
    operand rounding emulated (rae_oracle.bf16_round at the three R contractions), over the
    same first `steps` batches of an epoch from RandomState(2).  Returns dict of
    costs / params per run ("gpu", "exact", "emu") and the initial parameters."""
    import torch
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    data, gold = synthetic_dataset(N, d, ntrue, seed=seed_data)
    xs = data.split["train"]
    out = {}
    for name, bf in (("exact", False), ("emu", True)):
        tr = O.OracleTrainer(dec, xs.xFeats, xs.args1, xs.args2, data.negSamplingCum,
                             np.random.RandomState(2), m, r, s, l, lr=0.1, alpha=1.0, bf16=bf)
        if name == "exact":
            init = {k: v.copy() for k, v in tr.params.items()}
        neg1 = O.negative_samples(tr.rng, tr.cum, tr.N, s)
        neg2 = O.negative_samples(tr.rng, tr.cum, tr.N, s)
        c = [tr.train_batch(b, neg1[:, O.batch_rows(b, l)], neg2[:, O.batch_rows(b, l)])
             for b in range(steps)]
        out[name] = (np.array(c), tr.params)
        del tr
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "bf16", dec, False, True, False, 1.0, device=cuda_dev,
                             graph_chunk=graph_chunk, mfma_bf16=True)
    ind.compile_function()
    eng = ind.engine
    eng.set_epoch_negatives(neg1, neg2)
    eng.run(0, steps)
    torch.cuda.synchronize()
    eng.check()
    got = {k: v.detach().cpu().double().numpy() for k, v in ind.modelFunc.named_params().items()}
    out["gpu"] = (eng.costs[:steps].cpu().numpy().astype(np.float64), got)
    if labels:
        out["labels"] = _gpu_labels(eng)
        out["xs"] = xs
    ind._drop_engine()
    return out, init


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


# Derived bf16 tolerance: the GPU trajectory must be as close to the float64 one as bf16
# operand rounding itself allows (the emulated oracle's distance, x1.25 + 1e-4 slack for the
# fp32 accumulation), AND much closer to the emulated oracle than either is to the exact one
# (<= 0.25 x that distance + 1e-4): the kernels differ from the reference only by rounding
# the R-contraction operands to bf16.  Costs alike, per batch.
BF16_EXACT_FACTOR, BF16_EMU_FACTOR, BF16_SLACK = 1.25, 0.25, 1e-4


def check_bf16(out, init=None, what=""):
    ce, cm, cg = out["exact"][0], out["emu"][0], out["gpu"][0]
    dc_emu = np.abs(cm - ce)
    assert np.all(np.abs(cg - ce) <= BF16_EXACT_FACTOR * dc_emu + 2e-5 * np.abs(ce)), \
        (what, cg, ce, cm)
    assert np.all(np.abs(cg - cm) <= BF16_EMU_FACTOR * dc_emu + 2e-5 * np.abs(ce)), \
        (what, cg, ce, cm)
    pe, pm, pg = out["exact"][1], out["emu"][1], out["gpu"][1]
    rep = {}
    for k in pe:
        d_emu, d_gpu, d_ge = _rel(pm[k], pe[k]), _rel(pg[k], pe[k]), _rel(pg[k], pm[k])
        rep[k] = (d_emu, d_gpu, d_ge)
        assert d_gpu <= BF16_EXACT_FACTOR * d_emu + BF16_SLACK, (what, k, rep[k])
        assert d_ge <= BF16_EMU_FACTOR * d_emu + BF16_SLACK, (what, k, rep[k])
        if init is not None and k in ("W", "A"):
            untouched = np.all(pe[k] == init[k], axis=1)
            f32 = init[k][untouched].astype(np.float32).astype(np.float64)
            assert np.array_equal(pg[k][untouched], f32), (what, k)
    print(what, {k: "emu %.2e gpu %.2e gpu-emu %.2e" % v for k, v in rep.items()})
    return rep


@pytest.mark.timeout(900)
def test_c5_bench_size_bf16(built_lib, cuda_dev):
    """BASELINE config 5 at the size bench.py --config c5 times: 1M synthetic triples,
    d = 2^17, K = 100, embed 200, neg 20, l = 100, RESCAL, bf16 MFMA operands -- the row index,
    heavy-row classes and the k_bil_rows / k_update_bil dispatch at full scale -- against the
    float64 oracle with the derived bf16 tolerance (check_bf16) and the untouched-rows
    property."""
    out, init = bf16_trajectories(cuda_dev, "rescal", N=1_000_000, d=2 ** 17, m=100, r=200,
                                  s=20, l=100, ntrue=100, steps=4, labels=True)
    check_bf16(out, init, "c5 full size")
    # relation assignments: against the bf16-emulating oracle (the same operand rounding) and
    # against the exact float64 oracle, each where its top-2 margin is decisive
    pg = out["gpu"][1]
    for name, floor in (("emu", 0.9), ("exact", 0.5)):
        p = out[name][1]
        check_labels(out["labels"], out["xs"], p["W"], p["Wb"], what=f"c5 labels vs {name}",
                     W_gpu=pg["W"], Wb_gpu=pg["Wb"], min_decisive=floor)


def _run_oracle_only(N, d, m, r, s, l, ntrue, steps, seed_data=1234):
    from rae.data import synthetic_dataset
    data, gold = synthetic_dataset(N, d, ntrue, seed=seed_data)
    xs = data.split["train"]
    tr = O.OracleTrainer("sp", xs.xFeats, xs.args1, xs.args2, data.negSamplingCum,
                         np.random.RandomState(2), m, r, s, l, lr=0.1, alpha=1.0)
    init = {k: v.copy() for k, v in tr.params.items()}
    neg1 = O.negative_samples(tr.rng, tr.cum, tr.N, s)
    neg2 = O.negative_samples(tr.rng, tr.cum, tr.N, s)
    want = [tr.train_batch(b, neg1[:, O.batch_rows(b, l)], neg2[:, O.batch_rows(b, l)])
            for b in range(steps)]
    return np.array(want), None, tr.params, None, init


def _check(want_c, got_c, want_p, got_p, init, min_untouched=0.0):
    np.testing.assert_allclose(got_c, want_c, rtol=COST_RTOL, atol=0)
    for k in want_p:
        err = np.abs(got_p[k] - want_p[k])
        tol = 2e-4 + 2e-3 * np.abs(want_p[k])
        assert np.all(err <= tol), f"{k}: max err {err.max():.3e}"
        # rows the batches never touched: bit-unchanged from the fp32 initialisation
        if k in ("W", "A"):
            untouched = np.all(want_p[k] == init[k], axis=1)
            assert untouched.sum() >= min_untouched * untouched.size, k
            f32 = init[k][untouched].astype(np.float32).astype(np.float64)
            assert np.array_equal(got_p[k][untouched], f32), k


def test_headline_c3_full_size(built_lib, cuda_dev):
    want_c, got_c, want_p, got_p, init = _run(cuda_dev, N=1_000_000, d=2 ** 17, m=100, r=200,
                                              s=20, l=100, ntrue=100, steps=4, labels=True)
    _check(want_c, got_c, want_p, got_p, init, min_untouched=0.5)


def test_c4_shape(built_lib, cuda_dev):
    # BASELINE config 4's K / embed / neg (K=300, embed 300, neg 50): the general (non-fixed
    # shape) SP path, two float4 columns per lane in the row updates
    want_c, got_c, want_p, got_p, init = _run(cuda_dev, N=3000, d=20_000, m=300, r=300, s=50,
                                              l=100, ntrue=20, steps=6)
    _check(want_c, got_c, want_p, got_p, init)


@pytest.mark.parametrize("heavy_chunk", ["off", "on"])
def test_c3_global_batch_800(built_lib, cuda_dev, heavy_chunk):
    # the global batch of 8 data-parallel ranks at l = 100: Zipf-frequent rows carry hundreds
    # of records per step (workgroup rows split over four waves, or -- heavy_chunk on, the
    # default from L = 2048 -- into 128-record chunks summed in parallel and combined by
    # k_heavy_fin) and every K-chunk of the dense tiles is non-trivial
    want_c, got_c, want_p, got_p, init = _run(cuda_dev, N=1_000_000, d=2 ** 17, m=100, r=200,
                                              s=20, l=800, ntrue=100, steps=3,
                                              kernel_forms={"heavy_chunk": heavy_chunk})
    _check(want_c, got_c, want_p, got_p, init, min_untouched=0.5)


@pytest.mark.parametrize("dec,opt", [("rescal", "adagrad"), ("rescal+sp", "adagrad"),
                                     ("sp", "sgd"), ("rescal", "sgd")])
def test_bilinear_heavy_chunks(built_lib, cuda_dev, dec, opt):
    """The bilinear updates with the heavy-row chunks (heavy_chunk on: rows with >= 256 records of
    the global batch summed as parallel chunks, k_heavy_fin combining them) against the same
    run without them, at a Zipf global batch of 800 from the 1M-triple generator: costs and
    every parameter equal to fp32 summation-order noise (a lost or doubled chunk would not be)."""
    import torch
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    runs = {}
    for hc in ("off", "on"):
        data, gold = synthetic_dataset(1_000_000, 2 ** 17, 100, seed=1234)
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 800, 64, 30, 20,
                                 0.0, 0.0, opt, "hchunk", dec, False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=2, kernel_forms={"heavy_chunk": hc})
        ind.compile_function()
        eng = ind.engine
        assert eng.kernel_forms_in_use()["heavy_chunk"] == hc
        n1, n2 = ind.draw_epoch_negatives()
        if hc == "off":   # the batches do have rows past one chunk (the path is exercised)
            xs = data.split["train"]
            ids = np.concatenate([xs.args1[:800], xs.args2[:800], np.ravel(n1[:, :800]),
                                  np.ravel(n2[:, :800])])
            assert np.bincount(ids).max() >= 256      # at least two chunks
        eng.set_epoch_negatives(n1, n2)
        eng.run(0, 3)
        torch.cuda.synchronize()
        eng.check()
        runs[hc] = ({k: v.detach().cpu().double().numpy() for k, v in ind.modelFunc.named_params().items()},
                    eng.costs[:3].cpu().numpy().astype(np.float64))
        ind._drop_engine()
    (p0, c0), (p1, c1) = runs["off"], runs["on"]
    np.testing.assert_allclose(c1, c0, rtol=1e-5, atol=1e-6)
    for k in p0:
        err = np.abs(p1[k] - p0[k])
        assert np.all(err <= 1e-5 + 1e-4 * np.abs(p0[k])), f"{k}: max err {err.max():.3e}"


# --------------------------------------------------------------------------------------------
# config C4 at its real size: 10M synthetic triples, d = 2^20, K = 300, embed 300, neg 50, l=100
# --------------------------------------------------------------------------------------------
def _chunked_rows(draw, nrows, ncols, keep, chunk=1 << 16):
    """Rows `keep` (sorted) of a (nrows, ncols) RandomState draw made in row chunks -- the same
    stream as one whole draw (the legacy generator's doubles / cached Gaussians carry over
    between calls) without materialising the whole matrix."""
    out = np.empty((len(keep), ncols), dtype=np.float64)
    for r0 in range(0, nrows, chunk):
        blk = draw((min(chunk, nrows - r0), ncols))
        lo, hi = np.searchsorted(keep, [r0, r0 + blk.shape[0]])
        out[lo:hi] = blk[keep[lo:hi] - r0]
    return out


@pytest.mark.timeout(900)
def test_c4_full_size(built_lib, cuda_dev):
    """BASELINE config 4 on one GPU at full size: the first steps of an epoch (graph-captured
    epoch path, device negatives on the reference's RandomState stream) against the float64
    oracle.  The oracle keeps only the rows the steps reference -- exact for lambda = 0,
    because an AdaGrad step with zero gradient leaves a row bit-unchanged
    (learning/Optimizers.py:30-32) -- drawn from the same RandomState(2) stream
    in the reference's order (W, A, C1, C2; OieModel.py:49-63,105) without materialising the
    2.5 GB W / 4.5 GB A in float64.  Checked: per-batch costs, every referenced row of W, A,
    Ab and all of C1, C2, Wb; the initial values of the referenced rows; and a sample of
    100k unreferenced rows of W and of A bit-unchanged over the steps."""
    import torch
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    N, d, m, r, s, l, steps = 10_000_000, 2 ** 20, 300, 300, 50, 100, 3
    data, gold = synthetic_dataset(N, d, 300, seed=1234)
    xs = data.split["train"]
    n = data.get_arg_voc_size()
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, l, r, m, s, 0.0, 0.0,
                             "adagrad", "c4", "sp", False, True, False, 1.0, device=cuda_dev,
                             graph_chunk=2)
    ind.compile_function()
    eng = ind.engine
    eng.sample_epoch_negatives(ind.negativeSampler, "device")   # neg1 then neg2, (s, N) each
    rows = slice(0, steps * l)
    neg1 = eng.neg1[:, rows].cpu().numpy()
    neg2 = eng.neg2[:, rows].cpu().numpy()
    Xb = xs.xFeats[rows]
    tf = np.unique(Xb.indices)
    te = np.unique(np.concatenate([xs.args1[rows], xs.args2[rows], neg1.ravel(), neg2.ravel()]))
    named = ind.modelFunc.named_params()
    g = np.random.RandomState(99)
    uf = np.setdiff1d(g.choice(d, 100_000, replace=False), tf)
    ue = np.setdiff1d(g.choice(n, 100_000, replace=False), te)
    uf_t, ue_t = torch.as_tensor(uf, device=cuda_dev), torch.as_tensor(ue, device=cuda_dev)
    W0 = named["W"][uf_t].cpu().numpy()
    A0 = named["A"][ue_t].cpu().numpy()
    init_W = named["W"][torch.as_tensor(tf, device=cuda_dev)].cpu().double().numpy()
    init_A = named["A"][torch.as_tensor(te, device=cuda_dev)].cpu().double().numpy()
    init_C1 = named["C1"].cpu().double().numpy()

    eng.run(0, steps)
    torch.cuda.synchronize()
    eng.check()
    got_c = eng.costs[:steps].cpu().numpy().astype(np.float64)

    # the oracle on the referenced rows, same RandomState(2) draws
    rng = np.random.RandomState(2)
    p = {"W": _chunked_rows(lambda sh: rng.uniform(O.LOW, O.HIGH, sh), d, m, tf),
         "Wb": np.zeros(m)}
    p["A"] = _chunked_rows(lambda sh: rng.uniform(-0.01, 0.01, sh), n, r, te)
    p["C1"] = rng.normal(0, np.sqrt(0.1), (r, m))
    p["C2"] = rng.normal(0, np.sqrt(0.1), (r, m))
    p["Ab"] = np.zeros(len(te))
    assert np.array_equal(init_W, p["W"].astype(np.float32).astype(np.float64))
    assert np.array_equal(init_A, p["A"].astype(np.float32).astype(np.float64))
    assert np.array_equal(init_C1, p["C1"].astype(np.float32).astype(np.float64))
    acc = {k: np.zeros_like(v) for k, v in p.items()}
    fmap = np.full(d, -1, np.int64)
    fmap[tf] = np.arange(len(tf))
    emap = np.full(n, -1, np.int64)
    emap[te] = np.arange(len(te))
    want_c = []
    for b in range(steps):
        rb = slice(b * l, (b + 1) * l)
        Xs = xs.xFeats[rb]
        Xc = sp.csr_matrix((Xs.data, fmap[Xs.indices], Xs.indptr), shape=(l, len(tf)))
        res = O.train_step_grads("sp", p, Xc, emap[xs.args1[rb]], emap[xs.args2[rb]],
                                 emap[neg1[:, rb]], emap[neg2[:, rb]], alpha=1.0)
        O.adagrad_apply(p, acc, res.grads, 0.1)
        want_c.append(res.cost)
    np.testing.assert_allclose(got_c, np.array(want_c), rtol=COST_RTOL, atol=0)
    got = {"W": named["W"][torch.as_tensor(tf, device=cuda_dev)],
           "A": named["A"][torch.as_tensor(te, device=cuda_dev)],
           "Ab": named["Ab"][torch.as_tensor(te, device=cuda_dev)],
           "C1": named["C1"], "C2": named["C2"], "Wb": named["Wb"]}
    for k, v in got.items():
        v = v.cpu().double().numpy()
        err = np.abs(v - p[k])
        tol = 2e-4 + 2e-3 * np.abs(p[k])
        assert np.all(err <= tol), f"{k}: max err {err.max():.3e}"
    assert np.array_equal(named["W"][uf_t].cpu().numpy(), W0)
    assert np.array_equal(named["A"][ue_t].cpu().numpy(), A0)


@pytest.mark.parametrize("dp_update,heavy_chunk", [("replicated", "auto"), ("partitioned", "auto"),
                                                   ("partitioned", "on")])
def test_c3_global_batch_800_two_ranks(built_lib, cuda_dev, tmp_path, dp_update, heavy_chunk):
    """The data-parallel path itself at C3's full size: 2 ranks x l = 400 (the global batch of
    8 ranks at l = 100), records all-gathered between the forward and the update (replicated:
    every rank updates every row; partitioned: each rank its own rows, rows pulled from their
    owners before each forward), against the float64 oracle at the global batch L = 800; the
    two replicas bit-identical (partitioned: after the final gather)."""
    import test_dist
    test_dist._launch(["gpu_c3", str(tmp_path), dp_update, heavy_chunk], timeout=600)
    want_c, _, want_p, _, init = _run_oracle_only(N=1_000_000, d=2 ** 17, m=100, r=200, s=20,
                                                  l=800, ntrue=100, steps=3)
    c0 = np.load(tmp_path / "c3_costs_0.npy").astype(np.float64)
    c1 = np.load(tmp_path / "c3_costs_1.npy").astype(np.float64)
    np.testing.assert_array_equal(c0, c1)
    got = {}
    for k in want_p:
        g0 = np.load(tmp_path / f"c3_{k}_0.npy")
        g1 = np.load(tmp_path / f"c3_{k}_1.npy")
        assert np.array_equal(g0, g1), f"replicas differ in {k}"
        got[k] = g0.astype(np.float64)
    _check(want_c, c0, want_p, got, init, min_untouched=0.5)


@pytest.mark.parametrize("dec", ["sp", "rescal+sp"])
def test_heavy_chunks_tiny_vocabulary(built_lib, cuda_dev, dec):
    """a batch dominated by a few hot rows -- 24 entities and 40 features at a global
    batch of 2048 (every entity row ~850 records, every feature row ~256: 2..7 chunks each) --
    with heavy_chunk on: the chunk tasks, the combine list and k_heavy_fin fit their slots (no
    error flag, no lost chunk), and training equals the float64 oracle and the unchunked run."""
    import torch
    from rae.data import DatasetManager
    from rae.inducer import ReconstructInducer
    g = np.random.RandomState(11)
    N, d, n, m, r, s, l = 4096, 40, 24, 8, 16, 4, 2048
    nf = 5
    rows = np.repeat(np.arange(N), nf)
    cols = np.concatenate([g.choice(d, nf, replace=False) for _ in range(N)])
    X = sp.csr_matrix((np.ones(N * nf, np.float32), (rows, cols)), shape=(N, d))
    a1 = g.randint(0, n, N).astype(np.int32)
    a2 = g.randint(0, n, N).astype(np.int32)
    data = DatasetManager.from_arrays(X, a1, a2, n_entities=n)
    runs = {}
    for hc in ("off", "on"):
        ind = ReconstructInducer(data, {"train": {}}, np.random.RandomState(2), 1, 0.1, l, r, m, s,
                                 0.0, 0.0, "adagrad", "tiny", dec, False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=1, kernel_forms={"heavy_chunk": hc})
        ind.learn(verbose=False)
        torch.cuda.synchronize()
        ind.engine.check()
        assert ind.engine.kernel_forms_in_use()["heavy_chunk"] == hc
        runs[hc] = ({k: v.detach().cpu().double().numpy() for k, v in
                     ind.modelFunc.named_params().items()}, np.array(ind.epoch_costs))
        ind._drop_engine()
    tr = O.OracleTrainer(dec, X, a1, a2, data.negSamplingCum, np.random.RandomState(2), m, r, s, l,
                         lr=0.1, alpha=1.0)
    want_c = np.array([tr.epoch()[0]])
    for hc, (p, c) in runs.items():
        np.testing.assert_allclose(c, want_c, rtol=2e-5, atol=2e-5)
        for k, want in tr.params.items():
            err = np.abs(p[k] - want)
            assert np.all(err <= 2e-4 + 2e-3 * np.abs(want)), f"{hc} {k}: max err {err.max():.3e}"
