"""The CPU oracle pinned against golden vectors produced by the reference's own model code
(oracle/gen_golden.py) and against finite differences."""
import glob
import os

import numpy as np
import pytest
import scipy.sparse as sp

import rae_oracle as O
from conftest import GOLDEN

CASES = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
               if "sampler" not in p and "c1_sample" not in p)   # c1: a dataset, not a golden run


def load_case(path):
    z = np.load(path)
    cfg = {k: z[k].item() if z[k].shape == () else z[k] for k in z.files}
    cfg["decoder"] = str(z["decoder"])
    cfg["optimizer"] = str(z["optimizer"])
    X = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(int(z["N"]), int(z["d"])))
    return z, cfg, X


def make_trainer(z, cfg, X):
    return O.OracleTrainer(cfg["decoder"], X, z["args1"], z["args2"], z["cum"],
                           np.random.RandomState(int(z["seed"])), int(z["m"]), int(z["r"]),
                           int(z["s"]), int(z["l"]), lr=float(z["lr"]), alpha=float(z["alpha"]),
                           lambda1=float(z["l1"]), lambda2=float(z["l2"]),
                           optimizer=cfg["optimizer"], ext_reg=bool(int(z["ext_reg"])))


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[:-4] for p in CASES])
def test_oracle_matches_reference_golden(path):
    z, cfg, X = load_case(path)
    tr = make_trainer(z, cfg, X)
    # init + RNG draw order (bit-exact)
    for k, v in tr.params.items():
        assert np.array_equal(v, z["init_" + k]), k
    # the CDF (bit-exact)
    assert np.array_equal(O.neg_sampling_cum(z["freqs"]), z["cum"])
    l = int(z["l"])
    res = O.train_step_grads(cfg["decoder"], tr.params, X[:l], z["args1"][:l], z["args2"][:l],
                             z["neg1_e0"][:, :l], z["neg2_e0"][:, :l], alpha=float(z["alpha"]),
                             lambda1=float(z["l1"]), lambda2=float(z["l2"]),
                             adjust=l / int(z["N"]), ext_reg=bool(int(z["ext_reg"])))
    assert abs(res.cost - float(z["step0_cost"])) < 1e-12
    np.testing.assert_allclose(res.scores, z["step0_scores"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(res.P, z["step0_P"], rtol=0, atol=1e-14)
    for k, g in res.grads.items():
        np.testing.assert_allclose(g, z["step0_grad_" + k], rtol=1e-9, atol=1e-15, err_msg=k)
    for ep in range(int(z["epochs"])):
        costs, err = tr.epoch()
        np.testing.assert_allclose(costs, z["costs"][ep], rtol=1e-10, atol=1e-12)
        assert abs(err - z["errs"][ep]) < 1e-10
    for k, v in tr.params.items():
        np.testing.assert_allclose(v, z["final_" + k], rtol=1e-7, atol=1e-11, err_msg=k)
        if cfg["optimizer"] == "adagrad":
            np.testing.assert_allclose(tr.acc[k], z["final_acc_" + k], rtol=1e-7, atol=1e-15)
    labels, probs = tr.labels()
    assert np.array_equal(labels, z["labels"])
    np.testing.assert_allclose(probs, z["probs"], rtol=0, atol=1e-12)


def test_oracle_sampler_matches_reference():
    z = np.load(os.path.join(GOLDEN, "sampler.npz"))
    cum = O.neg_sampling_cum(z["freqs"])
    assert np.array_equal(cum, z["cum"])
    rng = np.random.RandomState(int(z["seed"]))
    a = O.negative_samples(rng, cum, int(z["N"]), int(z["s"]))
    b = O.negative_samples(rng, cum, int(z["N"]), int(z["s"]))
    assert np.array_equal(a, z["neg1"]) and np.array_equal(b, z["neg2"])


@pytest.mark.parametrize("decoder", ["sp", "rescal", "rescal+sp"])
@pytest.mark.parametrize("lam", [(0.0, 0.0), (0.01, 0.1)])
def test_oracle_gradients_finite_difference(decoder, lam):
    g = np.random.RandomState(3)
    N, d, n, m, r, s, l = 6, 10, 7, 3, 4, 2, 3
    X = sp.csr_matrix((g.rand(N, d) < 0.3).astype(np.float32))
    e1, e2 = g.randint(0, n, l), g.randint(0, n, l)
    n1, n2 = g.randint(0, n, (s, l)), g.randint(0, n, (s, l))
    p = O.init_params(np.random.RandomState(1), decoder, d, m, n, r)
    for k in p:          # move away from the symmetric init so all terms matter
        p[k] = p[k] + 0.3 * g.standard_normal(p[k].shape)
    kw = dict(alpha=0.7, lambda1=lam[0], lambda2=lam[1], adjust=0.5, ext_reg=True)
    res = O.train_step_grads(decoder, p, X[:l], e1, e2, n1, n2, **kw)
    eps = 1e-6
    for k in p:
        flat = p[k].reshape(-1)
        idx = g.choice(flat.size, size=min(12, flat.size), replace=False)
        for i in idx:
            old = flat[i]
            if lam[0] and abs(old) < 1e-4:
                continue        # |x| kink
            flat[i] = old + eps
            cp = O.train_step_grads(decoder, p, X[:l], e1, e2, n1, n2, **kw).cost
            flat[i] = old - eps
            cm = O.train_step_grads(decoder, p, X[:l], e1, e2, n1, n2, **kw).cost
            flat[i] = old
            fd = (cp - cm) / (2 * eps)
            an = res.grads[k].reshape(-1)[i]
            assert abs(fd - an) < 1e-6 + 1e-5 * abs(fd), (decoder, k, i, fd, an)


def test_oracle_zero_grad_rows_unchanged():
    """The exactness fact behind the sparse update: rows with zero gradient
    are bit-unchanged by the dense AdaGrad sweep."""
    p = {"A": np.random.RandomState(0).standard_normal((5, 3))}
    acc = {"A": np.abs(np.random.RandomState(1).standard_normal((5, 3)))}
    acc["A"][0] = 0.0
    g = {"A": np.zeros((5, 3))}
    g["A"][2] = 1.0
    before = p["A"].copy()
    O.adagrad_apply(p, acc, g, 0.1)
    assert np.array_equal(p["A"][[0, 1, 3, 4]], before[[0, 1, 3, 4]])
    assert not np.array_equal(p["A"][2], before[2])


def test_bf16_round_matches_torch_bfloat16():
    """The oracle's bf16 operand emulation rounds exactly as a float32 -> bfloat16 conversion
    (round to nearest, ties to even) -- the v_mfma_f32_16x16x32_bf16 operand rounding."""
    import torch
    g = np.random.RandomState(0)
    x = np.concatenate([g.standard_normal(10000) * 10.0 ** g.randint(-8, 8, 10000),
                        [0.0, -0.0, 1.0, 1.00390625, 1.01171875, 65504.0, 1e-40]])
    want = torch.as_tensor(x.astype(np.float32)).to(torch.bfloat16).to(torch.float64).numpy()
    assert np.array_equal(O.bf16_round(x), want)
