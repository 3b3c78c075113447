"""CPU oracle for the discrete-state relation-VAE training step.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (relation-autoencoder_amd/)
imports this module; only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, and only as the checker / the timed CPU baseline.

It is a float64 numpy restatement of the reference's (Theano) graph, written from
the reference's source (citations are /root/reference-relative file:line):

* data layout / batch slicing ...... learning/OieData.py:72-90, learning/OieInduction.py:96-98,146-149,186-188
* negative-sampling CDF ............ learning/OieData.py:53-59,115-118
* negative sampler ................. learning/NegativeExampleGenerator.py:14-32
* parameter init + RNG order ....... learning/models/encoders/RelationClassifier.py:24-25,
                                     learning/OieModel.py:49-63,103-105,
                                     learning/models/decoders/{SelectionalPreferences.py:13-19,
                                     Bilinear.py:14-17, BilinearPlusSP.py:14-23}
* encoder ........................... learning/models/encoders/RelationClassifier.py:28-48
* entropy + loss ................... learning/OieModel.py:80-90
* decoders ......................... SelectionalPreferences.py:30-51, Bilinear.py:28-79, BilinearPlusSP.py:34-102
* regularisers + cost .............. learning/OieModel.py:54-62, decoders' get_l{1,2}_*, learning/OieInduction.py:131-135
* optimisers ....................... learning/Optimizers.py:18-52

The gradients are derived analytically (the reference uses Theano's T.grad); they are
pinned against the reference's own modules executed eagerly (oracle/gen_golden.py ->
tests/golden/) and against central finite differences (tests/test_oracle.py).

It follows Theano's *dense* schedule: every gradient is a dense array of the
parameter's shape and every optimiser step sweeps every parameter, exactly as
``theano.function(..., updates=AdaGrad.update(...))`` does.  That is also what makes it
the honest CPU baseline for bench.py.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp

# settings.py:23-24 -- encoder init range
LOW, HIGH = -1.0e-3, 1.0e-3
# learning/Optimizers.py:31 -- AdaGrad epsilon
ADAGRAD_EPS = 1e-6

DECODERS = ("sp", "rescal", "rescal+sp")


# --------------------------------------------------------------------------------------
# data: CDF, sampler, batch slicing
# --------------------------------------------------------------------------------------
def neg_sampling_cum(freqs, power: float = 0.75) -> np.ndarray:
    """learning/OieData.py:57-59 + :115-118.

    ``norm1 = float(sum(f**p for f in freqs))`` is a sequential Python sum, the
    normalised list is cumsum'd sequentially; np.cumsum is sequential too, so the
    last element of the un-normalised cumsum reproduces ``norm1`` bit for bit.
    """
    powered = np.array([float(f) ** power for f in freqs], dtype=np.float64)
    norm1 = float(np.cumsum(powered)[-1]) if len(powered) else 0.0
    distr = powered / norm1
    return np.cumsum(distr)


def negative_samples(rng: np.random.RandomState, cum: np.ndarray, num_positive: int,
                     num_neg: int) -> np.ndarray:
    """learning/NegativeExampleGenerator.py:24,32.

    ``np.array(map(cum.searchsorted, rng.uniform(0, cum[-1], n*s)), dtype=int32)``
    reshaped to (s, n).  searchsorted's default side is 'left'; the vectorised call is
    element-wise identical to the per-scalar map.
    """
    u = rng.uniform(0, cum[-1], num_positive * num_neg)
    return np.asarray(cum.searchsorted(u), dtype=np.int32).reshape((num_neg, num_positive))


def batch_count(num_examples: int, batch_size: int) -> int:
    """learning/OieInduction.py:98 -- Py2 integer division: the tail batch is dropped."""
    return num_examples // batch_size


def batch_rows(batch_index: int, batch_size: int) -> slice:
    """learning/OieInduction.py:147-149 -- givens slice [b*l, (b+1)*l)."""
    return slice(batch_index * batch_size, (batch_index + 1) * batch_size)


# --------------------------------------------------------------------------------------
# parameters
# --------------------------------------------------------------------------------------
def param_names(decoder: str):
    """Parameter list order: learning/OieModel.py:50,63 + decoders' get_parameters()
    (SelectionalPreferences.py:21-22, Bilinear.py:19-20, BilinearPlusSP.py:31-32)."""
    dec = {"sp": ["A", "C1", "C2", "Ab"],
           "rescal": ["R", "A", "Ab"],
           "rescal+sp": ["C", "A", "Ab", "C1", "C2"]}[decoder]
    return ["W", "Wb"] + dec


def reg_names(decoder: str, ext_reg: bool):
    """Parameters inside L1/L2: W always (OieModel.py:54-56), decoder weights if
    extended_regularizer (OieModel.py:60-62; SelectionalPreferences.py:24-28,
    Bilinear.py:22-26, BilinearPlusSP.py:25-29).  Never A, Ab, Wb."""
    dec = {"sp": ["C1", "C2"], "rescal": ["R"], "rescal+sp": ["C1", "C2", "C"]}[decoder]
    return ["W"] + (dec if ext_reg else [])


def init_params(rng: np.random.RandomState, decoder: str, d: int, m: int, n: int, r: int,
                dtype=np.float64) -> dict:
    """Draw order on the single RandomState:
    W (RelationClassifier.py:24), A (OieModel.py:105), then the decoder's weights
    (SP: C1, C2 -- SelectionalPreferences.py:13-14; RESCAL: R -- Bilinear.py:14;
    hybrid: C, C1, C2 -- BilinearPlusSP.py:14-17).  Wb, Ab start at zero."""
    p = {}
    p["W"] = np.asarray(rng.uniform(low=LOW, high=HIGH, size=(d, m)), dtype=dtype)
    p["Wb"] = np.zeros(m, dtype=dtype)
    p["A"] = np.asarray(rng.uniform(-0.01, 0.01, size=(n, r)), dtype=dtype)
    sd = math.sqrt(0.1)
    if decoder == "sp":
        p["C1"] = np.asarray(rng.normal(0, sd, size=(r, m)), dtype=dtype)
        p["C2"] = np.asarray(rng.normal(0, sd, size=(r, m)), dtype=dtype)
    elif decoder == "rescal":
        p["R"] = np.asarray(rng.normal(0, sd, size=(r, r, m)), dtype=dtype)
    elif decoder == "rescal+sp":
        p["C"] = np.asarray(rng.normal(0, sd, size=(r, r, m)), dtype=dtype)
        p["C1"] = np.asarray(rng.normal(0, sd, size=(r, m)), dtype=dtype)
        p["C2"] = np.asarray(rng.normal(0, sd, size=(r, m)), dtype=dtype)
    else:
        raise ValueError(f"unknown decoder {decoder!r}")
    p["Ab"] = np.zeros(n, dtype=dtype)
    return {k: p[k] for k in param_names(decoder)}


# --------------------------------------------------------------------------------------
# numerics helpers (Theano's stabilising rewrites: log(softmax) -> logsoftmax,
# log(sigmoid(x)) -> -softplus(-x))
# --------------------------------------------------------------------------------------
def _log_sigmoid(x):
    return -np.logaddexp(0.0, -x)


def _sigmoid(x):
    return np.exp(-np.logaddexp(0.0, -x))


def encoder_forward(X, W, Wb):
    """RelationClassifier.py:35-36,45-47: S = X.W + Wb, P = softmax(S), labels = argmax(S)."""
    S = np.asarray(X @ W) + Wb
    mx = S.max(axis=1, keepdims=True)
    Z = np.exp(S - mx)
    lse = np.log(Z.sum(axis=1, keepdims=True))
    logP = S - mx - lse
    P = np.exp(logP)
    return S, P, logP


def label(X, W, Wb):
    """comp_probs_and_labels (RelationClassifier.py:39-48): (argmax(S) int64, softmax(S)).
    np.argmax returns the first maximum, as Theano's argmax does."""
    S, P, _ = encoder_forward(X, W, Wb)
    return np.argmax(S, axis=1).astype(np.int64), P


# --------------------------------------------------------------------------------------
# one training step: forward, loss, dense gradients
# --------------------------------------------------------------------------------------
@dataclass
class StepResult:
    cost: float                 # scalar returned by func['train']
    scores: np.ndarray          # all_scores vector (4l + 2ls,) in the reference's order
    P: np.ndarray               # (l, m) relation probabilities
    H: np.ndarray               # (l,) alpha-scaled entropy
    grads: dict = field(default_factory=dict)   # dense, param-shaped


def bf16_round(x):
    """Round to bfloat16 (nearest even, via float32) and back to float64: the operand
    rounding of v_mfma_f32_16x16x32_bf16 (no NaN/inf inputs here)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def _decoder_forward_backward(decoder, p, P, H, e1, e2, neg1, neg2, D, bf16=False):
    """Returns (scores_without_entropy_parts, dP, grads-dict) for the decoder.

    bf16 (bilinear decoders only): emulate rae_config.mfma_bf16 -- the three R contractions
    take bf16-rounded operands (fp32 / here float64 accumulation), exactly where the MI355X
    kernels round: M = P.R (k_bil_mt: bf16 P and R), dP = sum_ij U_ij R_ij (U = x a2^T + a1 y^T
    formed in fp32, then rounded), dR = sum_b P_b U_b (U formed from bf16 copies of x, a1, a2,
    y, then rounded; P bf16).  Not the reference's arithmetic: it measures how far bf16
    operands alone move a trajectory, which is what the bf16 path's tolerance is derived from
    (tests/test_gpu_fullscale.py)."""
    A, Ab = p["A"], p["Ab"]
    l = P.shape[0]
    s = neg1.shape[0]
    g = {}
    gA = np.zeros_like(A)
    gAb = np.zeros_like(Ab)
    a1 = A[e1]
    n1e = A[neg1]       # (s, l, r)  SelectionalPreferences.py:41
    n2e = A[neg2]

    if decoder == "sp":
        C1, C2 = p["C1"], p["C2"]
        wC1 = P @ C1.T                              # SelectionalPreferences.py:31
        wC2 = P @ C2.T                              # :32
        left = np.einsum("br,br->b", wC1, a1)       # :34
        right = np.einsum("br,br->b", wC2, a1)      # :35  (A[args1] twice: reference behaviour)
        one = left + right                          # :36
        u = np.concatenate([one + Ab[e1], one + Ab[e2]])            # :38
        negL = np.einsum("br,tbr->tb", wC1, n1e)    # :43 (transposed to (s,l))
        negR = np.einsum("br,tbr->tb", wC2, n2e)    # :44
        negOne = negL + right[None, :]              # :46
        negTwo = negR + left[None, :]               # :47
        gneg = np.concatenate([negOne + Ab[neg1], negTwo + Ab[neg2]])  # (2s, l) :48
        pos = _log_sigmoid(u)
        negs = _log_sigmoid(-gneg).ravel()          # s-major flatten :49-50
        # ---- backward
        du = -_sigmoid(-u) / D
        du1, du2 = du[:l], du[l:]
        dg = _sigmoid(gneg) / D
        dg1, dg2 = dg[:s], dg[s:]                   # (s, l)
        d_left = du1 + du2 + dg2.sum(0)
        d_right = du1 + du2 + dg1.sum(0)
        dwC1 = d_left[:, None] * a1 + np.einsum("tb,tbr->br", dg1, n1e)
        dwC2 = d_right[:, None] * a1 + np.einsum("tb,tbr->br", dg2, n2e)
        np.add.at(gA, e1, d_left[:, None] * wC1 + d_right[:, None] * wC2)
        np.add.at(gA, neg1, dg1[..., None] * wC1[None])
        np.add.at(gA, neg2, dg2[..., None] * wC2[None])
        np.add.at(gAb, e1, du1)
        np.add.at(gAb, e2, du2)
        np.add.at(gAb, neg1, dg1)
        np.add.at(gAb, neg2, dg2)
        g["C1"] = dwC1.T @ P
        g["C2"] = dwC2.T @ P
        dP = dwC1 @ C1 + dwC2 @ C2
    else:
        Rk = p["R"] if decoder == "rescal" else p["C"]      # (r, r, m)
        r_ = Rk.shape[0]
        a2 = A[e2]
        # M_b = sum_k P_bk R[:,:,k]  (Bilinear.py:33 / BilinearPlusSP.py:37) as one GEMM
        Rb = (bf16_round(Rk) if bf16 else Rk).reshape(r_ * r_, -1)
        M = ((bf16_round(P) if bf16 else P) @ Rb.T).reshape(l, r_, r_)
        Ma2 = np.einsum("bij,bj->bi", M, a2)        # M a2
        MTa1 = np.einsum("bij,bi->bj", M, a1)       # M^T a1
        one = np.einsum("bi,bi->b", a1, Ma2)        # Bilinear.py:58-59
        negOne = np.einsum("tbi,bi->bt", n1e, Ma2)  # Bilinear.py:68-69   (l, s)
        negTwo = np.einsum("bj,tbj->bt", MTa1, n2e)  # Bilinear.py:78-79  (l, s)
        if decoder == "rescal+sp":
            C1, C2 = p["C1"], p["C2"]
            wC1 = P @ C1.T                          # BilinearPlusSP.py:35-36
            wC2 = P @ C2.T
            sp1 = np.einsum("br,br->b", wC1, a1)     # :70
            sp2 = np.einsum("br,br->b", wC2, a2)     # :71
            one = one + sp1 + sp2                    # :72
            negOne = negOne + np.einsum("br,tbr->bt", wC1, n1e) + sp2[:, None]   # :85-87
            negTwo = negTwo + np.einsum("br,tbr->bt", wC2, n2e) + sp1[:, None]   # :100-102
        u = np.concatenate([one + Ab[e1], one + Ab[e2]])
        gneg = np.concatenate([negOne + Ab[neg1].T, negTwo + Ab[neg2].T])   # (2l, s) b-major
        pos = _log_sigmoid(u)
        negs = _log_sigmoid(-gneg).ravel()
        # ---- backward
        du = -_sigmoid(-u) / D
        du1, du2 = du[:l], du[l:]
        dOne = du1 + du2
        dg = _sigmoid(gneg) / D
        dg1, dg2 = dg[:l], dg[l:]                   # (l, s)
        x = dOne[:, None] * a1 + np.einsum("bt,tbi->bi", dg1, n1e)   # left factor of dM
        y = np.einsum("bt,tbj->bj", dg2, n2e)                         # right factor (with a1)
        # dM_b = x_b a2_b^T + a1_b y_b^T
        g_a1 = dOne[:, None] * Ma2 + np.einsum("bij,bj->bi", M, y)
        g_a2 = np.einsum("bij,bi->bj", M, x)
        g_n1 = dg1.T[..., None] * Ma2[None]          # (s, l, r)
        g_n2 = dg2.T[..., None] * MTa1[None]
        # U_b = dCost/dM_b = x_b a2_b^T + a1_b y_b^T;  dP_bk = <U_b, R_k>;  dR_k = sum_b P_bk U_b
        U = (x[:, :, None] * a2[:, None, :] + a1[:, :, None] * y[:, None, :]).reshape(l, -1)
        if bf16:
            dP = bf16_round(U) @ Rb
            bx, b1, b2, by = bf16_round(x), bf16_round(a1), bf16_round(a2), bf16_round(y)
            Uf = (bx[:, :, None] * b2[:, None, :] + b1[:, :, None] * by[:, None, :]).reshape(l, -1)
            gR = (bf16_round(Uf).T @ bf16_round(P)).reshape(r_, r_, -1)
        else:
            dP = U @ Rb
            gR = (U.T @ P).reshape(r_, r_, -1)
        if decoder == "rescal+sp":
            c_a1 = dOne + dg2.sum(1)     # <wC1,a1> appears in one and in every negRight
            c_a2 = dOne + dg1.sum(1)     # <wC2,a2> appears in one and in every negLeft
            dwC1 = c_a1[:, None] * a1 + np.einsum("bt,tbr->br", dg1, n1e)
            dwC2 = c_a2[:, None] * a2 + np.einsum("bt,tbr->br", dg2, n2e)
            g_a1 = g_a1 + c_a1[:, None] * wC1
            g_a2 = g_a2 + c_a2[:, None] * wC2
            g_n1 = g_n1 + dg1.T[..., None] * wC1[None]
            g_n2 = g_n2 + dg2.T[..., None] * wC2[None]
            g["C1"] = dwC1.T @ P
            g["C2"] = dwC2.T @ P
            dP = dP + dwC1 @ C1 + dwC2 @ C2
            g["C"] = gR
        else:
            g["R"] = gR
        np.add.at(gA, e1, g_a1)
        np.add.at(gA, e2, g_a2)
        np.add.at(gA, neg1, g_n1)
        np.add.at(gA, neg2, g_n2)
        np.add.at(gAb, e1, du1)
        np.add.at(gAb, e2, du2)
        np.add.at(gAb, neg1, dg1.T)
        np.add.at(gAb, neg2, dg2.T)

    g["A"] = gA
    g["Ab"] = gAb
    return pos, negs, dP, g


def train_step_grads(decoder: str, p: dict, X, e1, e2, neg1, neg2, *, alpha: float,
                     lambda1: float = 0.0, lambda2: float = 0.0, adjust: float = 0.0,
                     ext_reg: bool = True, denom: float | None = None,
                     bf16: bool = False) -> StepResult:
    """Forward + loss + dense gradients of one ``func['train']`` call.

    cost = -mean(all_scores) + lambda1*adjust*L1 + lambda2*adjust*L2
    (learning/OieModel.py:90, learning/OieInduction.py:131-135), all_scores =
    [logsig(u) (2l), H (l), H (l), logsig(-g) (2ls)] (SelectionalPreferences.py:39,50;
    Bilinear.py:39,48; BilinearPlusSP.py:47,56).
    """
    e1 = np.asarray(e1, dtype=np.int64)
    e2 = np.asarray(e2, dtype=np.int64)
    neg1 = np.asarray(neg1, dtype=np.int64)
    neg2 = np.asarray(neg2, dtype=np.int64)
    l = e1.shape[0]
    s = neg1.shape[0]
    D = 4 * l + 2 * l * s
    if denom is not None:       # data-parallel emulation: a rank's slice of a global batch
        D = denom
    S, P, logP = encoder_forward(X, p["W"], p["Wb"])
    H = alpha * -(P * logP).sum(axis=1)                     # OieModel.py:81
    pos, negs, dP, g = _decoder_forward_backward(decoder, p, P, H, e1, e2, neg1, neg2, D,
                                                 bf16=bf16)
    scores = np.concatenate([pos, H, H, negs])
    assert scores.shape[0] == 4 * l + 2 * l * s
    cost = -float(scores.sum()) / D                         # OieModel.py:90 (mean)
    # entropy: cost has -(2/D) * sum_b H_b; dH_b/dP_bk = -alpha (logP_bk + 1)
    dP = dP + (2.0 * alpha / D) * (logP + 1.0)
    dS = P * (dP - (P * dP).sum(axis=1, keepdims=True))     # softmax backward
    g["W"] = np.asarray(X.T @ dS)
    g["Wb"] = dS.sum(axis=0)
    # regularisers (OieInduction.py:131-135)
    if lambda1 != 0.0 or lambda2 != 0.0:
        L1 = L2 = 0.0
        for name in reg_names(decoder, ext_reg):
            w = p[name]
            L1 += float(np.abs(w).sum())
            L2 += float(np.square(w).sum())
            g[name] = g[name] + lambda1 * adjust * np.sign(w) + 2.0 * lambda2 * adjust * w
        cost += lambda1 * L1 * adjust + lambda2 * L2 * adjust
    grads = {k: g[k] for k in param_names(decoder)}
    return StepResult(cost=cost, scores=scores, P=P, H=H, grads=grads)


# --------------------------------------------------------------------------------------
# optimisers
# --------------------------------------------------------------------------------------
def adagrad_apply(p: dict, acc: dict, grads: dict, lr: float) -> None:
    """learning/Optimizers.py:29-32: acc <- acc + g^2; p <- p - lr*g/(sqrt(acc)+1e-6),
    using the *new* accumulator, for every parameter (dense sweep)."""
    for k, gk in grads.items():
        acc[k] += np.square(gk)
        p[k] -= lr * gk / (np.sqrt(acc[k]) + ADAGRAD_EPS)


def sgd_apply(p: dict, grads: dict, lr: float) -> None:
    """learning/Optimizers.py:48-51."""
    for k, gk in grads.items():
        p[k] -= lr * gk


# --------------------------------------------------------------------------------------
# a whole trainer (ReconstructInducer.learn restated, learning/OieInduction.py:172-203)
# --------------------------------------------------------------------------------------
@dataclass
class OracleTrainer:
    decoder: str
    X: sp.csr_matrix            # train split feature matrix (N, d), float32 values
    args1: np.ndarray
    args2: np.ndarray
    cum: np.ndarray             # negative-sampling CDF
    rng: np.random.RandomState
    m: int
    r: int
    s: int
    l: int
    lr: float = 0.1
    alpha: float = 1.0
    lambda1: float = 0.0
    lambda2: float = 0.0
    optimizer: str = "adagrad"
    ext_reg: bool = True
    dtype: type = np.float64
    bf16: bool = False          # emulate the bf16-operand R contractions (see bf16_round)

    def __post_init__(self):
        n = len(self.cum)
        d = self.X.shape[1]
        self.params = init_params(self.rng, self.decoder, d, self.m, n, self.r, self.dtype)
        self.acc = {k: np.zeros_like(v) for k, v in self.params.items()}
        self.N = self.X.shape[0]
        self.nb = batch_count(self.N, self.l)
        self.adjust = float(self.l) / float(self.N)           # OieInduction.py:131

    def train_batch(self, b: int, neg1: np.ndarray, neg2: np.ndarray) -> float:
        rows = batch_rows(b, self.l)
        res = train_step_grads(self.decoder, self.params, self.X[rows], self.args1[rows],
                               self.args2[rows], neg1, neg2, alpha=self.alpha,
                               lambda1=self.lambda1, lambda2=self.lambda2,
                               adjust=self.adjust, ext_reg=self.ext_reg, bf16=self.bf16)
        if self.optimizer == "adagrad":
            adagrad_apply(self.params, self.acc, res.grads, self.lr)
        elif self.optimizer == "sgd":
            sgd_apply(self.params, res.grads, self.lr)
        else:
            raise Exception("Optimizer '{}' not implemented".format(self.optimizer))
        return res.cost

    def epoch(self):
        """One epoch: neg1 then neg2 drawn for all N (OieInduction.py:183-184), then
        batches in order; returns (per-batch costs, err = sequential sum)."""
        neg1 = negative_samples(self.rng, self.cum, self.N, self.s)
        neg2 = negative_samples(self.rng, self.cum, self.N, self.s)
        costs = []
        err = 0.0
        for b in range(self.nb):
            cols = batch_rows(b, self.l)
            c = self.train_batch(b, neg1[:, cols], neg2[:, cols])
            costs.append(c)
            err += c
        return np.array(costs), err

    def labels(self, X=None):
        X = self.X if X is None else X
        nrows = batch_count(X.shape[0], self.l) * self.l       # tail dropped (OieInduction.py:337)
        return label(X[:nrows], self.params["W"], self.params["Wb"])
