"""CPU baseline: the reference's Theano training step restated on torch (CPU, all threads).

TEST / MEASUREMENT INFRASTRUCTURE ONLY.  Nothing in relation-autoencoder_amd/ imports this
module; bench.py's cpu_baseline leg times it and tests/test_cpu_ref.py pins it against the
float64 oracle (oracle/rae_oracle.py, itself pinned to the reference's golden vectors).

Theano cannot run here (Python-2-only trainer, no Theano install), so the
baseline is this restatement of what ``theano.function(..., updates=AdaGrad.update(...))``
executes per ``func['train']`` call (learning/OieInduction.py:146-149,189):

* the forward graph of learning/models/encoders/RelationClassifier.py:35-36,
  learning/OieModel.py:81,90 and the decoder's get_scores (SelectionalPreferences.py:30-51,
  Bilinear.py:28-79, BilinearPlusSP.py:34-102), with the tensors Theano builds (the
  (s, l, r) negative-row tensors, the (l, r, r) weighted RESCAL tensor);
* T.grad of the cost (learning/Optimizers.py:27) -- here torch autograd, which, like
  Theano, produces DENSE gradients: dW (d, m) from the sparse dot, dA (n, r) / dAb (n) by
  inc-subtensor scatter-adds into zeros;
* the dense AdaGrad / SGD sweep over every parameter (learning/Optimizers.py:29-33,48-51).

Runs in float64 (Theano's default floatX, which the reference never sets) or float32
(THEANO_FLAGS=floatX=float32), with torch.set_num_threads() chosen by the caller.
"""
from __future__ import annotations

import math

import numpy as np
import torch

ADAGRAD_EPS = 1e-6          # learning/Optimizers.py:31
LOW, HIGH = -1.0e-3, 1.0e-3  # settings.py:23-24


def param_names(decoder):
    """learning/OieModel.py:50,63 + the decoders' get_parameters()."""
    return ["W", "Wb"] + {"sp": ["A", "C1", "C2", "Ab"], "rescal": ["R", "A", "Ab"],
                          "rescal+sp": ["C", "A", "Ab", "C1", "C2"]}[decoder]


def init_params(rng, decoder, d, m, n, r, dtype):
    """Same RandomState draw order as the reference (W, A, decoder weights)."""
    p = {"W": rng.uniform(LOW, HIGH, size=(d, m)), "Wb": np.zeros(m)}
    p["A"] = rng.uniform(-0.01, 0.01, size=(n, r))
    sd = math.sqrt(0.1)
    if decoder == "sp":
        p["C1"] = rng.normal(0, sd, size=(r, m))
        p["C2"] = rng.normal(0, sd, size=(r, m))
    elif decoder == "rescal":
        p["R"] = rng.normal(0, sd, size=(r, r, m))
    else:
        p["C"] = rng.normal(0, sd, size=(r, r, m))
        p["C1"] = rng.normal(0, sd, size=(r, m))
        p["C2"] = rng.normal(0, sd, size=(r, m))
    p["Ab"] = np.zeros(n)
    return {k: torch.tensor(p[k], dtype=dtype).requires_grad_(True) for k in param_names(decoder)}


def _log_sigmoid(x):
    return torch.nn.functional.logsigmoid(x)     # Theano's log(sigmoid) -> -softplus(-x)


def cost_graph(decoder, p, X, e1, e2, neg1, neg2, alpha):
    """The symbolic cost of one batch (learning/OieModel.py:65-92), eagerly."""
    W, Wb, A, Ab = p["W"], p["Wb"], p["A"], p["Ab"]
    l, s = e1.shape[0], neg1.shape[0]
    S = torch.sparse.mm(X, W) + Wb                                   # RelationClassifier.py:35
    logP = torch.log_softmax(S, dim=1)                               # :36 (+ log rewrite)
    P = logP.exp()
    H = alpha * -(logP * P).sum(dim=1)                               # OieModel.py:81
    a1 = A[e1]
    n1e = A[neg1.reshape(-1)].reshape(s, l, -1)                      # SelectionalPreferences.py:41
    n2e = A[neg2.reshape(-1)].reshape(s, l, -1)                      # :42
    if decoder == "sp":
        wC1 = P @ p["C1"].T                                          # :31
        wC2 = P @ p["C2"].T                                          # :32
        left = (wC1 * a1).sum(1)                                     # :34
        right = (wC2 * a1).sum(1)                                    # :35 (A[args1] twice)
        one = left + right                                           # :36
        u = torch.cat([one + Ab[e1], one + Ab[e2]])                  # :38
        negOne = (wC1[None] * n1e).sum(2) + right[None]              # :43,46
        negTwo = (wC2[None] * n2e).sum(2) + left[None]               # :44,47
        g = torch.cat([negOne + Ab[neg1], negTwo + Ab[neg2]])        # :48 (2s, l)
        negs = _log_sigmoid(-g).reshape(-1)                          # :49
    else:
        Rk = p["R"] if decoder == "rescal" else p["C"]
        a2 = A[e2]
        M = torch.einsum("bk,ijk->bij", P, Rk)                       # Bilinear.py:33 (l, r, r)
        Ma2 = torch.einsum("bij,bj->bi", M, a2)
        MTa1 = torch.einsum("bij,bi->bj", M, a1)
        one = (a1 * Ma2).sum(1)                                      # Bilinear.py:58-59
        negOne = torch.einsum("tbi,bi->bt", n1e, Ma2)                # :68-69
        negTwo = torch.einsum("bj,tbj->bt", MTa1, n2e)               # :78-79
        if decoder == "rescal+sp":
            wC1 = P @ p["C1"].T                                      # BilinearPlusSP.py:35-36
            wC2 = P @ p["C2"].T
            sp1 = (wC1 * a1).sum(1)                                  # :70
            sp2 = (wC2 * a2).sum(1)                                  # :71
            one = one + sp1 + sp2                                    # :72
            negOne = negOne + torch.einsum("br,tbr->bt", wC1, n1e) + sp2[:, None]   # :85-87
            negTwo = negTwo + torch.einsum("br,tbr->bt", wC2, n2e) + sp1[:, None]   # :100-102
        u = torch.cat([one + Ab[e1], one + Ab[e2]])
        g = torch.cat([negOne + Ab[neg1].T, negTwo + Ab[neg2].T])   # Bilinear.py:46 (2l, s)
        negs = _log_sigmoid(-g).reshape(-1)
    scores = torch.cat([_log_sigmoid(u), H, H, negs])                # :39,50
    return -scores.mean()                                            # OieModel.py:90


class DenseScheduleStep:
    """One func['train'] call at a time: forward, T.grad (dense), dense AdaGrad/SGD."""

    def __init__(self, decoder, params, lr=0.1, alpha=1.0, optimizer="adagrad"):
        self.decoder = decoder
        self.p = params
        self.names = param_names(decoder)
        self.lr = lr
        self.alpha = alpha
        self.optimizer = optimizer
        self.acc = {k: torch.zeros_like(v, requires_grad=False) for k, v in params.items()}

    def __call__(self, X, e1, e2, neg1, neg2):
        cost = cost_graph(self.decoder, self.p, X, e1, e2, neg1, neg2, self.alpha)
        grads = torch.autograd.grad(cost, [self.p[k] for k in self.names])   # Optimizers.py:27
        with torch.no_grad():
            for k, gk in zip(self.names, grads):
                pk = self.p[k]
                if gk.is_sparse:
                    gk = gk.to_dense()
                if self.optimizer == "adagrad":                      # Optimizers.py:30-32
                    ak = self.acc[k]
                    ak.addcmul_(gk, gk)
                    pk.addcdiv_(gk, ak.sqrt().add_(ADAGRAD_EPS), value=-self.lr)
                else:                                                # Optimizers.py:51
                    pk.add_(gk, alpha=-self.lr)
        return float(cost.detach())


def batch_csr(xfeats, rows, dtype):
    """The givens slice xFeats[b*l:(b+1)*l] (learning/OieInduction.py:147) as a torch
    sparse COO tensor (the layout torch.sparse.mm differentiates through)."""
    x = xfeats[rows].tocoo()
    idx = torch.tensor(np.vstack([x.row, x.col]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.tensor(x.data, dtype=dtype), x.shape).coalesce()
