"""Eager restatement of the Theano op semantics the reference's model files use.

TEST INFRASTRUCTURE ONLY (fixture generation in this container; never shipped, never
imported by the product path, never run on the GPU box).

Theano is a third-party dependency of the reference that is absent here (its version is
unpinned: README.md:8 names it, there is no requirements/lock file).  Per its published
semantics, the ops used on the hot path are restated below on torch float64 tensors, so
that the reference's *own* files -- learning/models/encoders/RelationClassifier.py,
learning/models/decoders/{Decoder,SelectionalPreferences,Bilinear,BilinearPlusSP}.py,
learning/Optimizers.py, learning/NegativeExampleGenerator.py -- execute unmodified and
produce golden vectors.  Symbolic graph building becomes eager evaluation; ``T.grad``
becomes reverse-mode autodiff (torch.autograd), which computes the same derivative.

Op semantics restated (Theano >= 0.9):
  theano.shared(v)          -> a leaf variable holding v (get_value/set_value)
  T.dot(a, b)               -> matrix product
  sparse.dot(X, W)          -> sparse x dense product (X densified; values as given)
  T.nnet.softmax(x)         -> row softmax
  T.nnet.sigmoid, T.log     -> elementwise
  T.batched_dot(a, b)       -> a[i] . b[i] per leading index (2-D: rowwise dot)
  T.batched_tensordot(a,b,axes=[[i],[j]]) -> per-batch tensordot over (i, j) (axes count
                               the batch axis 0, as in Theano)
  T.tensordot(a, b, axes)   -> numpy tensordot
  x.dimshuffle(*perm)       -> permute
  T.argmax(x, axis)         -> first maximum
"""
from __future__ import annotations

import sys
import types

import numpy as np
import torch

_DT = torch.float64


def _t(x):
    if isinstance(x, Var):
        return x.t
    if isinstance(x, torch.Tensor):
        return x
    a = np.asarray(x)
    if a.dtype.kind in "iu":
        return torch.as_tensor(a.astype(np.int64))
    return torch.as_tensor(a.astype(np.float64))


class Var:
    """A Theano variable evaluated eagerly."""
    __array_priority__ = 1000

    def __init__(self, t, name=None):
        self.t = t
        self.name = name

    # -- shared-variable API
    def get_value(self, borrow=False):
        return self.t.detach().cpu().numpy().copy()

    def set_value(self, v, borrow=False):
        self.t = torch.as_tensor(np.asarray(v, dtype=np.float64)).clone().requires_grad_(True)

    # -- tensor API
    @property
    def shape(self):
        return tuple(self.t.shape)

    @property
    def ndim(self):
        return self.t.dim()

    def dimshuffle(self, *perm):
        if len(perm) == 1 and isinstance(perm[0], (tuple, list)):
            perm = tuple(perm[0])
        return Var(self.t.permute(*perm))

    def flatten(self, ndim=1):
        return Var(self.t.reshape(-1))

    def reshape(self, shape):
        return Var(self.t.reshape(tuple(int(s) for s in shape)))

    def __getitem__(self, idx):
        if isinstance(idx, Var):
            idx = idx.t
        return Var(self.t[idx])

    def __add__(self, o):
        return Var(self.t + _t(o))

    __radd__ = __add__

    def __sub__(self, o):
        return Var(self.t - _t(o))

    def __rsub__(self, o):
        return Var(_t(o) - self.t)

    def __mul__(self, o):
        return Var(self.t * _t(o))

    __rmul__ = __mul__

    def __truediv__(self, o):
        return Var(self.t / _t(o))

    def __rtruediv__(self, o):
        return Var(_t(o) / self.t)

    def __neg__(self):
        return Var(-self.t)

    def __abs__(self):
        return Var(self.t.abs())


def _batched_tensordot(a, b, axes):
    (ia,), (ib,) = axes
    a, b = _t(a), _t(b)
    # move the contracted axis last / first (excluding batch axis 0)
    ar = a.movedim(ia, -1)
    br = b.movedim(ib, 1)
    # ar: (B, ..., K), br: (B, K, ...)
    B = ar.shape[0]
    ash = ar.shape[1:-1]
    bsh = br.shape[2:]
    out = torch.bmm(ar.reshape(B, -1, ar.shape[-1]), br.reshape(B, br.shape[1], -1))
    return Var(out.reshape((B,) + tuple(ash) + tuple(bsh)))


def _batched_dot(a, b):
    a, b = _t(a), _t(b)
    if a.dim() == 2 and b.dim() == 2:
        return Var((a * b).sum(1))
    return Var(torch.bmm(a, b))


def _tensordot(a, b, axes):
    a, b = _t(a), _t(b)
    return Var(torch.tensordot(a, b, dims=([ax for ax in axes[0]], [bx for bx in axes[1]])))


def _concatenate(xs, axis=0):
    return Var(torch.cat([_t(x) for x in xs], dim=axis))


def _grad(cost, params):
    gs = torch.autograd.grad(_t(cost), [p.t for p in params], retain_graph=True)
    return [Var(g) for g in gs]


def _sparse_dot(x, w):
    return Var(_t(x) @ _t(w))


def install():
    """Insert ``theano``, ``theano.tensor``, ``theano.tensor.nnet``, ``theano.sparse``
    into sys.modules."""
    theano = types.ModuleType("theano")
    theano.config = types.SimpleNamespace(floatX="float64")
    theano.shared = lambda value, name=None, borrow=False: Var(
        torch.as_tensor(np.asarray(value, dtype=np.float64)).clone().requires_grad_(True), name)

    T = types.ModuleType("theano.tensor")
    T.dot = lambda a, b: Var(_t(a) @ _t(b))
    T.batched_dot = _batched_dot
    T.batched_tensordot = _batched_tensordot
    T.tensordot = _tensordot
    T.concatenate = _concatenate
    T.log = lambda x: Var(torch.log(_t(x)))
    T.sqrt = lambda x: Var(torch.sqrt(_t(x)))
    T.sqr = lambda x: Var(_t(x) ** 2)
    T.sum = lambda x, axis=None: Var(_t(x).sum() if axis is None else _t(x).sum(axis))
    T.mean = lambda x, axis=None: Var(_t(x).mean() if axis is None else _t(x).mean(axis))
    T.argmax = lambda x, axis=None: Var(torch.as_tensor(np.argmax(_t(x).detach().numpy(), axis=axis)))
    T.grad = _grad
    nnet = types.ModuleType("theano.tensor.nnet")
    nnet.softmax = lambda x: Var(torch.softmax(_t(x), dim=1))
    nnet.sigmoid = lambda x: Var(torch.sigmoid(_t(x)))
    T.nnet = nnet

    sparse = types.ModuleType("theano.sparse")
    sparse.dot = _sparse_dot

    theano.tensor = T
    theano.sparse = sparse
    sys.modules["theano"] = theano
    sys.modules["theano.tensor"] = T
    sys.modules["theano.tensor.nnet"] = nnet
    sys.modules["theano.sparse"] = sparse
    return theano
