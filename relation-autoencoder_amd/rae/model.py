"""Model objects of the training path: encoder, decoders, OieModelFunctions, optimizers.

Mirrors the reference's object model (learning/OieModel.py, learning/models/encoders/
RelationClassifier.py, learning/models/decoders/*.py, learning/Optimizers.py): the same
constructor arguments, the same single-RandomState draw order for initialisation, the same
``params`` list order -- but the parameters are fp32 tensors resident in HBM and the
computation they feed is the HIP training step (engine.py), not a symbolic graph.
"""
from __future__ import annotations

import math

import numpy as np
import torch

LOW, HIGH = -1.0e-3, 1.0e-3          # settings.py:23-24


def _dev(x, device):
    return torch.as_tensor(np.asarray(x, dtype=np.float32), device=device).contiguous()


class IndependentRelationClassifiers:
    """learning/models/encoders/RelationClassifier.py:8-26: W ~ U(low, high) (d, m), Wb = 0."""

    def __init__(self, rng, feature_dim, relation_num, device=None):
        self.d = int(feature_dim)
        self.m = int(relation_num)
        self.W = _dev(rng.uniform(low=LOW, high=HIGH, size=(self.d, self.m)), device)
        self.Wb = torch.zeros(self.m, dtype=torch.float32, device=device)
        self.params = [self.W, self.Wb]


class Decoder:
    """learning/models/decoders/Decoder.py:4-81 (parameter bookkeeping only; the scores are
    computed by the HIP step)."""
    model_type = None
    param_names: tuple = ()
    reg_names: tuple = ()

    def __init__(self, rng, neg_samples_num, batch_size, embeddings_size, relation_num,
                 entity_vocab_size, init_embds=None, device=None):
        self.type = self.model_type
        self.rng = rng
        self.s = int(neg_samples_num)
        self.l = int(batch_size)
        self.r = int(embeddings_size)
        self.m = int(relation_num)
        self.n = int(entity_vocab_size)
        self.A_np = init_embds
        self.device = device

    def get_parameters(self):
        return [getattr(self, k) for k in self.param_names]

    def regularized(self):
        """Tensors entering L1/L2 when extended_regularizer (get_l{1,2}_...)."""
        return [getattr(self, k) for k in self.reg_names]


class SelectionalPreferences(Decoder):
    """SelectionalPreferences.py:9-22: C1, C2 ~ N(0, sqrt(0.1)) (r, m) drawn in that order."""
    model_type = "sp"
    param_names = ("A", "C1", "C2", "Ab")
    reg_names = ("C1", "C2")

    def __init__(self, rng, s, l, r, m, n, ex_emb=None, device=None):
        super().__init__(rng, s, l, r, m, n, ex_emb, device)
        sd = math.sqrt(0.1)
        self.C1 = _dev(rng.normal(0, sd, size=(self.r, self.m)), device)
        self.C2 = _dev(rng.normal(0, sd, size=(self.r, self.m)), device)
        self.A = _dev(self.A_np, device)
        self.Ab = torch.zeros(self.n, dtype=torch.float32, device=device)


class Bilinear(Decoder):
    """Bilinear.py:10-20: R ~ N(0, sqrt(0.1)) (r, r, m)."""
    model_type = "rescal"
    param_names = ("R", "A", "Ab")
    reg_names = ("R",)

    def __init__(self, rng, s, l, r, m, n, A_np=None, device=None):
        super().__init__(rng, s, l, r, m, n, A_np, device)
        self.R = _dev(rng.normal(0, math.sqrt(0.1), size=(self.r, self.r, self.m)), device)
        self.A = _dev(self.A_np, device)
        self.Ab = torch.zeros(self.n, dtype=torch.float32, device=device)


class BilinearPlusSP(Decoder):
    """BilinearPlusSP.py:10-32: C (r, r, m), then C1, C2 (r, m), all N(0, sqrt(0.1))."""
    model_type = "rescal+sp"
    param_names = ("C", "A", "Ab", "C1", "C2")
    reg_names = ("C1", "C2", "C")

    def __init__(self, rng, s, l, r, m, n, ex_emb=None, device=None):
        super().__init__(rng, s, l, r, m, n, ex_emb, device)
        sd = math.sqrt(0.1)
        self.C = _dev(rng.normal(0, sd, size=(self.r, self.r, self.m)), device)
        C1 = rng.normal(0, sd, size=(self.r, self.m))
        C2 = rng.normal(0, sd, size=(self.r, self.m))
        self.A = _dev(self.A_np, device)
        self.Ab = torch.zeros(self.n, dtype=torch.float32, device=device)
        self.C1 = _dev(C1, device)
        self.C2 = _dev(C2, device)


def construct_decoder(model_type, rng, neg_samples_num, batch_size, embeddings_size,
                      relation_num, entity_vocab_size, init_embds=None, device=None):
    """learning/models/decoders/Decoder.py:84-93.  (An unknown type is an error here; the
    reference returns None and crashes later.)"""
    cls = {"rescal": Bilinear, "rescal+sp": BilinearPlusSP, "sp": SelectionalPreferences}
    if model_type not in cls:
        raise ValueError(f"unknown decoder {model_type!r}: expected one of {sorted(cls)}")
    return cls[model_type](rng, neg_samples_num, batch_size, embeddings_size, relation_num,
                           entity_vocab_size, init_embds, device=device)


class OieModelFunctions:
    """learning/OieModel.py:12-63 (+ initialize_entity_embeddings :103-123).

    Parameter order ``params`` = [W, Wb] + decoder.get_parameters(); regularised tensors:
    W, plus the decoder's weights when ``extended_regularizer`` (OieModel.py:54-62)."""

    def __init__(self, rng, embed_size, nb_relations, neg_samples_num, batch_size, model, data,
                 extended_regularizer, alpha, external_embeddings=False, device=None):
        self.rng = rng
        self.r = int(embed_size)
        self.s = int(neg_samples_num)
        self.l = int(batch_size)
        self.m = int(nb_relations)
        self.n = data.get_arg_voc_size()
        self.model = model
        self.external_emb = external_embeddings
        self.extended_reg = _as_bool(extended_regularizer)
        self.alpha = float(alpha)
        self.device = device
        self.relationClassifiers = IndependentRelationClassifiers(rng, data.get_dimensionality(),
                                                                  nb_relations, device)
        self.params = list(self.relationClassifiers.params)
        embds = self.initialize_entity_embeddings(data, self.external_emb)
        self.decoder = construct_decoder(model, rng, self.s, self.l, self.r, self.m, self.n,
                                         init_embds=embds, device=device)
        self.params.extend(self.decoder.get_parameters())
        self.param_names = ["W", "Wb"] + list(self.decoder.param_names)

    def initialize_entity_embeddings(self, data, word2vecflag):
        """OieModel.py:103-123: A ~ U(-0.01, 0.01) (n, r).  word2vec initialisation (gensim)
        is outside this path."""
        A_np = self.rng.uniform(-0.01, 0.01, size=(data.get_arg_voc_size(), self.r))
        if _as_bool(word2vecflag):
            raise NotImplementedError("--ext-emb (gensim word2vec initialisation) is not part "
                                      "of the MI355X training path")
        return A_np

    def named_params(self):
        return dict(zip(self.param_names, self.params))


class AdaGrad:
    """learning/Optimizers.py:6-33: one zero accumulator per parameter, same order."""
    name = "adagrad"

    def __init__(self, params):
        self.accumulator = [torch.zeros_like(p) for p in params]


class SGD:
    """learning/Optimizers.py:36-52."""
    name = "sgd"

    def __init__(self, params=None):
        self.accumulator = None


def make_optimizer(optimization, params):
    """learning/OieInduction.py:261-269."""
    if optimization == "adagrad":
        return AdaGrad(params)
    if optimization == "sgd":
        return SGD(params)
    raise Exception("Optimizer '{}' not implemented".format(optimization))


def _as_bool(v):
    """learning/OieInduction.py:452-458 fix_parsing (strings 'True'/'False' or bools)."""
    if v == "True":
        return True
    if v == "False":
        return False
    return bool(v)
