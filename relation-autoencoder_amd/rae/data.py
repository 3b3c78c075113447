"""Dataset layout of the training path (learning/OieData.py restated for device residency).

The reference keeps, per split, a CSR feature matrix ``xFeats`` (N, d) float32 with all
stored values 1.0 (duplicates collapse, OieData.py:83-90), int32 entity-id vectors
``args1``/``args2`` (OieData.py:80-87), and one negative-sampling CDF over entities
(``negSamplingCum``, OieData.py:53-59).  Here the same arrays are uploaded once to HBM as
int32 CSR (indptr, indices; values dropped when binary) and int32 id vectors.

Also: the deterministic synthetic triple generator that BASELINE.json's configs are
measured on.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

SPLIT_LABELS = ["train", "valid", "test"]          # settings.py:26


def neg_sampling_cum(freqs, power: float = 0.75) -> np.ndarray:
    """learning/OieData.py:57-59,115-118: cumsum of freq**0.75 / sum(freq**0.75), entity-id
    order; the normaliser is the sequential sum (== last element of the raw cumsum).
    ``f ** p`` is evaluated with Python's float pow (C pow), as the reference does -- numpy's
    vectorised power differs in the last bit for ~5 % of integers, which would change the
    CDF and therefore the sampled ids."""
    f = np.asarray(freqs, dtype=np.int64)
    uniq, inv = np.unique(f, return_inverse=True)
    upow = np.array([float(int(x)) ** power for x in uniq], dtype=np.float64)
    powered = upow[inv]
    raw = np.cumsum(powered)
    return np.cumsum(powered / raw[-1])


class DatasetSplit:
    """learning/OieData.py:8-26."""

    def __init__(self, arguments1, arguments2, arg_features):
        self.args1 = np.ascontiguousarray(arguments1, dtype=np.int32)
        self.args2 = np.ascontiguousarray(arguments2, dtype=np.int32)
        x = sp.csr_matrix(arg_features, dtype=np.float32)
        x.sort_indices()
        self.xFeats = x

    def get_size(self):
        return len(self.args1)


class DatasetManager:
    """Array-level counterpart of learning/OieData.py:29-140.

    ``splits`` maps split names to DatasetSplit; ``entity_freqs`` are the mention counts in
    entity-id order over all splits (OieData.py:53, generate_args :143-155).  Ingestion of
    the reference's pickle (processing/OiePreprocessor.py) is not part of this path.
    """

    def __init__(self, splits: dict, entity_freqs, n_features: int,
                 neg_sampling_distr_power: float = 0.75):
        if "train" not in splits:
            raise Exception("Dataset manager requires that the provided dataset contains a "
                            "'train' split.")
        self.split = dict(splits)
        self.negSamplingDistrPower = neg_sampling_distr_power
        self.entity_freqs = np.asarray(entity_freqs, dtype=np.int64)
        self.n_features = int(n_features)
        self.negSamplingCum = neg_sampling_cum(self.entity_freqs, neg_sampling_distr_power)

    def get_arg_voc_size(self):
        return int(len(self.entity_freqs))

    def get_dimensionality(self):
        return self.n_features

    def get_neg_sampling_cum(self):
        return self.negSamplingCum

    def generate_split_keys(self):
        for s in SPLIT_LABELS:
            if s in self.split:
                yield s

    @classmethod
    def from_arrays(cls, xfeats, args1, args2, n_entities=None, n_features=None, **extra):
        split = DatasetSplit(args1, args2, xfeats)
        n = int(n_entities) if n_entities is not None else int(max(split.args1.max(),
                                                                    split.args2.max()) + 1)
        freqs = np.bincount(np.concatenate([split.args1, split.args2]), minlength=n)
        splits = {"train": split}
        for k, v in extra.items():
            splits[k] = v
            freqs = freqs + np.bincount(np.concatenate([v.args1, v.args2]), minlength=n)
        return cls(splits, freqs, n_features or split.xFeats.shape[1])


# ---------------------------------------------------------------------------------------
# on-disk format (numpy .npz, no pickles): the arrays of every split + entity frequencies
# ---------------------------------------------------------------------------------------
def save_npz(path, data: DatasetManager, gold_standard=None):
    """Write a DatasetManager (+ gold standard {split: {index: [label, ...]}}) as .npz."""
    out = {"n_features": np.int64(data.n_features), "entity_freqs": data.entity_freqs,
           "power": np.float64(data.negSamplingDistrPower)}
    for name, sp_ in data.split.items():
        x = sp_.xFeats
        out[f"{name}/indptr"] = np.asarray(x.indptr, dtype=np.int64)
        out[f"{name}/indices"] = np.asarray(x.indices, dtype=np.int32)
        out[f"{name}/data"] = np.asarray(x.data, dtype=np.float32)
        out[f"{name}/args1"] = sp_.args1
        out[f"{name}/args2"] = sp_.args2
        g = (gold_standard or {}).get(name) or {}
        idx = np.array(sorted(g), dtype=np.int64)
        out[f"{name}/gold_index"] = idx
        out[f"{name}/gold_label"] = np.array([str(g[int(i)][0]) for i in idx], dtype=np.str_)
    np.savez(path, **out)


def load_npz(path):
    """Inverse of save_npz -> (DatasetManager, gold standard).  allow_pickle stays False."""
    z = np.load(path, allow_pickle=False)
    d = int(z["n_features"])
    splits, gold = {}, {}
    for name in SPLIT_LABELS:
        if f"{name}/indptr" not in z:
            continue
        indptr = z[f"{name}/indptr"]
        X = sp.csr_matrix((z[f"{name}/data"], z[f"{name}/indices"], indptr),
                          shape=(len(indptr) - 1, d))
        splits[name] = DatasetSplit(z[f"{name}/args1"], z[f"{name}/args2"], X)
        gold[name] = {int(i): [str(lbl)] for i, lbl in zip(z[f"{name}/gold_index"],
                                                              z[f"{name}/gold_label"])}
    return DatasetManager(splits, z["entity_freqs"], d, float(z["power"])), gold


# ---------------------------------------------------------------------------------------
# synthetic (e1, e2, feature-bag) triples, SURVEY.md 8d
# ---------------------------------------------------------------------------------------
def _zipf_sampler(rng, n, a, size):
    """Truncated Zipf(a) ranks in [0, n) by inverse CDF."""
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), a)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.searchsorted(cdf, rng.random_sample(size), side="right").clip(0, n - 1)


def synthetic_dataset(n_examples: int, n_features: int, n_relations_true: int, seed: int = 1234,
                      n_slots: int = 8, bow_mean: float = 6.0, max_bow: int = 31,
                      gold_fraction: float = 0.02):
    """Deterministic synthetic triples shaped like data-sample.txt:
    8 single-valued "slot" features from disjoint Zipf vocabularies (cf. the 8 slot-like
    extractors of definitions/OieFeatures.py:245-246) + Poisson(6) distinct Zipf "bow"
    features; entities n = N/5 with Zipf(1.0) mention frequency, ids in descending
    frequency; K_true planted relations bias slot features and entity pools; ~2 % of the
    examples carry a gold label.  Returns (DatasetManager, gold dict {index: label})."""
    rng = np.random.RandomState(seed)
    N, d, K = int(n_examples), int(n_features), int(n_relations_true)
    rel = rng.randint(K, size=N)
    slot_vocab = d // (2 * n_slots)
    bow_vocab = d - n_slots * slot_vocab
    cols = []
    rows = []
    ar = np.arange(N)
    for j in range(n_slots):
        z = _zipf_sampler(rng, slot_vocab, 1.0, N)
        # relation-specific rotation of the slot vocabulary for half of the mass
        mix = rng.random_sample(N) < 0.5
        v = np.where(mix, (z + rel * 7919 * (j + 1)) % slot_vocab, z)
        cols.append(j * slot_vocab + v)
        rows.append(ar)
    nb = np.clip(rng.poisson(bow_mean, N), 1, max_bow)
    brow = np.repeat(ar, nb)
    bcol = n_slots * slot_vocab + _zipf_sampler(rng, bow_vocab, 1.0, brow.shape[0])
    rows.append(brow)
    cols.append(bcol)
    rows = np.concatenate(rows).astype(np.int64)
    cols = np.concatenate(cols).astype(np.int64)
    key = np.unique(rows * d + cols)                      # duplicates collapse (OieData.py:88)
    r_ = (key // d).astype(np.int64)
    c_ = (key % d).astype(np.int32)
    indptr = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(np.bincount(r_, minlength=N), out=indptr[1:])
    X = sp.csr_matrix((np.ones(len(c_), dtype=np.float32), c_, indptr.astype(np.int32)),
                      shape=(N, d))
    # entities
    n = max(2, N // 5)
    ez1 = _zipf_sampler(rng, n, 1.0, N)
    ez2 = _zipf_sampler(rng, n, 1.0, N)
    pool = rng.random_sample(N) < 0.3
    e1 = np.where(pool, (ez1 + rel * 104729) % n, ez1)
    e2 = np.where(pool, (ez2 + rel * 15485863) % n, ez2)
    # relabel ids in descending frequency (stable), drop unseen entities
    cnt = np.bincount(np.concatenate([e1, e2]), minlength=n)
    order = np.argsort(-cnt, kind="stable")
    seen = cnt[order] > 0
    order = order[seen]
    remap = np.full(n, -1, dtype=np.int64)
    remap[order] = np.arange(len(order))
    a1 = remap[e1].astype(np.int32)
    a2 = remap[e2].astype(np.int32)
    freqs = cnt[order]
    gold_idx = np.nonzero(rng.random_sample(N) < gold_fraction)[0]
    gold = {int(i): [f"REL{int(rel[i])}"] for i in gold_idx}
    data = DatasetManager({"train": DatasetSplit(a1, a2, X)}, freqs, d)
    return data, {"train": gold}


def batch_nnz_stats(indptr: np.ndarray, global_batch: int):
    """(max nnz of a global batch, max nnz of an example row) for plan sizing."""
    indptr = np.asarray(indptr, dtype=np.int64)
    N = len(indptr) - 1
    nb = N // global_batch
    if nb == 0:
        return 1, int(np.diff(indptr).max(initial=1))
    starts = indptr[0:nb * global_batch:global_batch]
    ends = indptr[global_batch:nb * global_batch + 1:global_batch]
    return int((ends - starts).max(initial=1)), int(np.diff(indptr).max(initial=1))
