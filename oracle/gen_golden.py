"""Generate golden vectors by executing the reference's own model code.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (where /root/reference exists),
never on the GPU box; its outputs are committed as small .npz fixtures under
tests/golden/ and are pure data (inputs + expected outputs).

What runs *unmodified* from the reference (imported from /root/reference, bytecode
writing disabled so nothing is written there):
  learning/models/encoders/RelationClassifier.py  (IndependentRelationClassifiers)
  learning/models/decoders/Decoder.py              (construct_decoder)
  learning/models/decoders/SelectionalPreferences.py, Bilinear.py, BilinearPlusSP.py
  learning/Optimizers.py                           (AdaGrad, SGD)
  learning/NegativeExampleGenerator.py             (NegativeExampleGenerator)
on top of oracle/theano_shim.py (Theano's op semantics restated; Theano is absent).

What is restated here because those files are Python-2-only (print statements) and do
not parse under Python 3 -- each a handful of lines, cited:
  learning/OieModel.py:50,54-63,81,90,105   (param list, L1/L2, entropy, mean, A init)
  learning/OieInduction.py:98,131-135,183-189 (batch count, cost, per-epoch loop)
  learning/OieData.py:53-59,115-118         (CDF over entity frequencies)

Usage:  python oracle/gen_golden.py [outdir]
"""
from __future__ import annotations

import builtins
import importlib
import os
import sys

sys.dont_write_bytecode = True          # never write __pycache__ into /root/reference

import numpy as np                       # noqa: E402
import scipy.sparse as sp                # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("RAE_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")

sys.path.insert(0, HERE)
import theano_shim                       # noqa: E402
from rae_oracle import neg_sampling_cum  # noqa: E402  (restated CDF, also pinned here)


def _import_reference():
    theano_shim.install()
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "learning", "models", "decoders"))
    rc = importlib.import_module("learning.models.encoders.RelationClassifier")
    dec = importlib.import_module("learning.models.decoders.Decoder")
    opt = importlib.import_module("learning.Optimizers")
    neg = importlib.import_module("learning.NegativeExampleGenerator")
    # Py2 map() returned a list; the module's np.array(map(...)) relies on that.
    neg.map = lambda f, xs: list(builtins.map(f, xs))
    return rc, dec, opt, neg


def make_dataset(seed, N, d, n, min_f=2, max_f=6):
    """Tiny synthetic (features, e1, e2) triples; every entity id appears at least once
    (the reference's ids come from observed mentions, learning/OieData.py:53,56)."""
    g = np.random.RandomState(seed)
    rows, cols = [], []
    for i in range(N):
        k = g.randint(min_f, max_f + 1)
        feats = g.choice(d, size=k, replace=False)
        rows += [i] * k
        cols += list(feats)
    dok = sp.dok_matrix((N, d), dtype=np.float64)
    for i, f in zip(rows, cols):
        dok[i, f] = 1
    X = sp.csr_matrix(dok, dtype="float32")          # learning/OieData.py:90
    X.sort_indices()
    ents = np.concatenate([np.arange(n), g.zipf(1.6, size=2 * N - n) % n]) if 2 * N >= n \
        else g.randint(0, n, size=2 * N)
    g.shuffle(ents)
    args1 = ents[:N].astype(np.int32)
    args2 = ents[N:2 * N].astype(np.int32)
    freqs = np.bincount(np.concatenate([args1, args2]), minlength=n)
    return X, args1, args2, freqs


def run_case(mods, name, *, decoder, N, d, m, n, r, s, l, alpha, lr, l1, l2, optimizer,
             ext_reg, seed, epochs, data_seed):
    rc, dec, opt, negmod = mods
    import theano_shim as th
    T = sys.modules["theano.tensor"]

    X, args1, args2, freqs = make_dataset(data_seed, N, d, n)
    cum = neg_sampling_cum(freqs)
    rng = np.random.RandomState(seed=seed)                        # OieInduction.py:494
    sampler = negmod.NegativeExampleGenerator(rng, cum)          # OieInduction.py:85 (no draw)
    enc = rc.IndependentRelationClassifiers(rng, d, m)            # OieModel.py:49 -> draws W
    A_np = np.asarray(rng.uniform(-0.01, 0.01, size=(n, r)), dtype=np.float64)   # OieModel.py:105
    decoder_obj = dec.construct_decoder(decoder, rng, s, l, r, m, n, init_embds=A_np)  # :59
    params = list(enc.params) + list(decoder_obj.get_parameters())   # OieModel.py:50,63
    L1 = T.sum(abs(enc.W))                                        # OieModel.py:54
    L2 = T.sum(T.sqr(enc.W))                                      # :56
    if ext_reg:                                                   # :60-62
        L1 = L1 + decoder_obj.get_l1_regularization_term_computation()
        L2 = L2 + decoder_obj.get_l2_regularization_term_computation()
    names = ["W", "Wb"] + {"sp": ["A", "C1", "C2", "Ab"], "rescal": ["R", "A", "Ab"],
                           "rescal+sp": ["C", "A", "Ab", "C1", "C2"]}[decoder]
    out = dict(decoder=np.array(decoder), N=N, d=d, m=m, n=n, r=r, s=s, l=l, alpha=alpha,
               lr=lr, l1=l1, l2=l2, optimizer=np.array(optimizer), ext_reg=int(ext_reg),
               seed=seed, epochs=epochs,
               indptr=X.indptr.astype(np.int32), indices=X.indices.astype(np.int32),
               data=X.data.astype(np.float32), args1=args1, args2=args2,
               freqs=freqs.astype(np.int64), cum=cum)
    for nm, pv in zip(names, params):
        out["init_" + nm] = pv.get_value()

    if optimizer == "adagrad":
        optim = opt.AdaGrad(params)                                # OieInduction.py:264
    else:
        optim = opt.SGD()
    adjust = float(l) / float(N)                                   # OieInduction.py:131
    nb = N // l                                                    # OieInduction.py:98
    Xd = X.toarray().astype(np.float64)

    def build_cost(b, n1, n2):
        sl = slice(b * l, (b + 1) * l)
        x = th.Var(th.torch.as_tensor(Xd[sl]))
        a1 = th.Var(th.torch.as_tensor(args1[sl].astype(np.int64)))
        a2 = th.Var(th.torch.as_tensor(args2[sl].astype(np.int64)))
        ng1 = th.Var(th.torch.as_tensor(np.asarray(n1, dtype=np.int64)))
        ng2 = th.Var(th.torch.as_tensor(np.asarray(n2, dtype=np.int64)))
        P = enc.comp_relation_probs(x)                             # OieModel.py:80
        ent = alpha * -T.sum(T.log(P) * P, axis=1)                 # OieModel.py:81
        scores = decoder_obj.get_scores(a1, a2, P, ng1, ng2, ent)  # OieModel.py:82
        cost = -T.mean(scores)                                     # OieModel.py:90
        cost = cost + (l1 * L1_now() * adjust) + (l2 * L2_now() * adjust)   # OieInduction.py:134-135
        return cost, P, ent, scores

    # L1/L2 are symbolic in Theano (re-evaluated every call); rebuild them eagerly
    def L1_now():
        v = T.sum(abs(enc.W))
        if ext_reg:
            v = v + decoder_obj.get_l1_regularization_term_computation()
        return v

    def L2_now():
        v = T.sum(T.sqr(enc.W))
        if ext_reg:
            v = v + decoder_obj.get_l2_regularization_term_computation()
        return v

    costs = np.zeros((epochs, nb))
    errs = np.zeros(epochs)
    for ep in range(epochs):
        neg1 = sampler.get_negative_samples(N, s)                  # OieInduction.py:183
        neg2 = sampler.get_negative_samples(N, s)                  # :184
        out[f"neg1_e{ep}"] = neg1.astype(np.int32)
        out[f"neg2_e{ep}"] = neg2.astype(np.int32)
        err = 0.0
        for b in range(nb):                                        # :186-189
            n1 = neg1[:, b * l:(b + 1) * l]
            n2 = neg2[:, b * l:(b + 1) * l]
            cost, P, ent, scores = build_cost(b, n1, n2)
            if ep == 0 and b == 0:
                out["step0_P"] = P.t.detach().numpy()
                out["step0_H"] = ent.t.detach().numpy()
                out["step0_scores"] = scores.t.detach().numpy()
                out["step0_cost"] = float(cost.t)
                gs = T.grad(cost, params)
                for nm, gv in zip(names, gs):
                    out["step0_grad_" + nm] = gv.t.detach().numpy()
            if optimizer == "adagrad":
                updates = optim.update(lr, params, cost)           # Optimizers.py:18-33
            else:
                updates = optim.update(lr, params, cost)           # Optimizers.py:37-52
            vals = [(var, newv.t.detach().numpy().copy()) for var, newv in updates]
            for var, v in vals:                                    # simultaneous update
                var.set_value(v)
            c = float(cost.t)
            costs[ep, b] = c
            err += c
            if ep == 0 and b == 0:
                for nm, pv in zip(names, params):
                    out["step1_" + nm] = pv.get_value()
        errs[ep] = err
    out["costs"] = costs
    out["errs"] = errs
    for nm, pv in zip(names, params):
        out["final_" + nm] = pv.get_value()
    if optimizer == "adagrad":
        for nm, acc in zip(names, optim.accumulator):
            out["final_acc_" + nm] = acc.get_value()
    # labelling pass after training (RelationClassifier.py:39-48; tail dropped,
    # OieInduction.py:337)
    labs, probs = [], []
    for b in range(nb):
        x = th.Var(th.torch.as_tensor(Xd[b * l:(b + 1) * l]))
        lab, pr = enc.comp_probs_and_labels(x)
        labs.append(lab.t.numpy().astype(np.int64))
        probs.append(pr.t.detach().numpy())
    out["labels"] = np.concatenate(labs)
    out["probs"] = np.concatenate(probs)
    return out


CASES = {
    # name: kwargs
    "sp_basic": dict(decoder="sp", N=14, d=24, m=3, n=9, r=5, s=2, l=4, alpha=1.0, lr=0.1,
                     l1=0.0, l2=0.0, optimizer="adagrad", ext_reg=True, seed=2, epochs=2,
                     data_seed=11),
    "sp_reg": dict(decoder="sp", N=12, d=20, m=4, n=8, r=6, s=3, l=3, alpha=0.1, lr=0.05,
                   l1=0.01, l2=0.1, optimizer="adagrad", ext_reg=True, seed=7, epochs=2,
                   data_seed=12),
    "sp_sgd_noext": dict(decoder="sp", N=10, d=16, m=3, n=7, r=4, s=2, l=5, alpha=0.5,
                         lr=0.2, l1=0.0, l2=0.1, optimizer="sgd", ext_reg=False, seed=3,
                         epochs=2, data_seed=13),
    "rescal_basic": dict(decoder="rescal", N=14, d=24, m=3, n=9, r=5, s=2, l=4, alpha=1.0,
                         lr=0.1, l1=0.0, l2=0.0, optimizer="adagrad", ext_reg=True, seed=2,
                         epochs=2, data_seed=11),
    "rescal_reg": dict(decoder="rescal", N=12, d=20, m=4, n=8, r=6, s=3, l=3, alpha=0.1,
                       lr=0.05, l1=0.01, l2=0.1, optimizer="adagrad", ext_reg=True, seed=7,
                       epochs=2, data_seed=12),
    "hybrid_basic": dict(decoder="rescal+sp", N=14, d=24, m=3, n=9, r=5, s=2, l=4,
                         alpha=1.0, lr=0.1, l1=0.0, l2=0.0, optimizer="adagrad",
                         ext_reg=True, seed=2, epochs=2, data_seed=11),
    # test.py:33 hyper-parameters (lr 0.1, batch 100->4 here, embed 10->5, 5 relations,
    # 5 negatives, l1 0, l2 0.1, adagrad, rescal+sp, ext_reg True, alpha 0.1)
    "hybrid_testpy": dict(decoder="rescal+sp", N=18, d=30, m=5, n=11, r=5, s=5, l=4,
                          alpha=0.1, lr=0.1, l1=0.0, l2=0.1, optimizer="adagrad",
                          ext_reg=True, seed=2, epochs=2, data_seed=14),
}


def sampler_case(mods):
    _, _, _, negmod = mods
    freqs = np.array([5, 1, 3, 9, 2, 2, 7, 1, 4, 6, 1, 1, 3])
    cum = neg_sampling_cum(freqs)
    rng = np.random.RandomState(seed=7)
    gen = negmod.NegativeExampleGenerator(rng, cum)
    a = gen.get_negative_samples(37, 4)
    b = gen.get_negative_samples(37, 4)
    return dict(freqs=freqs, cum=cum, seed=7, N=37, s=4, neg1=a.astype(np.int32),
                neg2=b.astype(np.int32))


def main(outdir=OUT):
    os.makedirs(outdir, exist_ok=True)
    mods = _import_reference()
    for name, kw in CASES.items():
        out = run_case(mods, name, **kw)
        np.savez_compressed(os.path.join(outdir, f"{name}.npz"), **out)
        print(f"wrote {name}: cost0={out['step0_cost']:.12f} errs={out['errs']}")
    np.savez_compressed(os.path.join(outdir, "sampler.npz"), **sampler_case(mods))
    print("wrote sampler")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else OUT)
