"""Generate the B^3 golden vectors by executing the reference's own evaluator.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (where /root/reference exists), never
on the GPU box.  It imports /root/reference/evaluation/OieEvaluation.py unmodified (bytecode
writing disabled, so nothing is written there) with two stand-ins for its Python-2
environment:
  * a ``settings`` module holding only ``split_labels`` (settings.py:26), which the
    evaluator's constructor asserts against (OieEvaluation.py:17);
  * dicts with Python 2's ``iteritems`` / ``itervalues`` (OieEvaluation.py:31,92,123,195):
    the inputs, and the induced-cluster mapping feed_induced_clusters rebuilds (:30-34).
Everything the metric computes -- feed_induced_clusters (:23-34), compute_metrics (:36-44),
b3_total_element_precision / recall (:90-96,121-127), _parse_first_relation_label
(:185-203), _find_cluster (:205-209) -- is the reference's code.

Output: tests/golden/b3_cases.json -- per case the induced clusters, the gold labels and the
reference's (f1, precision, recall); pure data.

Usage:  python oracle/gen_b3_fixture.py [out.json]
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import types

sys.dont_write_bytecode = True          # never write __pycache__ into /root/reference

import numpy as np                       # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("RAE_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "b3_cases.json")


class Py2Dict(dict):
    """dict with the Python 2 iteration methods the evaluator calls."""

    def iteritems(self):
        return iter(self.items())

    def itervalues(self):
        return iter(self.values())


def load_reference_evaluator():
    settings = types.ModuleType("settings")
    settings.split_labels = ["train", "valid", "test"]     # settings.py:26
    sys.modules["settings"] = settings
    path = os.path.join(REF, "evaluation", "OieEvaluation.py")
    spec = importlib.util.spec_from_file_location("ref_OieEvaluation", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def source_sha256():
    """sha256 of the evaluator file the fixture was produced from (recorded in the fixture)."""
    with open(os.path.join(REF, "evaluation", "OieEvaluation.py"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def _cases():
    g = np.random.RandomState(17)
    cases = []
    # hand-made: empty induced cluster, unlabelled members, a cluster without any assessable
    # member, multi-label gold (first label only), a first label '' with a later label
    cases.append(dict(
        name="edges",
        induced={0: [0, 1, 2, 3], 1: [], 2: [4, 5, 6], 3: [7, 8], 4: [9]},
        gold={0: ["A", "B"], 1: ["A"], 2: ["B"], 4: ["B", "A"], 5: ["C"], 6: ["B"],
              9: ["", "A"], 3: [""], 8: ["C"]}))
    cases.append(dict(name="perfect", induced={0: [0, 1], 1: [2, 3], 2: [4]},
                      gold={0: ["x"], 1: ["x"], 2: ["y"], 3: ["y"], 4: ["z"]}))
    cases.append(dict(name="one_cluster", induced={0: list(range(8))},
                      gold={i: ["ab"[i % 2]] for i in range(8)}))
    cases.append(dict(name="singletons", induced={i: [i] for i in range(6)},
                      gold={i: ["q" if i < 4 else "r"] for i in range(6)}))
    # random: the training loop's shape (cluster id -> example ids over range(N); ~20 % of the
    # examples labelled, some with several labels, some with '' first)
    for k, (N, K, G, frac) in enumerate([(60, 5, 3, 0.5), (400, 30, 8, 0.2),
                                         (1500, 100, 12, 0.05)]):
        lab = g.randint(0, K, size=N)
        induced = {c: [int(i) for i in np.nonzero(lab == c)[0]] for c in range(K)}
        gold = {}
        for i in range(N):
            if g.rand() < frac:
                first = f"REL{g.randint(G)}" if g.rand() > 0.05 else ""
                extra = [f"REL{g.randint(G)}" for _ in range(g.randint(0, 3))]
                gold[i] = [first] + extra
        cases.append(dict(name=f"random{k}", induced=induced, gold=gold))
    return cases


def main(out=OUT):
    mod = load_reference_evaluator()
    res = []
    for c in _cases():
        gold = Py2Dict({i: list(v) for i, v in c["gold"].items()})
        ev = mod.construct_split_evaluator(gold, "train")               # :220-230
        ev.feed_induced_clusters(Py2Dict({cid: set(m) for cid, m in c["induced"].items()}))
        # feed_induced_clusters rebuilds the mapping as a plain {} literal (:30-34), which
        # Python 3 has no iteritems() for: re-type it (same contents)
        ev.induced_clusters = Py2Dict(ev.induced_clusters)
        f1, pre, rec = ev.compute_metrics()                             # :36-44
        res.append({"name": c["name"],
                    "induced": {str(k): v for k, v in c["induced"].items()},
                    "gold": {str(k): v for k, v in c["gold"].items()},
                    "f1": f1, "precision": pre, "recall": rec,
                    "number_of_elements": ev.numberOfElements})
        print(f"{c['name']}: f1 {f1:.12f} pre {pre:.12f} rec {rec:.12f}")
    with open(out, "w") as fh:
        json.dump({"source": "evaluation/OieEvaluation.py executed by oracle/gen_b3_fixture.py",
                   "source_sha256": source_sha256(), "cases": res}, fh, indent=0, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else OUT)
