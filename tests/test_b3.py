"""B^3 evaluation (rae/evaluation.py) pinned to the reference's own evaluator.

tests/golden/b3_cases.json was produced by executing evaluation/OieEvaluation.py itself
(oracle/gen_b3_fixture.py): induced clusters incl. empty ones, unlabelled members, clusters
without assessable members, multi-label gold (first label only) and a '' first label."""
import json
import os

import pytest

from conftest import GOLDEN
from rae.evaluation import construct_split_evaluator

with open(os.path.join(GOLDEN, "b3_cases.json")) as fh:
    CASES = json.load(fh)["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_b3_matches_reference_evaluator(case):
    gold = {int(k): v for k, v in case["gold"].items()}
    induced = {int(k): set(v) for k, v in case["induced"].items()}
    ev = construct_split_evaluator(gold, "train")
    ev.feed_induced_clusters(induced)
    f1, pre, rec = ev.compute_metrics()
    assert ev.numberOfElements == case["number_of_elements"]
    assert pre == pytest.approx(case["precision"], rel=1e-12, abs=1e-15)
    assert rec == pytest.approx(case["recall"], rel=1e-12, abs=1e-15)
    assert f1 == pytest.approx(case["f1"], rel=1e-12, abs=1e-15)


def test_b3_from_training_loop_labels():
    """The inducer's path: labels -> get_clusters_sets-style mapping -> metrics (the random
    cases are exactly that shape: cluster id -> example ids over range(N))."""
    case = CASES[-1]
    N = 1 + max(max(v) for v in case["induced"].values() if v)
    labels = [0] * N
    for cid, members in case["induced"].items():
        for i in members:
            labels[i] = int(cid)
    clusters = {c: set() for c in range(len(case["induced"]))}
    for i, c in enumerate(labels):
        clusters[c].add(i)
    ev = construct_split_evaluator({int(k): v for k, v in case["gold"].items()}, "train")
    ev.feed_induced_clusters(clusters)
    assert ev.compute_metrics()[0] == pytest.approx(case["f1"], rel=1e-12)


def _b3_by_definition(gold, induced):
    """Clean-room B^3 straight from the per-element definition (no contingency table):
    precision = mean_{e in A} |C(e) & G(e)| / |C(e) & A|, recall = mean |C(e) & G(e)| / |G(e)|,
    A = examples whose first gold label is not ''."""
    first = {e: v[0] for e, v in gold.items() if v and v[0] != ""}
    A = set(first)
    if not A:
        return 0.0, 0.0, 0.0
    G = {}
    for e, lab in first.items():
        G.setdefault(lab, set()).add(e)
    C = {}
    for members in induced.values():
        for e in members:
            C[e] = set(members)
    pre = sum(len(C[e] & G[first[e]]) / len(C[e] & A) for e in A if e in C) / len(A)
    rec = sum(len(C[e] & G[first[e]]) / len(G[first[e]]) for e in A if e in C) / len(A)
    f1 = 0.0 if pre + rec == 0 else 2 * pre * rec / (pre + rec)
    return f1, pre, rec


def test_b3_hand_computed():
    # P: e0 2/3, e1 2/3, e2 1/3, e3 1, e4 1 -> 11/15;  R: 1, 1, 1/3, 2/3, 2/3 -> 11/15
    gold = {0: ["A"], 1: ["A"], 2: ["B"], 3: ["B"], 4: ["B", "A"], 5: [""]}
    induced = {0: {0, 1, 2}, 1: {3, 4, 5}, 2: set()}
    ev = construct_split_evaluator(gold, "train")
    ev.feed_induced_clusters(induced)
    f1, pre, rec = ev.compute_metrics()
    assert ev.numberOfElements == 6
    assert pre == pytest.approx(11 / 15, rel=1e-15)
    assert rec == pytest.approx(11 / 15, rel=1e-15)
    assert f1 == pytest.approx(11 / 15, rel=1e-15)
    assert (f1, pre, rec) == pytest.approx(_b3_by_definition(gold, induced), rel=1e-15)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_b3_fixture_matches_clean_room_definition(case):
    """The executed-reference fixture agrees with an independent per-element computation."""
    gold = {int(k): v for k, v in case["gold"].items()}
    induced = {int(k): set(v) for k, v in case["induced"].items() if v}
    f1, pre, rec = _b3_by_definition(gold, induced)
    assert pre == pytest.approx(case["precision"], rel=1e-12, abs=1e-15)
    assert rec == pytest.approx(case["recall"], rel=1e-12, abs=1e-15)
    assert f1 == pytest.approx(case["f1"], rel=1e-12, abs=1e-15)
