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
