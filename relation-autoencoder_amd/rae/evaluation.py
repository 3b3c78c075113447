"""B^3 cluster evaluation of the induced relation assignments
(evaluation/OieEvaluation.py:5-44,90-127,215-220).

Element-level B^3 over the examples that carry a gold label (first label only):
  precision = (1/|A|) sum_{e in A} |C(e) n G(e)| / |C(e) n A|
  recall    = (1/|A|) sum_{e in A} |C(e) n G(e)| / |G(e)|
computed here from the cluster x gold contingency table (same values as the reference's
per-element set intersections, without its O(|A| * |C|) set work).
"""
from __future__ import annotations

import numpy as np


class SingleLabelClusterEvaluation:
    def __init__(self, split_goldstandard, split_label):
        assert split_label in ("train", "valid", "test")
        self.split_label = split_label
        self.numberOfElements = 0
        self.induced_clusters = {}
        self.gold_clusters, self.assessableElemSet = self._parse_first_relation_label(
            split_goldstandard)

    @staticmethod
    def _parse_first_relation_label(relations):
        """OieEvaluation.py:190-210."""
        gold, labeled = {}, set()
        for ex_id, labels in relations.items():
            first = labels[0]
            if first != "":
                labeled.add(ex_id)
                gold.setdefault(first, set()).add(ex_id)
        return gold, labeled

    def feed_induced_clusters(self, response):
        """OieEvaluation.py:23-34: drop empty clusters."""
        self.numberOfElements = 0
        self.induced_clusters = {}
        for cid, members in response.items():
            if len(members) > 0:
                self.numberOfElements += len(members)
                self.induced_clusters[cid] = set(members)

    def _contingency(self):
        gold_of = {}
        for gi, (_, members) in enumerate(sorted(self.gold_clusters.items())):
            for e in members:
                gold_of[e] = gi
        ng = len(self.gold_clusters)
        rows = []
        for _, members in sorted(self.induced_clusters.items()):
            row = np.zeros(ng, dtype=np.float64)
            for e in members:
                g = gold_of.get(e)
                if g is not None:
                    row[g] += 1
            rows.append(row)
        return np.array(rows).reshape(-1, ng)

    def b3_total_element_precision(self):
        n = self._contingency()
        nc = n.sum(axis=1, keepdims=True)
        with np.errstate(invalid="ignore", divide="ignore"):
            t = np.where(nc > 0, n * n / np.where(nc > 0, nc, 1), 0.0)
        return float(t.sum()) / float(len(self.assessableElemSet))

    def b3_total_element_recall(self):
        n = self._contingency()
        sizes = np.array([len(v) for _, v in sorted(self.gold_clusters.items())],
                         dtype=np.float64)
        t = n * n / np.where(sizes > 0, sizes, 1)[None, :]
        return float(t.sum()) / float(len(self.assessableElemSet))

    def compute_metrics(self):
        """OieEvaluation.py:36-44 -> (f1, precision, recall)."""
        if not self.assessableElemSet:
            return 0.0, 0.0, 0.0
        rec = self.b3_total_element_recall()
        pre = self.b3_total_element_precision()
        if rec == 0.0 and pre == 0.0:
            return 0.0, pre, rec
        return (2 * rec * pre) / (rec + pre), pre, rec


def construct_split_evaluator(split_goldstandard, split_label):
    """OieEvaluation.py:220-230."""
    return SingleLabelClusterEvaluation(split_goldstandard or {}, split_label)
