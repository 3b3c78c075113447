"""Dataset ingestion: the Yao-format relation file -> feature lexicon -> indexed splits
(processing/OiePreprocessor.py, definitions/OieFeatures.py, definitions/OieExample.py,
learning/OieData.py:36-90).  SURVEY 8(f) #2; BASELINE config 1 (data-sample.txt).

    python -m rae.preprocess data-sample.txt sample.json [--batch train] [--thres 0]
    python -m rae sample.json --model-name m --decoder sp --relations_number 10 ...

The reference pickles its output (feature-extractor functions, FeatureLexicon, the OieExample
lists and the gold standard; OiePreprocessor.py:290-321).  Pickles execute code on load, so
the same four objects are written here as JSON instead (the extractors by name), and a file
can be extended with further splits exactly like the reference's ``--batch valid`` reruns.

Reference behaviour kept on purpose:
* the input is read as Python 2 byte strings: ASCII-only lower-casing and whitespace
  splitting (``_lower`` / ``_split``), the label field keeps its newline until
  ``strip()`` (OiePreprocessor.py:230, 283);
* ``--test-mode`` is accepted and, as in the reference (parsed at :373, never read), has no
  effect: the lexicon is always expanded;
* feature frequencies count every occurrence, thresholding is ``freq > thres`` (:202) and
  pruned ids are assigned in first-pass order (:57-61); duplicate ids inside one example
  collapse to a single 1.0 in the CSR matrix (OieData.py:88).

Entity ids: the reference numbers entities in ``Counter`` iteration order over all splits
(OieData.py:53,126-140), which is Python 2 hash order and cannot be reproduced; here they are
numbered in first-mention order (train, valid, test; arg1 before arg2), the order Python 3's
``Counter`` iterates in.  ``bow_clean`` filters with nltk's English stopword list
(OieFeatures.py:19); nltk and its data are absent here, so the list below is the nltk 3.x
``stopwords.words('english')`` list written out -- parity for that one feature family is
unpinned (the reference pins no nltk version).
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import re
import sys
import time

import numpy as np
import scipy.sparse as sp

from .data import SPLIT_LABELS, DatasetManager, DatasetSplit

# ---------------------------------------------------------------------------------------
# Python 2 byte-string semantics
# ---------------------------------------------------------------------------------------
_ASCII_LOWER = {c: c + 32 for c in range(ord("A"), ord("Z") + 1)}
_PUNCT = "!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~"          # string.punctuation (Py2 == Py3)
_WS = re.compile(r"[ \t\n\r\x0b\x0c]+")
_DIGITS = re.compile(r"\d", re.ASCII)                  # OieFeatures.py:20


def _lower(s: str) -> str:
    return s.translate(_ASCII_LOWER)


def _split(s: str) -> list:
    """str.split() with no argument on a Py2 byte string: ASCII whitespace only."""
    return [w for w in _WS.split(s) if w]


def _strip(s: str) -> str:
    return s.strip(" \t\n\r\x0b\x0c")


STOPWORDS_EN = frozenset("""
i me my myself we our ours ourselves you you're you've you'll you'd your yours yourself
yourselves he him his himself she she's her hers herself it it's its itself they them their
theirs themselves what which who whom this that that'll these those am is are was were be been
being have has had having do does did doing a an the and but if or because as until while of at
by for with about against between into through during before after above below to from up down
in out on off over under again further then once here there when where why how all any both each
few more most other some such no nor not only own same so than too very s t can will just don
don't should should've now d ll m o re ve y ain aren aren't couldn couldn't didn didn't doesn
doesn't hadn hadn't hasn hasn't haven haven't isn isn't ma mightn mightn't mustn mustn't needn
needn't shan shan't shouldn shouldn't wasn wasn't weren weren't won won't wouldn wouldn't
""".split())

# info[] positions (OieFeatures.py:9-14)
PARSING, ENTITIES, TRIG, SENTENCE, POS, DOCPATH = range(6)


# ---------------------------------------------------------------------------------------
# feature extractors: getBasicCleanFeatures (OieFeatures.py:230-247)
# ---------------------------------------------------------------------------------------
def _between_tokens(info, arg1, arg2):
    """Words from the first mention of arg1 through the last of arg2, each stripped of every
    punctuation character in turn, lower-cased, empties dropped (OieFeatures.py:32-39)."""
    sent = info[SENTENCE]
    span = sent[sent.find(arg1):sent.rfind(arg2) + len(arg2)]
    out = []
    for word in _split(span):
        for pun in _PUNCT:
            word = word.strip(pun)
        if word != "":
            out.append(_lower(word))
    return out


def trigger(info, arg1, arg2):              # OieFeatures.py:136-137
    return info[TRIG].replace("TRIGGER:", "")


def entityTypes(info, arg1, arg2):          # :140-141
    return info[ENTITIES]


def arg1_lower(info, arg1, arg2):           # :156-157
    return _lower(arg1)


def arg2_lower(info, arg1, arg2):           # :168-169
    return _lower(arg2)


def bow_clean(info, arg1, arg2):            # :27-43
    return [w for w in _between_tokens(info, arg1, arg2)
            if w not in STOPWORDS_EN and not _DIGITS.search(w) and not ("A" <= w[0] <= "Z")]


def entity1Type(info, arg1, arg2):          # :144-145
    return info[ENTITIES].split("-")[0]


def entity2Type(info, arg1, arg2):          # :148-149
    return info[ENTITIES].split("-")[1]


def lexicalPattern(info, arg1, arg2):       # :176-187: every second token of the path
    p = _split(info[PARSING].replace("->", " ").replace("<-", " "))
    return "_".join(x for num, x in enumerate(p) if num % 2 != 0)


def posPatternPath(info, arg1, arg2):       # :204-227
    words, tags = _split(info[SENTENCE]), _split(info[POS])
    assert len(tags) == len(words), "error"
    if not words:
        return ""
    last1, first2 = _split(arg1)[-1], _split(arg2)[0]
    begin = next((i for i, w in enumerate(words) if w == last1), None)
    end = next((i for i, w in enumerate(words) if w == first2), None)
    if begin is None or end is None:
        return ""
    return "_".join(tags[i] for i in range(len(words)) if begin < i < end)


def get_basic_clean_features():
    return [trigger, entityTypes, arg1_lower, arg2_lower, bow_clean, entity1Type, entity2Type,
            lexicalPattern, posPatternPath]


getBasicCleanFeatures = get_basic_clean_features
_EXTRACTORS = {f.__name__: f for f in get_basic_clean_features()}


# ---------------------------------------------------------------------------------------
# FeatureLexicon (OiePreprocessor.py:9-110) and OieExample (definitions/OieExample.py)
# ---------------------------------------------------------------------------------------
class FeatureLexicon:
    def __init__(self):
        self.nextId = 0
        self.id2Str, self.str2Id, self.id2freq = {}, {}, {}
        self.nextIdPruned = 0
        self.id2StrPruned, self.str2IdPruned = {}, {}

    def get_or_add(self, s):
        i = self.str2Id.get(s)
        if i is None:
            i = self.nextId
            self.id2Str[i], self.str2Id[s], self.id2freq[i] = s, i, 1
            self.nextId += 1
        else:
            self.id2freq[i] += 1
        return i

    def get_or_add_pruned(self, s):
        i = self.str2IdPruned.get(s)
        if i is None:
            i = self.nextIdPruned
            self.id2StrPruned[i], self.str2IdPruned[s] = s, i
            self.nextIdPruned += 1
        return i

    def get_id(self, s):
        return self.str2Id.get(s)

    def get_str(self, idx):
        return self.id2Str.get(idx)

    def get_str_pruned(self, idx):
        return self.id2StrPruned.get(idx)

    def get_freq(self, idx):
        return self.id2freq.get(idx)

    def get_feature_space_dimensionality(self):
        return self.nextIdPruned

    def to_json(self):
        return {"strs": [self.id2Str[i] for i in range(self.nextId)],
                "freqs": [self.id2freq[i] for i in range(self.nextId)],
                "pruned": [self.id2StrPruned[i] for i in range(self.nextIdPruned)]}

    @classmethod
    def from_json(cls, d):
        lex = cls()
        for i, (s, f) in enumerate(zip(d["strs"], d["freqs"])):
            lex.id2Str[i], lex.str2Id[s], lex.id2freq[i] = s, i, int(f)
        lex.nextId = len(d["strs"])
        for i, s in enumerate(d["pruned"]):
            lex.id2StrPruned[i], lex.str2IdPruned[s] = s, i
        lex.nextIdPruned = len(d["pruned"])
        return lex


class OieExample:
    def __init__(self, arg1, arg2, features, trigger, relation=""):
        self.features = features
        self.arg1 = arg1
        self.arg2 = arg2
        self.relation = relation
        self.trigger = trigger


def _generate_feature_element(res):         # OiePreprocessor.py:183-188
    if isinstance(res, list):
        yield from res
    else:
        yield res


def get_features(lexicon, feature_extractors, info, arg1=None, arg2=None, expand=False):
    """OiePreprocessor.py:121-148."""
    feats = []
    for f in feature_extractors:
        res = f(info, arg1, arg2)
        if res is not None:
            for el in _generate_feature_element(res):
                key = f.__name__ + "#" + el
                if expand:
                    feats.append(lexicon.get_or_add(key))
                else:
                    i = lexicon.get_id(key)
                    if i is not None:
                        feats.append(i)
    return feats


def get_thresholded_features(lexicon, feature_extractors, info, arg1, arg2, threshold,
                             expand=False):
    """OiePreprocessor.py:151-180, 200-208: ids of the features seen more than ``threshold``
    times, in the pruned numbering."""
    feats = []
    for f in feature_extractors:
        res = f(info, arg1, arg2)
        if res is not None:
            for el in _generate_feature_element(res):
                key = f.__name__ + "#" + el
                i = lexicon.get_id(key)
                if expand:
                    if lexicon.id2freq[i] > threshold:      # KeyError on an unseen key, as :202
                        feats.append(lexicon.get_or_add_pruned(key))
                elif i is not None and lexicon.id2freq[i] > threshold:
                    feats.append(lexicon.get_or_add_pruned(key))
    return feats


def _info(ex):
    """[parsing, entities, trigger, sentence, pos, docPath] (OiePreprocessor.py:117, 280)."""
    return [ex[1], ex[4], ex[5], ex[7], ex[8], ex[6]]


def read_examples(file_name):
    """OiePreprocessor.py:211-241: tab-separated, 9 fields per line; each example is
    ``[str(counter)] + fields`` (the last field keeps its newline)."""
    out = []
    with open(file_name, "rb") as fp:
        for line in fp:
            line = line.decode("latin-1")
            if len(line) == 0 or len(_split(line)) == 0:
                raise IOError(f"{file_name}: empty line {len(out) + 1}")
            fields = line.split("\t")
            assert len(fields) == 9, ("a problem with the file format (# fields is wrong) len is "
                                      + str(len(fields)) + "instead of 9")
            out.append([str(len(out))] + fields)
    return out


def build_feature_lexicon(raw_features, feature_extractors, lexicon):
    """OiePreprocessor.py:113-118: first pass, counts every feature occurrence."""
    for ex in raw_features:
        get_features(lexicon, feature_extractors, _info(ex), ex[2], ex[3], expand=True)


def load_features(raw_features, lexicon, examples_list, labels_dict, threshold,
                  feature_extractors=None):
    """OiePreprocessor.py:244-287: second pass, thresholded ids -> OieExample; gold labels
    ``feats[-1].strip().split(' ')`` keyed by position in the split."""
    fx = feature_extractors or get_basic_clean_features()
    index = len(labels_dict)
    for ex in raw_features:
        ids = get_thresholded_features(lexicon, fx, _info(ex), ex[2], ex[3], threshold,
                                       expand=True)
        examples_list.append(OieExample(ex[2], ex[3], ids, ex[5], relation=ex[9]))
        labels_dict[index] = _strip(ex[-1]).split(" ")
        index += 1


# ---------------------------------------------------------------------------------------
# the preprocessed dataset file (JSON in place of OiePreprocessor.py:290-364's pickle)
# ---------------------------------------------------------------------------------------
def save_preprocessed(path, feat_extrs, lexicon, dataset, goldstandard):
    for k in dataset:
        assert k in SPLIT_LABELS, f"split '{k}' not in {SPLIT_LABELS}"
    doc = {"format": "rae-preprocessed-v1",
           "extractors": [f.__name__ for f in feat_extrs],
           "lexicon": lexicon.to_json(),
           "dataset": {k: [[e.arg1, e.arg2, e.features, e.trigger, e.relation] for e in v]
                       for k, v in dataset.items()},
           "goldstandard": {k: [[i, lab] for i, lab in sorted(v.items())]
                            for k, v in goldstandard.items()}}
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "wt", encoding="utf-8") as fp:
        json.dump(doc, fp)


def load_preprocessed(path):
    """-> (feature extractors, FeatureLexicon, {split: [OieExample]}, {split: {i: labels}})."""
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rt", encoding="utf-8") as fp:
        doc = json.load(fp)
    if doc.get("format") != "rae-preprocessed-v1":
        raise ValueError(f"{path}: not a file written by rae.preprocess")
    fx = [_EXTRACTORS[n] for n in doc["extractors"]]
    lex = FeatureLexicon.from_json(doc["lexicon"])
    dataset = {k: [OieExample(a1, a2, f, t, r) for a1, a2, f, t, r in v]
               for k, v in doc["dataset"].items()}
    gold = {k: {int(i): list(lab) for i, lab in v} for k, v in doc["goldstandard"].items()}
    return fx, lex, dataset, gold


def index_dataset(oie_dataset, n_features, power: float = 0.75):
    """learning/OieData.py:36-90 -> DatasetManager: entity ids over all splits (first-mention
    order, see the module docstring), binary CSR features, int32 argument vectors."""
    if "train" not in oie_dataset:
        raise Exception("Dataset manager requires that the provided dataset contains a "
                        "'train' split.")
    arg2id, freqs = {}, []
    for split in SPLIT_LABELS:                      # generate_args, OieData.py:143-155
        for ex in oie_dataset.get(split, ()):
            for a in (ex.arg1, ex.arg2):
                i = arg2id.get(a)
                if i is None:
                    arg2id[a] = len(freqs)
                    freqs.append(1)
                else:
                    freqs[i] += 1
    splits = {}
    for split in SPLIT_LABELS:
        exs = oie_dataset.get(split)
        if exs is None:
            continue
        n = len(exs)
        a1 = np.fromiter((arg2id[e.arg1] for e in exs), dtype=np.int32, count=n)
        a2 = np.fromiter((arg2id[e.arg2] for e in exs), dtype=np.int32, count=n)
        rows = np.repeat(np.arange(n), [len(e.features) for e in exs])
        cols = np.fromiter((f for e in exs for f in e.features), dtype=np.int64,
                           count=len(rows))
        X = sp.csr_matrix((np.ones(len(rows), np.float32), (rows, cols)), shape=(n, n_features))
        X.sum_duplicates()
        X.data[:] = 1.0                             # dok assignment: duplicates collapse
        splits[split] = DatasetSplit(a1, a2, X)
    dm = DatasetManager(splits, np.asarray(freqs, dtype=np.int64), n_features, power)
    dm.arg2Id = arg2id
    dm.id2Arg = {i: a for a, i in arg2id.items()}
    return dm


def load_data(path, rng=None, verbose=False):
    """learning/OieInduction.py:417-436: preprocessed file -> (DatasetManager, gold standard)."""
    if not os.path.exists(path):
        print(f"Pickled '{path}' dataset not found", file=sys.stderr)
        sys.exit(1)
    _, lex, data, gold = load_preprocessed(path)
    dm = index_dataset(data, lex.get_feature_space_dimensionality())
    dm.featureLex = lex
    return dm, gold


def preprocess(input_file, output_file, batch="train", thres=0, test_mode=False, verbose=False):
    """The OiePreprocessor.py:377-414 main: add ``batch`` from ``input_file`` to the
    (possibly existing) preprocessed file."""
    t0 = time.time()
    raw = read_examples(input_file)
    fx, lex, dataset, gold = get_basic_clean_features(), FeatureLexicon(), {}, {}
    if os.path.exists(output_file):
        fx, lex, dataset, gold = load_preprocessed(output_file)
    examples = dataset.setdefault(batch, [])
    labels = gold.setdefault(batch, {})
    build_feature_lexicon(raw, fx, lex)
    load_features(raw, lex, examples, labels, thres, fx)
    save_preprocessed(output_file, fx, lex, dataset, gold)
    if verbose:
        print(f"{len(raw)} examples, {lex.nextId} lexicon entries, {lex.nextIdPruned} "
              f"thresholded features, {time.time() - t0:.2f} s", file=sys.stderr)
    return fx, lex, dataset, gold


def main(argv=None):
    p = argparse.ArgumentParser(description="Processes an Oie file and add its representations "
                                            "to a preprocessed dataset file.")
    p.add_argument("input_file", metavar="input-file", help="input file in the Yao format, "
                                                             "like data-sample.txt")
    p.add_argument("pickled_dataset", metavar="pickled-dataset",
                   help="output .json / .json.gz (created if absent, else extended)")
    p.add_argument("--batch", "--batch-name", dest="batch", metavar="batch-name", default="train",
                   nargs="?", help="split name: train, valid or test (README.md:32-34 spells the "
                                   "flag --batch-name)")
    p.add_argument("--thres", metavar="threshold-value", default=0, nargs="?", type=int)
    p.add_argument("--test-mode", action="store_true")
    a = p.parse_args(argv)
    preprocess(a.input_file, a.pickled_dataset, a.batch, a.thres, a.test_mode, verbose=True)


if __name__ == "__main__":
    main()
