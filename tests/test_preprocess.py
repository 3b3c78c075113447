"""Dataset ingestion (rae.preprocess): the reference's OiePreprocessor.py / OieFeatures.py
restated, and BASELINE config 1 (data-sample.txt, m=10, r=10, s=5, l=100) end to end on the
CPU oracle -- the reference's own C1 is "plumbing, no GPU".

The feature extractors are checked on a line written here (a made-up sentence in the Yao
format), each expected value derived by hand from the cited reference lines.  data-sample.txt
is read from /root/reference when present (this container); the GPU box only has the derived
fixture tests/golden/c1_sample.npz (oracle/gen_c1_fixture.py), which is checked here to be
exactly what the ingestion produces.  bow_clean's stopword list (nltk) is unpinned.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

SAMPLE = "/root/reference/data-sample.txt"
have_sample = pytest.mark.skipif(not os.path.exists(SAMPLE), reason="reference data absent")

# path, e1, e2, types, trigger, doc, sentence, pos, label (+ newline, as read from a file)
LINE = ["->nsubj->wrote->dobj->", "Ada Lovelace", "The Notes", "PERSON-WORK",
        "TRIGGER:wrote", "./2000/01/02/1.xml",
        "In 1843 , Ada Lovelace famously wrote The Notes on engines .",
        "IN CD , NNP NNP RB VBD DT NNPS IN NNS .", "/book/author/works_written\n"]


def _ex():
    return ["0"] + LINE


def _info(ex):
    from rae.preprocess import _info
    return _info(ex)


def test_feature_extractors_follow_reference_lines():
    from rae import preprocess as P
    ex = _ex()
    info, a1, a2 = _info(ex), ex[2], ex[3]
    assert P.trigger(info, a1, a2) == "wrote"                      # OieFeatures.py:136-137
    assert P.entityTypes(info, a1, a2) == "PERSON-WORK"            # :140-141
    assert P.entity1Type(info, a1, a2) == "PERSON"                 # :144-145
    assert P.entity2Type(info, a1, a2) == "WORK"                   # :148-149
    assert P.arg1_lower(info, a1, a2) == "ada lovelace"            # :156-157
    assert P.arg2_lower(info, a1, a2) == "the notes"               # :168-169
    # span 'Ada Lovelace famously wrote The Notes' -> lower, drop stopwords ('the')
    assert P.bow_clean(info, a1, a2) == ["ada", "lovelace", "famously", "wrote", "notes"]
    # path tokens: nsubj wrote dobj -> odd positions: 'wrote'
    assert P.lexicalPattern(info, a1, a2) == "wrote"               # :176-187
    # tags strictly between 'Lovelace' (idx 4) and 'The' (idx 7): RB VBD
    assert P.posPatternPath(info, a1, a2) == "RB_VBD"              # :204-227


def test_extractor_edge_cases():
    from rae import preprocess as P
    info = ["<-a->b<-c->", "X-Y", "TRIGGER:x", "Foo 12abc bar-baz Qux", "NN NN NN NN", "d"]
    # digits drop '12abc'; punctuation is stripped only at the ends ('bar-baz' stays)
    assert P.bow_clean(info, "Foo", "Qux") == ["foo", "bar-baz", "qux"]
    assert P.lexicalPattern(info, "Foo", "Qux") == "b"             # tokens a b c -> odd: b
    # arg2's first token not in the sentence -> '' (OieFeatures.py:224-225)
    assert P.posPatternPath(info, "Foo", "Nope") == ""
    with pytest.raises(AssertionError):                           # :210 length check
        P.posPatternPath(["", "", "", "a b", "NN", ""], "a", "b")


def test_lexicon_threshold_and_pruned_ids():
    """Two passes (OiePreprocessor.py:113-118, 244-287): frequencies count every
    occurrence; pruned ids in first-pass order; thres=1 keeps features seen twice+."""
    from rae import preprocess as P
    ex0 = _ex()
    ex1 = _ex()
    ex1[0] = "1"
    ex1[2] = "Charles Babbage"
    ex1[7] = ex1[7].replace("Ada Lovelace", "Charles Babbage")
    raw = [ex0, ex1]
    for thres in (0, 1):
        lex, exs, gold = P.FeatureLexicon(), [], {}
        P.build_feature_lexicon(raw, P.get_basic_clean_features(), lex)
        P.load_features(raw, lex, exs, gold, thres)
        assert lex.get_freq(lex.get_id("trigger#wrote")) == 2
        assert gold == {0: ["/book/author/works_written"], 1: ["/book/author/works_written"]}
        names0 = [lex.get_str_pruned(i) for i in exs[0].features]
        names1 = [lex.get_str_pruned(i) for i in exs[1].features]
        if thres == 0:
            assert "arg1_lower#ada lovelace" in names0 and "arg1_lower#charles babbage" in names1
            assert exs[0].features[0] == 0 and lex.get_str_pruned(0) == "trigger#wrote"
        else:
            # only the features both examples share survive
            assert set(names0) == set(names1)
            assert "arg1_lower#ada lovelace" not in names0
        assert lex.get_feature_space_dimensionality() == lex.nextIdPruned


def test_unseen_feature_in_expand_mode_raises_like_reference():
    from rae import preprocess as P
    lex = P.FeatureLexicon()
    with pytest.raises(KeyError):                                 # OiePreprocessor.py:202
        P.get_thresholded_features(lex, [P.trigger], _info(_ex()), "a", "b", 0, expand=True)


def test_read_examples_format_checks(tmp_path):
    from rae import preprocess as P
    f = tmp_path / "x.txt"
    f.write_text("\t".join(LINE))
    ex = P.read_examples(str(f))
    assert ex[0][0] == "0" and ex[0][-1] == LINE[-1]               # newline kept
    f.write_text("a\tb\n")
    with pytest.raises(AssertionError):                           # :235 nine fields
        P.read_examples(str(f))
    f.write_text("\t".join(LINE) + "   \n")
    with pytest.raises(IOError):                                  # :231-232 blank line
        P.read_examples(str(f))


def test_json_file_round_trip_and_split_extension(tmp_path):
    """The CLI flow of README.md:30-34: the same file added as train, valid, test."""
    from rae import preprocess as P
    src = tmp_path / "in.txt"
    rows = []
    for i, name in enumerate(["Ada Lovelace", "Charles Babbage", "Alan Turing"]):
        ln = list(LINE)
        ln[0], ln[1] = LINE[0], name
        ln[6] = LINE[6].replace("Ada Lovelace", name)
        ln[8] = "\n" if i == 2 else LINE[8]
        rows.append("\t".join(ln))
    src.write_text("".join(rows))
    out = tmp_path / "ds.json.gz"
    for split in ("train", "valid", "test"):
        P.main([str(src), str(out), "--batch-name", split])
    fx, lex, ds, gold = P.load_preprocessed(str(out))
    assert [f.__name__ for f in fx] == [f.__name__ for f in P.get_basic_clean_features()]
    assert set(ds) == {"train", "valid", "test"} and all(len(v) == 3 for v in ds.values())
    assert gold["test"][2] == [""]                                # unlabelled example
    assert ds["valid"][1].features == ds["train"][1].features     # same lexicon ids
    assert lex.get_freq(lex.get_id("trigger#wrote")) == 9          # 3 passes x 3 lines
    dm, g = P.load_data(str(out))
    assert dm.get_arg_voc_size() == 4                             # 3 authors + 'The Notes'
    assert dm.arg2Id["Ada Lovelace"] == 0 and dm.arg2Id["The Notes"] == 1
    np.testing.assert_array_equal(dm.entity_freqs, [3, 9, 3, 3])
    for s in ("train", "valid", "test"):
        x = dm.split[s].xFeats
        assert x.shape == (3, lex.get_feature_space_dimensionality())
        assert np.all(x.data == 1.0)
    with pytest.raises(AssertionError):                           # OiePreprocessor.py:312
        P.main([str(src), str(out), "--batch", "dev"])


@have_sample
def test_data_sample_matches_committed_fixture():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import gen_c1_fixture as G
    from rae.data import load_npz
    dm, gold = G.build(SAMPLE)
    want, wgold = load_npz(os.path.join(GOLDEN, "c1_sample.npz"))
    a, b = dm.split["train"], want.split["train"]
    assert a.xFeats.shape == b.xFeats.shape == (1000, 6271)
    assert (a.xFeats != b.xFeats).nnz == 0
    np.testing.assert_array_equal(a.args1, b.args1)
    np.testing.assert_array_equal(a.args2, b.args2)
    np.testing.assert_array_equal(dm.entity_freqs, want.entity_freqs)
    labelled = {k: v for k, v in gold["train"].items() if v[0] != ""}
    assert len(labelled) == 22                                    # 22/1000 labelled
    assert labelled == {k: v for k, v in wgold["train"].items() if v[0] != ""}
    nnz = np.diff(a.xFeats.indptr)
    assert nnz.min() == 9 and np.median(nnz) == 13                # SURVEY 8(d) stats


def test_c1_plumbing_on_the_oracle():
    """BASELINE config 1 (README.md:44 hyper-parameters: m=10, r=10, s=5, l=100, l2=0.1,
    alpha=0.1, seed 2) through the CPU restatement, plus the B^3 evaluation of its labels."""
    import rae_oracle as O
    from rae.data import load_npz
    from rae.evaluation import construct_split_evaluator
    dm, gold = load_npz(os.path.join(GOLDEN, "c1_sample.npz"))
    tr = dm.split["train"]
    ot = O.OracleTrainer("sp", tr.xFeats, tr.args1, tr.args2, dm.negSamplingCum,
                         np.random.RandomState(2), 10, 10, 5, 100, lr=0.1, alpha=0.1,
                         lambda2=0.1)
    errs = [ot.epoch()[1] for _ in range(2)]
    assert np.all(np.isfinite(errs)) and errs[1] < errs[0]
    lab, _ = ot.labels()
    clusters = {i: set(np.flatnonzero(lab == i).tolist()) for i in range(10)}
    ev = construct_split_evaluator(gold["train"], "train")
    ev.feed_induced_clusters(clusters)
    f1, pre, rec = ev.compute_metrics()
    assert 0.0 < pre <= 1.0 and 0.0 < rec <= 1.0


def test_cli_loads_preprocessed_file(tmp_path):
    """python -m rae <file.json.gz>: the trainer's dataset loader takes the preprocessor's
    output (learning/OieInduction.py:495 load_data)."""
    from rae import preprocess as P
    from rae.cli import get_command_args, load_dataset
    src = tmp_path / "in.txt"
    src.write_text("\t".join(LINE) * 1)
    out = tmp_path / "ds.json"
    P.main([str(src), str(out)])
    a = get_command_args([str(out), "--model-name", "x", "--decoder", "sp"])
    dm, gold = load_dataset(a.dataset)
    assert dm.split["train"].xFeats.shape[0] == 1 and gold["train"][0] == [LINE[-1].strip()]
