"""Test infrastructure: regenerate tests/golden/c1_sample.npz, BASELINE config 1's dataset.

data-sample.txt (the reference's sample input, /root/reference/data-sample.txt) run through
this repo's ingestion (rae.preprocess: OiePreprocessor.py's two passes, threshold 0) into the
array layout of rae.data.save_npz: the train split's CSR features, entity ids, per-entity
mention counts and the gold labels.  The GPU box has no /root/reference, so the GPU C1 test
reads this fixture; tests/test_preprocess.py re-derives it here and checks it is unchanged.

    python oracle/gen_c1_fixture.py [/root/reference/data-sample.txt]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))

from rae.data import save_npz  # noqa: E402
from rae.preprocess import FeatureLexicon, build_feature_lexicon, get_basic_clean_features, \
    index_dataset, load_features, read_examples  # noqa: E402

SAMPLE = "/root/reference/data-sample.txt"
OUT = os.path.join(ROOT, "tests", "golden", "c1_sample.npz")


def build(path=SAMPLE):
    raw = read_examples(path)
    fx, lex = get_basic_clean_features(), FeatureLexicon()
    examples, labels = [], {}
    build_feature_lexicon(raw, fx, lex)
    load_features(raw, lex, examples, labels, 0, fx)
    dm = index_dataset({"train": examples}, lex.get_feature_space_dimensionality())
    return dm, {"train": labels}


if __name__ == "__main__":
    dm, gold = build(sys.argv[1] if len(sys.argv) > 1 else SAMPLE)
    save_npz(OUT, dm, gold)
    x = dm.split["train"].xFeats
    print(f"{OUT}: {x.shape[0]} examples, d={x.shape[1]}, nnz={x.nnz}, "
          f"entities={dm.get_arg_voc_size()}")
