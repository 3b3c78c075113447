"""Command line of the trainer: the flags of learning/OieInduction.py:461-500 (same names,
defaults and meaning), plus the README's aliases (README.md:44: --pickled_dataset,
--model_name, --batch_size, --relations_number, --negative_samples_number,
--l2_regularization, --embed_size, --learning_rate, --optimization).

    python -m rae DATASET --model-name NAME --decoder sp [--epochs 100 ...]

DATASET is a preprocessed file written by ``python -m rae.preprocess`` (.json / .json.gz: the
reference's OiePreprocessor output, stored without pickles), an array dataset written by
rae.data.save_npz, or ``synthetic:N[:d[:K]]`` for the SURVEY 8(d) generator.  Multi-GPU: launch with torch.distributed.run, one process per GPU.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np


def _str_bool(v):
    """learning/OieInduction.py fix_parsing: 'True'/'False' strings from store_true defaults."""
    if isinstance(v, bool):
        return v
    return str(v).lower() in ("true", "1", "yes")


def get_command_args(argv=None, program_name="rae"):
    p = argparse.ArgumentParser(prog=program_name,
                                description="Trains a basic Open Information Extraction Model",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("dataset", nargs="?", default=None,
                   help="preprocessed .json[.gz] (rae.preprocess), dataset .npz "
                        "(rae.data.save_npz) or synthetic:N[:d[:K]]")
    p.add_argument("--pickled_dataset", dest="dataset_alias", default=None, help=argparse.SUPPRESS)
    p.add_argument("--epochs", type=int, default=100, help="the number of training epochs")
    p.add_argument("--learning-rate", "--learning_rate", dest="learning_rate", type=float,
                   default=0.1, help="the initial learning rate")
    p.add_argument("--batch-size", "--batch_size", dest="batch_size", type=int, default=50,
                   help="the size of the minibatches (per GPU)")
    p.add_argument("--embed-size", "--embed_size", dest="embed_size", type=int, default=30,
                   help="the embedding space dimensionality")
    p.add_argument("--relations", "--relations_number", dest="relations", type=int, default=3,
                   help="the number of semantic relation to induce")
    p.add_argument("--neg-samples", "--negative_samples_number", dest="neg_samples", type=int,
                   default=5, help="the number of negative samples to take per entity")
    p.add_argument("--l1", metavar="lambda_1", type=float, default=0.0,
                   help="the value of the L1-norm regularization coefficient")
    p.add_argument("--l2", "--l2_regularization", metavar="lambda_2", dest="l2", type=float,
                   default=0.0, help="the value of the L2-norm regulatization coefficient")
    p.add_argument("--optimizer", choices=["adagrad", "sgd"], type=str, default="adagrad",
                   help="the optimization algorithm")
    p.add_argument("--optimization", type=int, default=None, help=argparse.SUPPRESS)
    p.add_argument("--model-name", "--model_name", dest="model_name", type=str, default=None,
                   help="a name to be given to the trained model instance")
    p.add_argument("--model", dest="legacy_model", default=None, help=argparse.SUPPRESS)
    p.add_argument("--decoder", choices=["rescal", "sp", "rescal+sp"], type=str,
                   help="the type of factorization model to be used as the decoder")
    p.add_argument("--ext-emb", dest="ext_emb", action="store_true", default="False",
                   help="use external embeddings (not supported: SURVEY 8a11 marks it out)")
    p.add_argument("--ext-reg", dest="ext_reg", action="store_true", default="True",
                   help="regularize the factorization (decoder) model parameters as well")
    p.add_argument("--freq-eval", dest="freq_eval", action="store_true", default="False",
                   help="use frequent evaluation")
    p.add_argument("--alpha", type=float, default=1.0,
                   help="the alpha coefficient for scaling the entropy term")
    p.add_argument("--seed", type=int, default=2, help="a seed number")
    p.add_argument("--graph-chunk", type=int, default=64,
                   help="training steps captured per HIP graph (1 = eager launches)")
    if argv is not None and len(argv) == 0:
        p.print_help()
        raise SystemExit(1)
    a = p.parse_args(argv)
    if a.dataset is None:
        a.dataset = a.dataset_alias
    if a.dataset is None:
        p.error("a dataset is required")
    if a.model_name is None:
        p.error("--model-name is required")
    if a.optimization is not None:        # README.md:44 --optimization 1 (AdaGrad) / 0 (SGD)
        a.optimizer = "adagrad" if a.optimization else "sgd"
    if a.decoder is None:
        p.error("--decoder is required (rescal, sp or rescal+sp)")
    a.ext_emb = _str_bool(a.ext_emb)
    a.ext_reg = _str_bool(a.ext_reg)
    a.freq_eval = _str_bool(a.freq_eval)
    if a.ext_emb:
        p.error("--ext-emb (gensim external embeddings) is out of scope")
    return a


def load_dataset(spec: str, seed: int = 1234):
    from .data import load_npz, synthetic_dataset
    if spec.startswith("synthetic:"):
        parts = [int(x) for x in spec.split(":")[1:]]
        N = parts[0]
        d = parts[1] if len(parts) > 1 else 2 ** 17
        K = parts[2] if len(parts) > 2 else 10
        return synthetic_dataset(N, d, K, seed=seed)
    if spec.endswith((".json", ".json.gz")):
        from .preprocess import load_data
        return load_data(spec)
    return load_npz(spec)


def main(argv=None):
    args = get_command_args(sys.argv[1:] if argv is None else argv)
    import torch

    from . import dist as rdist
    from .inducer import ReconstructInducer
    ws, rk, lrank = rdist.init()
    dev = torch.device("cuda", lrank)
    torch.cuda.set_device(dev)
    print("Relation Learner", file=sys.stderr)
    rand = np.random.RandomState(seed=args.seed)
    data, gold = load_dataset(args.dataset)
    exchange = rdist.make_exchange(ws, rk)
    ind = ReconstructInducer(data, gold, rand, args.epochs, args.learning_rate, args.batch_size,
                             args.embed_size, args.relations, args.neg_samples, args.l1, args.l2,
                             args.optimizer, args.model_name, args.decoder, args.ext_emb,
                             args.ext_reg, args.freq_eval, args.alpha, device=dev, world_size=ws,
                             rank=rk, exchange=exchange, graph_chunk=args.graph_chunk)
    if exchange is not None:
        ind.compile_function()
        rdist.warm_up(exchange, ind.engine.exchange_buf)
    ind.train()
    return ind


if __name__ == "__main__":
    main()
