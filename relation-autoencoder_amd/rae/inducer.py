"""ReconstructInducer: the trainer that drives the training path
(learning/OieInduction.py:26-319), same constructor, same ``func`` dictionary, same epoch
loop and RNG consumption -- with the step running on MI355X.
"""
from __future__ import annotations

import sys
import time
from collections import Counter

import numpy as np
import torch

from .data import SPLIT_LABELS
from .engine import DeviceSplit, TrainEngine
from .evaluation import construct_split_evaluator
from .model import OieModelFunctions, _as_bool, make_optimizer
from .negatives import NegativeExampleGenerator


class _TrainFunction:
    """``func['train'](batch_index, neg1, neg2) -> cost`` (OieInduction.py:146-149)."""

    def __init__(self, engine):
        self.engine = engine

    def __call__(self, batch_index, neg1, neg2):
        return self.engine.train_call(batch_index, neg1, neg2)


class _LabelFunction:
    """``func['label_<split>'](batch_index) -> (labels, probs)`` (OieInduction.py:151-155)."""

    def __init__(self, engine, split, batch_size):
        self.engine = engine
        self.split = split
        self.l = batch_size

    def __call__(self, batch_index):
        b = int(batch_index)
        lab, pr = self.engine.label(self.split, b * self.l, self.l)
        return lab.cpu().numpy(), pr.cpu().numpy()

    def all_labels(self, nb_batches):
        """Labels of the first nb_batches*l rows in one launch (tail dropped as the
        reference's per-batch loop does, OieInduction.py:337)."""
        lab, _ = self.engine.label(self.split, 0, nb_batches * self.l, probs=False)
        return lab.cpu().numpy()


class ReconstructInducer:
    def __init__(self, data, gold_standard, rng, nb_epochs, learning_rate, batch_size,
                 embed_size, nb_relations, nb_neg_samples, lambda1, lambda2, optimization,
                 model_name, decoder_model, external_embeddings, extended_regularizer,
                 frequent_eval, alpha, *, device=None, world_size=1, rank=0, exchange=None,
                 graph_chunk=64, neg_sampler="device", neg_seed=0, mfma_bf16=False,
                 kernel_forms=None, dp_update="replicated", index_window=0,
                 index_overlap=True, p2p_cross_device=False, p2p_timeout=5.0):
        self.data = data
        self.goldStandard = gold_standard
        self.rng = rng
        self.nb_epochs = nb_epochs
        self.learningRate = learning_rate
        self.batch_size = batch_size
        self.embedSize = embed_size
        self.relationNum = nb_relations
        self.neg_sample_num = nb_neg_samples
        self.lambdaL1 = lambda1
        self.lambdaL2 = lambda2
        self.optimization = optimization
        self.modelName = model_name
        self.decoder_type = decoder_model
        self.extEmb = external_embeddings
        self.extendedReg = extended_regularizer
        self.frequentEval = _as_bool(frequent_eval)
        self.alpha = alpha
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.world_size = int(world_size)
        self.rank = int(rank)
        self.exchange = exchange
        self.graph_chunk = graph_chunk
        if neg_sampler not in ("host", "device", "philox"):
            raise ValueError("neg_sampler must be 'host', 'device' or 'philox'")
        self.neg_sampler = neg_sampler     # host / device: the reference's RNG stream
        self.neg_seed = int(neg_seed)
        self.mfma_bf16 = bool(mfma_bf16)   # RESCAL / hybrid: bf16 MFMA operands (config 5)
        self.kernel_forms = dict(kernel_forms or {})   # engine.TrainEngine kernel_forms
        self.index_window = int(index_window)          # engine.TrainEngine row-index ring
        self.index_overlap = bool(index_overlap)       # next window's index beside the steps
        self.dp_update = dp_update         # "replicated" | "partitioned" (rae/dist.py)
        # peer-to-peer exchange (kernel_forms dp_xchg="p2p"): ranks on different GPUs only
        # when asked for (engine.TrainEngine._p2p_setup); a wait's bound in seconds
        self.p2p_cross_device = bool(p2p_cross_device)
        self.p2p_timeout = float(p2p_timeout)
        self.negativeSampler = NegativeExampleGenerator(rng, data.negSamplingCum)   # :85
        self.modelID = (f"{decoder_model}_{model_name}_maxepoch{nb_epochs}_lr{learning_rate}"
                        f"_embedsize{embed_size}_l1{lambda1}_l2{lambda2}_opt{optimization}"
                        f"_rel_num{nb_relations}_batch{batch_size}_negs{nb_neg_samples}")
        self.modelFunc = OieModelFunctions(rng, embed_size, nb_relations, nb_neg_samples,
                                           batch_size, decoder_model, data, extended_regularizer,
                                           alpha, external_embeddings=external_embeddings,
                                           device=self.device)          # :90
        self.func = dict(zip([SPLIT_LABELS[0]] + ["label_" + s for s in SPLIT_LABELS],
                             [None] * (1 + len(SPLIT_LABELS))))         # :91
        self.cur_epoch = 0
        self.evaluator = {s: None for s in SPLIT_LABELS}
        for split in self.data.generate_split_keys():
            self.evaluator[split] = construct_split_evaluator(
                (gold_standard or {}).get(split, {}), split)
        self.batch_reps = {s: None for s in SPLIT_LABELS}
        for split in self.data.generate_split_keys():
            # Py2 integer division: tail dropped (:98); data-parallel global batch
            self.batch_reps[split] = self.data.split[split].args1.shape[0] // (
                self.batch_size * (self.world_size if split == "train" else 1))
        self.cluster = {s: None for s in SPLIT_LABELS}
        self.train_errors = []
        self.epoch_costs = []
        self.engine = None
        self.optimizer = None
        self._resume = False        # set by load_checkpoint: keep optimizer state + epoch cursor

    def initialize(self):
        """OieInduction.py:103-108: re-draw all parameters from the shared RNG.  Like the
        reference, the next train()/learn() then starts from epoch 0 with a fresh optimizer
        (compile_function builds a new zero-accumulator AdaGrad, OieInduction.py:137)."""
        self._drop_engine()
        self.optimizer = None
        self._resume = False
        self.cur_epoch = 0
        self.train_errors = []
        self.epoch_costs = []
        self.modelFunc = OieModelFunctions(self.rng, self.embedSize, self.relationNum,
                                           self.neg_sample_num, self.batch_size,
                                           self.decoder_type, self.data, self.extendedReg,
                                           self.alpha, external_embeddings=self.extEmb,
                                           device=self.device)

    def _drop_engine(self):
        if self.engine is not None:
            self.engine.close()
        self.engine = None
        self.func = {k: None for k in self.func}

    # ------------------------------------------------------------------ compile
    def compile_function(self):
        """OieInduction.py:118-155: build the train function and one labelling function
        per split."""
        if self.optimizer is None or not self._resume:
            # a fresh zero-accumulator optimizer per compile, as the reference builds one
            # (:137); only a loaded checkpoint keeps its accumulators
            self.optimizer = make_optimizer(self.optimization, self.modelFunc.params)
        self.engine = TrainEngine(self.modelFunc, self.optimizer, self.data.split["train"],
                                  learning_rate=self.learningRate, lambda1=self.lambdaL1,
                                  lambda2=self.lambdaL2, world_size=self.world_size,
                                  rank=self.rank, exchange=self.exchange,
                                  graph_chunk=self.graph_chunk, device=self.device,
                                  mfma_bf16=self.mfma_bf16, kernel_forms=self.kernel_forms,
                                  dp_update=self.dp_update, index_window=self.index_window,
                                  index_overlap=self.index_overlap,
                                  p2p_cross_device=self.p2p_cross_device,
                                  p2p_timeout=self.p2p_timeout)
        self.func["train"] = _TrainFunction(self.engine)
        for key in self.data.generate_split_keys():
            ds = self.engine.split if key == "train" else DeviceSplit(self.data.split[key], self.device)
            self.func["label_" + key] = _LabelFunction(self.engine, ds, self.batch_size)

    def _check_for_compiled_functions(self):
        return self.func.get("train") is not None

    # ------------------------------------------------------------------ train / learn
    def train(self, debug=False):
        """OieInduction.py:157-170 (wall-clock timers instead of process CPU time)."""
        t0 = time.perf_counter()
        if not self._check_for_compiled_functions():
            self.compile_function()
        compile_duration = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.learn(debug=debug)
        train_duration = time.perf_counter() - t0
        print("Compiling completed in {:.1f}s".format(compile_duration), file=sys.stderr)
        print("Training completed in {:.1f}s".format(train_duration), file=sys.stderr)
        if self.cur_epoch:
            print("Trained for {} epochs. Avg epoch duration: {:.1f}s".format(
                self.cur_epoch, train_duration / float(self.cur_epoch)))

    def draw_epoch_negatives(self):
        """OieInduction.py:183-184: neg1 then neg2, each (s, N), from the shared RNG."""
        N = self.data.split["train"].args1.shape[0]
        neg1 = self.negativeSampler.get_negative_samples(N, self.neg_sample_num)
        neg2 = self.negativeSampler.get_negative_samples(N, self.neg_sample_num)
        return neg1, neg2

    def learn(self, debug=False, verbose=True):
        """OieInduction.py:172-219.  Per epoch: draw negatives on the host RNG (parity mode),
        upload once, run every batch on the device, read the per-batch costs back and sum
        them in batch order (err += cost, :189)."""
        if not self._check_for_compiled_functions():
            self.compile_function()
        nb = self.batch_reps["train"]
        # the reference always starts at epoch 0 (:175); a loaded checkpoint resumes at the
        # epoch it was taken at
        epoch = self.cur_epoch if self._resume else 0
        self._resume = False
        while epoch < self.nb_epochs:
            t0 = time.perf_counter()
            epoch += 1
            self.cur_epoch = epoch
            if self.neg_sampler == "host":
                neg1, neg2 = self.draw_epoch_negatives()
                self.engine.set_epoch_negatives(neg1, neg2)
            else:
                self.engine.sample_epoch_negatives(self.negativeSampler, self.neg_sampler,
                                                   self.neg_seed, epoch - 1)
            if self.frequentEval:
                # per-batch evaluation needs the host between batches (:190-198)
                for b in range(nb):
                    self.engine.run(b, 1, graph=False)
                    if self._mode() == 1:
                        print(b * self.batch_size, b, "#" * 60)
                        print(self.get_clusters_size(), "\n")
                    else:                       # mode 2: valid + test after every batch
                        print(b * self.batch_size, b, "#" * 60)
                        for split in SPLIT_LABELS[1:]:
                            self.cluster[split] = self.get_clusters_sets(split)
                            self._evaluate(split, verbose=verbose)
            else:
                self.engine.run(0, nb)
            costs = self.engine.costs[:nb].double().cpu().numpy()
            self.engine.check()
            self.epoch_costs.append(costs)
            err = 0.0
            for c in costs:
                err += float(np.float32(c))
            self.train_errors.append(err)
            if verbose:
                print("\nEPOCH", epoch)
                print("Training error: {:.4f}".format(err))
                print("Epoch duration: {:.1f}s".format(time.perf_counter() - t0))
            if self._mode() == 1:
                self.cluster["train"] = self.get_clusters_sets("train")
                self._evaluate("train", verbose=verbose)
            else:
                for split in SPLIT_LABELS[1:]:
                    self.cluster[split] = self.get_clusters_sets(split)
                    self._evaluate(split, verbose=verbose)
        return self.train_errors

    # ------------------------------------------------------------------ clusters / eval
    def _labels(self, split):
        nbs = self.data.split[split].args1.shape[0] // self.batch_size
        return self.func["label_" + split].all_labels(nbs)

    def get_clusters_sets(self, split):
        """get_clusters_sets (OieInduction.py:321-340): cluster id -> set of example ids."""
        clusters = {i: set() for i in range(self.relationNum)}
        for idx, pred in enumerate(self._labels(split)):
            clusters[int(pred)].add(idx)
        return clusters

    def get_clusters_size(self, split="train"):
        """get_clusters_size (OieInduction.py:248-259)."""
        return Counter(int(x) for x in self._labels(split))

    def _evaluate(self, split, verbose=True):
        ev = self.evaluator.get(split)
        if ev is None:
            return None
        ev.feed_induced_clusters(self.cluster[split])
        f1, pre, rec = ev.compute_metrics()
        if verbose:
            print("{} f1: {:.4f} pre: {:.4f} rec: {:.4f}".format(split, f1, pre, rec))
        return f1, pre, rec

    def _mode(self):
        """OieInduction.py:300-312."""
        if len(self.data.split) == 1 and "train" in self.data.split:
            return 1
        if len(self.data.split) == 3 and all(k in self.data.split for k in SPLIT_LABELS):
            return 2
        raise Exception("Either 'train' split or 'train', 'valid' and 'test' splits should be defined")

    def gather(self):
        """Make this rank's replica whole (partitioned data-parallel update: every A / Ab / W
        row and accumulator from its owner).  A collective -- call it on EVERY rank, e.g. before
        a rank-0-only save_checkpoint or labelling pass; a no-op when nothing is stale and for
        the replicated update."""
        if self.engine is not None:
            self.engine.sync_replicas(accumulators=True)

    def state_dict(self):
        """Parameters + AdaGrad accumulators + RNG state + epoch cursor (the reference's
        save() keeps only the parameters and loses the accumulators and the RNG position,
        OieInduction.py:110-116, so a reloaded model cannot continue the same run).
        Partitioned data-parallel update: if rows are stale this gathers them (a collective:
        all ranks must call it) -- call gather() on every rank first to save from one rank."""
        if self.engine is not None and self.engine.stale(accumulators=True):
            self.engine.sync_replicas(accumulators=True)
        sd = {"params": {k: v.detach().cpu() for k, v in self.modelFunc.named_params().items()},
              "rng": self.rng.get_state(), "epoch": self.cur_epoch,
              "train_errors": list(self.train_errors)}
        if self.optimizer is not None and self.optimizer.accumulator is not None:
            sd["acc"] = {k: v.detach().cpu() for k, v in
                         zip(self.modelFunc.param_names, self.optimizer.accumulator)}
        return sd

    def save_checkpoint(self, path):
        """state_dict() as a flat .npz (no pickles)."""
        sd = self.state_dict()
        name, key, pos, has_gauss, gauss = sd["rng"]
        out = {"epoch": np.int64(sd["epoch"]), "train_errors": np.array(sd["train_errors"]),
               "rng_key": key, "rng_pos": np.int64(pos), "rng_has_gauss": np.int64(has_gauss),
               "rng_gauss": np.float64(gauss), "decoder": np.str_(self.decoder_type)}
        for k, v in sd["params"].items():
            out["param/" + k] = v.numpy()
        for k, v in sd.get("acc", {}).items():
            out["acc/" + k] = v.numpy()
        np.savez(path, **out)

    def load_checkpoint(self, path):
        """Restore a save_checkpoint() file into this inducer (same shapes/decoder): the
        parameters and accumulators are copied into the existing device tensors (a built
        engine keeps its pointers), the shared RNG resumes its stream and learn() continues
        at the next epoch."""
        z = np.load(path, allow_pickle=False)
        if str(z["decoder"]) != self.decoder_type:
            raise ValueError(f"checkpoint decoder {z['decoder']} != {self.decoder_type}")
        for k, v in self.modelFunc.named_params().items():
            v.copy_(torch.as_tensor(z["param/" + k]))
        if self.optimizer is None and self.optimization is not None:
            self.optimizer = make_optimizer(self.optimization, self.modelFunc.params)
        if self.optimizer is not None and self.optimizer.accumulator is not None:
            for k, v in zip(self.modelFunc.param_names, self.optimizer.accumulator):
                v.copy_(torch.as_tensor(z["acc/" + k]))
        self.rng.set_state(("MT19937", z["rng_key"], int(z["rng_pos"]), int(z["rng_has_gauss"]),
                            float(z["rng_gauss"])))
        self.cur_epoch = int(z["epoch"])
        self.train_errors = [float(x) for x in z["train_errors"]]
        self._resume = True
