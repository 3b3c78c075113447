"""Host-side pieces that need no GPU: the command line (learning/OieInduction.py:461-500 and
the README aliases), the .npz dataset format, batch sizing, and the product path's refusal to
run without the HIP library."""
import os
import subprocess
import sys

import numpy as np
import pytest

from rae import cli
from rae.data import batch_nnz_stats, load_npz, save_npz, synthetic_dataset


def test_cli_flags_and_defaults_match_reference():
    a = cli.get_command_args(["data.npz", "--model-name", "m", "--decoder", "sp"])
    # learning/OieInduction.py:464-480 defaults
    assert (a.epochs, a.learning_rate, a.batch_size, a.embed_size, a.relations, a.neg_samples,
            a.l1, a.l2, a.optimizer, a.alpha, a.seed) == (100, 0.1, 50, 30, 3, 5, 0.0, 0.0,
                                                           "adagrad", 1.0, 2)
    assert a.ext_reg is True and a.ext_emb is False and a.freq_eval is False


def test_cli_readme_aliases():
    # README.md:44 / BASELINE.json config 1
    a = cli.get_command_args(["--pickled_dataset", "x.npz", "--model_name", "discrete-autoencoder",
                              "--decoder", "sp", "--optimization", "1", "--epochs", "10",
                              "--batch_size", "100", "--relations_number", "10",
                              "--negative_samples_number", "5", "--l2_regularization", "0.1",
                              "--alpha", "0.1", "--seed", "2", "--embed_size", "10",
                              "--learning_rate", "0.1"])
    assert (a.dataset, a.model_name, a.optimizer, a.epochs, a.batch_size, a.relations,
            a.neg_samples, a.l2, a.alpha, a.embed_size) == ("x.npz", "discrete-autoencoder",
                                                            "adagrad", 10, 100, 10, 5, 0.1, 0.1, 10)


def test_cli_requires_model_name_and_decoder():
    with pytest.raises(SystemExit):
        cli.get_command_args(["d.npz", "--decoder", "sp"])
    with pytest.raises(SystemExit):
        cli.get_command_args(["d.npz", "--model-name", "x"])
    with pytest.raises(SystemExit):
        cli.get_command_args(["d.npz", "--model-name", "x", "--decoder", "bogus"])


def test_npz_round_trip(tmp_path):
    data, gold = synthetic_dataset(500, 700, 4, seed=3)
    p = tmp_path / "ds.npz"
    save_npz(p, data, gold)
    d2, g2 = load_npz(p)
    x1, x2 = data.split["train"].xFeats, d2.split["train"].xFeats
    assert (x1 != x2).nnz == 0
    assert np.array_equal(data.split["train"].args1, d2.split["train"].args1)
    assert np.array_equal(data.negSamplingCum, d2.negSamplingCum)
    assert g2 == gold


def test_batch_nnz_stats():
    indptr = np.array([0, 3, 4, 9, 10, 12])
    assert batch_nnz_stats(indptr, 2) == (6, 5)     # batches [0,2) -> 4, [2,4) -> 6; max row 5


def test_product_path_fails_loudly_without_library(tmp_path):
    code = ("import os, sys; os.environ['RAE_LIB'] = os.path.join(sys.argv[1], 'missing.so');"
            "sys.path.insert(0, sys.argv[2]);"
            "from rae import _lib\n"
            "try:\n    _lib.load()\nexcept _lib.RaeError as e:\n    print('refused', e)\n")
    out = subprocess.run([sys.executable, "-c", code, str(tmp_path),
                          os.path.join(os.path.dirname(os.path.dirname(__file__)),
                                       "relation-autoencoder_amd")],
                         capture_output=True, text=True, timeout=120)
    assert "refused" in out.stdout, out.stdout + out.stderr


def test_checkpoint_round_trip_cpu(tmp_path):
    """Params, AdaGrad accumulators, the shared RNG position and the epoch cursor survive a
    save/load (the reference's save() keeps only the parameters, OieInduction.py:110-116)."""
    import torch
    from rae.inducer import ReconstructInducer
    data, gold = synthetic_dataset(300, 400, 3, seed=5)

    def make():
        return ReconstructInducer(data, gold, np.random.RandomState(2), 3, 0.1, 50, 8, 5, 3, 0.0,
                                  0.0, "adagrad", "ck", "rescal+sp", False, True, False, 1.0,
                                  device=torch.device("cpu"))
    a = make()
    from rae.model import make_optimizer
    a.optimizer = make_optimizer("adagrad", a.modelFunc.params)
    g = torch.Generator().manual_seed(0)
    for t in a.modelFunc.params + a.optimizer.accumulator:
        t.add_(torch.rand(t.shape, generator=g))
    a.rng.uniform(size=17)
    a.cur_epoch, a.train_errors = 1, [3.5]
    a.save_checkpoint(tmp_path / "ck.npz")
    b = make()
    b.load_checkpoint(tmp_path / "ck.npz")
    for (k, x), y in zip(a.modelFunc.named_params().items(), b.modelFunc.params):
        assert torch.equal(x, y), k
    for x, y in zip(a.optimizer.accumulator, b.optimizer.accumulator):
        assert torch.equal(x, y)
    assert b.cur_epoch == 1 and b.train_errors == [3.5]
    assert np.array_equal(a.rng.uniform(size=5), b.rng.uniform(size=5))


def test_bench_attaches_traffic_of_the_same_batch_size():
    """bench.py's roofline 'traffic' comes from the committed PMC passes taken at the run's own
    per-rank batch size (the passes' bench arguments name it; none = the default 100)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    t = bench.pmc_traffic("c3", 100)
    assert t is not None and "--batch-size" not in t["source"]
    t8 = bench.pmc_traffic("c3", 800)
    assert t8 is not None and "--batch-size 800" in t8["source"]
    assert bench.pmc_traffic("c3", 37) is None


def test_p2p_device_guard():
    """the peer-to-peer exchange refuses ranks on different GPUs unless asked
    (engine.check_p2p_devices, called by TrainEngine._p2p_setup with every rank's device)."""
    from rae.engine import check_p2p_devices
    check_p2p_devices(["gpu-a"] * 8, False)              # ranks sharing one GPU
    with pytest.raises(ValueError, match="p2p_cross_device"):
        check_p2p_devices(["gpu-a", "gpu-b"], False)
    check_p2p_devices(["gpu-a", "gpu-b"], True)


def test_integration_names_every_export():
    """every entry point include/rae.h declares has its binding row or
    recipe in INTEGRATION.md."""
    import re
    from conftest import ROOT
    from test_abi import header_symbols
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    named = set(re.findall(r"\b(rae_[a-z_0-9]+)", doc))
    missing = [s for s in header_symbols() if s not in named]
    assert not missing, missing
