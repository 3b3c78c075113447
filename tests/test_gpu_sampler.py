"""Device negative sampler (rae_neg_sample / rae_neg_sample_philox) vs the reference sampler
(learning/NegativeExampleGenerator.py:14-32): parity mode must be bit-identical to
``cum.searchsorted(RandomState.uniform(0, cum[-1], N*s))``; the Philox perf mode must follow
the CDF's distribution and be deterministic in (seed, offset)."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _search(lib, cum_t, u_t, out_t):
    from rae import _lib
    _lib.check(lib.rae_neg_sample(C.c_void_p(cum_t.data_ptr()), cum_t.numel(),
                                  C.c_void_p(u_t.data_ptr()), u_t.numel(),
                                  C.c_void_p(out_t.data_ptr()), None))


def test_parity_mode_matches_reference_golden(built_lib, cuda_dev):
    import torch
    z = np.load(os.path.join(GOLDEN, "sampler.npz"))
    rng = np.random.RandomState(int(z["seed"]))
    N, s = int(z["N"]), int(z["s"])
    cum = torch.as_tensor(z["cum"], device=cuda_dev)
    for key in ("neg1", "neg2"):                  # neg1 then neg2 on the same stream
        u = torch.as_tensor(rng.uniform(0, z["cum"][-1], N * s), device=cuda_dev)
        out = torch.empty(N * s, dtype=torch.int32, device=cuda_dev)
        _search(built_lib, cum, u, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().reshape(s, N), z[key]), key


def test_parity_mode_large_and_ties(built_lib, cuda_dev):
    import torch
    from rae.data import synthetic_dataset
    data, _ = synthetic_dataset(20000, 3000, 5, seed=4)
    cum_np = data.negSamplingCum
    rng = np.random.RandomState(9)
    u_np = np.concatenate([rng.uniform(0, cum_np[-1], 2_000_000),
                           cum_np[::97], [0.0], np.nextafter(cum_np[:50], 0)])  # exact ties
    cum = torch.as_tensor(cum_np, device=cuda_dev)
    u = torch.as_tensor(u_np, device=cuda_dev)
    out = torch.empty(u_np.size, dtype=torch.int32, device=cuda_dev)
    _search(built_lib, cum, u, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), cum_np.searchsorted(u_np).astype(np.int32))


def test_philox_mode_distribution_and_determinism(built_lib, cuda_dev):
    import torch
    from rae import _lib
    freqs = np.array([50, 20, 10, 5, 5, 3, 2, 2, 1, 1, 1], dtype=np.int64)
    from rae.data import neg_sampling_cum
    cum_np = neg_sampling_cum(freqs)
    cum = torch.as_tensor(cum_np, device=cuda_dev)
    n = 4_000_000

    def draw(seed, off):
        out = torch.empty(n, dtype=torch.int32, device=cuda_dev)
        _lib.check(built_lib.rae_neg_sample_philox(C.c_void_p(cum.data_ptr()), cum.numel(), seed,
                                                   off, n, C.c_void_p(out.data_ptr()), None))
        torch.cuda.synchronize()
        return out.cpu().numpy()
    a, b, c = draw(7, 0), draw(7, 0), draw(7, n)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, c)
    pmf = np.diff(np.concatenate([[0.0], cum_np]))
    freq = np.bincount(a, minlength=len(cum_np)) / n
    assert np.all(np.abs(freq - pmf) <= 5 * np.sqrt(pmf * (1 - pmf) / n) + 1e-6)


def test_epoch_with_device_sampler_equals_host_sampler(built_lib, cuda_dev):
    """The whole training run is identical with the host and the device parity sampler."""
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    data, gold = synthetic_dataset(800, 900, 5, seed=12)
    out = []
    for mode in ("host", "device"):
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 2, 0.1, 40, 12, 6, 3, 0.0,
                                 0.0, "adagrad", "neg", "sp", False, True, False, 1.0,
                                 device=cuda_dev, graph_chunk=4, neg_sampler=mode)
        ind.learn(verbose=False)
        out.append({k: v.detach().cpu().numpy() for k, v in ind.modelFunc.named_params().items()})
    for k in out[0]:
        assert np.array_equal(out[0][k], out[1][k]), k
