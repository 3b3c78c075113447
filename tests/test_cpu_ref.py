"""The torch CPU baseline (oracle/cpu_ref.py, Theano's dense schedule on all host threads)
computes the same training steps as the pinned float64 oracle (oracle/rae_oracle.py), so the
cpu_baseline bench.py reports is the reference's algorithm, not a cheaper one."""
import numpy as np
import pytest
import torch

import cpu_ref
import rae_oracle as O


@pytest.mark.parametrize("decoder", ["sp", "rescal", "rescal+sp"])
def test_dense_schedule_matches_oracle(decoder):
    g = np.random.RandomState(3)
    N, d, n, m, r, s, l = 24, 40, 15, 4, 6, 3, 6
    import scipy.sparse as sp
    rows = np.repeat(np.arange(N), 4)
    X = sp.csr_matrix((np.ones(N * 4), (rows, g.randint(0, d, N * 4))), shape=(N, d))
    X.data[:] = 1.0
    X = X.astype(np.float32)
    a1 = g.randint(0, n, N)
    a2 = g.randint(0, n, N)
    p_t = cpu_ref.init_params(np.random.RandomState(2), decoder, d, m, n, r, torch.float64)
    p_o = O.init_params(np.random.RandomState(2), decoder, d, m, n, r)
    for k in p_o:
        np.testing.assert_array_equal(p_t[k].detach().numpy(), p_o[k])
    acc = {k: np.zeros_like(v) for k, v in p_o.items()}
    step = cpu_ref.DenseScheduleStep(decoder, p_t, lr=0.1, alpha=0.7)
    for b in range(N // l):
        rws = slice(b * l, (b + 1) * l)
        n1 = g.randint(0, n, (s, l))
        n2 = g.randint(0, n, (s, l))
        c_t = step(cpu_ref.batch_csr(X, rws, torch.float64), torch.as_tensor(a1[rws]),
                   torch.as_tensor(a2[rws]), torch.as_tensor(n1), torch.as_tensor(n2))
        res = O.train_step_grads(decoder, p_o, X[rws], a1[rws], a2[rws], n1, n2, alpha=0.7)
        O.adagrad_apply(p_o, acc, res.grads, 0.1)
        assert abs(c_t - res.cost) <= 1e-12 * max(1.0, abs(res.cost))
        for k in p_o:
            np.testing.assert_allclose(p_t[k].detach().numpy(), p_o[k], rtol=1e-9, atol=1e-11,
                                       err_msg=k)
