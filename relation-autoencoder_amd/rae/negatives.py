"""Negative-example generator: learning/NegativeExampleGenerator.py, host parity mode.

The reference draws, once per epoch, ``N*s`` float64 uniforms on the model's single
``numpy.random.RandomState`` and maps each through ``negSamplingCum.searchsorted``
(side='left') -- as a Python-level ``map`` over every scalar (NegativeExampleGenerator.py:32).
Here the same draw is one vectorised searchsorted, element-for-element identical, so the
RNG stream (and therefore every later draw) is unchanged.
"""
from __future__ import annotations

import numpy as np


class NegativeExampleGenerator:
    def __init__(self, rand: np.random.RandomState, neg_sampling_cum):
        self._rand = rand
        self._negSamplingCum = np.asarray(neg_sampling_cum, dtype=np.float64)
        assert abs(self._negSamplingCum[-1] - 1) < 1.e-4, (
            "Negative example generator initialized with a cumulative distribution derived "
            "from a non-normalized one")

    def get_negative_samples(self, num_positive_entities: int, num_negative_samples: int):
        """(s, l) int32 array of sampled entity ids (NegativeExampleGenerator.py:14-24)."""
        return self._get_sample(num_positive_entities * num_negative_samples).reshape(
            (num_negative_samples, num_positive_entities))

    def _get_sample(self, num_samples: int):
        u = self.draw_uniforms(num_samples)
        return np.asarray(self._negSamplingCum.searchsorted(u), dtype=np.int32)

    def draw_uniforms(self, num_samples: int) -> np.ndarray:
        """The float64 draws of one get_negative_samples call (NegativeExampleGenerator.py:
        32): U(0, cum[-1]) from the shared RandomState -- the device sampler searches them."""
        return self._rand.uniform(0, self._negSamplingCum[-1], num_samples)

    @property
    def cum(self) -> np.ndarray:
        return self._negSamplingCum
