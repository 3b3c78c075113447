"""MI355X-native relation-autoencoder training path (discrete-state relation VAE).

Public surface mirrors the reference (boromir674/relation-autoencoder):
  ReconstructInducer          learning/OieInduction.py:26
  OieModelFunctions           learning/OieModel.py:12
  construct_decoder           learning/models/decoders/Decoder.py:84
  NegativeExampleGenerator    learning/NegativeExampleGenerator.py:4
  DatasetManager/DatasetSplit learning/OieData.py:8,29
  AdaGrad / SGD               learning/Optimizers.py:6,36
The step itself runs as HIP kernels for gfx950 behind the C ABI in include/rae.h.
"""
from .data import DatasetManager, DatasetSplit, neg_sampling_cum, synthetic_dataset  # noqa: F401
from .model import (AdaGrad, SGD, Bilinear, BilinearPlusSP, IndependentRelationClassifiers,  # noqa: F401
                    OieModelFunctions, SelectionalPreferences, construct_decoder)
from .negatives import NegativeExampleGenerator  # noqa: F401


def __getattr__(name):
    # torch-dependent pieces load lazily so the pure-host modules import without a GPU
    if name in ("ReconstructInducer",):
        from .inducer import ReconstructInducer
        return ReconstructInducer
    if name in ("TrainEngine", "DeviceSplit"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
