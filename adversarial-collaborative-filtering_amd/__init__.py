"""MI355X-native APR (adversarial BPR-MF) training path.

Drop-in surface of feay1234/Adversarial-Collaborative-Filtering's APR path:
``MF`` / ``Session`` (APR.py:85-202), ``training`` / ``training_batch`` /
``training_loss_acc`` (APR.py:206-292, utils.py:106-175), ``sampling`` /
``shuffle`` (APR.py:30-61), ``init_eval_model`` / ``evaluate`` (utils.py:178-267),
``OriginalDataset`` (Dataset.py:226-327), ``Recommender`` / ``APR``
(Recommender.py, run.py:157), CLIs of run_adv_ori.py / run_adv.py.

The package directory name contains hyphens; import it with
``importlib.import_module("adversarial-collaborative-filtering_amd")`` (the
module also registers itself as ``acf_amd``).
"""
import sys as _sys

from . import _native  # noqa: F401
from .data import (DeviceDataset, OriginalDataset, SyntheticDataset, get_dataset, ml1m_like, pinterest_like,
                   synthetic_dataset, synthetic_large, yelp_like)
from .evaluate import evaluate, init_eval_model
from .evaluation import evaluate_apr_mode, evaluate_model
from .model import MF, Session
from .neumf import AdversarialNeuMF, NeuMF
from .fast_adversarial_mf import FastAdversarialMF
from .recommender import APR, Recommender
from .sampler import DeviceSampler, EpochTriplets, sampling, shuffle
from .train import (output_evaluate, prediction2file, training, training_batch, training_loss_acc,
                    write2file)

_sys.modules.setdefault("acf_amd", _sys.modules[__name__])

__all__ = [
    "APR", "AdversarialNeuMF", "DeviceDataset", "FastAdversarialMF", "DeviceSampler", "EpochTriplets", "MF", "NeuMF", "OriginalDataset", "Recommender", "Session",
    "SyntheticDataset", "evaluate", "evaluate_apr_mode", "evaluate_model", "get_dataset", "init_eval_model", "ml1m_like", "output_evaluate",
    "pinterest_like", "prediction2file", "sampling", "shuffle", "synthetic_dataset", "synthetic_large", "training",
    "training_batch", "training_loss_acc", "write2file", "yelp_like",
]
