"""
heat_amd - an MI355X-native distributed tensor and data-analytics framework with Heat's
NumPy-like ``DNDarray`` API and split-axis semantics.

One process per GPU (``python -m heat_amd.run -n 8 script.py`` or ``torchrun``); process-local
data are PyTorch-ROCm tensors; communication is RCCL over xGMI through ``torch.distributed``;
hot paths are hand-written CDNA4 (gfx950) HIP kernels in :mod:`heat_amd.ops`.

Usage mirrors the reference: ``import heat_amd as ht; x = ht.random.rand(10**6, 64, split=0)``.
"""
from .core import *
from .core import __version__
from .core import linalg
from .core import random
from . import ops
from . import parallel
from . import spatial
from . import cluster
from . import graph
from . import regression
from . import naive_bayes
from . import classification
from . import nn
from . import optim
from . import utils
from . import profiling
from . import datasets
from . import testing

profiling._auto_enable()
