"""tgnx — MI355X-native TGN temporal link-prediction hot path (HIP kernels behind a C ABI).

Drop-in surface of cseduashraful/tgb-tgn-dgl:
  LastNeighborLoader        neighbor_loader.py:15-109
  NegLinkSamplerDest        neg_sampler.py:3-23
  getModel / getOptimizer   model_utils.py:700-710
  train / test              epoch_utils.py:15-318
  parse_config / getDataWithDependecyBlock   utils.py:17-67
"""
from ._lib import LIB_PATH, lib  # noqa: F401

__version__ = "0.1.0"
