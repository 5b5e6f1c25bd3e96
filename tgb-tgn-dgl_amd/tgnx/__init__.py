"""tgnx — MI355X-native TGN temporal link-prediction hot path (HIP kernels behind a C ABI).

Drop-in surface of cseduashraful/tgb-tgn-dgl:
  LastNeighborLoader        neighbor_loader.py:15-109
  NegLinkSamplerDest        neg_sampler.py:3-23
  getModel / getOptimizer   model_utils.py:700-710
  train / test              epoch_utils.py:15-318
  parse_config / getDataWithDependecyBlock   utils.py:17-67
"""
import os as _os

# The train / eval steps are replayed from HIP graphs. With CLR's graph packet capture (its default) the replayed
# wiki step ran 0.0917 ms, without it 0.0878 ms (launch gaps; profiles/r5/r5_graph_packet_ab.txt). CLR reads the
# flag when the HIP runtime initialises: effective when tgnx is imported before the first HIP call (the reference
# script's import block comes first); an explicit setting wins.
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from ._lib import LIB_PATH, lib  # noqa: F401,E402

__version__ = "0.1.0"
