"""tgnx — MI355X-native TGN temporal link-prediction hot path (HIP kernels behind a C ABI).

Drop-in surface of cseduashraful/tgb-tgn-dgl:
  LastNeighborLoader        neighbor_loader.py:15-109
  NegLinkSamplerDest        neg_sampler.py:3-23
  getModel / getOptimizer   model_utils.py:700-710
  train / test              epoch_utils.py:15-318
  parse_config / getDataWithDependecyBlock   utils.py:17-67
"""
import os as _os
import sys as _sys
import warnings as _warnings

# The train / eval steps are replayed from HIP graphs. With CLR's graph packet capture (its default) the replayed
# wiki step ran 0.0917 ms, without it 0.0878 ms (launch gaps; profiles/r5/r5_graph_packet_ab.txt). CLR reads the
# flag once, when the HIP runtime initialises: effective when tgnx is imported before the first HIP call (the
# reference script's import block comes first).  An explicit setting wins; TGNX_GRAPH_PACKET_CAPTURE=keep leaves
# the runtime's default alone.  The flag is process-wide: it applies to every HIP graph of the process
# ("Runtime settings").
GRAPH_PACKET_ENV = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
_preset = GRAPH_PACKET_ENV in _os.environ
if _os.environ.get("TGNX_GRAPH_PACKET_CAPTURE", "") != "keep":
    _os.environ.setdefault(GRAPH_PACKET_ENV, "0")


def _hip_initialized() -> bool:
    """Whether this process already initialised the HIP runtime through torch (without importing torch)."""
    torch = _sys.modules.get("torch")
    try:
        return bool(torch is not None and torch.cuda.is_initialized())
    except Exception:
        return False


# effective = the runtime will read the setting: set before the first HIP call (or set by the user beforehand)
graph_packet_setting_effective = _preset or not _hip_initialized()
if not graph_packet_setting_effective and _os.environ.get("TGNX_GRAPH_PACKET_CAPTURE", "") != "keep":
    _warnings.warn("tgnx was imported after the HIP runtime was initialised (torch.cuda is already in use): "
                   f"{GRAPH_PACKET_ENV}=0 cannot take effect, so replayed steps keep CLR's graph packet capture "
                   "(~4 % slower on the wiki-shaped step). Import tgnx before the first torch.cuda call, or set "
                   f"{GRAPH_PACKET_ENV}=0 in the environment.", RuntimeWarning, stacklevel=2)

from ._lib import LIB_PATH, lib  # noqa: F401,E402

__version__ = "0.1.0"
