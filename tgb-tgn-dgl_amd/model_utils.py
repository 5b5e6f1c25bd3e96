"""Drop-in for the reference's model_utils.py (getModel / getOptimizer, TGNN) — tgnx HIP path."""
from tgnx.model import TGNN, FusedAdam, getModel, getOptimizer  # noqa: F401
