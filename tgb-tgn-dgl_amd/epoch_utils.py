"""Drop-in for the reference's epoch_utils.py (train / test) — fused HIP step."""
from tgnx.epoch import test, train  # noqa: F401
