"""Drop-in for the reference's pyg_epoch_utils.py (train / test of the PyG TGN memory path) — fused HIP
step (tgnx/tgn_epoch.py; epoch_utils.train / test dispatch there for a TGN model as well)."""
from tgnx.tgn_epoch import test, train  # noqa: F401
