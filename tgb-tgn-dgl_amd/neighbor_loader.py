"""Drop-in for the reference's neighbor_loader.py (LastNeighborLoader) — HIP ring kernels."""
from tgnx.sampler import LastNeighborLoader  # noqa: F401
