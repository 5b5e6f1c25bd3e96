"""Drop-in for the reference's temporal_dataset.py (TemporalGraphDataset)."""
from tgnx.data import TemporalGraphDataset  # noqa: F401
