"""Drop-in for the reference's dependencyGraph.py (get_block / dependecyAwareBatch) — native block ids."""
from tgnx.data import block_ids, dependecyAwareBatch, get_block  # noqa: F401
