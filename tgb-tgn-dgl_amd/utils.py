"""Drop-in for the reference's utils.py (parse_config / getDataWithDependecyBlock)."""
from tgnx.data import Evaluator, getDataWithDependecyBlock, parse_config  # noqa: F401
