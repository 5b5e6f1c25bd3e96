"""ORACLE (test infrastructure only) — TGB link-prediction MRR.

[ext] py-tgb `linkproppred.evaluate.Evaluator` (not installed; called at
/root/reference/epoch_utils.py:108-113): per positive,
rank = 0.5 * (#neg > pos + #neg >= pos) + 1, MRR = mean(1 / rank).
PARITY UNPINNED: restated from TGB's published evaluator, no reference fixture.
"""
from __future__ import annotations

import numpy as np


def mrr_batch(y_pred_pos: np.ndarray, y_pred_neg: np.ndarray) -> float:
    pos = np.asarray(y_pred_pos, dtype=np.float64).reshape(-1, 1)
    neg = np.asarray(y_pred_neg, dtype=np.float64)
    opt = (neg > pos).sum(axis=1)
    pes = (neg >= pos).sum(axis=1)
    rank = 0.5 * (opt + pes) + 1.0
    return float((1.0 / rank).mean())
