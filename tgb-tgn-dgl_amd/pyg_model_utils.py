"""Drop-in for the reference's pyg_model_utils.py (getModel / getOptimizer of the PyG TGN: TGNMemory +
IdentityMessage + LastAggregator, GraphAttentionEmbedding, LinkPredictor) — tgnx HIP path.

getModel(feature_dim, hidden_dim, num_nodes, device) keeps the reference signature
(pyg_model_utils.py:10-36) and returns {'memory', 'gnn', 'link_pred'} (+ 'model', the flat-buffer
owner); getOptimizer(model, lr) is Adam over the three modules' parameters (:38-43), run on the
device inside the train step.  Keyword extras: ring (sampler K), max_batch, max_neg (eval
negatives per event), aggr ('last' as the reference, or 'mean'), dropout (attention, 0.1), layers (2:
2-hop attention), updater ('gru' | 'rnn': TGNMemory's memory_updater_cell, memory_module.py:57,70-78),
memory ('tgn', or 'dyrep': DyRepMemory, memory_module.py:218-421, with the same updater choice)."""
from tgnx.tgn import TGNModel, TgnAdam, getModel, getOptimizer  # noqa: F401
