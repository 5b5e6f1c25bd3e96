"""ORACLE — CPU restatement of the reference's hot path. TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import anything from this package, and only as the checker / the timed CPU
baseline.  The product (`tgb-tgn-dgl_amd/`) never imports it: its path runs on
the HIP library and fails loudly when that library is missing.

Pinning:
  sampler_ref   LastNeighborLoader  neighbor_loader.py:15-109  pinned: tests/golden/sampler_*.npz
  blocks_ref    get_block           dependencyGraph.py:8-49    pinned: tests/golden/blocks.npz
  negs_ref      NegLinkSamplerDest  neg_sampler.py:3-23        pinned: tests/golden/negs.npz (exact RNG replay)
  tgnn_ref      TGNN per-block loop model_utils.py:14-237,422-697  TimeEncode/EdgePredictor pinned by
                tests/golden/model.npz; the DGL graph ops (in_subgraph, edge_softmax, update_all)
                are restated from DGL's documented semantics: PARITY UNPINNED against DGL itself
                (dgl is not installed; no reference fixture covers them).
  epoch_ref     train/test loops    epoch_utils.py:15-318      built on the above
  memory_ref    TGNMemory + msg/agg modules/memory_module.py:25-215, msg_func.py, msg_agg.py:
                PARITY UNPINNED (torch_geometric / torch_scatter / modules/time_enc.py absent);
                IdentityMessage pinned by tests/golden/msg.npz
  mrr_ref       TGB Evaluator MRR   [ext] py-tgb linkproppred evaluator: PARITY UNPINNED
"""
