"""Entry script with the reference's CLI (pyg-mem-tgn.py --data <name> --config <yml>).

Runs the running reference path (TGNN, dependency-block batching; --path dgl, the default) or the
PyG TGN memory path (--path pyg: pyg_model_utils + the canonical loop in pyg_epoch_utils, the
import swap at pyg-mem-tgn.py:23-25) on the fused HIP step: train + validation MRR per epoch,
wall-clock per phase.  Extra flags: --epochs overrides train.epoch (the reference's 3000 is a run
length, not a smoke test), --batch overrides train.batch_size.  Data: a TGB dataset name
(synthetic stream of that shape; no network here) or an .npz with src/dst/t/msg, see tgnx/data.py.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from neg_sampler import NegLinkSamplerDest  # noqa: E402
from neighbor_loader import LastNeighborLoader  # noqa: E402
from utils import getDataWithDependecyBlock, parse_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", type=str, default="tgbl-wiki", help="dataset name")
    ap.add_argument("--config", type=str, default=os.path.join(os.path.dirname(__file__), "config", "TGN.yml"))
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--path", choices=["dgl", "pyg"], default="dgl", help="#change based on dgl/pyg")
    args = ap.parse_args()
    # the reference's imports (pyg-mem-tgn.py:16-25): epoch_utils for both paths (it hands a TGN model to the
    # PyG loop), the model module per the "#change based on dgl/pyg" swap
    from epoch_utils import test, train
    if args.path == "dgl":
        from model_utils import getModel, getOptimizer
    else:
        from pyg_model_utils import getModel, getOptimizer

    device = torch.device("cuda")
    sample_param, memory_param, gnn_param, train_param = parse_config(args.config)
    if args.batch:
        train_param["batch_size"] = args.batch
    epochs = args.epochs if args.epochs is not None else train_param["epoch"]
    data, train_dl, val_dl, test_dl, neg_sampler, evaluator, metric = getDataWithDependecyBlock(args.data, train_param)
    neg_dest_sampler = NegLinkSamplerDest(torch.unique(data.dst), device=device)
    neighbor_loader = LastNeighborLoader(data.num_nodes, size=sample_param["neighbor"][0], device=device)
    assoc = torch.empty(data.num_nodes, dtype=torch.long, device=device)
    # pyg-mem-tgn.py:49: the config's other sections (memory.mail_combine / memory_update, neighbor,
    # batch_size) reach the model through gnn_param (tgnx parse_config records the file)
    model = getModel(data.msg.shape[1], gnn_param["dim_out"], data.num_nodes, device, gnn_param=gnn_param)
    optimizer = getOptimizer(model, train_param["lr"])
    criterion = torch.nn.BCEWithLogitsLoss()
    t_start = time.time()
    for e in range(epochs):
        print("Epoch {:d}:".format(e))
        t0 = time.time()
        loss = train(model, data.msg, train_dl, neighbor_loader, neg_dest_sampler, assoc, device, optimizer, criterion)
        t1 = time.time()
        print(f"Epoch: {e + 1:02d}, Loss: {loss:.4f}, Training elapsed Time (s): {t1 - t0: .4f}")
        t0 = time.time()
        mrr = test(model, data.msg, val_dl, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion,
                   evaluator, metric, "val")
        t1 = time.time()
        print(f"Validation {metric}: {mrr: .4f}, elapsed Time (s): {t1 - t0: .4f}")
    print(f"Execution Time: {time.time() - t_start:.6f} seconds")


if __name__ == "__main__":
    main()
