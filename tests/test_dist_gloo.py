"""World-size-2 `gloo` test (CPU) of the data-parallel decomposition the HIP step uses:
every rank replays the whole global batch's ring / time_assoc state, computes the loss only on
the rows of its event slice [B*r/W, B*(r+1)/W) (normalised by the global B), all-reduces the
gradients, and applies the same Adam step.  The result must equal the single-process step."""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, out_dir, steps):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import blocks_ref
    from oracle.epoch_ref import _assemble
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgnn_ref import RefTGNN
    from tgnx.synth import make_stream

    torch.set_num_threads(1)
    if world > 1:
        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    N, B, d = 300, 120, 16
    s = make_stream("tgbl-wiki", seed=11, num_events=B * steps, num_nodes=N, msg_dim=d)
    blk_all = blocks_ref.block_ids(s.src, s.dst, B)
    torch.manual_seed(0)
    model = RefTGNN(d, 100, N, feat_drop=0.0, attn_drop=0.0)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    loader = RefLastNeighborLoader(N, 10)
    feats = torch.from_numpy(s.msg)
    rng = np.random.default_rng(5)
    lo, hi = B * rank // world, B * (rank + 1) // world
    losses = []
    for st in range(steps):
        sl = slice(st * B, (st + 1) * B)
        src, dst = torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl])
        neg = torch.from_numpy(rng.choice(s.dst_nodes, size=B))      # same draws on every rank
        t = torch.from_numpy(s.t[sl].astype(np.float32))
        msg, blk = torch.from_numpy(s.msg[sl]), torch.from_numpy(blk_all[sl])
        opt.zero_grad()
        g, bf, bt, blocks = _assemble(loader, feats, src, dst, neg, t, msg, blk)
        pos_out, neg_out = model(g, bf, bt, blocks)
        order = np.argsort(blk.numpy(), kind="stable")              # reference rows are in block order
        mine = torch.from_numpy((order >= lo) & (order < hi))
        loss = (torch.nn.functional.softplus(-pos_out.view(-1))[mine].sum()
                + torch.nn.functional.softplus(neg_out.view(-1))[mine].sum()) / B
        loss.backward()
        if world > 1:
            for p in model.parameters():
                if p.grad is not None:
                    dist.all_reduce(p.grad)
            lt = loss.detach().clone()
            dist.all_reduce(lt)
            loss = lt
        opt.step()
        loader.insert(src.numpy(), dst.numpy(), t.numpy())       # whole global batch on every rank
        losses.append(float(loss.detach()))
    params = {k: v.detach().numpy() for k, v in model.named_parameters() if v.requires_grad}
    np.savez(os.path.join(out_dir, f"r{rank}_w{world}.npz"), losses=np.array(losses), **params)
    if world > 1:
        dist.destroy_process_group()


def test_dp_decomposition_gloo_world2():
    steps = 3
    with tempfile.TemporaryDirectory() as td:
        _run(0, 1, 0, td, steps)
        mp.spawn(_run, args=(2, _free_port(), td, steps), nprocs=2, join=True)
        ref = np.load(os.path.join(td, "r0_w1.npz"))
        for r in (0, 1):
            got = np.load(os.path.join(td, f"r{r}_w2.npz"))
            np.testing.assert_allclose(got["losses"], ref["losses"], rtol=1e-5, atol=1e-6)
            for k in ref.files:
                if k == "losses":
                    continue
                np.testing.assert_allclose(got[k], ref[k], rtol=0, atol=5e-6, err_msg=k)
