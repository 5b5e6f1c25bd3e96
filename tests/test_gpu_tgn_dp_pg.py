"""The TGN data-parallel step through a real process group: two processes on one device, gloo
(RCCL refuses two ranks on one GPU), each driving TgnEngine exactly as bench.py does at world 2 —
bind_resident, begin_epoch, capture_resident, replay_resident — so the exchange is the engine's own
asynchronous dist.all_reduce over [gradients | memory-row slots], with the next batch's scan
(tgnx_tgn_scan_next, split_scan) replayed on the compute stream while the collective is in flight, then
the apply-rows + Adam graph (tgnx/tgn.py TgnEngine._allreduce / replay_resident).

Checks, per step:
  * lr = 0 (parameters fixed, so states compare step after step): each rank's memory, last_update, ring
    and message stores against a world-1 engine on the same global batches (memory 1e-5 abs, the rest
    exact), and the two ranks bit-identical;
  * lr = 1e-3: the two ranks' parameters, Adam moments and memory bit-identical after every step (the
    replicas never drift), parameters moved.
The step includes a partial last batch and one step past the split (B = 0)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, d, D, B, NB = 2000, 16, 32, 128, 6


def _stream():
    from tgnx.synth import make_stream
    return make_stream("tgbl-wiki", seed=41, num_events=B * NB, num_nodes=N, msg_dim=d)


def _engine(s, rank, world, lr):
    from oracle.tgn_ref import RefTGN
    from tgnx.sampler import LastNeighborLoader
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    torch.manual_seed(0)
    sd = RefTGN(N, d, hidden=D, aggr="last", dropout=0.1).state_dict()
    dev = torch.device("cuda", 0)
    model = TGNModel(N, s.num_events, d, D, dev, ring=10, max_batch=B, max_neg=1, aggr="last", dropout=0.1)
    model.load_reference_state(sd)
    eng = TgnEngine(model, LastNeighborLoader(N, 10, device=dev),
                    dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg), TgnAdam(model, lr),
                    dst_nodes=s.dst_nodes, seed=99, rank=rank, world=world)
    return eng


def _split_hi():
    return (NB - 3) * B + 40     # NB - 3 full batches, a partial one, then steps past the split


def _snapshot(eng):
    m = eng.model
    return dict(memory=m.memory.memory.cpu().numpy(), last_update=m.memory.last_update.cpu().numpy(),
                flat=m.flat.cpu().numpy(), adam_m=eng.adam_m.cpu().numpy(), adam_v=eng.adam_v.cpu().numpy(),
                eid=eng.loader.e_id.cpu().numpy(), nbr=eng.loader.neighbors.cpu().numpy(),
                store=m.store.cpu().numpy())


def _worker(rank, world, port, lr, split, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tgb-tgn-dgl_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        s = _stream()
        eng = _engine(s, rank, world, lr)
        eng.split_scan = split
        eng.bind_resident(0, _split_hi(), B, dropout=True)
        eng.begin_epoch()
        eng.capture_resident()
        for st in range(NB - 1):
            eng.replay_resident()
            torch.cuda.synchronize()
            eng.check()
            np.savez(os.path.join(out_dir, f"r{rank}_s{st}.npz"), **_snapshot(eng))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _run_ranks(lr, split, out_dir):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, lr, split, str(out_dir))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
        assert p.exitcode == 0, f"rank process exit code {p.exitcode}"


@pytest.mark.parametrize("split", [True, False])
def test_tgn_dp_process_group_lr0_matches_world1(tmp_path, split):
    _run_ranks(0.0, split, tmp_path)
    s = _stream()
    e1 = _engine(s, 0, 1, 0.0)
    # world 1 over the same GLOBAL batches (the ranks' batch B is the global batch, sliced per rank)
    e1.bind_resident(0, _split_hi(), B, dropout=True)
    e1.begin_epoch()
    for st in range(NB - 1):
        e1.resident_train_step()
        torch.cuda.synchronize()
        e1.check()
        ref = _snapshot(e1)
        r0, r1 = (np.load(tmp_path / f"r{r}_s{st}.npz") for r in (0, 1))
        for k in ("memory", "last_update", "eid", "nbr", "store"):
            assert np.array_equal(r0[k], r1[k]), (st, k)
        assert np.array_equal(r0["last_update"], ref["last_update"]), st
        assert np.array_equal(r0["eid"], ref["eid"]) and np.array_equal(r0["store"], ref["store"]), st
        live = ref["eid"] >= 0
        assert np.array_equal(r0["nbr"][live], ref["nbr"][live]), st
        err = float(np.abs(r0["memory"] - ref["memory"]).max())
        assert err < 1e-5, (st, err)
        assert np.array_equal(r0["flat"], ref["flat"]), st   # lr = 0: parameters never move


def test_tgn_dp_process_group_replicas_stay_identical(tmp_path):
    _run_ranks(1e-3, True, tmp_path)
    first = None
    for st in range(NB - 1):
        r0, r1 = (np.load(tmp_path / f"r{r}_s{st}.npz") for r in (0, 1))
        for k in ("flat", "adam_m", "adam_v", "memory", "last_update", "store", "eid"):
            assert np.array_equal(r0[k], r1[k]), (st, k)
        if first is None:
            first = r0["flat"]
    s = _stream()
    init = _engine(s, 0, 1, 0.0).model.flat.cpu().numpy()
    assert not np.array_equal(first, init)       # Adam moved the parameters on both ranks alike
