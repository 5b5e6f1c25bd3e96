"""World-size-2 `gloo` test (CPU) of the TGN data-parallel exchange (tgnx/tgn.py
TgnEngine._exchange): ONE all-reduce over [gradients | world x xcap memory-row slots], each rank
writing only its own slot (rows with float-integer headers, include/tgnx.h TGNX_TGN_ROW; the other
slots zero).  The summed row part must equal the all-gather of the slots bit for bit — node ids,
int64 last_update values beyond 2^32 and negative ones, unused-slot markers, arbitrary memory floats —
and the gradient part the element-wise sum."""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

G, XCAP, D = 1000, 6, 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _slot(rank):
    import sys
    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    from tgnx.tgn import row_header
    rng = np.random.default_rng(100 + rank)
    rows = np.zeros((XCAP, D + 4), dtype=np.float32)
    lus = [0, 1_700_000_123, (1 << 40) + 12345, -5, (1 << 62) + 7]
    for u in range(XCAP):
        if u < XCAP - 1:
            rows[u, :4] = row_header(rank * 100_000 + 16_000_000 * (u == 0) + u, lus[u % len(lus)])
            rows[u, 4:] = rng.standard_normal(D).astype(np.float32) * 10.0 ** rng.integers(-20, 20, D)
        else:
            rows[u, 0] = -1.0          # unused slot
    return rows


def _run(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rw = D + 4
    comm = torch.zeros(G + world * XCAP * rw, dtype=torch.float32)
    comm[:G] = torch.from_numpy(np.random.default_rng(rank).standard_normal(G).astype(np.float32))
    xg = comm[G:].view(world * XCAP, rw)
    xg[rank * XCAP:(rank + 1) * XCAP] = torch.from_numpy(_slot(rank))
    dist.all_reduce(comm)
    np.save(os.path.join(out_dir, f"r{rank}.npy"), comm.numpy())
    dist.destroy_process_group()


def test_exchange_all_reduce_is_all_gather():
    import sys
    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    from tgnx.tgn import row_decode, row_header
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_run, args=(world, _free_port(), d), nprocs=world, join=True)
        outs = [np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)]
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    want = np.concatenate([_slot(r) for r in range(world)])
    got = outs[0][G:].reshape(world * XCAP, D + 4)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    gsum = sum(np.random.default_rng(r).standard_normal(G).astype(np.float32) for r in range(world))
    assert np.allclose(outs[0][:G], gsum, rtol=1e-6, atol=1e-6)
    # header round trip
    for v, lu in ((0, 0), (16_777_215, (1 << 63) - 1), (5, -(1 << 40)), (123, 1_700_000_000)):
        assert row_decode(np.asarray(row_header(v, lu), dtype=np.float32)) == (v, lu)


def _run_modes(rank, world, port, out_dir):
    import sys
    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    from tgnx.tgn import exchange_collectives
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rw = D + 4
    for mode in ("fused", "split"):
        for async_op in (False, True):
            comm = torch.zeros(G + world * XCAP * rw, dtype=torch.float32)
            comm[:G] = torch.from_numpy(np.random.default_rng(rank).standard_normal(G).astype(np.float32))
            xg = comm[G:].view(world * XCAP, rw)
            xg[rank * XCAP:(rank + 1) * XCAP] = torch.from_numpy(_slot(rank))
            for w in exchange_collectives(comm, G, rank, world, mode, async_op=async_op):
                w.wait()
            np.save(os.path.join(out_dir, f"{mode}_{int(async_op)}_r{rank}.npy"), comm.numpy())
    dist.destroy_process_group()


def test_exchange_modes_agree():
    """The engine's exchange knob (TgnEngine.exchange_mode / TGNX_EXCHANGE; tgnx.tgn.exchange_collectives):
    'split' = gradient all-reduce + in-place all_gather_into_tensor of the row slots gives bit for bit the buffer
    that 'fused' (one all-reduce of [gradients | slots]) gives, on every rank, blocking and async."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_run_modes, args=(world, _free_port(), d), nprocs=world, join=True)
        outs = {(m, a, r): np.load(os.path.join(d, f"{m}_{a}_r{r}.npy"))
                for m in ("fused", "split") for a in (0, 1) for r in range(world)}
    ref = outs[("fused", 0, 0)]
    want = np.concatenate([_slot(r) for r in range(world)])
    assert np.array_equal(ref[G:].reshape(world * XCAP, D + 4).view(np.uint32), want.view(np.uint32))
    for k, v in outs.items():
        assert np.array_equal(v.view(np.uint32), ref.view(np.uint32)), k
