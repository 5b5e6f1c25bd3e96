"""Phase timing of the single-workgroup kernels (assemble) from a -DTGNX_TIMING build.

    TGNX_LIB=build_var/timing/libtgnx.so python tools/phase_timing.py
Runs the bench workload eagerly and reports the mean wall-clock time of each phase (µs)."""
import ctypes
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tgb-tgn-dgl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import block_ids  # noqa: E402
from tgnx import _lib  # noqa: E402
from tgnx.engine import TgnnEngine  # noqa: E402
from tgnx.model import TGNN, getOptimizer  # noqa: E402
from tgnx.sampler import LastNeighborLoader  # noqa: E402
from tgnx.synth import SHAPES, make_stream  # noqa: E402

NAMES = {1: "negs+keys", 2: "touch sort", 3: "sp scan", 4: "runs+nodemap", 5: "seg counts", 6: "block sort",
         7: "offset scan"}


def main(steps=200, B=200):
    dev = torch.device("cuda", 0)
    shape = SHAPES["tgbl-wiki"]
    s = make_stream(shape, seed=0)
    blk = block_ids(s.src, s.dst, B)
    ev = dict(src=torch.from_numpy(s.src).to(dev), dst=torch.from_numpy(s.dst).to(dev),
              t=torch.from_numpy(s.t.astype(np.float32)).to(dev), blk=torch.from_numpy(blk).to(dev),
              msg=torch.from_numpy(s.msg).to(dev))
    model = TGNN(shape.msg_dim, 100, shape.num_nodes, dev, ring=10, max_batch=B, max_neg=1,
                 generator=torch.Generator().manual_seed(0))
    opt = getOptimizer({"gnn": model}, 1e-4)
    loader = LastNeighborLoader(shape.num_nodes, 10, device=dev)
    eng = TgnnEngine(model, loader, ev["msg"], opt, dst_nodes=torch.from_numpy(np.unique(s.dst)), seed=1)
    neg_buf = torch.zeros(s.num_events, dtype=torch.long, device=dev)
    eng.bind_resident(ev["src"], ev["dst"], ev["t"], ev["blk"], ev["msg"], neg_buf, 0, s.train_end, B)
    off = _lib.lib().tgnx_tgnn_ws_misc_offset(ctypes.byref(model.cfg))
    nb_epoch = math.ceil(s.train_end / B)
    acc = {}
    for i in range(steps):
        if i % nb_epoch == 0:
            eng.begin_epoch()
        eng.resident_train_step()
        torch.cuda.synchronize()
        st = eng.ws[off + 64: off + 64 + 8 * 11].cpu().view(torch.int64).numpy()
        if i < 10:
            continue
        for k in range(1, 8):
            acc.setdefault(NAMES[k], []).append((st[k] - st[k - 1]) * 0.01)   # 100 MHz wall clock
        acc.setdefault("total wg0", []).append((st[7] - st[0]) * 0.01)
        acc.setdefault("ring plan wg1", []).append((st[10] - st[8]) * 0.01)
    for k, v in acc.items():
        print(f"{k:16s} {np.mean(v):8.2f} us")


if __name__ == "__main__":
    main(B=int(sys.argv[1]) if len(sys.argv) > 1 else 200)
