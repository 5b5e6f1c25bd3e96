"""CPU checks of the C-ABI library: it loads, exports every declared symbol, and its host-side
entry points (no GPU needed) match the oracle / goldens."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT


def _declared():
    hdr = open(os.path.join(ROOT, "include", "tgnx.h")).read()
    return sorted(set(re.findall(r"\b(tgnx_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    from tgnx import _lib
    L = _lib.lib()
    names = _declared()
    assert len(names) >= 8
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.SIGNATURES, f"{n} declared in include/tgnx.h but not bound in tgnx/_lib.py"
    assert L.tgnx_version() >= 1


def test_block_ids_host_matches_golden(golden):
    from tgnx import _lib
    z = golden("blocks.npz")
    src = np.ascontiguousarray(z["src"])
    dst = np.ascontiguousarray(z["dst"])
    out = np.empty_like(src)
    rc = _lib.lib().tgnx_block_ids_host(src.ctypes.data, dst.ctypes.data, src.shape[0], int(z["batch"][0]),
                                        out.ctypes.data)
    assert rc == 0
    np.testing.assert_array_equal(out, z["blocks"])


def test_block_ids_host_rejects_bad_input():
    from tgnx import _lib
    src = np.array([1, -2], dtype=np.int64)
    out = np.empty_like(src)
    rc = _lib.lib().tgnx_block_ids_host(src.ctypes.data, src.ctypes.data, 2, 2, out.ctypes.data)
    assert rc != 0
    assert b"negative" in _lib.lib().tgnx_last_error()


def test_torch_ops_library_registers_every_op():
    """torch.ops.tgnx (csrc/tgnx_torch.cpp, TORCH_LIBRARY over the C ABI) loads without a GPU and
    registers its schemas; the host op (block_ids) runs and matches the oracle (dependencyGraph.py:8-49)."""
    import numpy as np
    import torch

    from oracle import blocks_ref
    from tgnx import ops
    ns = ops.load()
    for name in ops.OPS:
        assert hasattr(ns, name), name
    assert "Tensor(a!) assoc" in str(ns.ring_sample.default._schema)
    rng = np.random.default_rng(0)
    src, dst = rng.integers(0, 50, 600), rng.integers(0, 50, 600)
    got = ns.block_ids(torch.from_numpy(src), torch.from_numpy(dst), 200).numpy()
    assert np.array_equal(got, blocks_ref.block_ids(src, dst, 200))
