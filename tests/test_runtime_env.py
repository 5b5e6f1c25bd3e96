"""The graph-replay runtime setting `tgnx` applies at import (tgnx/__init__.py, INTEGRATION.md "Runtime settings"):
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 is read by the HIP runtime once, when it initialises, so an import after the first
torch.cuda call cannot apply it — that case must warn instead of failing silently.  CPU-only: the initialised
runtime is simulated (torch.cuda.is_initialized patched) in a fresh interpreter."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tgb-tgn-dgl_amd")

PROBE = r"""
import json, os, sys, warnings
sys.path.insert(0, {pkg!r})
import torch
if {initialised}:
    torch.cuda.is_initialized = lambda: True
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    import tgnx
print(json.dumps({{"warned": any("cannot take effect" in str(x.message) for x in w),
                   "effective": tgnx.graph_packet_setting_effective,
                   "env": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")}}))
"""


def _probe(initialised, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "TGNX_GRAPH_PACKET_CAPTURE")}
    e.update(env or {})
    out = subprocess.run([sys.executable, "-c", PROBE.format(pkg=PKG, initialised=initialised)], env=e,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def test_import_before_hip_sets_the_flag_silently():
    r = _probe(False)
    assert r == {"warned": False, "effective": True, "env": "0"}


def test_import_after_hip_init_warns():
    r = _probe(True)
    assert r["warned"] and not r["effective"]


def test_explicit_setting_wins_and_does_not_warn():
    r = _probe(True, {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "1"})
    assert r == {"warned": False, "effective": True, "env": "1"}


def test_keep_leaves_the_runtime_default():
    r = _probe(True, {"TGNX_GRAPH_PACKET_CAPTURE": "keep"})
    assert not r["warned"] and r["env"] is None
