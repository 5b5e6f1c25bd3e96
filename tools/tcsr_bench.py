"""The bench's t-CSR sampler leg alone (bench.tcsr_sampler_bench): one JSON line.  The kernel variant is
chosen by TGNX_TCSR_GROUPS in the environment (0: wave per root, 1: G-lane groups, 2: two roots per group)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps({"TGNX_TCSR_GROUPS": os.environ.get("TGNX_TCSR_GROUPS"),
                      **bench.tcsr_sampler_bench(None)}))
