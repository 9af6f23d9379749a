"""Diagnostic: bench.copy_probe (co_probe_copy, the streaming ceiling beside the roofline)
for the headline's byte volume and 2 GiB.  CO_LIB picks a variant library."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rl4co_slap_amd import _native  # noqa: E402

if os.environ.get("CO_LIB"):
    _native.LIB_PATH = os.environ["CO_LIB"]
_native.load()
dev = torch.device("cuda:0")
res = bench.copy_probe(65536 * (17 * 100 + 30), dev, 50)
print(json.dumps({"lib": os.environ.get("CO_LIB", "base"),
                  **{k: {"us": round(v["us"], 2), "GBps": round(v["GBps"], 1)} for k, v in res.items()}}))
