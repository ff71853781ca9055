"""Mistral-7B int2-g64 policy decode token (bench.decode_workload, no prefill): development tool for A/B builds
(NAD_LIB_PATH)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402

cfg = bench.MISTRAL if (len(sys.argv) < 2 or sys.argv[1] == "mistral") else bench.LLAMA_ASYM
print(json.dumps(bench.decode_workload(cfg, torch, reps=20, prefill=False)), flush=True)
