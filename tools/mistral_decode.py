"""Decode token (Mistral-7B int2-g64 policy; `llama` / `llama_asym` for the Llama-2-7B stacks) (bench.decode_workload, no prefill): development tool for A/B builds
(NAD_LIB_PATH)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "mistral"
cfg = {"mistral": bench.MISTRAL, "llama": bench.LLAMA, "llama_asym": bench.LLAMA_ASYM}[which]
print(json.dumps(bench.decode_workload(cfg, torch, reps=20, prefill=False)), flush=True)
