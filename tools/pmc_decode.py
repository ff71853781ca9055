"""Workload for the PMC traffic pass (development tool): a few decode tokens through the per-op launches and a few
prefill GEMMs, on the bench's synthetic Llama-2-7B stack (fewer layers: the per-launch
counters do not depend on the layer count)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

cfg = dict(bench.LLAMA, layers=int(os.environ.get("PMC_LAYERS", "4")))
stack = bench.Stack(cfg, 0, 1)
dec = bench.Runner(stack, 1, None, "cuda")
for _ in range(3):
    dec.step()
pre = bench.Runner(stack, 2048, None, "cuda")
pre.step()
torch.cuda.synchronize()
# algorithmic bytes of the per-op decode launches above (tools/pmc_traffic.py divides the counters by these)
if os.environ.get("PMC_ALG_OUT"):
    import json
    L1 = stack.launches(1)
    launches = sum(c for *_, c in L1)
    json.dump({"decode_bytes_per_token": sum(b * c for _, b, _, c in L1), "decode_launches_per_token": launches,
               "decode_tokens": 3}, open(os.environ["PMC_ALG_OUT"], "w"))
