"""config 2 (K = N = 4096 int4 g128) M = 1: single launches vs 64-problem batches (bench.synthetic_sweep), for A/B
builds (NAD_LIB_PATH).  Prints the M = 1 entries only."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402

bench.SYN_MS = [1, 4096]
r = bench.synthetic_sweep(torch, copies=128, reps=5)
print(json.dumps({k: r[k] for k in ("config2_m1_single_launches", "config2_m1_batched")}), flush=True)
