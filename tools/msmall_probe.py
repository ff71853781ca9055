"""K = N = 4096 int4 g128 at M = 1..16 (bench.synthetic_sweep rows): per-launch device time, for knob / build A/B
(knobs are read once per process: one configuration per run)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402

bench.SYN_MS = [1, 2, 4, 8, 16, 4096]
r = bench.synthetic_sweep(torch, copies=128, reps=5)
print(os.environ.get("NAD_GEMV_NST", "auto"), " ".join(f"M={x['m']}:{x['us_median']}us" for x in r["per_m"][:-1]),
      "batched:", r["config2_m1_batched"]["us_per_problem_median"], flush=True)
