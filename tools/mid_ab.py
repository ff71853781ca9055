"""Mid-M A/B (development tool): bench.py's synthetic cold-rotation graph timing (K = N = 4096 int4 g128, fp16
activations) per M, alternating runtime knob settings inside one process.

Usage: python tools/mid_ab.py [--m 17,32,48,64] [--rounds 3] [--knob NAD_MID_XCD] [--values 0,1] [--n 4096] [--act fp16]
Each line: round, knob value, M, median / min us per launch over the graph replays.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="17,32,48,64")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--knob", default="NAD_MID_XCD")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--copies", type=int, default=128)
    ap.add_argument("--act", default="fp16", help="activation dtype: fp16, bf16 or fp32")
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--bits", type=int, default=4)
    args = ap.parse_args()
    import torch
    import bench
    from neural_amd import _lib, bestla
    K, N = 4096, args.n
    ws = [bestla.DeviceWeight.synthetic(args.bits, N, K, args.group, "fp16", False, seed=9000 + i)
          for i in range(args.copies)]
    gen = torch.Generator(device="cpu").manual_seed(11)
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[args.act]
    xs = {m: (torch.rand((m, K), generator=gen) - 0.5).to(dt).cuda() for m in map(int, args.m.split(","))}
    for r in range(args.rounds):
        for v in args.values.split(","):
            os.environ[args.knob] = v
            _lib.reload_knobs()
            for m, x in xs.items():
                y = torch.empty((m, N), dtype=torch.float32, device="cuda")
                n = 128

                def fn(st, x=x, y=y, n=n):
                    for i in range(n):
                        ws[i % args.copies].forward(x, out=y, stream=st)
                per = sorted(t / n for t in bench.graph_times(fn, 5, torch))
                print(f"round {r} {args.knob}={v} M={m:4d} median {per[len(per) // 2] * 1e6:7.2f} us  "
                      f"min {per[0] * 1e6:7.2f}", flush=True)


if __name__ == "__main__":
    main()
