"""Batch-size sweep of one WOQ linear (development tool): device time per forward of a K x N int4 g128 weight at
M = 1 .. 4096 (the SURVEY.md §8(d) GEMM config), cold weights (rotating copies past the 256 MB Infinity Cache), HIP
graph replay, HIP events on the launch stream.  Prints per M: us, GB/s of algorithmic bytes (bestla_benchmark.cpp
formula, act bytes at the given dtype), TFLOP/s, and which path nad_device_forward takes.

Usage: python tools/m_sweep.py [--m 1,2,...] [--act fp16|fp32] [--n 4096] [--k 4096] [--bits 4] [--group 128]
"""
import argparse
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="1,2,4,8,16,17,24,32,48,64,96,128,192,256,512,1024,2048,4096")
    ap.add_argument("--act", default="fp16")
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--reps", type=int, default=32)
    ap.add_argument("--mb", type=float, default=400.0, help="MB of rotated weight copies (past 256 MB: cold)")
    args = ap.parse_args()
    import torch
    from neural_amd import bestla
    n, k, g, bits = args.n, args.k, args.group, args.bits
    wb = n * k * bits // 8 + n * math.ceil(k / g) * 2
    copies = max(2, math.ceil(args.mb * 1e6 / wb))
    ws = [bestla.DeviceWeight.synthetic(bits, n, k, g, "fp16", False, seed=77 + i) for i in range(copies)]
    dt = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[args.act]
    esz = torch.tensor([], dtype=dt).element_size()
    print(f"{torch.cuda.get_device_name()}  N={n} K={k} int{bits} g{g} act {args.act}, {copies} weight copies")
    for m in [int(v) for v in args.m.split(",")]:
        x = (torch.rand((m, k), device="cuda") - 0.5).to(dt)
        out = torch.empty((m, n), device="cuda")
        reps = args.reps if m <= 256 else max(4, args.reps // 4)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(min(copies, reps)):
                ws[i % copies].forward(x, out=out)
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph, stream=s):
                for i in range(reps):
                    ws[i % copies].forward(x, out=out)
            gph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(3):
                gph.replay()
            e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (3 * reps)
        byts = wb + m * k * esz + m * n * 4
        print(f"  M={m:5d} {us:9.2f} us {byts / us / 1e3:8.1f} GB/s {2 * m * n * k / us / 1e6:8.1f} TFLOP/s", flush=True)
        del gph


if __name__ == "__main__":
    main()
