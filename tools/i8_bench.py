"""int8-compute mode timing (development tool): one Llama-2-7B-shaped linear quantized with the reference Python
default (int4, group 32, sym, compute int8) by the product packer, timed in compute mode 0 (fp16 MFMA on exact weights)
and mode 1 (the reference's u8 x s8 kblock arithmetic), at decode and prefill M.  Also a GGUF Q4_0 matrix of the same
shape (Q8_0 x Q4_0 in mode 1).

Usage: python tools/i8_bench.py [--shapes o,gate] [--m 1,16,2048] [--reps 20]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
SHAPES = {"o": (4096, 4096), "gate": (11008, 4096), "down": (4096, 11008)}


def q4_0_blocks(W):
    """numpy restatement of quantize_row_q4_0_reference for synthetic inputs (timing only)"""
    n, k = W.shape
    x = W.reshape(n, k // 32, 32)
    idx = np.abs(x).argmax(axis=2)
    mx = np.take_along_axis(x, idx[..., None], axis=2)[..., 0]
    d = (mx / -8).astype(np.float32)
    idv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0).astype(np.float32)
    q = np.minimum(15, (x * idv[..., None] + 8.5).astype(np.int8)).astype(np.uint8)
    out = np.zeros((n, k // 32, 18), np.uint8)
    out[:, :, :2] = d.astype(np.float16).view(np.uint8).reshape(n, k // 32, 2)
    out[:, :, 2:] = q[:, :, :16] | (q[:, :, 16:] << 4)
    return out.reshape(n, -1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="o,gate")
    ap.add_argument("--m", default="1,16,2048")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from neural_amd import bestla
    rng = np.random.default_rng(0)
    for name in args.shapes.split(","):
        n, k = SHAPES[name]
        W = rng.uniform(-1, 1, size=(n, k)).astype(np.float32)
        weights = {"btla_g32_int8comp": bestla.DeviceWeight(bestla.quantize(W, 32, "int4", "fp32", "sym", "int8")),
                   "gguf_q4_0": bestla.DeviceWeight.from_q4_0(q4_0_blocks(W), n, k)}
        for wname, w in weights.items():
            for m in (int(v) for v in args.m.split(",")):
                x = torch.rand((m, k), device="cuda") - 0.5
                out = torch.empty((m, n), device="cuda")
                for mode in (0, 1):
                    bestla.set_compute_mode(mode)
                    for _ in range(3):
                        w.forward(x, out=out)
                    s = torch.cuda.current_stream()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record(s)
                    for _ in range(args.reps):
                        w.forward(x, out=out)
                    e1.record(s)
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / args.reps
                    gbs = (n * k / 2 + n * k / 32 * 4) / us / 1e3
                    tf = 2.0 * m * n * k / us / 1e6
                    print(f"{name:5s} {wname:18s} M={m:5d} mode{mode}: {us:9.1f} us  {gbs:7.0f} GB/s(weights)  "
                          f"{tf:7.1f} TFLOP/s", flush=True)
                bestla.set_compute_mode(0)


if __name__ == "__main__":
    main()
