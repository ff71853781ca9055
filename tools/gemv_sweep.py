"""Decode GEMV tuning sweep -- development tool, not part of the product.

For each Llama-2-7B decode shape, rotates enough distinct weight copies to defeat the 256 MB Infinity Cache, captures
`reps` launches in one HIP graph and reports device time per launch (HIP events on the launch stream) and GB/s of
algorithmic bytes, for every configuration given as NAME=VAL[,NAME=VAL...] env settings (NAD_GEMV_*).  With --trace
(phase-trace library, `make -C neural_amd trace`) it also prints per-workgroup phase spans of the last launch.

Usage: python tools/gemv_sweep.py [--trace] [--shapes qkv,o,...] CONFIG [CONFIG ...]
       CONFIG e.g. "base"  or  "NAD_GEMV_WAVES=8,NAD_GEMV_WPC=2"
"""
import argparse
import ctypes as C
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--trace", action="store_true")
ap.add_argument("--shapes", default="qkv,o,gate_up,down,lm_head")
ap.add_argument("--reps", type=int, default=64)
ap.add_argument("configs", nargs="*")
args = ap.parse_args()
if args.trace:
    os.environ.setdefault("NAD_LIB_PATH", os.path.join(REPO, "neural_amd", "libneural_amd_trace.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from neural_amd import _lib, bestla  # noqa: E402

G = int(os.environ.get("SWEEP_GROUP", "128"))  # quantization group of the synthetic weights
BITS = int(os.environ.get("SWEEP_BITS", "4"))  # weight bits (4, or 2 for the Mistral int2 policy)
SHAPES = {  # name: (n, k, weights per launch)
    "qkv": (4096, 4096, 3), "o": (4096, 4096, 1), "gate_up": (11008, 4096, 2), "down": (4096, 11008, 1), "down14": (4096, 14336, 1),
    "lm_head": (32000, 4096, 1)}


def wbytes(n, k):
    return n * k * BITS // 8 + n * (k // G) * 2


def set_env(cfg):
    for k in list(os.environ):
        if k.startswith("NAD_GEMV_"):
            del os.environ[k]
    if cfg and cfg != "base":
        for kv in cfg.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    _lib.reload_knobs()  # the library reads its switches once


def main():
    dev = torch.device("cuda")
    x = torch.empty((1, 16384), device=dev).uniform_(-1, 1)
    configs = args.configs or ["base"]
    L = _lib.lib()
    if args.trace:
        L.nad_trace_fetch.restype = C.c_int
        L.nad_trace_fetch.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int]
        L.nad_trace_clock_khz.restype = C.c_int
        tick_us = 1e3 / L.nad_trace_clock_khz()
    print(f"{torch.cuda.get_device_name()}  reps {args.reps}")
    for name in args.shapes.split(","):
        n, k, nw = SHAPES[name]
        per = nw * wbytes(n, k) + 4 * (k + nw * n)
        copies = max(2, math.ceil(600e6 / per))
        if os.environ.get("SWEEP_COPIES"):  # e.g. 1-2: weights stay in the Infinity Cache (warm-MALL experiment)
            copies = int(os.environ["SWEEP_COPIES"])
        ws = [[bestla.DeviceWeight.synthetic(BITS, n, k, G, "fp16", False, seed=1000 * i + j) for j in range(nw)]
              for i in range(copies)]
        xa = x[:, :k].contiguous()
        out = torch.empty((3, 1, n), device=dev)
        tmp = torch.empty((2, 1, n), device=dev)

        def launch(i):
            w = ws[i % copies]
            if name == "qkv":
                bestla.qkv_forward(xa, w[0], w[1], w[2], out=out)
            elif name == "gate_up":
                # the dual gate/up launch alone: nad_device_ffn_forward's first kernel, via the C-ABI
                r = L.nad_device_ffn_gate_up(xa.data_ptr(), 0, w[0].desc, w[1].desc, tmp[0].data_ptr(),
                                             tmp[1].data_ptr(), 1, k, n, k, 2, torch.cuda.current_stream().cuda_stream)
                assert r == 0, _lib.last_error()
            else:
                w[0].forward(xa, out=out[0])

        print(f"\n== {name}: N={n} K={k} x{nw}, {per / 1e6:.2f} MB/launch, {copies} copies")
        for cfg in configs:
            set_env(cfg)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for i in range(copies):
                    launch(i)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for i in range(args.reps):
                        launch(i)
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(3):
                    g.replay()
                e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (3 * args.reps)
            print(f"  {cfg:48s} {us:8.2f} us  {per / us / 1e3:8.1f} GB/s")
            del g
            if args.trace:
                buf = np.zeros((8, 16384), np.uint64)
                assert L.nad_trace_fetch(None, 0, 1, 0) == 0
                with torch.cuda.stream(s):
                    for i in range(copies):
                        launch(i)
                assert L.nad_trace_fetch(buf.ctypes.data, buf.nbytes, 0, 0) == 0
                nz = buf[0] > 0
                grid = int(nz.sum())
                s0, s1, s2, s3, s4 = (buf[i, :grid].astype(np.int64) for i in range(5))
                t0 = s0.min()
                q = lambda v: "p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f" % tuple(  # noqa: E731
                    np.percentile(v * tick_us, [10, 50, 90, 100]))
                print(f"    traced span {(s3.max() - t0) * tick_us:7.2f} us, grid {grid}")
                print(f"    wg start offset   {q(s0 - t0)}")
                print(f"    A + stage0 issued {q(s4 - s0)}")
                print(f"    A staged (->bar)  {q(s1 - s0)}")
                print(f"    main loop         {q(s2 - s1)}")
                print(f"    reduce+epilogue   {q(s3 - s2)}")
                print(f"    wg end offset     {q(s3 - t0)}")
        set_env(None)
        del ws


if __name__ == "__main__":
    main()
